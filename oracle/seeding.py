"""Deterministic (numpy PCG64) parameters for parity tests.  TEST INFRASTRUCTURE ONLY.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may import
anything under `oracle/`.  The same (name, shape) list -> same arrays on every machine
and numpy version, so golden fixtures store a seed instead of megabytes of weights.

Rules (by state_dict key, in state_dict order, one shared generator):
  4-D  *.weight  (conv)         N(0, 1) * sqrt(2 / fan_in)        (He init)
  1-D  *.weight  (InstanceNorm) 1 + 0.1 * N(0, 1)
  1-D  *.bias                   0.1 * N(0, 1)
"""
import numpy as np


def seeded_arrays(named_shapes, seed):
    rng = np.random.default_rng(seed)
    out = {}
    for name, shape in named_shapes:
        shape = tuple(int(s) for s in shape)
        if len(shape) == 4:
            fan_in = shape[1] * shape[2] * shape[3]
            a = rng.standard_normal(shape) * np.sqrt(2.0 / fan_in)
        elif name.endswith("weight"):
            a = 1.0 + 0.1 * rng.standard_normal(shape)
        else:
            a = 0.1 * rng.standard_normal(shape)
        out[name] = a.astype(np.float32)
    return out


def seed_module(module, seed):
    """Overwrite every floating parameter/buffer of `module` in place; returns the dict."""
    import torch

    sd = module.state_dict()
    arrs = seeded_arrays([(k, v.shape) for k, v in sd.items() if v.is_floating_point()], seed)
    with torch.no_grad():
        for k, a in arrs.items():
            sd[k].copy_(torch.from_numpy(a))
    return arrs
