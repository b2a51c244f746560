"""Oracle = CPU restatement of the reference's hot path.  TEST INFRASTRUCTURE ONLY.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may import this
package, and only as the checker / the timed CPU baseline.  The product path
(`video-style-transfer_amd/vst`) never imports it and has no CPU fallback.

Pinned by golden vectors produced by running the reference itself in the build container
(`tests/golden/gen_golden.py`); see tests/test_oracle_golden.py.
"""
import torch

from . import adaattn_ref, reconet_ref, rtnstv_ref, seeding, shapes  # noqa: F401


def seeded_params(spec, seed, requires_grad=False):
    """{name: fp32 CPU tensor} for a shapes.* list, identical to gen_golden's seeding."""
    arrs = seeding.seeded_arrays(spec, seed)
    return {k: torch.from_numpy(v).requires_grad_(requires_grad) for k, v in arrs.items()}
