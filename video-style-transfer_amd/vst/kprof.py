"""Live per-kernel-family timing with HIP events (used by bench.py for the roofline line).

`conv_gemm` launches (forward + data-gradient implicit GEMM, `conv_gemm_kernel<...>`) record a
start/stop event pair on the stream they are launched on, plus their algorithmic FLOPs
(2 * N * Cout * Ho * Wo * Cin * k^2 of the reference convolution they implement, no padding or
stride-2 zero-tap redundancy counted) and algorithmic bytes (source + packed weights + output, once).
"""
import torch

_active = None


class KernelTimer:
    def __init__(self, detail=False):
        self.detail = detail
        self.records = []  # (start, stop, flops, family, algorithmic bytes, tag)

    def __enter__(self):
        global _active
        _active = self
        return self

    def __exit__(self, *exc):
        global _active
        _active = None

    def summary(self, family="conv_gemm"):
        torch.cuda.synchronize()
        recs = [r for r in self.records if r[3] == family]
        ms = sum(r[0].elapsed_time(r[1]) for r in recs)
        flops = sum(r[2] for r in recs)
        nbytes = sum(r[4] for r in recs)
        n = len(recs)
        return {"launches": n, "total_ms": ms, "avg_us": 1e3 * ms / max(n, 1), "flops": flops, "bytes": nbytes,
                "tflops": flops / (ms * 1e-3) / 1e12 if ms > 0 else 0.0}


    def by_tag(self, family="conv_gemm"):
        """{tag: [launches, ms, flops]} (detail mode)."""
        torch.cuda.synchronize()
        out = {}
        for r in self.records:
            if r[3] != family:
                continue
            a = out.setdefault(r[5], [0, 0.0, 0.0])
            a[0] += 1
            a[1] += r[0].elapsed_time(r[1])
            a[2] += r[2]
        return out


def begin(flops, nbytes=0.0, tag=None):
    """nbytes: algorithmic HBM bytes of the launch (each operand read once, output written once);
    tag: launch shape, kept only when the timer was created with detail=True."""
    if _active is None:
        return None
    s = torch.cuda.Event(enable_timing=True)
    s.record()
    return (s, flops, nbytes, tag if _active.detail else None)


def end(tok, family="conv_gemm"):
    if tok is None:
        return
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    _active.records.append((tok[0], e, tok[1], family, tok[2], tok[3]))
