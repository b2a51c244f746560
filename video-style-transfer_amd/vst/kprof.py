"""Live per-kernel-family timing with HIP events (used by bench.py for the roofline line).

`conv_gemm` launches (forward + data-gradient implicit GEMM, `conv_gemm_kernel<...>`) record a
start/stop event pair on the stream they are launched on, plus their algorithmic FLOPs
(2 * N * Cout * Ho * Wo * Cin * k^2 of the reference convolution they implement, no padding or
stride-2 zero-tap redundancy counted) and algorithmic bytes (source + packed weights + output, once).
"""
import torch

_active = None

# MFMA peak per GEMM arithmetic mode (vst_set_gemm_mode), in algorithmic fp32-operand TFLOP/s:
# f32 = v_mfma_f32_32x32x2_f32 (157.3 TF); bf16x3 = 3 bf16 MFMAs per product (2500 / 3);
# bf16 = 2500 (dense bf16 MFMA, MI355X_MICROARCH.md); bf16x6 = 6 bf16 MFMAs per product;
# f16 = 2500 (dense fp16 MFMA)
MODE_PEAK_TFLOPS = {0: 157.3, 1: 2500.0 / 3.0, 2: 2500.0, 3: 2500.0 / 6.0, 4: 2500.0}


class KernelTimer:
    def __init__(self, detail=False):
        self.detail = detail
        self.records = []  # (start, stop, flops, family, algorithmic bytes, tag, gemm mode)

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
        # effective peak of a mixed-mode launch set: the time the launches would take at their
        # modes' peaks, flops / sum(flops_i / peak_i)
        by_mode = {}
        for r in recs:
            a = by_mode.setdefault(r[6] & 7 if r[6] is not None else r[6], [0, 0.0, 0.0])  # arithmetic bits only
            a[0] += 1
            a[1] += r[0].elapsed_time(r[1])
            a[2] += r[2]
        t_peak = sum(f / (MODE_PEAK_TFLOPS.get(m, 157.3) * 1e12) for m, (_, _, f) in by_mode.items())
        return {"launches": n, "total_ms": ms, "avg_us": 1e3 * ms / max(n, 1), "flops": flops, "bytes": nbytes,
                "tflops": flops / (ms * 1e-3) / 1e12 if ms > 0 else 0.0,
                "peak_tflops": flops / t_peak / 1e12 if t_peak > 0 else 157.3,
                "by_mode": {m: {"launches": c, "ms": t, "gflop": f / 1e9, "tflops": f / (t * 1e-3) / 1e12 if t > 0 else 0.0}
                            for m, (c, t, f) in by_mode.items()}}


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


def begin(flops, nbytes=0.0, tag=None, mode=None):
    """nbytes: algorithmic HBM bytes of the launch (each operand read once, output written once);
    tag: launch shape, kept only when the timer was created with detail=True; mode: the GEMM
    arithmetic mode of the launch."""
    if _active is None:
        return None
    s = torch.cuda.Event(enable_timing=True)
    s.record()
    return (s, flops, nbytes, tag if _active.detail else None, mode)


def end(tok, family="conv_gemm"):
    if tok is None:
        return
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    _active.records.append((tok[0], e, tok[1], family, tok[2], tok[3], tok[4]))
