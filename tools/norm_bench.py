"""Microbenchmark of the InstanceNorm forward / backward entries (vst_instnorm_fwd / _bwd) on the
config-3 plane shapes, optionally across library builds.  Interleaved rounds, HIP-event timing;
prints ms per call and the effective HBM rate of the plane-sized transfers the kernel makes.

    python tools/norm_bench.py [lib.so ...]
"""
import ctypes
import statistics
import sys

import torch

sys.path.insert(0, "video-style-transfer_amd")
from vst._lib import LIB_PATH, _CTYPES, parse_header  # noqa: E402

# name, N, C, H, W, relu (the ReCoNet planes: conv1 / deconv2 output, conv2 / deconv1 output, residual)
SHAPES = [
    ("full48", 16, 48, 256, 512, 1),
    ("half96", 16, 96, 128, 256, 1),
    ("res192", 16, 192, 64, 128, 1),
]


def load(path):
    lib = ctypes.CDLL(path)
    for name, (rt, argts) in parse_header().items():
        fn = getattr(lib, name, None)
        if fn is not None:
            fn.restype = _CTYPES[rt] if rt != "char*" else ctypes.c_char_p
            fn.argtypes = [_CTYPES[a] for a in argts]
    return lib


def main():
    paths = sys.argv[1:] or [LIB_PATH]
    libs = [load(p) for p in paths]
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    bufs = {}
    for name, N, C, H, W, relu in SHAPES:
        x = torch.randn(N, C, H, W, device="cuda")
        w = 1 + 0.1 * torch.randn(C, device="cuda")
        b = 0.1 * torch.randn(C, device="cuda")
        y = torch.empty_like(x)
        stats = torch.empty(N * C * 2, device="cuda")
        gy = torch.randn_like(x)
        gx = torch.empty_like(x)
        gw, gb = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
        part = torch.empty(N * C * 3, device="cuda")
        bufs[name] = (x, w, b, y, stats, gy, gx, gw, gb, part)
    outs = {}
    for _ in range(5):
        for p, lib in zip(paths, libs):
            for name, N, C, H, W, relu in SHAPES:
                x, w, b, y, stats, gy, gx, gw, gb, part = bufs[name]
                fwd = (x.data_ptr(), w.data_ptr(), b.data_ptr(), None, y.data_ptr(), stats.data_ptr(), N, C, H * W,
                       1e-5, relu, st)
                bwd = (gy.data_ptr(), x.data_ptr(), None, b.data_ptr(), stats.data_ptr(), w.data_ptr(), gx.data_ptr(),
                       gw.data_ptr(), gb.data_ptr(), None, part.data_ptr(), N, C, H * W, relu, 0, st)
                for tag, fn, args in (("fwd", lib.vst_instnorm_fwd, fwd), ("bwd", lib.vst_instnorm_bwd, bwd)):
                    assert fn(*args) == 0
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(5):
                        fn(*args)
                    e1.record()
                    torch.cuda.synchronize()
                    res.setdefault((p, name, tag), []).append(e0.elapsed_time(e1) / 5)
                outs[(p, name)] = (gx.clone(), gw.clone(), gb.clone())
    for name, N, C, H, W, relu in SHAPES:
        plane_bytes = 4.0 * N * C * H * W
        for tag, nplanes in (("fwd", 2), ("bwd", 3)):  # one-pass floor: x -> y; gy, x -> gx
            line = f"{name:8s} {tag}"
            for p in paths:
                ms = statistics.median(res[(p, name, tag)])
                line += f"  {ms * 1e3:7.1f} us"
            print(line + f"   (one-pass floor {nplanes * plane_bytes / 1e6:.0f} MB)")
        if len(paths) > 1:
            a = outs[(paths[0], name)]
            for p in paths[1:]:
                bq = outs[(p, name)]
                print(f"{name:8s} vs {p}: max |dgx| {(a[0] - bq[0]).abs().max().item():.3e} "
                      f"rel {((a[0] - bq[0]).norm() / a[0].norm()).item():.3e}; "
                      f"dgw {(a[1] - bq[1]).abs().max().item():.3e} dgb {(a[2] - bq[2]).abs().max().item():.3e}")


if __name__ == "__main__":
    main()
