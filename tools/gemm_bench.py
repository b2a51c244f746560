import os
"""Microbenchmark of the implicit-GEMM conv kernel on the step's layer shapes, across library
builds (tuning variants compiled with different -D flags).  Interleaved rounds in one process.

    python tools/gemm_bench.py video-style-transfer_amd/vst/libvst_hip.so video-style-transfer_amd/vst/variants/*.so
"""
import ctypes
import statistics
import sys

import torch

# GEMM arithmetic passed to every call (vst_hip.h VST_GEMM_*): 0 f32, 1 bf16x3, 2 bf16, 3 bf16x6
# (BENCH_GEMM_MODES="3,19": one column per mode and library; 19 = bf16x6 | VST_GEMM_KBLOCK)
MODES = [int(m) for m in os.environ.get("BENCH_GEMM_MODES", os.environ.get("BENCH_GEMM_MODE", "3")).split(",")]

sys.path.insert(0, "video-style-transfer_amd")
from vst._lib import _CTYPES, parse_header  # noqa: E402

# name, N, Cs, Hs, Ws, M, KH, KW, Ho, Wo, gmode, stride, pad, up, algo_flops
SHAPES = []


def conv(name, N, Cin, H, W, Cout, k, stride=1, pad_mode="reflect", up=1):
    pad = k // 2
    Ho = (H * up + 2 * pad - k) // stride + 1
    Wo = (W * up + 2 * pad - k) // stride + 1
    fl = 2.0 * N * Cout * Ho * Wo * Cin * k * k
    SHAPES.append((name + ".fwd", N, Cin, H, W, Cout, k, k, Ho, Wo, 0 if pad_mode == "reflect" else 1, stride, pad, up, fl))
    if pad_mode == "zero":
        SHAPES.append((name + ".dgrad", N, Cout, Ho, Wo, Cin, k, k, H, W, 2, stride, pad, 1, fl))
    else:
        SHAPES.append((name + ".dgrad", N, Cout, Ho, Wo, Cin, k, k, H * up + 2 * pad, W * up + 2 * pad, 2, stride, 0, 1, fl))


conv("vgg1_2", 16, 64, 256, 512, 64, 3, pad_mode="zero")
conv("vgg2_2", 16, 128, 128, 256, 128, 3, pad_mode="zero")
conv("vgg3_2", 16, 256, 64, 128, 256, 3, pad_mode="zero")
conv("vgg4_2", 16, 512, 32, 64, 512, 3, pad_mode="zero")
conv("res", 16, 192, 64, 128, 192, 3)
conv("deconv1", 16, 192, 64, 128, 96, 3, up=2)
conv("deconv2", 16, 96, 128, 256, 48, 3, up=2)
conv("conv2", 16, 48, 256, 512, 96, 3, stride=2)
conv("conv3", 16, 96, 128, 256, 192, 3, stride=2)
# AdaAttN config 4 (4 triples at 256x512: 8 content images) decoder 3x3 layers and VGG19 conv4 / conv5
conv("aa4_dec256", 8, 256, 32, 64, 256, 3)
conv("aa4_dec128", 8, 128, 64, 128, 128, 3)
conv("aa4_vgg4", 12, 512, 32, 64, 512, 3, pad_mode="zero")
conv("aa4_vgg5", 12, 512, 16, 32, 512, 3, pad_mode="zero")
# VGG conv1_1 over the kw-unfolded input (3 channels x 3 kw, padded to 16): K = 48, output-bound
# (KW = 1 with pad 1 shifts the columns by one -- same cost as the real pad_x = 0 launch)
SHAPES.append(("vgg1_1u.fwd", 16, 16, 256, 512, 64, 3, 1, 256, 512, 1, 1, 1, 1, 2.0 * 16 * 64 * 256 * 512 * 48))


def load(path):
    lib = ctypes.CDLL(path)
    for name, (rt, argts) in parse_header().items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = _CTYPES[rt] if rt != "char*" else ctypes.c_char_p
        fn.argtypes = [_CTYPES[a] for a in argts]
    return lib


def main():
    paths = sys.argv[1:]
    libs = [load(p) for p in paths]
    cols = [(p, lib, m) for p, lib in zip(paths, libs) for m in MODES]
    dev = "cuda"
    st = torch.cuda.current_stream().cuda_stream
    only = os.environ.get("BENCH_ONLY")  # comma-separated substrings of the shape names to run
    sel = (lambda nm: any(o in nm for o in only.split(","))) if only else (lambda nm: True)
    results = {(p, m, s[0]): [] for p in paths for m in MODES for s in SHAPES}
    bufs = {}
    for s in SHAPES:
        name, N, Cs, Hs, Ws, M, KH, KW, Ho, Wo, gm, stride, pad, up, fl = s
        if not sel(name):
            continue
        src = torch.randn(N, Cs, Hs, Ws, device=dev)
        out = torch.empty(N, M, Ho, Wo, device=dev)
        bufs[name] = (src, out)
    for rnd in range(3):
        for p, lib, MODE in cols:
            for s in SHAPES:
                name, N, Cs, Hs, Ws, M, KH, KW, Ho, Wo, gm, stride, pad, up, fl = s
                if not sel(name):
                    continue
                src, out = bufs[name]
                mp, kp = ctypes.c_int(), ctypes.c_int()
                lib.vst_conv_pack_dims(M, KH * KW * Cs, ctypes.byref(mp), ctypes.byref(kp))
                # packed A floats per mode (bf16x6 blocks are 96 B per 16 k, the others 64 B)
                pf = kp.value * mp.value * 3 // 2 if (MODE & 15) == 3 else kp.value * mp.value
                wp = torch.randn(pf, device=dev) * 0.05
                nb = lib.vst_conv_splitk_workspace(N, Cs, M, Ho, Wo, KH, KW, gm, stride, pad, pad, up, 0, 0, MODE)
                wsb = torch.empty((nb + 3) // 4, device=dev) if nb else None
                args = (src.data_ptr(), wp.data_ptr(), None, None, out.data_ptr(), N, Cs, Hs, Ws, M, KH * KW * Cs, Ho, Wo,
                        KH, KW, gm, stride, pad, up, 0, 0, None, None, None if wsb is None else wsb.data_ptr(), nb,
                        MODE, st)
                for _ in range(2):
                    assert lib.vst_conv_gemm(*args) == 0
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                reps = 5
                for _ in range(reps):
                    lib.vst_conv_gemm(*args)
                e1.record()
                torch.cuda.synchronize()
                results[(p, MODE, name)].append(e0.elapsed_time(e1) / reps)
    hdr = "shape".ljust(16) + "".join(
        (p.split("/")[-1].replace("libvst_hip", "").replace(".so", "")[:10] + f" m{m}").rjust(16) for p, _, m in cols)
    print(hdr)
    tot = {(p, m): 0.0 for p, _, m in cols}
    for s in SHAPES:
        if not sel(s[0]):
            continue
        line = s[0].ljust(16)
        for p, _, m in cols:
            ms = statistics.median(results[(p, m, s[0])])
            tot[(p, m)] += ms
            line += f"{ms*1e3:8.0f}us{s[-1]/ms/1e9:5.0f}TF".rjust(16)
        print(line)
    print("total".ljust(16) + "".join(f"{tot[(p, m)]:14.2f}ms" for p, _, m in cols))


if __name__ == "__main__":
    main()
