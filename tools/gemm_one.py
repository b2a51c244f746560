"""Run a few GEMM launches of one layer shape (for rocprofv3 PMC passes on a single kernel).

    python tools/gemm_one.py [fwd|dgrad|wgrad|attn|vgg1|vgg3|vgg3kb] [reps]

The GEMM policy comes from VST_GEMM_POLICY (default f32); vgg3kb runs the channel-blocked K order.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-style-transfer_amd")]

import torch  # noqa: E402

from vst import ops  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "fwd"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    g = torch.Generator(device="cuda").manual_seed(0)
    N, C, H, W = 16, 192, 64, 128
    if which.startswith("vgg"):
        C, H, W = {"vgg1": (64, 256, 512), "vgg3": (256, 64, 128), "vgg3kb": (256, 64, 128)}[which]
        N = 8
    x = torch.randn(N, C, H, W, device="cuda", generator=g)
    w = torch.randn(C, C, 3, 3, device="cuda", generator=g) * 0.05
    gy = torch.randn(N, C, H, W, device="cuda", generator=g)
    for _ in range(reps):
        if which == "fwd":
            with ops.gemm_scope("stylizer"):
                ops.gemm_role("fwd")
                ops.conv_gemm(x, ops.packed_weight(w, False), C, 3, H, W, ops.GM_REFLECT, 1, 1, 1)
        elif which.startswith("vgg"):
            scope = "stylizer" if which != "vgg3kb" else "vgg"
            with ops.gemm_scope(scope):
                ops.gemm_role("fwd")
                ops.conv_gemm(x, ops.packed_weight(w, False), C, 3, H, W, ops.GM_ZERO, 1, 1, 1)
        elif which == "dgrad":
            ops.gemm_role("dgrad")
            ops.conv_gemm(gy, ops.packed_weight(w, True), C, 3, H, W, ops.GM_TRANSPOSED, 1, 1, 1)
        elif which == "wgrad":
            ops.conv_wgrad(gy, x, w.shape, 3, 1, 1, "reflect", 1)
        elif which == "attn":
            from vst.adaattn.attention import bmm_at_b
            q = torch.randn(4, 448, 8192, device="cuda", generator=g)
            bmm_at_b(q, 8192, 448, False, q, 8192)
    torch.cuda.synchronize()
    print("done", which)


if __name__ == "__main__":
    main()
