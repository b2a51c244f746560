"""Time vst_resize_bilinear on the config-5 (AdaAttN, B=8, 512x1024) shapes: the decoder's x2 upsamples
and the attention keys' downsamples (AA/utilities.py:98-109), with the HBM rate of each launch
(bytes = the output written + the input rows the bilinear taps touch)."""
import sys

import torch

sys.path.insert(0, "video-style-transfer_amd")
from vst import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = "cuda"
cases = [  # (C, H, W, Ho, Wo)
    (512, 32, 64, 64, 128), (256, 64, 128, 128, 256), (128, 128, 256, 256, 512), (64, 256, 512, 512, 1024),
    (64, 512, 1024, 128, 256), (128, 256, 512, 128, 256),
    (64, 512, 1024, 64, 128), (128, 256, 512, 64, 128), (256, 128, 256, 64, 128),
    (64, 512, 1024, 32, 64), (128, 256, 512, 32, 64), (256, 128, 256, 32, 64), (512, 64, 128, 32, 64),
]
tot = 0.0
for C, H, W, Ho, Wo in cases:
    x = torch.randn(B, C, H, W, device=dev)
    for _ in range(3):
        y = ops.resize_bilinear(x, (Ho, Wo))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    e0.record()
    for _ in range(n):
        y = ops.resize_bilinear(x, (Ho, Wo))
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000 / n
    rows = min(H, 2 * Ho)  # input rows a launch touches
    nbytes = 4.0 * B * C * (Ho * Wo + rows * W)
    tot += us
    print(f"C={C:4d} {H}x{W} -> {Ho}x{Wo}: {us:8.1f} us  {nbytes / us / 1e6:6.2f} TB/s", flush=True)
print(f"sum {tot:.1f} us")

# reference points: a pure write (fill_) and a copy of the largest output; the per-element kernel on
# the upsample shapes (a misaligned input routes the call to it)
y = torch.empty(B, 64, 512, 1024, device=dev)
for name, fn, nbytes in (("fill", lambda: y.fill_(1.0), y.numel() * 4.0),
                         ("copy", lambda: y.copy_(y2), y.numel() * 8.0)) if (y2 := torch.empty_like(y)) is not None else ():
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000 / 20
    print(f"{name} {nbytes / 1e9:.2f} GB: {us:8.1f} us  {nbytes / us / 1e6:6.2f} TB/s", flush=True)
del y, y2
for C, H, W, Ho, Wo in cases[:4]:
    buf = torch.randn(B * C * H * W + 4, device=dev)
    x = buf[1:1 + B * C * H * W].view(B, C, H, W)
    for _ in range(3):
        ops.resize_bilinear(x, (Ho, Wo))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.resize_bilinear(x, (Ho, Wo))
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000 / 20
    nbytes = 4.0 * B * C * (Ho * Wo + H * W)
    print(f"per-element C={C:4d} {H}x{W} -> {Ho}x{Wo}: {us:8.1f} us  {nbytes / us / 1e6:6.2f} TB/s", flush=True)

# torch's own upsample (a reference point for the achievable rate of this access pattern)
import torch.nn.functional as F  # noqa: E402
for C, H, W, Ho, Wo in cases[:4]:
    x = torch.randn(B, C, H, W, device=dev)
    for _ in range(3):
        F.interpolate(x, size=(Ho, Wo), mode="bilinear", align_corners=False)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        F.interpolate(x, size=(Ho, Wo), mode="bilinear", align_corners=False)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000 / 20
    nbytes = 4.0 * B * C * (Ho * Wo + H * W)
    print(f"torch C={C:4d} {H}x{W} -> {Ho}x{Wo}: {us:8.1f} us  {nbytes / us / 1e6:6.2f} TB/s", flush=True)

# the x2 upsample's adjoint (with the fused ReLU mask, as the decoder calls it)
for C, H, W, Ho, Wo in cases[:4]:
    x = torch.randn(B, C, H, W, device=dev)
    gout = torch.randn(B, C, Ho, Wo, device=dev)
    for _ in range(3):
        ops.upsample2x_bwd(gout, x, relu_mask=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.upsample2x_bwd(gout, x, relu_mask=True)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000 / 20
    nbytes = 4.0 * B * C * (Ho * Wo + 2 * H * W)
    print(f"up2 bwd C={C:4d} {H}x{W} <- {Ho}x{Wo}: {us:8.1f} us  {nbytes / us / 1e6:6.2f} TB/s", flush=True)
