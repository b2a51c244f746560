"""Error of the GEMM kernels in each arithmetic mode vs an fp64 reference (diagnostic)."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, "video-style-transfer_amd")
from vst import ops  # noqa: E402
from vst.adaattn.attention import gemm_abt  # noqa: E402

g = torch.Generator().manual_seed(0)
x = torch.randn(2, 64, 16, 24, generator=g)
w = torch.randn(96, 64, 3, 3, generator=g) * 0.05
ref = F.conv2d(x.double(), w.double(), padding=1)
a = torch.randn(2, 40, 300, generator=g)
b = torch.randn(2, 56, 300, generator=g)
refg = torch.bmm(a.double(), b.double().transpose(1, 2))
for mode in ("f32", "bf16x6", "bf16x3", "bf16"):
    ops.set_gemm_mode(mode)
    y = ops.conv2d(x.cuda(), w.cuda(), None, pad=1).cpu().double()
    e = ((y - ref).abs().max() / ref.abs().max()).item()
    z = gemm_abt(a.cuda(), b.cuda()).cpu().double()
    e2 = ((z - refg).abs().max() / refg.abs().max()).item()
    print(f"{mode:7s} conv fwd rel err {e:.3e}   gemm_abt rel err {e2:.3e}", flush=True)
