"""Time the stride-1 reflect-pad data gradient of the residual convs (RC/network.py:145-150) on its
two paths: the padded-grid GEMM (conv_dgrad_padout: per-tap kernel, interior + border side buffer)
and core + ring (conv_dgrad_ring: the 3x3 core on the halo kernel, the padded grid's border ring as
small GEMMs folded into dx's border band).  bf16x6 policy; interleaved rounds, median."""
import statistics
import sys

import torch

sys.path.insert(0, "video-style-transfer_amd")
from vst import ops  # noqa: E402


def main():
    ops.use_policy("bf16x6")
    dev = "cuda"
    N, C, H, W = 16, 192, 64, 128
    gz = torch.randn(N, C, H, W, device=dev)
    w = torch.randn(C, C, 3, 3, device=dev) * 0.05
    flops = 2.0 * N * C * H * W * C * 9
    paths = {"padout": lambda: ops.conv_dgrad_padout(gz, w, (N, C, H, W), 3, 1, flops),
             "ring": lambda: ops.conv_dgrad_ring(gz, w, (N, C, H, W), 3, 1, flops)}
    with ops.gemm_scope("stylizer"), ops.gemm_scope("res"):
        ops.gemm_role("dgrad")
        out = {k: f() for k, f in paths.items()}
        torch.cuda.synchronize()
        d = float((out["padout"] - out["ring"]).abs().max() / out["padout"].abs().max())
        times = {k: [] for k in paths}
        for _ in range(5):
            for k, f in paths.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    f()
                e1.record()
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) / 5)
    for k, v in times.items():
        ms = statistics.median(v)
        print(f"{k:8s} {ms*1e3:8.1f} us  {flops/ms/1e9:6.1f} TF/s")
    print(f"max |padout - ring| / max |padout| = {d:.2e}")


if __name__ == "__main__":
    main()
