"""Where does the data-parallel gradient sum differ from the sum of the single-process shard gradients?
Runs tests/test_gpu_ddp.py's two-rank gloo step on cuda:0 and prints the parameters whose summed
gradient differs, largest first.  usage: python tools/ddp_diag.py [reconet|adaattn]"""
import os
import sys
import tempfile

import numpy as np
import torch
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-style-transfer_amd"), os.path.join(REPO, "tests")]

import test_gpu_ddp as T  # noqa: E402


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "reconet"
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(T._worker, args=(2, T._free_port(), d, kind), nprocs=2, join=True)
        g_dp = np.load(os.path.join(d, "g0.npy"))
    gs = []
    for r in (0, 1):
        tr = T._trainer(kind)
        tr.flat.zero_grad()
        out = tr.losses(*T._batch(kind, r))
        out["loss"].backward()
        torch.cuda.synchronize()
        gs.append(tr.flat.g.cpu().numpy().copy())
    gsum = gs[0] + gs[1]
    names = [(n, p.numel()) for n, p in tr.model.named_parameters()]
    offs = 0
    rows = []
    gmax = np.abs(gsum).max()
    for n, k in names:
        a, b = g_dp[offs:offs + k], gsum[offs:offs + k]
        e = np.abs(a - b).max()
        rows.append((e / gmax, e / max(np.abs(b).max(), 1e-30), n, np.abs(b).max(), int((a != b).sum()), k))
        offs += k
    rows.sort(reverse=True)
    for r in rows[:15]:
        print(f"{r[2]:40s} err/gmax {r[0]:.2e} err/own {r[1]:.2e} own max {r[3]:.3e} differing {r[4]}/{r[5]}")
    s0 = np.abs(gs[0]).max()
    print("flat offsets check:", offs, g_dp.size)


if __name__ == "__main__":
    main()
