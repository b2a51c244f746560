"""hipGraph capture of the config-3 training step (torch.cuda.graph over the whole sync-free step:
forward, autograd backward with the side-stream weight gradients, Adam) vs eager issue, A/B/A/B on
one box.  Also checks that a replay computes what the eager step computes on the same state and
batch (loss terms and flat gradient bitwise: the step has no float atomics).

    python tools/graph_ab.py [steps]        (GPU; one JSON line)
"""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-style-transfer_amd")]


def main():
    from vst import ops
    from vst.reconet import network as N
    from vst.reconet.train import ReCoNetTrainer
    from vst.synthetic import frame_pair_parts, style_image

    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    ops.use_policy("bf16x6")
    dev = torch.device("cuda")
    B, H, W = 8, 256, 512
    tr = ReCoNetTrainer.for_script("train_candy", N.ReCoNet().to(dev), N.Vgg16().to(dev), style_image(7, H, W).to(dev))
    batches = []
    for i in range(6):
        img1, img2, f01, f10, motion = (t.to(dev) for t in frame_pair_parts(1234 + i, B, H, W))
        mask = torch.stack([ops.flow_warp_mask(f01[b], f10[b]) for b in range(B)]) * motion
        batches.append((torch.stack([img1, img2]).contiguous(), f10.contiguous(), mask.contiguous()))
    static = tuple(t.clone() for t in batches[0])

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for i in range(3):
            tr.step(*batches[i % len(batches)])
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()

    # capture
    g = torch.cuda.CUDAGraph()
    state = (tr.flat.p.clone(), tr.flat.m.clone(), tr.flat.v.clone(), tr.step_count)
    with torch.cuda.graph(g):
        gout = tr.step(*static)
    torch.cuda.synchronize()

    # replay == eager on the same state and batch (losses, flat gradient)
    def restore():
        tr.flat.p.copy_(state[0])
        tr.flat.m.copy_(state[1])
        tr.flat.v.copy_(state[2])
        tr.step_count = state[3]

    restore()
    for s, b in zip(static, batches[1]):
        s.copy_(b)
    g.replay()
    torch.cuda.synchronize()
    rep = ({k: float(v) for k, v in gout.items()}, tr.flat.g.clone())
    restore()
    eo = tr.step(*batches[1])
    torch.cuda.synchronize()
    eag = ({k: float(v) for k, v in eo.items()}, tr.flat.g.clone())
    check = {"loss_equal": rep[0] == eag[0], "grad_bitwise": bool(torch.equal(rep[1], eag[1])),
             "grad_maxdiff": float((rep[1] - eag[1]).abs().max()), "losses": [rep[0]["loss"], eag[0]["loss"]]}

    def run_eager():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            tr.step(*batches[i % len(batches)])
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    def run_graph():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            for s, b in zip(static, batches[i % len(batches)]):
                s.copy_(b, non_blocking=True)
            g.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    res = {"eager_ms": [], "graph_ms": []}
    for _ in range(2):
        res["eager_ms"].append(run_eager())
        res["graph_ms"].append(run_graph())
    print(json.dumps({"check": check, **res}), flush=True)


if __name__ == "__main__":
    main()
