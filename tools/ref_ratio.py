"""Oracle / reference CPU time ratio, measured in the BUILD CONTAINER (the reference never travels
to the GPU box): the reference's own train_candy.train() and train_video.train() loop bodies vs
the oracle restatement of the same step (oracle/reconet_ref.py, oracle/adaattn_ref.py), same
B=1 full-size synthetic inputs, same thread count, median of timed steps after a warm-up.

bench.py reports cpu_baseline = the oracle timed on the GPU box's host; this ratio relates that
number to the reference itself (reference time ~= oracle time / ratio).

    python tools/ref_ratio.py [--threads 8] [--steps 3]   -> profiles/r02_oracle_ref_ratio.json
"""
import argparse
import json
import os
import sys
import time
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(REPO, "tests", "golden"), REPO, os.path.join(REPO, "video-style-transfer_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gen_golden as GG  # noqa: E402  (reference loading helpers: stubs, recorders)


class _Clock:
    """tqdm stand-in: the reference calls set_postfix once per step, after adam.step()."""
    stamps = []

    def __init__(self, it, **_):
        self.it = it

    def __iter__(self):
        _Clock.stamps.append(time.perf_counter())
        return iter(self.it)

    def set_postfix(self, _d):
        _Clock.stamps.append(time.perf_counter())


def _median_step(stamps, warm):
    d = np.diff(stamps)[warm:]
    return float(np.median(d)), [float(x) for x in d]


def reference_reconet(H, W, steps, warm):
    from oracle.seeding import seed_module
    from vst.synthetic import frame_pair_batch, style_image

    GG._fresh_project(GG.RC_DIR)
    rc_util = GG._load("utilities", os.path.join(GG.RC_DIR, "utilities.py"))
    sys.modules["utilities"] = rc_util
    rc_net = GG._load("network", os.path.join(GG.RC_DIR, "network.py"))
    sys.modules["network"] = rc_net
    style = style_image(3, H, W)
    fake = types.ModuleType("datasets")
    fake.FlyingThings3D_Monkaa = lambda *a, **k: None
    fake.toTensor255 = lambda _i: style[0].clone()
    sys.modules["datasets"] = fake
    tc = GG._load("rc_ratio_candy", os.path.join(GG.RC_DIR, "train_single", "train_candy.py"))
    batch = frame_pair_batch(1234, 1, H, W, mask_fn=rc_util.flow_warp_mask)

    def net(n=1):
        m = rc_net.ReCoNet(n)
        seed_module(m, 1)
        return m

    def vgg(device="cpu"):
        v = rc_net.Vgg16(device)
        seed_module(v, 2)
        return v

    class _Img:
        BILINEAR = 2

        @staticmethod
        def open(_p):
            class _O:
                def convert(self, *_):
                    return self

                def resize(self, *_):
                    return self

            return _O()

    tc.device, tc.batch_size, tc.IMG_SIZE, tc.epoch_start, tc.epoch_end = "cpu", 1, (W, H), 1, 1
    tc.DataLoader = lambda *a, **k: [tuple(t.clone() for t in batch) for _ in range(warm + steps)]
    tc.ReCoNet, tc.Vgg16, tc.Image, tc.tqdm = net, vgg, _Img, _Clock
    _Clock.stamps = []
    save = torch.save
    torch.save = lambda *a, **k: None
    try:
        tc.train()
    finally:
        torch.save = save
    return _median_step(_Clock.stamps, warm)


def oracle_reconet(H, W, steps, warm):
    import oracle
    from oracle import reconet_ref as R
    from oracle import shapes
    from vst.synthetic import frame_pair_batch, style_image

    P = oracle.seeded_params(shapes.reconet(), 1, requires_grad=True)
    VP = oracle.seeded_params(shapes.vgg16(), 2)
    grams = R.style_grams(VP, style_image(3, H, W))
    img1, img2, flow, mask = frame_pair_batch(1234, 1, H, W, mask_fn=R.flow_warp_mask)
    state, stamps = {}, [time.perf_counter()]
    for _ in range(warm + steps):
        L = R.reconet_losses(P, VP, img1.clone(), img2.clone(), flow, mask, grams)
        for p in P.values():
            p.grad = None
        L["loss"].backward()
        with torch.no_grad():
            R.adam_step(P, {k: p.grad for k, p in P.items()}, state)
        stamps.append(time.perf_counter())
    return _median_step(stamps, warm)


def reference_adaattn(H, W, steps, warm):
    from oracle.seeding import seed_module
    from vst.synthetic import content_style_batch

    GG._fresh_project(GG.AA_DIR)
    for n in ("utilities", "vgg19", "network", "lossfn"):
        sys.modules[n] = GG._load(n, os.path.join(GG.AA_DIR, n + ".py"))
    fake = types.ModuleType("datasets")
    fake.VidevoWikiArt = lambda *a, **k: None
    sys.modules["datasets"] = fake
    tv = GG._load("aa_ratio_video", os.path.join(GG.AA_DIR, "train_video.py"))
    c1, c2, s = content_style_batch(99, 1, H, W)

    def net(activation="softmax"):
        m = sys.modules["network"].StylizingNetwork(activation)
        seed_module(m, 1)
        return m

    def vgg():
        v = sys.modules["vgg19"].VGG19()
        seed_module(v, 2)
        return v

    tv.EPOCH_START, tv.EPOCH_END = 1, 1
    tv.DataLoader = lambda *a, **k: [(c1.clone(), c2.clone(), s.clone()) for _ in range(warm + steps)]
    tv.StylizingNetwork, tv.VGG19, tv.tqdm = net, vgg, _Clock
    _Clock.stamps = []
    save = torch.save
    torch.save = lambda *a, **k: None
    try:
        tv.train()
    finally:
        torch.save = save
    return _median_step(_Clock.stamps, warm)


def oracle_adaattn(H, W, steps, warm):
    import oracle
    from oracle import adaattn_ref as A
    from oracle import reconet_ref as R
    from oracle import shapes
    from vst.synthetic import content_style_batch

    P = oracle.seeded_params(shapes.stylizing_network(), 1, requires_grad=True)
    VP = oracle.seeded_params(shapes.vgg19(), 2)
    c1, c2, s = content_style_batch(99, 1, H, W)
    state, stamps = {}, [time.perf_counter()]
    for _ in range(warm + steps):
        L = A.adaattn_losses(P, VP, c1, c2, s)
        for p in P.values():
            p.grad = None
        L["loss"].backward()
        with torch.no_grad():
            R.adam_step(P, {k: p.grad for k, p in P.items()}, state, lr=1e-4)
        stamps.append(time.perf_counter())
    return _median_step(stamps, warm)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r02_oracle_ref_ratio.json"))
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    res = {"host": f"build container, {a.threads} threads (os.cpu_count() = {os.cpu_count()})",
           "method": f"median of {a.steps} timed steps after {a.warmup} warm-up, B=1, 3x256x512, same seeded "
                     "weights and synthetic inputs; ratio = oracle step time / reference step time"}
    for kind, ref, orc in (("reconet", reference_reconet, oracle_reconet), ("adaattn", reference_adaattn, oracle_adaattn)):
        r, rs = ref(256, 512, a.steps, a.warmup)
        o, os_ = orc(256, 512, a.steps, a.warmup)
        res[kind] = o / r
        res[kind + "_detail"] = {"reference_s": r, "oracle_s": o, "reference_steps": rs, "oracle_steps": os_}
        print(kind, "reference", r, "oracle", o, "ratio", o / r, flush=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
