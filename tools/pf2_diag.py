"""Per-tensor gradient norms of the aa_step golden train_video step under a GEMM policy (argv[1]),
written to argv[2] (run once per build switch and compare)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-style-transfer_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from oracle import shapes  # noqa: E402
from vst import ops  # noqa: E402
from vst.adaattn.network import StylizingNetwork  # noqa: E402
from vst.adaattn.train import AdaAttNTrainer  # noqa: E402
from vst.adaattn.vgg19 import VGG19  # noqa: E402

s = np.load(os.path.join(REPO, "tests", "golden", "aa_step.npz"), allow_pickle=False)
seeds = s["seeds"]
ops.use_policy(sys.argv[1])
m = StylizingNetwork("cosine")
m.load_state_dict(oracle.seeded_params(shapes.stylizing_network(), int(seeds[0])))
v = VGG19()
v.load_state_dict(oracle.seeded_params(shapes.vgg19(), int(seeds[1])))
tr = AdaAttNTrainer(m.cuda(), v.cuda(), activation="cosine")
frames = torch.stack([torch.from_numpy(s[k]).cuda() for k in ("c1", "c2", "style")])
tr.flat.zero_grad()
out = tr.losses(frames)
un = tr.backward(out["loss"])
torch.cuda.synchronize()
res = {n: [float((p.grad * un).double().norm()), float(s[f"gnorm/{n}"])] for n, p in m.named_parameters()}
res["_loss"] = [float(out["loss"].item()), float(s["loss"])]
json.dump(res, open(sys.argv[2], "w"), indent=0)
