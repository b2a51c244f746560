"""Run-to-run reproducibility of the f16 AdaAttN step (AA/train_video.py:78-122) in one process:
K fresh trainers on the same weights and batch per side-stream setting (both side streams, content
branch only, weight gradients only, none), caches emptied before each, forward losses and flat
gradients compared bitwise with the first run of the setting.  (GPU; diagnostic for the one
side-stream difference recorded in DESIGN.md 4.6.)

    python tools/f16_repro.py [K]
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-style-transfer_amd"), os.path.join(REPO, "tests")]


def main():
    from test_gpu_streams import _batch, _fresh_caches, _trainer
    from vst import ops

    K = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    ops.gemm_role("fwd")
    ops.use_policy("f16")
    batch = _batch("adaattn")
    for wg, ct in ((True, True), (False, True), (True, False), (False, False)):
        ops.WGRAD_SIDE, ops.CONTENT_SIDE = wg, ct
        ref = None
        diffs = []
        for k in range(K):
            _fresh_caches()
            tr = _trainer("adaattn")
            out = tr.step(*batch)
            torch.cuda.synchronize()
            cur = ({n: float(v) for n, v in out.items()}, tr.flat.g.clone())
            if ref is None:
                ref = cur
                continue
            same_l = cur[0] == ref[0]
            same_g = torch.equal(cur[1], ref[1])
            if not (same_l and same_g):
                diffs.append((k, same_l, same_g, {n: cur[0][n] - ref[0][n] for n in ref[0]}))
        print(f"wgrad_side={wg} content_side={ct}: {K} runs, {len(diffs)} differ", diffs[:3], flush=True)


if __name__ == "__main__":
    main()
