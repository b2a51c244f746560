"""Run-to-run reproducibility of the f16 AdaAttN step (AA/train_video.py:78-122) in one process:
K fresh trainers on the same weights and batch per side-stream setting (both side streams, content
branch only, weight gradients only, none), caches emptied before each, forward losses and flat
gradients compared bitwise with the first run of the setting.  (GPU; diagnostic for the one
side-stream difference recorded in DESIGN.md 4.6.)

    python tools/f16_repro.py [K] [out.json] [--poison-scratch]

--poison-scratch: before every run, vst_test_scratch_poison fills the private (scratch) slots of both
streams with NaN, so a kernel that read a private slot before writing it shows a NaN instead of a stale
copy of the previous run's identical data.
"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-style-transfer_amd"), os.path.join(REPO, "tests")]


def main():
    from test_gpu_streams import _batch, _fresh_caches, _trainer
    from vst import ops
    from vst._lib import lib

    poison = "--poison-scratch" in sys.argv
    argv = [a for a in sys.argv if a != "--poison-scratch"]
    K = int(argv[1]) if len(argv) > 1 else 6
    ops.gemm_role("fwd")
    ops.use_policy("f16")
    out_path = argv[2] if len(argv) > 2 else None
    batch = _batch("adaattn")
    res = {"runs_per_setting": K, "poison_scratch": poison, "device": torch.cuda.get_device_name(0), "settings": []}
    for wg, ct in ((True, True), (False, True), (True, False), (False, False)):
        ops.WGRAD_SIDE, ops.CONTENT_SIDE = wg, ct
        ref = None
        diffs = []
        for k in range(K):
            if poison:
                dev = batch[0].device
                for st in (torch.cuda.current_stream(dev), ops._side_stream(dev)):
                    lib.vst_test_scratch_poison(4096, float("nan"), st.cuda_stream)
                torch.cuda.synchronize()
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
        res["settings"].append({"wgrad_side": wg, "content_side": ct, "differ": len(diffs),
                                "first_diffs": [{"run": d[0], "losses_equal": d[1], "grad_equal": d[2],
                                                 "loss_delta": d[3]} for d in diffs[:3]],
                                "losses": ref[0]})
    if out_path:
        with open(out_path, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
