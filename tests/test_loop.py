"""vst.reconet.loop: sync-free step logging and the reference's epoch loop (host logic, CPU)."""
import json

import pytest
import torch

from vst.reconet.loop import StepLog, fit


def test_steplog_window_means_and_jsonl(tmp_path):
    path = tmp_path / "log.jsonl"
    log = StepLog(str(path), every=2, units_per_step=8)
    vals = [1.0, 3.0, 5.0, 7.0, 11.0]
    for i, v in enumerate(vals):
        log.add({"loss": torch.tensor(v), "CL": torch.tensor(2 * v), "not_scalar": torch.ones(3)}, epoch=1)
    assert len(log.records) == 2 and log.window  # the last step waits for the next flush
    log.flush()
    recs = [json.loads(line) for line in open(path)]
    assert [r["steps"] for r in recs] == [2, 2, 1]
    assert [r["loss"] for r in recs] == [2.0, 6.0, 11.0]
    assert [r["CL"] for r in recs] == [4.0, 12.0, 22.0]
    assert all("not_scalar" not in r and r["frame-pairs/s"] > 0 and r["epoch"] == 1 for r in recs)
    assert recs[-1]["step"] == 5


class _StubTrainer:
    """records the batches it is stepped with; returns the reference's loss terms as 0-d tensors"""

    def __init__(self):
        self.model = torch.nn.Linear(2, 2)
        self.seen = []

    def step(self, frames, flow=None, mask=None):
        self.seen.append((tuple(frames.shape), tuple(flow.shape), tuple(mask.shape)))
        n = float(len(self.seen))
        return {"loss": torch.tensor(n), "FTL": torch.tensor(n / 2)}


def test_fit_epochs_batches_and_checkpoints(tmp_path):
    B, H, W = 2, 4, 6
    batch = (torch.zeros(B, 3, H, W), torch.zeros(B, 3, H, W), torch.zeros(B, 2, H, W), torch.zeros(B, H, W))
    tr = _StubTrainer()
    log = StepLog(every=10)
    fit(tr, [batch] * 3, epochs=2, log=log, checkpoint=str(tmp_path / "m_epoch_{epoch}.pth"))
    assert tr.seen == [((2, B, 3, H, W), (B, 2, H, W), (B, H, W))] * 6
    assert [r["steps"] for r in log.records] == [3, 3]          # flushed at each epoch end
    assert [r["loss"] for r in log.records] == [2.0, 5.0]
    for e in (1, 2):
        sd = torch.load(tmp_path / f"m_epoch_{e}.pth", weights_only=True)
        assert sorted(sd) == ["bias", "weight"]


class _StubAdaAttN:
    """an AdaAttN-style trainer: consumes (content1, content2, style) triples through step_batch"""

    def __init__(self):
        self.model = torch.nn.Conv2d(3, 3, 1)
        self.seen = []

    def step_batch(self, batch):
        c1, c2, s = batch
        self.seen.append(tuple(torch.stack([c1, c2, s]).shape))
        n = float(len(self.seen))
        return {"loss": torch.tensor(n), "loss_gs": torch.tensor(n / 4), "loss_lf": torch.tensor(n / 4),
                "loss_is": torch.tensor(n / 2)}


def test_fit_adaattn_triples_and_reference_checkpoint_name(tmp_path):
    from vst.reconet.loop import AA_VIDEO_CHECKPOINT

    B, H, W = 4, 8, 16
    triple = tuple(torch.zeros(B, 3, H, W) for _ in range(3))
    tr = _StubAdaAttN()
    log = StepLog(every=2, units_per_step=B)
    ck = str(tmp_path / AA_VIDEO_CHECKPOINT.replace("./models/", "").format(epoch="{epoch}", batch=B))
    fit(tr, [triple] * 3, epochs=1, log=log, checkpoint=ck)
    assert tr.seen == [(3, B, 3, H, W)] * 3
    assert [r["steps"] for r in log.records] == [2, 1]
    assert [r["loss_is"] for r in log.records] == [0.75, 1.5]
    assert (tmp_path / "AdaAttN-video_epoch_1_batchSize_4.pth").exists()


def test_fit_fills_the_batch_field_of_the_reference_pattern(tmp_path):
    """AA_VIDEO_CHECKPOINT (AA/train_video.py:138) passed as is: {batch} comes from checkpoint_fields
    or the loader's batch_size; a pattern the loop cannot fill raises before training."""
    from vst.reconet.loop import AA_VIDEO_CHECKPOINT

    B = 4
    triple = tuple(torch.zeros(B, 3, 8, 16) for _ in range(3))
    pat = str(tmp_path / AA_VIDEO_CHECKPOINT.replace("./models/", ""))
    fit(_StubAdaAttN(), [triple], epochs=1, checkpoint=pat, checkpoint_fields={"batch": B})
    assert (tmp_path / "AdaAttN-video_epoch_1_batchSize_4.pth").exists()

    class Loader(list):
        batch_size = 2

    fit(_StubAdaAttN(), Loader([triple]), epochs=1, checkpoint=pat)
    assert (tmp_path / "AdaAttN-video_epoch_1_batchSize_2.pth").exists()
    with pytest.raises(ValueError):
        fit(_StubAdaAttN(), [triple], epochs=1, checkpoint=pat)


def test_train_state_roundtrip_restores_adam_and_scaler():
    """train_state / load_train_state (vst/reconet/_flat.py): Adam moments, step count and the loss
    scaler's state survive a save / load (CPU tensors; the scaler's device state is a plain tensor)."""
    import io

    from vst.reconet import _flat

    class _Tr:
        pass

    class _Flat:
        def __init__(self):
            self.numel = 5
            self.m, self.v, self.p = torch.arange(5.0), torch.arange(5.0) * 2, torch.zeros(5)

    src = _Tr()
    src.flat, src.step_count = _Flat(), 7
    src.scaler = _flat.LossScaler("cpu", init_scale=2.0 ** 10)
    src.scaler.state[1] = 3.0
    buf = io.BytesIO()
    torch.save(_flat.train_state(src), buf)
    buf.seek(0)
    from vst import ops

    ops.gemm_role("fwd")
    saved = ops.POLICY_NAME[0]
    try:
        for policy in ("f16", "bf16x6"):
            ops.use_policy(policy)
            buf.seek(0)
            dst = _Tr()
            dst.flat, dst.step_count, dst.scaler = _Flat(), 0, None
            dst.flat.m.zero_(), dst.flat.v.zero_()
            if policy == "f16":
                _flat.load_train_state(dst, torch.load(buf, weights_only=True))
                assert dst.scaler.state_dict() == src.scaler.state_dict()
            else:
                # a loss-scaled checkpoint resumed under an unscaled policy: the scaler is not restored
                with pytest.warns(UserWarning, match="loss scaler"):
                    _flat.load_train_state(dst, torch.load(buf, weights_only=True))
                assert dst.scaler is None
            assert dst.step_count == 7 and torch.equal(dst.flat.m, src.flat.m) and torch.equal(dst.flat.v, src.flat.v)
    finally:
        ops.use_policy(saved)
