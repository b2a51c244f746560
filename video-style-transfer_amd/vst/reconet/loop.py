"""The reference's epoch loops (RC/train_single/train_candy.py:58-170, AA/train_video.py:64-138)
around a trainer step, without a host synchronisation per step.

The reference reads six `.item()` loss terms every step for its tqdm postfix
(train_candy.py:155-166) -- six device->host syncs that stall the launch queue.  `StepLog` keeps
the steps' 0-d device scalars as they are (no kernel, no sync), and every `every` steps reads them
all in ONE transfer and writes one JSONL line: the mean of every term over the window and the
window's wall-clock throughput (AA/train_video.py:124-134 reads four `.item()` per step the same
way).  `fit` is the loop: per batch `trainer.step_batch` (the trainer unpacks its loader's batch as
the reference's loop does), per epoch a `state_dict` checkpoint under the reference's file-name
pattern (train_candy.py:168-170, train_video.py:137-138: `AA_VIDEO_CHECKPOINT`).
"""
import json
import time

import torch

# AA/train_video.py:138
AA_VIDEO_CHECKPOINT = "./models/AdaAttN-video_epoch_{epoch}_batchSize_{batch}.pth"


class StepLog:
    """Sync-free per-step loss logging.

    add(out): out = the dict of 0-d tensors a trainer step returns; nothing is read back.
    Every `every` steps (and at flush()) the window's terms are stacked and copied to the host
    once; a JSONL record {"epoch", "step", "steps", <term>: mean, "units_per_s"} is appended to
    `path` (if given) and kept in `records`.  units_per_step: frame pairs per step (B x world)."""

    def __init__(self, path=None, every=50, units_per_step=None, unit="frame-pairs/s"):
        self.path, self.every = path, max(1, int(every))
        self.units_per_step, self.unit = units_per_step, unit
        self.window, self.records = [], []
        self.step, self.epoch = 0, 0
        self.t0 = time.perf_counter()

    def add(self, out, epoch=None):
        if epoch is not None:
            self.epoch = epoch
        self.window.append({k: v for k, v in out.items() if isinstance(v, torch.Tensor) and v.dim() == 0})
        self.step += 1
        if len(self.window) >= self.every:
            self.flush()

    def flush(self):
        if not self.window:
            return None
        keys = sorted(self.window[0])
        vals = torch.stack([torch.stack([w[k].detach().float() for k in keys]) for w in self.window]).cpu()  # one sync
        dt = time.perf_counter() - self.t0
        rec = {"epoch": self.epoch, "step": self.step, "steps": len(self.window)}
        rec.update({k: float(vals[:, i].double().mean()) for i, k in enumerate(keys)})
        if self.units_per_step:
            rec[self.unit] = self.units_per_step * len(self.window) / dt
        self.records.append(rec)
        if self.path:
            with open(self.path, "a") as f:
                f.write(json.dumps(rec) + "\n")
        self.window = []
        self.t0 = time.perf_counter()
        return rec


def fit(trainer, loader, epochs, epoch_start=1, log=None, checkpoint=None, checkpoint_fields=None,
        train_state=False):
    """train_candy.py:62-170 / train_video.py:64-138: for each epoch, one trainer step per batch of
    the loader (ReCoNet: FramePairLoader (img1, img2, flow, mask) or ImageLoader images; AdaAttN:
    (content1, content2, style) triples), the terms to `log` (StepLog) without a per-step sync, and
    `torch.save(model.state_dict(), checkpoint.format(epoch=e, **checkpoint_fields))` at the end of
    each epoch when `checkpoint` is given (the reference's patterns, e.g.
    "./models/Flow_input_1_epoch_{epoch}_batchSize_2.pth", or AA_VIDEO_CHECKPOINT with
    checkpoint_fields={"batch": B}; a {batch} field left unfilled is the loader's batch size when
    it has one).  train_state: also save the trainer's resume state (Adam moments, step count, the
    fp16 loss scaler; trainer.train_state()) next to it as <checkpoint>.train_state -- the
    reference's checkpoint holds the model alone."""
    fields = dict(checkpoint_fields or {})
    if checkpoint and "{batch}" in checkpoint and "batch" not in fields:
        bs = getattr(loader, "batch_size", None)
        if bs is None:
            raise ValueError(f"checkpoint pattern {checkpoint!r} has a {{batch}} field: pass checkpoint_fields")
        fields["batch"] = bs
    for epoch in range(epoch_start, epochs + 1):
        trainer.model.train()
        for batch in loader:
            if hasattr(trainer, "step_batch"):
                out = trainer.step_batch(batch)
            elif getattr(trainer, "single", False):
                out = trainer.step(batch)
            else:
                img1, img2, flow, mask = batch
                out = trainer.step(torch.stack([img1, img2]), flow, mask)
            if log is not None:
                log.add(out, epoch)
        if log is not None:
            log.flush()
        if checkpoint:
            path = checkpoint.format(epoch=epoch, **fields)
            torch.save(trainer.model.state_dict(), path)
            if train_state:
                torch.save(trainer.train_state(), path + ".train_state")
    return log
