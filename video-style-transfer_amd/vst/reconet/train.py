"""ReCoNet training step (RC/train_single/train_candy.py:63-152) on MI355X, single- or multi-GPU.

Semantics per step are the reference loop body's:
  styled = ReCoNet(img1), ReCoNet(img2); vgg_normalize everything; Vgg16 of the 4 images;
  FTL (feature-level masked temporal, train_candy.py:91-106), OTL (output-level, :109-123),
  content (relu3_3 MSE, :126-129), style (Gram MSE over 4 layers, :132-138), TV (:141-145),
  backward, Adam(lr=1e-3) step.
The reference's clones of that loop body are the same step with a different loss-term set
(`terms`) and weights, selected by name with `ReCoNetTrainer.for_script(...)`:
  train_candy / train_starry-night  FTL OTL CL SL RL   frame pairs
  train_Flow_noFTL                  OTL CL SL RL       frame pairs (train_Flow_noFTL.py:124-125)
  train_multiple/train_Flow         FTL OTL CL SL RL   frame pairs of input_frame_num=4 stacked
                                                       frames; VGG sees the last 3 channels
                                                       (train_Flow.py:58-60,83-84)
  train_coco2014                    CL SL              single images (train_coco2014.py:65-90):
                                                       content + style only, no TV, BETA 1e10
Batching choices that do not change the arithmetic:
  * both frames of a pair go through the stylizer / VGG as ONE batch of 2B (InstanceNorm is
    per sample, so this is the reference's two passes fused);
  * mean(a1) + mean(a2) over equal-size halves is evaluated as 2 * mean(a1 ++ a2).
No host synchronisation inside a step: the nnz counts of the temporal masks stay on device and
the loss terms are returned as device scalars.

Multi-GPU: one process per GPU (torchrun), frame pairs sharded across ranks, one RCCL
all-reduce (sum) of the flat gradient buffer per step, Adam applies the 1/world average.  The
FTL/OTL denominators are rank-local nnz and TV is a sum, exactly as the reference computes them
on its (per-rank) batch.
"""
import torch

from .. import ops
from ._flat import FlatParams, backward_and_adam, load_train_state, train_state
from .dist import GradBuckets, broadcast_params, world_info

LOSS_WEIGHTS = dict(ALPHA=1e5, BETA=2e10, GAMMA=1e-2, LAMBDA_F=1e12, LAMBDA_O=1e7)
# RC/train_single/train_Flow_SD{1,2}.py:24-29
SD_LOSS_WEIGHTS = dict(ALPHA=1e5, BETA=1e10, GAMMA=1e-2, LAMBDA_F=1e11, LAMBDA_O=1e7)
ALL_TERMS = ("FTL", "OTL", "CL", "SL", "RL")

# the reference's training scripts: (loss terms, weight overrides, single-image batches)
SCRIPTS = {
    "train_candy": (ALL_TERMS, {}, False),                                    # train_candy.py:23-28,148
    "train_starry-night": (ALL_TERMS, {"BETA": 1e11}, False),                 # train_starry-night.py:24
    "train_Flow_noFTL": (("OTL", "CL", "SL", "RL"), {"BETA": 1e10}, False),  # train_Flow_noFTL.py:24,125
    "train_Flow": (ALL_TERMS, {"BETA": 1e10}, False),                         # train_multiple/train_Flow.py:22-25,148
    "train_coco2014": (("CL", "SL"), {"BETA": 1e10}, True),                   # train_coco2014.py:23-24,86
}


class ReCoNetTrainer:
    def __init__(self, model, vgg, style, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weights=None, temporal=True,
                 process_group=None, teacher=None, sd_index=(0, 0), terms=None, single=False):
        """model: ReCoNet / ReCoNetSD1 / ReCoNetSD2 (feature map and styled image are its last two
        outputs).  teacher + sd_index=(teacher output, student output): the distillation trainers
        (train_Flow_SD{1,2}.py), whose symmetric distillation term SDL is reported but, as in the
        reference, not part of the optimised loss.
        terms: the loss terms summed into the optimised loss (subset of FTL OTL CL SL RL; default
        all, or CL SL RL with temporal=False).  single: batches are single images [B, C, H, W]
        (train_coco2014) instead of frame pairs [2, B, C, H, W]; only CL / SL / RL apply."""
        self.model = model
        self.teacher = teacher
        self.sd_index = sd_index
        self.vgg = vgg
        self.w = dict(LOSS_WEIGHTS if weights is None else weights)
        if terms is None:
            terms = ALL_TERMS if temporal and not single else ("CL", "SL", "RL")
        unknown = set(terms) - set(ALL_TERMS)
        if unknown or not terms:
            raise ValueError(f"loss terms must be a non-empty subset of {ALL_TERMS}, got {tuple(terms)}")
        if single and set(terms) & {"FTL", "OTL"}:
            raise ValueError("single-image batches have no temporal terms (FTL / OTL need frame pairs)")
        self.terms = tuple(t for t in ALL_TERMS if t in terms)
        self.single = single
        self.temporal = bool(set(self.terms) & {"FTL", "OTL"})
        self.lr, self.betas, self.eps = lr, betas, eps
        self.flat = FlatParams(model)
        self.step_count = 0
        self.pg = process_group
        self.rank, self.world = world_info(process_group)
        # DP: rank 0's initial parameters everywhere; gradient buckets all-reduced from backward
        broadcast_params(self.flat.p, process_group)
        self.dp = GradBuckets(model, self.flat, process_group)
        self.scaler = None  # LossScaler under a loss-scaled (fp16) policy, created at the first such step
        dev = self.flat.p.device
        self.chscale_cache = {}
        with torch.no_grad():
            feats = vgg(ops.VggNormalizeFn.apply(style.to(dev)))
            self.style_grams = [ops.gram_matrix(f) for f in feats]

    @classmethod
    def for_script(cls, script, model, vgg, style, **kw):
        """The trainer of one of the reference's training scripts (SCRIPTS): its loss terms, its
        weights (LOSS_WEIGHTS with the script's overrides) and its batch kind."""
        terms, over, single = SCRIPTS[script]
        w = dict(LOSS_WEIGHTS)
        w.update(over)
        w.update(kw.pop("weights", None) or {})
        return cls(model, vgg, style, weights=w, terms=terms, single=single, **kw)

    def _chscale(self, Hf, Wf, H, W, dev):
        key = (Hf, Wf, H, W)
        if key not in self.chscale_cache:
            self.chscale_cache[key] = torch.tensor([float(Wf) / W, float(Hf) / H], dtype=torch.float32, device=dev)
        return self.chscale_cache[key]

    def losses(self, frames, flow=None, mask=None):
        """frames: [2, B, C, H, W] frame pairs (img1 = frames[0], img2 = frames[1]), or [B, C, H, W]
        single images (single=True); returns dict of 0-d tensors."""
        w = self.w
        if self.single:
            if frames.dim() != 4:
                raise ValueError(f"single-image trainer: expected [B, C, H, W], got {tuple(frames.shape)}")
            B, C, H, W = frames.shape
            x, nf = frames, 1
        else:
            if frames.dim() != 5 or frames.shape[0] != 2:
                raise ValueError(f"frame-pair trainer: expected [2, B, C, H, W], got {tuple(frames.shape)}")
            _, B, C, H, W = frames.shape
            x, nf = frames.reshape(2 * B, C, H, W), 2
            if self.temporal and (flow is None or mask is None):
                raise ValueError("the temporal terms need flow and mask")
        # the content targets (normalized frames, their VGG features, the warped frame) depend on
        # the inputs only: computed on the side stream beside the stylizer's forward
        with ops.side_branch(x, flow) as side:
            with torch.no_grad():
                i_n = ops.VggNormalizeFn.apply(x if C == 3 else x[:, C - 3:].contiguous())
                # the content loss reads relu3_3 only (train_candy.py:126-128): the content pass stops
                # after slice 3 when the loss net supports it
                upto = getattr(self.vgg, "features_upto", None)
                cf = upto(i_n, 3) if upto is not None else self.vgg(i_n)
                warped_i = ops.warp(i_n[:B], flow) if "OTL" in self.terms else None
            side.produced(i_n, *cf, warped_i)
        mout = self.model(x)
        fmap, styled = mout[-2], mout[-1]
        s_n = ops.VggNormalizeFn.apply(styled)
        # the normalised stylised frames are read by the VGG pass, TV and (per frame) the output
        # temporal loss: one autograd output per consumer, their gradients summed in one pass
        s_vgg, s_tv, s_1, s_2 = ops.fork(s_n, 2, B) if nf == 2 else ops.fork(s_n, 2) + (None, None)
        sf = list(self.vgg(s_vgg))
        # relu3_3 feeds the content loss and its Gram matrix
        sf[2], f3_content = ops.fork(sf[2], 2)
        side.join()
        out = {}
        if "FTL" in self.terms:
            Hf, Wf = fmap.shape[2:]
            f_1, f_2 = ops.fork(fmap, 0, B)
            fflow = ops.resize_bilinear(flow, (Hf, Wf), chscale=self._chscale(Hf, Wf, H, W, flow.device))
            warped_f = ops.warp(f_1, fflow)
            fmask = ops.resize_bilinear(mask.unsqueeze(1), (Hf, Wf), binarize=True)
            out["FTL"] = ops.feature_temporal_loss(f_2, warped_f, fmask, w["LAMBDA_F"])
        if "OTL" in self.terms:
            warped_s = ops.warp(s_1, flow)
            out["OTL"] = ops.output_temporal_loss(s_2, warped_s, i_n[B:], warped_i, mask, w["LAMBDA_O"])
        # mean over the nf*B batch x nf = the reference's sum of nf per-frame means
        out["CL"] = ops.mse(f3_content, cf[2], nf * w["ALPHA"])
        out["SL"] = ops.sum_scalars(*[ops.mse(ops.gram_matrix(f), gs, nf * w["BETA"])
                                      for f, gs in zip(sf, self.style_grams)])
        if "RL" in self.terms:
            out["RL"] = ops.tv_loss(s_tv, w["GAMMA"])
        out["loss"] = ops.sum_scalars(*[out[k] for k in self.terms])
        if self.teacher is not None:
            ti, si = self.sd_index
            with torch.no_grad():
                # mean over the 2B batch = (mse(t1, s1) + mse(t2, s2)) / 2
                out["SDL"] = ops.mse(self.teacher(x)[ti], mout[si].detach(), nf * 0.01 * w["BETA"])
        return out

    def backward(self, loss):
        """loss.backward() seeded as a fresh trainer's first step seeds it (the policy's initial loss
        scale, `ops.loss_scale()`: 1 except under fp16); returns the factor that unscales the
        gradients.  Used by the parity tests that inspect gradients before Adam; `step` itself
        seeds with the dynamic scaler's device-resident scale."""
        s = ops.loss_scale()
        if s == 1.0:
            loss.backward()
            return 1.0
        loss.backward(torch.full((), s, device=loss.device))
        return 1.0 / s

    def train_state(self):
        """Adam moments / step count and the fp16 loss scaler's state, for a resume next to the
        model's state_dict checkpoint (_flat.train_state)."""
        return train_state(self)

    def load_train_state(self, sd):
        load_train_state(self, sd)

    def step_batch(self, batch):
        """One step on a loader batch: FramePairLoader's (img1, img2, flow, mask) or, for the
        single-image trainer, ImageLoader's images (train_candy.py:77-78, train_coco2014.py:65)."""
        if self.single:
            return self.step(batch)
        img1, img2, flow, mask = batch
        return self.step(torch.stack([img1, img2]), flow, mask)

    def step(self, frames, flow=None, mask=None):
        """One training step (train_candy.py:77-152): losses, backward, gradient exchange, Adam.
        `step_count` counts calls; under the fp16 policy Adam's own count lives in `scaler` and does
        not advance on a skipped (overflowed) step."""
        self.flat.zero_grad()
        self.dp.begin()
        out = self.losses(frames, flow, mask)
        backward_and_adam(self, out["loss"])
        return {k: v.detach() for k, v in out.items()}
