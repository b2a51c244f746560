"""RTNSTV training step (RT/train.py:36-61 spatial_loss, :98-145 loop body) on MI355X.

Per step, as the reference: styled_i = StylizingNetwork(img_i) for both frames; spatial loss of
each frame = ALPHA * MSE(relu4_2(content), relu4_2(styled)) + BETA * sum_l MSE(gram(styled_l),
gram_s_l) (gram / (H W)) + GAMMA * mean(sqrt(clamp(dx^2 + dy^2, 1e-8))); temporal loss =
LAMBDA * sum(mask * (styled2 - warp(styled1, flow))^2) / (sum(mask expanded to C) + 1e-8) on the
raw [0, 255] outputs; Adam(lr=1e-3).
Batching choices that do not change the arithmetic (as in the ReCoNet trainer): both frames of
a pair run as one 2B batch (InstanceNorm is per sample); the sum of the two frames' means over
equal-size halves is 2 * the mean over the 2B batch.  No host synchronisation inside a step.
Multi-GPU: frame pairs sharded, one RCCL all-reduce of the flat gradient (vst.reconet.dist).
"""
import torch

from .. import ops
from ..reconet._flat import FlatParams, backward_and_adam
from ..reconet.dist import GradBuckets, broadcast_params, world_info

# RT/train.py:28-31
LOSS_WEIGHTS = dict(ALPHA=1e7, BETA=5e7, GAMMA=5e-1, LAMBDA=1e6)


class RTNSTVTrainer:
    def __init__(self, model, vgg, style, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weights=None, process_group=None):
        self.model, self.vgg = model, vgg
        self.w = dict(LOSS_WEIGHTS if weights is None else weights)
        self.lr, self.betas, self.eps = lr, betas, eps
        self.flat = FlatParams(model)
        self.step_count = 0
        self.scaler = None  # LossScaler under a loss-scaled (fp16) policy
        self.pg = process_group
        self.rank, self.world = world_info(process_group)
        # DP: rank 0's initial parameters everywhere; gradient buckets all-reduced from backward
        broadcast_params(self.flat.p, process_group)
        self.dp = GradBuckets(model, self.flat, process_group)
        dev = self.flat.p.device
        with torch.no_grad():
            feats = vgg(style.to(dev))
            self.style_grams = [ops.gram_matrix(f, per_hw=True) for f in feats.values()]

    def losses(self, frames, flow, mask):
        """frames: [2, B, 3, H, W] (img1, img2); returns dict of 0-d device tensors."""
        w = self.w
        _, B, C, H, W = frames.shape
        x = frames.reshape(2 * B, C, H, W)
        styled = self.model(x)
        sf = self.vgg(styled)
        with torch.no_grad():
            cf = self.vgg(x)["relu4_2"]
        out = {"CL": ops.mse(sf["relu4_2"], cf, 2.0 * w["ALPHA"])}
        sl = None
        for f, gs in zip(sf.values(), self.style_grams):
            term = ops.mse(ops.gram_matrix(f, per_hw=True), gs, 2.0 * w["BETA"])
            sl = term if sl is None else sl + term
        out["SL"] = sl
        out["RL"] = ops.tv_sqrt_loss(styled, 2.0 * w["GAMMA"])
        warped = ops.warp(styled[:B], flow)
        # mask is 0/1 (flow_warp_mask): sum(mask) = nnz; an empty mask gives 0 like the reference's +1e-8
        out["TL"] = ops.feature_temporal_loss(styled[B:], warped, mask, w["LAMBDA"])
        out["loss"] = out["CL"] + out["SL"] + out["RL"] + out["TL"]
        return out

    def step(self, frames, flow, mask):
        self.flat.zero_grad()
        self.dp.begin()
        out = self.losses(frames, flow, mask)
        backward_and_adam(self, out["loss"])
        return {k: v.detach() for k, v in out.items()}
