"""AdaAttN training steps on MI355X, single- or multi-GPU: the video step (AA/train_video.py:78-118)
and the image step (AA/train_image.py:69-110, `image_step`).

Per step, exactly the reference loop body:
  fc1, fc2, fs = VGG19(content1), VGG19(content2), VGG19(style)          (no gradient: data)
  cs1, cs2 = model(fc1, fs), model(fc2, fs);  fcs1, fcs2 = VGG19(cs1), VGG19(cs2)
  loss_gs = LAMBDA_G  * sum_{relu2_1..relu5_1} global_stylized_loss(fcs1, fs)
  loss_lf = LAMBDA_L  * sum_{i=0..2} mse(fcs1[relu{i+3}_1], AdaAttnNoConv_i(fc1, fs))
  loss_is = LAMBDA_IS * sum_{relu2_1..relu4_1} image_similarity_loss(fc1, fc2, fcs1, fcs2)
  backward, Adam(lr=1e-4).
The loss weights are folded into the loss kernels' reductions.  The three data encodings run as
one VGG19 pass of 3B when the inputs are handed over as one [3, B, 3, H, W] buffer, and the two
stylisations (and the VGG19 passes of their outputs) as one batch of 2B: every op on the path is
per sample (InstanceNorm, attention per image), so this is the reference's two passes fused into
larger GEMMs.

Multi-GPU: one process per GPU, (content1, content2, style) triples sharded across ranks, one
RCCL all-reduce of the flat gradient per step; Adam applies the 1/world average.  Every loss term
is a per-rank mean or per-rank sum exactly as the reference computes it on its own batch.
"""

import torch

from .. import ops
from ..reconet._flat import FlatParams, backward_and_adam, load_train_state, train_state
from ..reconet.dist import GradBuckets, broadcast_params, world_info
from .lossfn import global_stylized_loss, image_similarity_loss, local_feature_loss
from .network import AdaAttnNoConv
from .utilities import feature_down_sample
from .vgg19 import FEATURES

LOSS_WEIGHTS = dict(LAMBDA_G=10.0, LAMBDA_L=3.0, LAMBDA_IS=100.0)


def _batch_pair(a, b):
    """{k: a[k] ++ b[k]} along the batch; a free view when b[k] directly follows a[k] in memory
    (the 3B encoding buffer), a copy otherwise."""
    out = {}
    for k, x in a.items():
        y = b[k]
        if (x.is_contiguous() and y.is_contiguous() and y.data_ptr() == x.data_ptr() + x.numel() * x.element_size()
                and x.untyped_storage().data_ptr() == y.untyped_storage().data_ptr()):
            out[k] = torch.as_strided(x, (x.shape[0] + y.shape[0],) + tuple(x.shape[1:]), x.stride())
        else:
            out[k] = _cat2(x, y)
    return out


def _cat2(x, y):
    """x ++ y along the batch with the library's plane-copy kernel."""
    out = torch.empty((x.shape[0] + y.shape[0],) + tuple(x.shape[1:]), device=x.device, dtype=torch.float32)
    ops.copy_into(x.contiguous(), out[:x.shape[0]])
    ops.copy_into(y.contiguous(), out[x.shape[0]:])
    return out


def _down_sampled(fc, fs):
    """({idx: feature_down_sample(fc, idx)}, {idx: feature_down_sample(fs, idx)}) for the three
    attention levels (AA/network.py:247-249, AA/train_video.py:96-101), data features only."""
    with torch.no_grad():
        lc, ls = list(fc.values()), list(fs.values())
        return ({idx: feature_down_sample(lc, idx) for idx in (2, 3, 4)},
                {idx: feature_down_sample(ls, idx) for idx in (2, 3, 4)})


class AdaAttNTrainer:
    def __init__(self, model, vgg, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weights=None, activation="cosine",
                 process_group=None):
        self.model, self.vgg = model, vgg
        self.w = dict(LOSS_WEIGHTS if weights is None else weights)
        self.lr, self.betas, self.eps = lr, betas, eps
        self.activation = activation
        self.flat = FlatParams(model)
        dev = self.flat.p.device
        self.noconv = [AdaAttnNoConv(v, q, activation).to(dev).eval()
                       for v, q in ((256, 64 + 128 + 256), (512, 64 + 128 + 256 + 512),
                                    (512, 64 + 128 + 256 + 512 + 512))]
        self.step_count = 0
        self.pg = process_group
        self.rank, self.world = world_info(process_group)
        # DP: rank 0's initial parameters everywhere; gradient buckets all-reduced from backward
        broadcast_params(self.flat.p, process_group)
        self.dp = GradBuckets(model, self.flat, process_group)
        self.scaler = None  # LossScaler under the fp16 policy (config 5), created at its first step

    def encode(self, c1, c2=None, s=None):
        """VGG19 features of the data images (no gradient).  c1 may be a [3, B, 3, H, W] buffer."""
        with torch.no_grad(), ops.gemm_scope("encode"):
            if c2 is None:
                T, B = c1.shape[:2]
                f = self.vgg(c1.reshape(T * B, *c1.shape[2:]))
                return tuple({k: v[t * B:(t + 1) * B] for k, v in f.items()} for t in range(T))
            return self.vgg(c1), self.vgg(c2), self.vgg(s)

    def losses(self, c1, c2=None, s=None):
        w = self.w
        fc1, fc2, fs = self.encode(c1, c2, s)
        B = next(iter(fc1.values())).shape[0]
        fc12 = _batch_pair(fc1, fc2)
        # cosine attention takes the style side once for both content frames (K / V broadcast over
        # the two halves of the batch: the style 1x1 convs, down-sampling and K U^T run on B images)
        fs2 = fs if self.activation == "cosine" else {k: _cat2(v, v) for k, v in fs.items()}
        # feature_down_sample of the data features, once per step: the stylizer takes both content
        # frames' and the style's, the AdaAttnNoConv loss targets frame 1's (the first half of the
        # content batch) and the style's (the first half when the style side is doubled)
        down = _down_sampled(fc12, fs2)
        # the local-feature targets (AdaAttnNoConv over frame 1's and the style's data features) depend
        # on the data only: computed on the side stream beside the stylizer and its VGG pass
        l1, ls = list(fc1.values()), list(fs.values())
        args = [(l1[i], ls[i], down[0][i][:B], down[1][i][:B]) for i in (2, 3, 4)]
        with ops.side_branch(*[t for a in args for t in a]) as side:
            with torch.no_grad():
                targets = [self.noconv[i](*args[i]) for i in range(3)]
            side.produced(*targets)
        cs = self.model(fc12, fs2, down=down)  # cs1 ++ cs2
        with ops.gemm_scope("lossnet"):
            fcs = self.vgg(cs)
        # each loss feature of the stylised pair is read by up to three loss terms (frame 1) and one
        # (frame 2): one autograd output per reader (ops.fork), their gradients summed per frame in one
        # pass -- no ATen adds, no slice zero-fills
        g_k, l_k, i_k = FEATURES[1:], FEATURES[2:5], FEATURES[1:4]
        views = {}
        for k, v in fcs.items():
            n1, n2 = (k in g_k) + (k in l_k) + (k in i_k), int(k in i_k)
            if n1 + n2:
                views[k] = list(ops.fork(v, 0, B, (n1, n2)))
        first = lambda k: views[k].pop(0)  # noqa: E731  (frame-1 views lead the list)
        second = lambda k: views[k].pop()  # noqa: E731  (the frame-2 view ends it)
        gs = ops.sum_scalars(*[global_stylized_loss(first(k), fs[k], weight=w["LAMBDA_G"]) for k in g_k])
        side.join()
        lf = ops.sum_scalars(*[local_feature_loss(first(l_k[i]), targets[i], weight=w["LAMBDA_L"]) for i in range(3)])
        isl = ops.sum_scalars(*[image_similarity_loss(fc1[k], fc2[k], first(k), second(k), weight=w["LAMBDA_IS"])
                                for k in i_k])
        return {"loss": ops.sum_scalars(gs, lf, isl), "loss_gs": gs, "loss_lf": lf, "loss_is": isl}

    def image_losses(self, c, s):
        """Loss terms of one train_image step (AA/train_image.py:76-106): content / style images,
        the trainer's activation (the reference script uses "softmax", :22), global-stylized and
        local-feature losses only (no image-similarity term)."""
        w = self.w
        with torch.no_grad():
            fc, fs = self.vgg(c), self.vgg(s)
        down = _down_sampled(fc, fs)
        fcs = self.vgg(self.model(fc, fs, down=down))
        gs = None
        for k in FEATURES[1:]:
            t = global_stylized_loss(fcs[k], fs[k], weight=w["LAMBDA_G"])
            gs = t if gs is None else gs + t
        lc, ls = list(fc.values()), list(fs.values())
        lf = None
        for i in range(3):
            idx = i + 2
            with torch.no_grad():
                target = self.noconv[i](lc[idx], ls[idx], down[0][idx], down[1][idx])
            t = local_feature_loss(fcs[FEATURES[idx]], target, weight=w["LAMBDA_L"])
            lf = t if lf is None else lf + t
        return {"loss": gs + lf, "loss_gs": gs, "loss_lf": lf}

    def image_step(self, c, s):
        """backward + Adam of `image_losses` (AA/train_image.py:109-110)."""
        return self._update(self.image_losses, c, s)

    def train_state(self):
        """Adam moments / step count and the fp16 loss scaler's state, for a resume next to the
        model's state_dict checkpoint (reconet._flat.train_state)."""
        return train_state(self)

    def load_train_state(self, sd):
        load_train_state(self, sd)

    def step(self, c1, c2=None, s=None):
        return self._update(self.losses, c1, c2, s)

    def step_batch(self, batch):
        """One step on a loader batch (content1, content2, style) (AA/train_video.py:78-81): the three
        encodings as one VGG19 pass of 3B (a [3, B, 3, H, W] buffer); an already stacked buffer is
        used as is."""
        if isinstance(batch, torch.Tensor):
            return self.step(batch)
        c1, c2, s = batch
        return self.step(torch.stack([c1, c2, s]))

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

    def _update(self, losses, *args):
        """losses, backward, gradient exchange, Adam (AA/train_video.py:120-122); under the fp16
        policy through the dynamic loss scaler (an overflowed step is skipped on the device)."""
        self.flat.zero_grad()
        self.dp.begin()
        out = losses(*args)
        backward_and_adam(self, out["loss"])
        return {k: v.detach() for k, v in out.items()}
