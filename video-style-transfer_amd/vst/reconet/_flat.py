"""Flat parameter / gradient / Adam-state buffers for a module.

Every parameter becomes a view into one contiguous fp32 buffer and its `.grad` a view into a
second one, so autograd accumulates straight into the flat gradient (AccumulateGrad adds in
place into an existing .grad), the DDP all-reduce is ONE RCCL call and Adam is ONE kernel
(`vst_adam`) over the whole model (62 tensors / 3,763,011 floats for ReCoNet).

`LossScaler` is the fp16 policy's overflow guard (the reference trains in fp32 and steps every
batch, AA/train_video.py:121-122): a device-resident dynamic loss scale with
torch.cuda.amp.GradScaler's rule (skip the step and halve the scale on an Inf / NaN gradient, double
it after `growth_interval` clean steps), applied by `vst_adam_loss_scaled` without a host sync.
"""
import warnings

import torch
from torch.autograd.graph import increment_version

from .._lib import lib, ptr, stream

SCALER_WS = 1024  # include/vst_hip.h VST_SCALER_WS


def _zeros_dev(n, dev):
    """A zero-filled fp32 buffer: the library's fill kernel on a HIP device (no ATen kernel in a
    training process), torch.zeros on the host."""
    t = torch.empty(n, device=dev, dtype=torch.float32)
    if t.is_cuda:
        lib.vst_fill(ptr(t), n, 0.0, stream())
    else:
        t.zero_()
    return t


class FlatParams:
    def __init__(self, module):
        params = [p for p in module.parameters() if p.requires_grad]
        n = sum(p.numel() for p in params)
        dev = params[0].device
        self.p = torch.empty(n, device=dev, dtype=torch.float32)
        self.g, self.m, self.v = (_zeros_dev(n, dev) for _ in range(3))
        off = 0
        with torch.no_grad():
            for prm in params:
                k = prm.numel()
                self.p[off:off + k].copy_(prm.reshape(-1))
                prm.data = self.p[off:off + k].view_as(prm)
                prm.grad = self.g[off:off + k].view_as(prm)
                off += k
        self.params = params
        self.numel = n

    def zero_grad(self):
        if self.g.is_cuda:
            lib.vst_fill(ptr(self.g), self.numel, 0.0, stream())
        else:  # (the CPU data-parallel tests' host stand-in of the flat buffers)
            self.g.zero_()
        for prm, (off, k) in zip(self.params, self._spans()):
            if prm.grad is None or prm.grad.data_ptr() != self.g[off:off + k].data_ptr():
                prm.grad = self.g[off:off + k].view_as(prm)

    def _spans(self):
        off = 0
        for prm in self.params:
            yield off, prm.numel()
            off += prm.numel()

    def _updated(self):
        # the kernel updated every parameter in place.  `prm.data = view` leaves each Parameter with
        # its OWN version counter (not the flat buffer's), so bump every parameter's counter: a
        # graph that saved a parameter before this step then refuses to run backward
        increment_version(self.params)
        increment_version(self.p)

    def adam(self, step, lr, betas, eps, gscale=1.0):
        lib.vst_adam(ptr(self.p), ptr(self.g), ptr(self.m), ptr(self.v), self.numel, float(lr), float(betas[0]),
                     float(betas[1]), float(eps), int(step), float(gscale), stream())
        self._updated()

    def adam_scaled(self, scaler, lr, betas, eps, world_scale=1.0):
        """One Adam step under `scaler` (skipped on device when the gradient holds an Inf / NaN)."""
        scaler.apply(self, lr, betas, eps, world_scale)
        self._updated()


class LossScaler:
    """Device-resident dynamic loss scale (state layout: include/vst_hip.h vst_adam_loss_scaled).

    `seed` is the backward's seed tensor (a 0-d view of the state, so the scale a step uses is the
    one the previous step left on the device); `apply` checks the flat gradient, then skips or
    applies Adam and advances the scale.  Nothing is read back to the host unless asked
    (`scale()`, `state_dict()`)."""

    def __init__(self, device, init_scale=2.0 ** 12, growth_factor=2.0, backoff_factor=0.5, growth_interval=2000,
                 step=0):
        if not (init_scale > 0 and growth_factor >= 1.0 and 0 < backoff_factor <= 1.0 and growth_interval > 0):
            raise ValueError("loss scaler: init_scale > 0, growth_factor >= 1, 0 < backoff_factor <= 1, "
                             "growth_interval > 0")
        init = torch.zeros(8, dtype=torch.float32)
        init[0], init[2] = float(init_scale), float(step)
        self.state = init.to(device)  # (host-built, one copy: no fill kernel on the device)
        self.ws = torch.empty(SCALER_WS, device=device, dtype=torch.float32)
        self.growth, self.backoff, self.interval = float(growth_factor), float(backoff_factor), int(growth_interval)

    @property
    def seed(self):
        return self.state[0]

    def apply(self, flat, lr, betas, eps, world_scale=1.0):
        lib.vst_adam_loss_scaled(ptr(flat.p), ptr(flat.g), ptr(flat.m), ptr(flat.v), flat.numel, float(lr),
                                 float(betas[0]), float(betas[1]), float(eps), float(world_scale), ptr(self.state),
                                 ptr(self.ws), self.interval, self.growth, self.backoff, stream())

    # host views (each one synchronises)
    def scale(self):
        return float(self.state[0].item())

    def skipped_last(self):
        return bool(self.state[3].item() != 0)

    def state_dict(self):
        st = self.state.cpu()
        return {"scale": float(st[0]), "growth_tracker": int(st[1]), "step": int(st[2]), "skipped": int(st[7]),
                "growth_factor": self.growth, "backoff_factor": self.backoff, "growth_interval": self.interval}

    def load_state_dict(self, sd):
        self.growth, self.backoff = float(sd["growth_factor"]), float(sd["backoff_factor"])
        self.interval = int(sd["growth_interval"])
        vals = torch.zeros(8, dtype=torch.float32)
        vals[0], vals[1], vals[2], vals[7] = sd["scale"], sd["growth_tracker"], sd["step"], sd.get("skipped", 0)
        self.state.copy_(vals)


def train_state(trainer):
    """What a resumed run needs beyond the model's state_dict (which the reference's checkpoint holds,
    train_candy.py:170 / train_video.py:138): Adam's moments and step count and, under a loss-scaled
    policy, the dynamic scaler's state -- without it a resumed fp16 run re-learns its scale over the
    first skipped steps and restarts Adam's bias correction."""
    return {"step_count": trainer.step_count, "adam_m": trainer.flat.m.detach().cpu(),
            "adam_v": trainer.flat.v.detach().cpu(),
            "scaler": None if trainer.scaler is None else trainer.scaler.state_dict()}


def load_train_state(trainer, sd):
    """Inverse of train_state (after the model's own load_state_dict)."""
    if sd["adam_m"].numel() != trainer.flat.numel:
        raise ValueError(f"train state holds {sd['adam_m'].numel()} Adam moments, the model {trainer.flat.numel}")
    trainer.step_count = int(sd["step_count"])
    trainer.flat.m.copy_(sd["adam_m"])
    trainer.flat.v.copy_(sd["adam_v"])
    if sd.get("scaler") is not None:
        from .. import ops  # (ops imports this module's siblings)

        if ops.loss_scale() == 1.0:
            # a loss-scaled (fp16) checkpoint resumed under an unscaled policy: the scaler, once
            # created, would stay in use and run loss-scaled Adam with skip-on-overflow there
            warnings.warn("train state holds a loss scaler but the current GEMM policy has no loss scale: "
                          "its state is ignored")
            return
        if trainer.scaler is None:
            trainer.scaler = LossScaler(trainer.flat.p.device)
        trainer.scaler.load_state_dict(sd["scaler"])


def backward_and_adam(trainer, loss):
    """loss.backward(), the data-parallel gradient exchange and one Adam step for a trainer holding
    `flat`, `dp`, `lr`, `betas`, `eps`, `step_count` and `scaler` (the reference's
    `loss.backward(); optimizer.step()`).  Under a policy with a loss scale (`ops.loss_scale()`,
    the fp16 policy) the backward is seeded with the device-resident dynamic scale and Adam runs
    through the `LossScaler` (skipped on overflow); the scaler, once created, stays in use (its
    Adam step count continues the trainer's)."""
    from .. import ops  # (ops imports this module's siblings)

    s = ops.loss_scale()
    if s != 1.0 and trainer.scaler is None:
        trainer.scaler = LossScaler(loss.device, init_scale=s, step=trainer.step_count)
    trainer.step_count += 1
    if trainer.scaler is None:
        loss.backward(ops.backward_seed(loss) if loss.is_cuda else None)
        trainer.flat.adam(trainer.step_count, trainer.lr, trainer.betas, trainer.eps, trainer.dp.finish())
        return
    loss.backward(trainer.scaler.seed)
    trainer.flat.adam_scaled(trainer.scaler, trainer.lr, trainer.betas, trainer.eps, trainer.dp.finish())
