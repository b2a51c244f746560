"""Data parallelism over frame pairs: one process per GPU, the model replicated
(rank 0's initial parameters broadcast once), frame pairs sharded, the flat gradient all-reduced
in ~8 MB buckets that are launched from backward as soon as the layers writing them are done, so
the RCCL ring over xGMI overlaps the rest of the backward pass.  Backend-agnostic host logic (also
runs on gloo/CPU, which is how tests/test_ddp.py covers it).

Bucket readiness.  The trainers keep every parameter as a view into one flat buffer
(`FlatParams`), in `module.parameters()` order, and the HIP backward writes weight gradients
straight into it.  The model's top-level blocks ("units": its children, with ModuleList /
ModuleDict expanded) are called once per forward; a forward pre-hook attaches a gradient hook to
each call's input.  That hook fires once the input's gradient is complete, i.e. after the block's
backward -- which wrote all of the block's parameter gradients -- has run.  A bucket (a contiguous
range of the flat gradient, cut at parameter boundaries, built from the end of the buffer because
backward reaches the last layers first) is launched as an async all-reduce when every unit owning
one of its parameters has had all its calls' input hooks fire.  Units whose input does not require
grad (the first conv on the images, AdaAttN levels fed by frozen VGG features) and parameters
outside any unit are reduced by `finish()` after backward returns.  Hooks fire in the same order
on every rank (same graph), so the collectives are issued in the same order everywhere.
"""
import torch
import torch.distributed as dist
from torch import nn

BUCKET_BYTES = 8 << 20


def world_info(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def shard_seed(base, rank):
    """Each rank draws its own frame pairs (weak scaling: per-GPU batch fixed)."""
    return base + rank


def allreduce_grads(flat_g, group=None):
    """Sum the flat gradient over ranks (one collective); return the scale (1/world) that the
    optimizer applies, so the update uses the mean of the per-shard reference gradients."""
    _, world = world_info(group)
    if world == 1:
        return 1.0
    dist.all_reduce(flat_g, op=dist.ReduceOp.SUM, group=group)
    return 1.0 / world


def broadcast_params(flat_p, group=None):
    """Replicas start from rank 0's parameters (one broadcast of the flat buffer)."""
    _, world = world_info(group)
    if world > 1:
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast(flat_p, src=src, group=group)


def _units(model):
    out = []
    for name, m in model.named_children():
        if isinstance(m, (nn.ModuleList, nn.ModuleDict)):
            out += [(f"{name}.{n}", c) for n, c in _units_of_container(m)]
        else:
            out.append((name, m))
    return out


def _units_of_container(c):
    out = []
    for n, m in c.named_children():
        if isinstance(m, (nn.ModuleList, nn.ModuleDict)):
            out += [(f"{n}.{k}", x) for k, x in _units_of_container(m)]
        else:
            out.append((n, m))
    return out


class GradBuckets:
    """Bucketed, backward-overlapped all-reduce of a FlatParams gradient (see module docstring).

    step protocol:  begin() -> forward + backward -> finish() (returns the 1/world scale)."""

    def __init__(self, model, flat, group=None, bucket_bytes=BUCKET_BYTES):
        self.flat, self.group = flat, group
        _, self.world = world_info(group)
        spans, off = {}, 0
        for p in flat.params:
            spans[id(p)] = (off, p.numel())
            off += p.numel()
        # buckets: contiguous [lo, hi) ranges, cut at parameter boundaries, from the end
        cap = max(1, bucket_bytes // 4)
        bounds, hi, size = [], off, 0
        for p in reversed(flat.params):
            o, k = spans[id(p)]
            size += k
            if size >= cap:
                bounds.append((o, hi))
                hi, size = o, 0
        if hi > 0:
            bounds.append((0, hi))
        self.buckets = bounds  # backward order: last parameters first
        owner = {}
        self.units = []
        for name, m in _units(model):
            ps = [p for p in m.parameters() if id(p) in spans]
            if not ps:
                continue
            self.units.append((name, m))
            u = len(self.units) - 1
            for p in ps:
                owner[id(p)] = u
            m.register_forward_pre_hook(self._make_pre_hook(u))
        # bucket -> the units owning its parameters (None = a parameter outside every unit)
        self.bucket_units = []
        for lo, hi in self.buckets:
            us = set()
            for p in flat.params:
                o, k = spans[id(p)]
                if o < hi and o + k > lo:
                    us.add(owner.get(id(p)))
            self.bucket_units.append(us)
        self.unit_buckets = [[b for b, us in enumerate(self.bucket_units) if u in us] for u in range(len(self.units))]
        self.active = False
        self.works = []
        self.launched = []

    def _make_pre_hook(self, u):
        def pre_hook(_module, inputs):
            if not self.active or not torch.is_grad_enabled():
                return
            t = next((x for x in inputs if isinstance(x, torch.Tensor) and x.requires_grad), None)
            if t is None:
                self.blocked[u] = True
                return
            self.calls[u] += 1
            t.register_hook(lambda g, u=u: self._unit_done(u))

        return pre_hook

    def begin(self):
        n = len(self.units)
        self.calls, self.done, self.blocked = [0] * n, [0] * n, [False] * n
        self.works, self.launched = [], [False] * len(self.buckets)
        self.active = self.world > 1

    def _unit_complete(self, u):
        return u is not None and not self.blocked[u] and self.done[u] == self.calls[u]

    def _unit_done(self, u):
        if not self.active:
            return None
        self.done[u] += 1
        if self.done[u] == self.calls[u]:
            for b in self.unit_buckets[u]:
                if not self.launched[b] and all(self._unit_complete(x) for x in self.bucket_units[b]):
                    self._launch(b)
        return None

    def _launch(self, b):
        lo, hi = self.buckets[b]
        self.launched[b] = True
        self.works.append(dist.all_reduce(self.flat.g[lo:hi], op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    def finish(self):
        """Reduce the buckets backward did not launch, wait for all (the current stream waits on
        the collectives' stream), return the optimizer's gradient scale 1/world."""
        if self.world == 1:
            return 1.0
        self.in_backward = len(self.works)  # buckets launched from backward hooks (overlapped)
        for b in range(len(self.buckets)):
            if not self.launched[b]:
                self._launch(b)
        for w in self.works:
            w.wait()
        self.active = False
        return 1.0 / self.world

    def stats(self):
        return {"buckets": len(self.buckets), "bucket_mb": [4 * (h - lo) / 2 ** 20 for lo, h in self.buckets],
                "launched_in_backward": getattr(self, "in_backward", None)}
