"""Data parallelism over frame pairs: one process per GPU, the model replicated
(rank 0's initial parameters broadcast once), frame pairs sharded, the flat gradient all-reduced
in ~8 MB buckets that are launched from backward as soon as the layers writing them are done, so
the RCCL ring over xGMI overlaps the rest of the backward pass.  Backend-agnostic host logic (also
runs on gloo/CPU, which is how tests/test_ddp.py covers it).

Bucket readiness.  The trainers keep every parameter as a view into one flat buffer
(`FlatParams`), in `module.parameters()` order, and the HIP backward writes weight gradients
straight into it (the Function then returns None for the parameter).  Every parameter carries a
post-accumulate-grad hook.  Autograd runs a leaf's AccumulateGrad node exactly once per backward,
after EVERY edge into it has delivered -- i.e. after the backward of every op that used the
parameter has run, and so after each of those ops has enqueued its write into the flat gradient on
the stream (whether it wrote in place and returned None, or returned the gradient to autograd).
A bucket (a contiguous range of the flat gradient, cut at parameter boundaries, built from the
end of the buffer because backward reaches the last layers first) is launched as an async
all-reduce when the hooks of all its parameters have fired.  No assumption about which input of a
module is consumed first is needed, and a parameter the graph never reaches (unused this step)
keeps its bucket back for `finish()`.  A hook that fires for a parameter whose bucket was already
launched (a second backward in the same step) raises instead of reducing a half-written slice.
Hooks fire in the same order on every rank (same graph), so the collectives are issued in the same
order everywhere.  Weight gradients that the HIP backward queued on its side stream
(ops.wgrad_into_sink) are joined into the current stream before each launch.
"""
import torch
import torch.distributed as dist

BUCKET_BYTES = 8 << 20


def world_info(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def shard_seed(base, rank):
    """Each rank draws its own frame pairs (weak scaling: per-GPU batch fixed)."""
    return base + rank


def step_seed(step, rank, base=1234):
    """numpy seed of the synthetic batch of training step `step` on `rank` (SURVEY.md §8(d):
    seed = 1234 + step; other ranks draw their own stream [1234 + step, rank], never another
    rank's or another step's)."""
    return base + step if rank == 0 else [base + step, rank]


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


class GradBuckets:
    """Bucketed, backward-overlapped all-reduce of a FlatParams gradient (see module docstring).

    step protocol:  begin() -> forward + backward -> finish() (returns the 1/world scale)."""

    def __init__(self, model, flat, group=None, bucket_bytes=BUCKET_BYTES):
        self.flat, self.group = flat, group
        _, self.world = world_info(group)
        spans, off = [], 0
        for p in flat.params:
            spans.append((off, p.numel()))
            off += p.numel()
        # buckets: contiguous [lo, hi) ranges, cut at parameter boundaries, from the end
        cap = max(1, bucket_bytes // 4)
        bounds, hi, size = [], off, 0
        for o, k in reversed(spans):
            size += k
            if size >= cap:
                bounds.append((o, hi))
                hi, size = o, 0
        if hi > 0:
            bounds.append((0, hi))
        self.buckets = bounds  # backward order: last parameters first
        self.bucket_of = [next(b for b, (lo, h) in enumerate(bounds) if lo <= o < h) for o, _ in spans]
        self.bucket_nparams = [self.bucket_of.count(b) for b in range(len(bounds))]
        self.names = {id(p): n for n, p in model.named_parameters()}
        self.active = False
        self.works = []
        self.launched = []
        if self.world > 1:
            for i, p in enumerate(flat.params):
                p.register_post_accumulate_grad_hook(self._make_hook(i))

    def _make_hook(self, i):
        def hook(p):
            if not self.active:
                return
            b = self.bucket_of[i]
            if self.launched[b]:
                raise RuntimeError(f"gradient of {self.names.get(id(p), '?')} accumulated after its bucket's "
                                   f"all-reduce was launched (a second backward before finish()?)")
            self.pending[b] -= 1
            if self.pending[b] == 0:
                self._launch(b)

        return hook

    def begin(self):
        self.pending = list(self.bucket_nparams)
        self.works, self.launched = [], [False] * len(self.buckets)
        self.active = self.world > 1

    def _launch(self, b):
        lo, hi = self.buckets[b]
        self.launched[b] = True
        if self.flat.g.is_cuda:
            from ..ops import join_side_streams  # weight gradients queued on the side stream

            join_side_streams()
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
