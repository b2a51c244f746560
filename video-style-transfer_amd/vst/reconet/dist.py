"""Data parallelism over frame pairs: one process per GPU, one RCCL
all-reduce of the flat gradient per step.  Backend-agnostic host logic (also runs on gloo/CPU,
which is how tests/test_ddp.py covers it)."""
import torch.distributed as dist


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
