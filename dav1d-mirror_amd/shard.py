"""Frame sharding across ranks: independent frames, one per
GPU, no collective on the data path.  Rank r reconstructs frame r; the only
communication is the max-over-ranks timing (and optional checksum) after
the timed region.  Works with the nccl (RCCL) and gloo backends."""
import dataclasses


def rank_config(base, rank):
    """The frame rank `rank` owns: same shape and mix, its own seed."""
    return dataclasses.replace(base, seed=base.seed + 7919 * rank)


def max_over_ranks(value, dist, device):
    import torch
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value, dist, device):
    import torch
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return int(value)
    t = torch.tensor([int(value)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def aggregate_gpix_per_s(pixels_per_frame, steps, world, elapsed_max_s):
    """Whole-job throughput: every rank's frames over the slowest rank's time."""
    return pixels_per_frame * steps * world / elapsed_max_s / 1e9
