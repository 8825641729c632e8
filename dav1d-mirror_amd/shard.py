"""Frame sharding across ranks: independent frames, one per
GPU, no collective on the data path.  Rank r reconstructs frame r; the only
communication is the max-over-ranks timing (and optional checksum) after
the timed region.  Works with the nccl (RCCL) and gloo backends.

Optionally (bench.py --feed rccl) rank 0 produces every frame and scatters
them over RCCL point-to-point before the timed region (feed_frame)."""
import dataclasses

import numpy as np


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


# ------------------------------------------------------------ frame feed ---
# BASELINE config 5 with the coded blocks coming from one producer: rank 0
# generates every rank's frame (standing in for the host-side decoder that
# parses the bitstream) and ships each rank its batch over RCCL point-to-point
# (xGMI on one node).  Frames are independent, so this is a scatter, not a
# broadcast: rank r receives only frame r.  The feed is timed on its own and
# stays outside the reconstruction's timed region.

_DTYPES = [np.uint8, np.int16, np.int32, np.uint16, np.int64]
_HDR = 4   # per array: dtype code, rows, cols, nbytes


def _frame_arrays(fd):
    arrs = [fd.units.view(np.uint8), fd.class_start.astype(np.int32), fd.coefs, fd.edges,
            fd.blk.astype(np.int32), fd.cfl_luma]
    arrs += [a for rp in fd.refs for a in rp]
    if fd.dst_init is not None:
        arrs += list(fd.dst_init)
    return arrs


def _header(arrs):
    h = [len(arrs)]
    for a in arrs:
        a2 = a.reshape(a.shape[0], -1) if a.ndim > 1 else a.reshape(1, -1)
        h += [_DTYPES.index(a.dtype.type), a2.shape[0], a2.shape[1], a.nbytes]
    return h


def feed_frame(cfg_of_rank, rank, world, dist, device, max_arrays=32):
    """Rank 0 builds world frames (cfg_of_rank(r)) and sends frame r to rank r;
    returns (FrameData of this rank, feed seconds, bytes received).  Works on
    any backend with send/recv (nccl = RCCL on device tensors, gloo on CPU)."""
    import time
    import torch
    from . import workload as wl
    hlen = 1 + _HDR * max_arrays
    t_total, nbytes = 0.0, 0
    if rank == 0:
        mine = None
        for r in range(world):
            fd = wl.make_frame(cfg_of_rank(r))
            if r == 0:
                mine = fd
                continue
            arrs = _frame_arrays(fd)
            h = _header(arrs)
            hdr = torch.zeros(hlen, dtype=torch.int64)
            hdr[:len(h)] = torch.tensor(h, dtype=torch.int64)
            bufs = [torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).to(device)
                    for a in arrs]
            if str(device) != "cpu":
                torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            dist.send(hdr.to(device), dst=r)
            for b in bufs:
                dist.send(b, dst=r)
            if str(device) != "cpu":
                torch.cuda.synchronize(device)
            t_total += time.perf_counter() - t0
            nbytes += sum(int(b.numel()) for b in bufs)
        return mine, t_total, nbytes
    hdr = torch.zeros(hlen, dtype=torch.int64, device=device)
    t0 = time.perf_counter()
    dist.recv(hdr, src=0)
    h = hdr.cpu().tolist()
    arrs = []
    for i in range(int(h[0])):
        code, rows, cols, nb = h[1 + _HDR * i: 1 + _HDR * (i + 1)]
        b = torch.empty(int(nb), dtype=torch.uint8, device=device)
        dist.recv(b, src=0)
        a = b.cpu().numpy().view(_DTYPES[int(code)])
        arrs.append(a.reshape(int(rows), int(cols)) if rows > 1 else a.reshape(-1))
        nbytes += int(nb)
    if str(device) != "cpu":
        torch.cuda.synchronize(device)
    t_total = time.perf_counter() - t0
    cfg = cfg_of_rank(rank)
    from . import abi
    units = arrs[0].reshape(-1).view(abi.UNIT_DTYPE)
    refs = [arrs[6:9], arrs[9:12]]
    dst_init = arrs[12:15] if len(arrs) > 12 else None
    W, H = cfg.width, cfg.height
    fd = wl.FrameData(cfg=cfg, units=units, class_start=arrs[1].reshape(-1), coefs=arrs[2].reshape(-1),
                      edges=arrs[3].reshape(-1), refs=refs, plane_wh=[(W, H), (W // 2, H // 2), (W // 2, H // 2)],
                      blk=arrs[4].reshape(-1), cfl_luma=arrs[5], dst_init=dst_init)
    fd.stats = wl.algorithmic_bytes(fd)
    return fd, t_total, nbytes
