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
_HDR = 5   # per array: name code, dtype code, rows, cols, nbytes
# every FrameData array the batch can read, by name; optional ones (None in
# the frame) are simply not sent, and the receiver leaves them None
_NAMES = (["units", "class_start", "coefs", "edges", "blk", "cfl_luma", "aux", "aux_pool", "class_warp", "src_xy"]
          + [f"ref{r}_{p}" for r in range(2) for p in range(3)] + [f"dst_init{p}" for p in range(3)])


def _frame_arrays(fd):
    """(name, array) of every array of the frame that is present."""
    out = [("units", fd.units.view(np.uint8)), ("class_start", fd.class_start.astype(np.int32)),
           ("coefs", fd.coefs), ("edges", fd.edges), ("blk", fd.blk.astype(np.int32)), ("cfl_luma", fd.cfl_luma)]
    for name in ("aux", "aux_pool", "class_warp", "src_xy"):
        a = getattr(fd, name)
        if a is not None:
            out.append((name, np.asarray(a)))
    assert len(fd.refs) <= 2, "feed ships at most 2 reference pictures"
    out += [(f"ref{r}_{p}", a) for r, rp in enumerate(fd.refs) for p, a in enumerate(rp)]
    if fd.dst_init is not None:
        out += [(f"dst_init{p}", a) for p, a in enumerate(fd.dst_init)]
    return out


def _header(named):
    h = [len(named)]
    for name, a in named:
        a2 = a.reshape(a.shape[0], -1) if a.ndim > 1 else a.reshape(1, -1)
        h += [_NAMES.index(name), _DTYPES.index(a.dtype.type), a2.shape[0], a2.shape[1], a.nbytes]
    return h


def feed_frame(cfg_of_rank, rank, world, dist, device, max_arrays=len(_NAMES)):
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
            named = _frame_arrays(fd)
            arrs = [a for _, a in named]
            h = _header(named)
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
    got = {}
    for i in range(int(h[0])):
        name, code, rows, cols, nb = h[1 + _HDR * i: 1 + _HDR * (i + 1)]
        b = torch.empty(int(nb), dtype=torch.uint8, device=device)
        dist.recv(b, src=0)
        a = b.cpu().numpy().view(_DTYPES[int(code)])
        got[_NAMES[int(name)]] = a.reshape(int(rows), int(cols)) if rows > 1 else a.reshape(-1)
        nbytes += int(nb)
    if str(device) != "cpu":
        torch.cuda.synchronize(device)
    t_total = time.perf_counter() - t0
    cfg = cfg_of_rank(rank)
    from . import abi
    flat = lambda k: None if k not in got else got[k].reshape(-1)   # noqa: E731
    refs = [[got[f"ref{r}_{p}"] for p in range(3)] for r in range(2) if f"ref{r}_0" in got]
    dst_init = [got[f"dst_init{p}"] for p in range(3)] if "dst_init0" in got else None
    W, H = cfg.width, cfg.height
    fd = wl.FrameData(cfg=cfg, units=got["units"].reshape(-1).view(abi.UNIT_DTYPE),
                      class_start=flat("class_start"), coefs=flat("coefs"), edges=flat("edges"), refs=refs,
                      plane_wh=[(W, H), (W // 2, H // 2), (W // 2, H // 2)], blk=flat("blk"),
                      cfl_luma=got["cfl_luma"], dst_init=dst_init, aux=flat("aux"), aux_pool=flat("aux_pool"),
                      class_warp=flat("class_warp"),
                      src_xy=None if "src_xy" not in got else got["src_xy"].reshape(-1, 2, 2))
    fd.stats = wl.algorithmic_bytes(fd)
    return fd, t_total, nbytes
