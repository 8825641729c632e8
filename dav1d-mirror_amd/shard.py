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


def gather_over_ranks(value, dist, device):
    """Every rank's float value, in rank order (all_gather; a 1-element list
    without a process group)."""
    import torch
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [float(value)]
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(o.item()) for o in out]


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
_HDR = 6   # per array: name code, dtype code, rows, cols, nbytes, byte offset in the flat buffer
_ALIGN = 16
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


def pack_frame(fd, pin=False):
    """(header int64 list, flat uint8 tensor): every array of the frame at a
    16-byte aligned offset of ONE buffer, so the feed is one send per rank
     instead of one per array.  pin: page-locked host memory,
    so the host-to-device copy before an RCCL send is one DMA."""
    import torch
    named = _frame_arrays(fd)
    h, off = [len(named)], 0
    for name, a in named:
        a2 = a.reshape(a.shape[0], -1) if a.ndim > 1 else a.reshape(1, -1)
        h += [_NAMES.index(name), _DTYPES.index(a.dtype.type), a2.shape[0], a2.shape[1], a.nbytes, off]
        off += (a.nbytes + _ALIGN - 1) // _ALIGN * _ALIGN
    flat = torch.empty(max(off, _ALIGN), dtype=torch.uint8, pin_memory=pin)
    fv = flat.numpy()
    for i, (_, a) in enumerate(named):
        nb, o = h[1 + _HDR * i + 4], h[1 + _HDR * i + 5]
        fv[o:o + nb] = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
    return h, flat


def unpack_frame(h, flat, cfg):
    """The FrameData a packed header + flat host buffer (numpy uint8) hold."""
    from . import abi
    from . import workload as wl
    got = {}
    for i in range(int(h[0])):
        name, code, rows, cols, nb, o = (int(v) for v in h[1 + _HDR * i: 1 + _HDR * (i + 1)])
        a = flat[o:o + nb].view(_DTYPES[code])
        got[_NAMES[name]] = a.reshape(rows, cols) if rows > 1 else a.reshape(-1)
    flat_ = lambda k: None if k not in got else got[k].reshape(-1)   # noqa: E731
    refs = [[got[f"ref{r}_{p}"] for p in range(3)] for r in range(2) if f"ref{r}_0" in got]
    dst_init = [got[f"dst_init{p}"] for p in range(3)] if "dst_init0" in got else None
    W, H = cfg.width, cfg.height
    fd = wl.FrameData(cfg=cfg, units=got["units"].reshape(-1).view(abi.UNIT_DTYPE),
                      class_start=flat_("class_start"), coefs=flat_("coefs"), edges=flat_("edges"), refs=refs,
                      plane_wh=[(W, H), (W // 2, H // 2), (W // 2, H // 2)], blk=flat_("blk"),
                      cfl_luma=got["cfl_luma"], dst_init=dst_init, aux=flat_("aux"), aux_pool=flat_("aux_pool"),
                      class_warp=flat_("class_warp"),
                      src_xy=None if "src_xy" not in got else got["src_xy"].reshape(-1, 2, 2))
    fd.stats = wl.algorithmic_bytes(fd)
    return fd


def feed_frame(cfg_of_rank, rank, world, dist, device, max_arrays=len(_NAMES)):
    """Rank 0 builds world frames (cfg_of_rank(r)) and sends frame r to rank r
    as one header and ONE flattened buffer (packed in page-locked memory on a
    GPU); returns (FrameData of this rank, feed seconds, bytes received).
    Works on any backend with send/recv (nccl = RCCL on device tensors, gloo
    on CPU)."""
    import time
    import torch
    from . import workload as wl
    hlen = 2 + _HDR * max_arrays   # [total bytes, n arrays, per-array fields...]
    gpu = str(device) != "cpu"
    t_total, nbytes = 0.0, 0
    if rank == 0:
        mine = None
        for r in range(world):
            fd = wl.make_frame(cfg_of_rank(r))
            if r == 0:
                mine = fd
                continue
            h, flat = pack_frame(fd, pin=gpu)
            hdr = torch.zeros(hlen, dtype=torch.int64)
            hdr[0] = flat.numel()
            hdr[1:1 + len(h)] = torch.tensor(h, dtype=torch.int64)
            if gpu:
                torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            buf = flat.to(device, non_blocking=True)
            dist.send(hdr.to(device), dst=r)
            dist.send(buf, dst=r)
            if gpu:
                torch.cuda.synchronize(device)
            t_total += time.perf_counter() - t0
            nbytes += int(flat.numel())
        return mine, t_total, nbytes
    hdr = torch.zeros(hlen, dtype=torch.int64, device=device)
    t0 = time.perf_counter()
    dist.recv(hdr, src=0)
    h = hdr.cpu().tolist()
    buf = torch.empty(int(h[0]), dtype=torch.uint8, device=device)
    dist.recv(buf, src=0)
    flat = buf.cpu().numpy()
    if gpu:
        torch.cuda.synchronize(device)
    t_total = time.perf_counter() - t0
    nbytes = int(h[0])
    return unpack_frame(h[1:], flat, cfg_of_rank(rank)), t_total, nbytes
