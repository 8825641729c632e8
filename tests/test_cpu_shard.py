"""The N>1 path on CPU: world_size-2 gloo, each rank reconstructs its own
frame (oracle on the host, standing in for the GPU kernel), timings reduce
with MAX and pixel counts with SUM exactly as bench.py does over RCCL."""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    import __graft_entry__ as ge
    ge.load_package()
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.shard as sh
    orc = ge.load_oracle()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    cfg = sh.rank_config(wl.FrameConfig(width=256, height=128), rank)
    fd = wl.make_frame(cfg)
    hf = orc.HostFrame(fd)
    hf.run()
    digest = int(np.bitwise_xor.reduce(hf.dst[0].view(np.uint8).ravel().astype(np.int64)
                                       * np.arange(hf.dst[0].size, dtype=np.int64)))
    el = sh.max_over_ranks(0.01 * (rank + 1), dist, "cpu")
    px = sh.sum_over_ranks(fd.stats["pixels"], dist, "cpu")
    q.put((rank, cfg.seed, digest, el, px, fd.stats["pixels"]))
    dist.destroy_process_group()


def test_two_rank_frame_sharding_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    seeds = {r[1] for r in res}
    assert len(seeds) == world                      # distinct frame per rank
    assert res[0][2] != res[1][2]                   # different content
    assert all(abs(r[3] - 0.02) < 1e-12 for r in res)   # MAX over ranks
    assert all(r[4] == res[0][5] + res[1][5] for r in res)  # SUM of pixels


def _feed_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    import __graft_entry__ as ge
    ge.load_package()
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.shard as sh
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    # world 2: a full frame; 3: an itx frame (dst_init); 4: an ext frame (aux,
    # aux_pool and class_warp: mask / palette / warp / inter-intra units)
    base = wl.FrameConfig(width=256, height=128, kind={2: "full", 3: "itx", 4: "ext"}[world])
    fd, secs, nbytes = sh.feed_frame(lambda r: sh.rank_config(base, r), rank, world, dist, "cpu")
    ref = wl.make_frame(sh.rank_config(base, rank))   # what this rank must have received
    same = (fd.units.tobytes() == ref.units.tobytes() and np.array_equal(fd.class_start, ref.class_start)
            and np.array_equal(fd.coefs, ref.coefs) and np.array_equal(fd.edges, ref.edges)
            and np.array_equal(fd.cfl_luma, ref.cfl_luma)
            and all(np.array_equal(fd.refs[k][p], ref.refs[k][p]) for k in range(2) for p in range(3))
            and (ref.dst_init is None or all(np.array_equal(fd.dst_init[p], ref.dst_init[p]) for p in range(3)))
            and all((getattr(ref, k) is None and getattr(fd, k) is None)
                    or np.array_equal(getattr(fd, k), getattr(ref, k)) for k in ("aux", "aux_pool", "class_warp", "src_xy"))
            and fd.stats == ref.stats)
    q.put((rank, same, nbytes))
    dist.destroy_process_group()


def test_rccl_feed_scatter_gloo():
    """bench.py --feed rccl: rank 0 generates every frame and sends frame r
    to rank r (send/recv, the same calls RCCL runs over xGMI); each rank
    ends up with exactly the frame it would have generated itself."""
    for world in (2, 3, 4):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        ps = [ctx.Process(target=_feed_worker, args=(r, world, port, q)) for r in range(world)]
        for p in ps:
            p.start()
        res = sorted(q.get(timeout=240) for _ in range(world))
        for p in ps:
            p.join(timeout=60)
            assert p.exitcode == 0
        assert all(r[1] for r in res), res
        assert res[0][2] > 0 and all(r[2] > 0 for r in res[1:])


def test_pack_frame_one_buffer():
    """The feed's flat image: every array at a 16-byte
    aligned offset of one buffer, and unpacking gives the frame back."""
    sys.path.insert(0, ROOT)
    import __graft_entry__ as ge
    ge.load_package()
    import dav1d_mirror_amd.workload as wl
    import dav1d_mirror_amd.shard as sh
    for kind in ("full", "ext", "itx"):
        fd = wl.make_frame(wl.FrameConfig(width=256, height=128, kind=kind))
        h, flat = sh.pack_frame(fd)
        n = h[0]
        offs = [h[1 + sh._HDR * i + 5] for i in range(n)]
        assert all(o % 16 == 0 for o in offs) and offs == sorted(offs)
        back = sh.unpack_frame(h, flat.numpy(), fd.cfg)
        assert back.units.tobytes() == fd.units.tobytes() and np.array_equal(back.coefs, fd.coefs)
        assert all(np.array_equal(back.refs[k][p], fd.refs[k][p]) for k in range(2) for p in range(3))
        assert back.stats == fd.stats
