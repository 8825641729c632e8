"""Diagnostics for the superblock wavefront (DGPU_IS_SB): one small frame,
a short poll bound, then the error word, the superblock done flags and the
pixel mismatches against the oracle.  Run on the GPU box under a timeout,
with the diagnostics build (tools/build_variants.sh sbdiag,
DAV1D_GPU_LIB_VARIANT=sbdiag): product builds ignore DAV1D_GPU_SB_TRACE."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("DAV1D_GPU_FLOW_SPIN_LIMIT", "20000")
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
orc = ge.load_oracle()
import torch  # noqa: E402
import dav1d_mirror_amd.intra as intra  # noqa: E402

kw = dict(seed=31)
if len(sys.argv) > 1:
    kw.update(eval(sys.argv[1]))
fr = intra.make_intra_frame(intra.IntraConfig(**kw))
perm, cut, cls, sls, sds, sdeps = intra.sb_schedule(fr)
print("units", len(fr.units), "groups", len(cut) - 1, "sb", len(sls) - 1, "sb deps", len(sdeps), flush=True)
dev = intra.DeviceIntraFrame(fr, mode="sb")
print("workspace", dev.workspace.numel(), flush=True)
n_sb = len(sls) - 1
# the kernel's progress trace in page-locked host memory, read by a watcher
# thread while the main thread waits for the device
trace = torch.zeros(16 * n_sb + 16, dtype=torch.int32, pin_memory=True)
os.environ["DAV1D_GPU_SB_TRACE"] = str(trace.data_ptr())
phases = None
if os.environ.get("DAV1D_GPU_SB_PHASE_MARKS"):   # DGPU_TRACE builds: the class code's marks (group 8 = ALL_IE)
    phases = torch.zeros(9 << 20, dtype=torch.int64, pin_memory=True)
    os.environ["DAV1D_GPU_SB_PHASES"] = str(phases.data_ptr())


def show(tag):
    tr = trace.numpy().view(np.uint32).reshape(-1, 16)
    print(tag, flush=True)
    if phases is not None:
        m = phases.numpy()[8 << 20:(8 << 20) + 16]
        print("class-code marks reached:", [i for i in range(16) if m[i]], flush=True)
    for b in range(n_sb):
        r = tr[b]
        if not r.any():
            continue
        waves = " ".join("w%d last task %s" % (w, int(r[2 * w + 1]) & 0xffffff if r[2 * w + 1] else "-") for w in range(4))
        print("wg %3d sb %s done %s | %s" % (b, hex(r[8]), hex(r[9]), waves), flush=True)


def watch():
    time.sleep(20)
    show("TIMEOUT: trace after 20 s")
    os._exit(3)


import threading  # noqa: E402
threading.Thread(target=watch, daemon=True).start()
t0 = time.time()
dev.launch()
torch.cuda.synchronize()
show("trace")
print("launch+sync %.3f s" % (time.time() - t0), flush=True)
ws = dev.workspace.cpu().numpy()
ctr = ws[:128].view(np.int32)
done = ws[128:128 + 4 * n_sb].view(np.int32)
print("ticket", ctr[0], "error", ctr[1], "done", done.tolist()[:64], flush=True)
ho = orc.HostIntraFrame(fr)
ho.run()
got = dev.planes_host()
for p in range(3):
    d = np.argwhere(got[p] != ho.dst[p])
    print("plane", p, "mismatches", len(d), d[:5].tolist(), flush=True)
