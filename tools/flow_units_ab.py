"""Intra wavefront time per 4K frame (1 tile and 2x2 tiles, persistent
dataflow kernel) for the units-per-task cap in DAV1D_GPU_FLOW_UNITS (read
once per process: run one process per value).  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import __graft_entry__ as ge
    ge.load_package()
    import dav1d_mirror_amd.intra as intra
    orc = ge.load_oracle()
    out = {"units_cap": int(os.environ.get("DAV1D_GPU_FLOW_UNITS", "8")),
           "task_groups": os.environ.get("FLOW_TASK_GROUPS", "0") == "1"}
    for name, tiles in (("1_tile", (1, 1)), ("2x2_tiles", (2, 2))):
        fr = intra.make_intra_frame(intra.IntraConfig(width=3840, height=2160, tile_cols=tiles[0], tile_rows=tiles[1]))
        dev = intra.DeviceIntraFrame(fr, mode="persistent", task_groups=os.environ.get("FLOW_TASK_GROUPS", "0") == "1")
        s = torch.cuda.current_stream()
        for _ in range(2):
            dev.launch(s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(5):
            dev.launch(s)
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        got = dev.planes_host()
        ok = dev.flow_error() == 0
        if name == "1_tile":
            ho = orc.HostIntraFrame(fr)
            ho.run()
            ok = ok and all(np.array_equal(g, o) for g, o in zip(got, ho.dst))
        out[name] = {"ms_per_frame": round(ms, 3), "ok": bool(ok)}
        print(name, out[name], file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
