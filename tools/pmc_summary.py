#!/usr/bin/env python3
"""Summarise a tools/prof.sh run: per recon kernel, mean duration (kernel
trace) and mean per-dispatch value of every collected counter.

    python tools/pmc_summary.py gpurun_out/prof_TAG [-o profiles/rN/TAG_pmc.json]

FETCH_SIZE / WRITE_SIZE are in KB as rocprofv3 reports them; `*_MB` adds
the MB figure (x1.024e-3).  No gfx950 correction is applied here: the ½
factor of MI355X_MICROARCH.md holds for wide coalesced streaming reads,
which these scattered footprint loads are not -- see DESIGN.md."""
import argparse
import collections
import csv
import json
import os


def short(name):
    for k in ("k_recon", "k_tiles", "k_lr_frame", "k_cdef", "k_lpf", "k_grain"):
        if k in name:
            return name[name.index(k):].split("(")[0]
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("-o", "--out")
    a = ap.parse_args()
    res = collections.defaultdict(dict)
    tr = os.path.join(a.dir, "trace", "run_kernel_trace.csv")
    if os.path.exists(tr):
        durs = collections.defaultdict(list)
        for r in csv.DictReader(open(tr)):
            k = short(r["Kernel_Name"])
            if k:
                durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
        for k, v in durs.items():
            v = sorted(v)
            res[k]["launches"] = len(v)
            res[k]["mean_us"] = round(sum(v) / len(v), 2)
            res[k]["median_us"] = round(v[len(v) // 2], 2)
    for sub in sorted(os.listdir(a.dir)):
        f = os.path.join(a.dir, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        meta = {}
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if not k:
                continue
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = dict(vgpr=int(r["VGPR_Count"]), sgpr=int(r["SGPR_Count"]), lds=int(r["LDS_Block_Size"]),
                           scratch=int(r["Scratch_Size"]), wg=int(r["Workgroup_Size"]), grid=int(r["Grid_Size"]))
        for k, cs in acc.items():
            res[k].update(meta[k])
            for c, v in cs.items():
                m = sum(v) / len(v)
                res[k][c] = round(m, 1)
                if c in ("FETCH_SIZE", "WRITE_SIZE"):
                    res[k][c + "_MB"] = round(m * 1.024e-3, 3)
    txt = json.dumps(res, indent=1, sort_keys=True)
    print(txt)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()
