#!/usr/bin/env python3
"""Static instruction counts per kernel phase of one class: compiles
recon8.hip (or recon16) with DGPU_ONLY_CLASS=<tx> and DGPU_ASM_MARKS, then
counts VALU / SALU / LDS / VMEM instructions between the ;DGPU_MARK comments
(the phases of recon_units; a phase's count sums all its branch paths).

    python tools/phase_isa.py TX [8|16] [extra -D flags...]"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "dav1d-mirror_amd")


def main():
    tx = int(sys.argv[1])
    bpc = sys.argv[2] if len(sys.argv) > 2 else "8"
    extra = sys.argv[3:]
    out = f"/tmp/phase_{tx}_{bpc}.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I../include", "-Icsrc",
                    "--cuda-device-only", "-S", f"-DDGPU_ONLY_CLASS={tx}", "-DDGPU_ASM_MARKS", *extra,
                    f"csrc/recon{bpc}.hip", "-o", out], cwd=SRC, check=True, stderr=subprocess.DEVNULL)
    name = f"_ZN4dgpu7k_reconILi{bpc}ELi0EEEvNS_9ReconArgsIXT_EEE:"
    lines = open(out).read().split("\n")
    i = next(k for k, l in enumerate(lines) if l.startswith(name))
    phase = "prologue"
    cnt = collections.defaultdict(collections.Counter)
    ops = collections.defaultdict(collections.Counter)
    for l in lines[i + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.search(r";DGPU_MARK (\d+)", l)
        if m:
            phase = f"after mark {m.group(1)}"
            continue
        t = l.strip().split()
        if not t or t[0].startswith((";", ".")) or t[0].endswith(":"):
            continue
        op = t[0]
        kind = ("VALU" if op.startswith("v_") else "SALU" if op.startswith("s_") and not op.startswith(("s_load", "s_waitcnt", "s_cbranch", "s_branch", "s_buffer")) else
                "LDS" if op.startswith("ds_") else "VMEM" if op.startswith(("global_", "buffer_", "flat_")) else
                "SMEM" if op.startswith(("s_load", "s_buffer")) else "other")
        cnt[phase][kind] += 1
        ops[phase][op] += 1
    for ph, c in cnt.items():
        print(f"{ph:14s} " + "  ".join(f"{k} {v:5d}" for k, v in sorted(c.items())))
        if "-v" in os.environ.get("PHASE_ISA", ""):
            print("     ", ", ".join(f"{o} {n}" for o, n in ops[ph].most_common(25)))


if __name__ == "__main__":
    main()
