#!/usr/bin/env python3
"""Compare two tools/codeobj_dump.sh dumps kernel by kernel: instruction
text with comments, branch offsets and PC-relative literals masked (those
move when another kernel of the object changes size).  Prints, per object,
the kernels whose code differs and those that are identical.

    python tools/codeobj_cmp.py <dump A> <dump B> [object ...]
"""
import os
import re
import sys

BR = re.compile(r"^(s_cbranch_\w+|s_branch|s_call_b64.*)\s+.*$")
PCREL = re.compile(r"^(s_add_u32|s_addc_u32)\s+(s\d+), (s\d+), (0x[0-9a-f]+|\d+)$")


def kernels(path):
    out, cur, body = {}, None, []
    for line in open(path):
        line = line.split("//")[0].rstrip()
        m = re.match(r"^([0-9a-f]*\s*)?<?([_A-Za-z][\w.$]*)>?:$", line.strip())
        if m and not line.startswith("\t"):
            if cur:
                out[cur] = body
            cur, body = m.group(2), []
            continue
        t = line.strip()
        if not t or cur is None:
            continue
        if BR.match(t):
            t = t.split()[0] + " <off>"
        mm = PCREL.match(t)
        if mm:
            t = f"{mm.group(1)} {mm.group(2)}, {mm.group(3)}, <lit>"
        body.append(t)
    if cur:
        out[cur] = body
    return out


def main():
    a, b = sys.argv[1], sys.argv[2]
    objs = sys.argv[3:] or sorted(f[:-2] for f in os.listdir(a) if f.endswith(".s"))
    for o in objs:
        ka, kb = kernels(os.path.join(a, o + ".s")), kernels(os.path.join(b, o + ".s"))
        same = [k for k in ka if k in kb and ka[k] == kb[k]]
        diff = [k for k in ka if k in kb and ka[k] != kb[k]]
        only = sorted(set(ka) ^ set(kb))
        print(f"{o}: {len(same)} identical, {len(diff)} differ, {len(only)} only in one")
        for k in diff:
            print(f"   differs: {k} ({len(ka[k])} vs {len(kb[k])} instructions)")
        for k in only[:10]:
            print(f"   only in {'A' if k in ka else 'B'}: {k}")


if __name__ == "__main__":
    main()
