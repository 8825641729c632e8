"""Pin the committed constant tables (dav1d-mirror_amd/csrc/dsp_tables.h) to
the reference's own data, src/tables.c.

Every kernel, the C oracle and both numpy restatements read
csrc/dsp_tables.h, which tools/gen_tables.py extracted with regular
expressions; an extraction slip (the filter-intra [5][64] -> [5][8][7]
re-layout, the x86-vs-C tap order of src/tables.c:746-758, a dropped zero of
the sparse dr_intra_derivative) would pass every other test.  This test
parses tables.c by a different method: it cuts each table's definition out
of the file as whole lines (no value parsing in Python) and lets the C
compiler evaluate the initialisers (designated initialisers, the F() macro of
the filter-intra table, sparse zeros), once with ARCH_X86 = 0 and once with
ARCH_X86 = 1, next to the committed header; the program compares every
element in C.  The reference is read at test time only (skipped where
/root/reference is absent, e.g. on the GPU box); nothing of it is kept.

Tables (src/tables.c line of the definition): dav1d_sgr_params :415,
dav1d_sgr_x_by_x :422, dav1d_mc_subpel_filters :443, dav1d_mc_warp_filter
:547, dav1d_resize_filter :651, dav1d_sm_weights :686,
dav1d_dr_intra_derivative :714, dav1d_filter_intra_taps :759,
dav1d_obmc_masks :808, dav1d_gaussian_sequence :825; and the batch kernel's
packed banks dspt_mc8 / dspt_mc16 derived from the sub-pel filters (m = 0
the identity tap).
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
TABLES_C = os.path.join(REF, "src", "tables.c")

NAMES = ("dav1d_sgr_params", "dav1d_sgr_x_by_x", "dav1d_mc_subpel_filters", "dav1d_mc_warp_filter",
         "dav1d_resize_filter", "dav1d_sm_weights", "dav1d_dr_intra_derivative", "dav1d_filter_intra_taps",
         "dav1d_obmc_masks", "dav1d_gaussian_sequence")


def _cut(lines, name):
    """The definition of `name` as whole lines: from its `const` line to the
    first line that closes it (`};`)."""
    start = next(i for i, l in enumerate(lines) if l.startswith("const ") and re.search(r"\b%s\b" % name, l))
    end = next(i for i in range(start, len(lines)) if lines[i].strip() == "};")
    return lines[start:end + 1]


def _f_macro(lines):
    """The `#if ARCH_X86 ... #endif` block that defines F() for the
    filter-intra table."""
    i = next(i for i, l in enumerate(lines) if "dav1d_filter_intra_taps" in l)
    start = max(j for j in range(i) if lines[j].startswith("#if ARCH_X86"))
    end = next(j for j in range(start, i) if lines[j].startswith("#endif"))
    return lines[start:end + 1]


_CHECK = r"""
#define DSPT_QUAL static const
#include "dsp_tables.h"

static int bad = 0;
#define CMP(tab, i, got, want) do { if ((long)(got) != (long)(want)) { \
    if (bad < 20) printf("MISMATCH %s[%d]: header %ld, tables.c %ld\n", tab, (int)(i), (long)(got), (long)(want)); \
    bad++; } } while (0)

int main(void) {
    int n = 0;
    for (int i = 0; i < 16; i++) for (int k = 0; k < 2; k++, n++)
        CMP("sgr_params", n, dspt_sgr_params[2 * i + k], dav1d_sgr_params[i][k]);
    for (int i = 0; i < 256; i++, n++) CMP("sgr_x_by_x", i, dspt_sgr_x_by_x[i], dav1d_sgr_x_by_x[i]);
    for (int b = 0; b < 6; b++) for (int m = 0; m < 15; m++) for (int t = 0; t < 8; t++, n++)
        CMP("subpel", (b * 15 + m) * 8 + t, dspt_subpel[(b * 15 + m) * 8 + t], dav1d_mc_subpel_filters[b][m][t]);
    for (int b = 0; b < 6; b++) for (int m = 0; m < 16; m++) {
        signed char tap[8];
        for (int t = 0; t < 8; t++) tap[t] = m ? dav1d_mc_subpel_filters[b][m - 1][t] : (t == 3 ? 64 : 0);
        for (int i = 0; i < 2; i++, n++) {
            unsigned v = 0;
            for (int j = 0; j < 4; j++) v |= (unsigned)(unsigned char)tap[4 * i + j] << (8 * j);
            CMP("mc8", (b * 16 + m) * 2 + i, dspt_mc8[(b * 16 + m) * 2 + i], v);
        }
        for (int i = 0; i < 4; i++, n++) {
            unsigned v = (unsigned)(unsigned short)tap[2 * i] | (unsigned)(unsigned short)tap[2 * i + 1] << 16;
            CMP("mc16", (b * 16 + m) * 4 + i, dspt_mc16[(b * 16 + m) * 4 + i], v);
        }
    }
    for (int r = 0; r < 193; r++) for (int t = 0; t < 8; t++, n++)
        CMP("warp", r * 8 + t, dspt_warp[r * 8 + t], dav1d_mc_warp_filter[r][t]);
    for (int r = 0; r < 64; r++) for (int t = 0; t < 8; t++, n++)
        CMP("resize", r * 8 + t, dspt_resize[r * 8 + t], dav1d_resize_filter[r][t]);
    for (int i = 0; i < 128; i++, n++) CMP("sm_weights", i, dspt_sm_weights[i], dav1d_sm_weights[i]);
    for (int i = 0; i < 44; i++, n++) CMP("dr_deriv", i, dspt_dr_deriv[i], dav1d_dr_intra_derivative[i]);
    /* F(idx, f0..f6): the header's [filter][output idx][tap k] against the
       reference's flat [filter][64] in the layout ARCH_X86 selects */
    for (int f = 0; f < 5; f++) for (int idx = 0; idx < 8; idx++) for (int k = 0; k < 7; k++, n++) {
        const int pos = ARCH_X86 ? 2 * idx + 16 * (k >> 1) + (k & 1) : idx + 8 * k;
        CMP("filter_intra", (f * 8 + idx) * 7 + k, dspt_filter_intra[(f * 8 + idx) * 7 + k],
            dav1d_filter_intra_taps[f][pos]);
    }
    for (int i = 0; i < 64; i++, n++) CMP("obmc", i, dspt_obmc[i], dav1d_obmc_masks[i]);
    for (int i = 0; i < 2048; i++, n++) CMP("gaussian", i, dspt_gaussian[i], dav1d_gaussian_sequence[i]);
    printf("compared %d elements, %d mismatches\n", n, bad);
    return bad != 0;
}
"""


@pytest.mark.skipif(not os.path.exists(TABLES_C), reason="the reference tree is not present (GPU box)")
@pytest.mark.parametrize("x86", [0, 1])
def test_tables_match_reference(tmp_path, x86):
    lines = open(TABLES_C).read().splitlines()
    body = ["#include <stdint.h>", "#include <stdio.h>", "#include <dav1d/headers.h>",
            "#define ALIGN(decl, a) decl", f"#define ARCH_X86 {x86}"]
    for name in NAMES:
        if name == "dav1d_filter_intra_taps":
            body += _f_macro(lines)
        body += _cut(lines, name)
    src = tmp_path / "pin.c"
    src.write_text("\n".join(body) + "\n" + _CHECK)
    exe = tmp_path / "pin"
    subprocess.run(["cc", "-std=c11", "-O0", "-Werror=override-init", "-I", os.path.join(REF, "include"),
                    "-I", os.path.join(ROOT, "dav1d-mirror_amd", "csrc"), str(src), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    n = int(re.search(r"compared (\d+) elements", r.stdout).group(1))
    assert n == 32 + 256 + 720 + 96 * 6 + 1544 + 512 + 128 + 44 + 280 + 64 + 2048, r.stdout
