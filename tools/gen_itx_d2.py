#!/usr/bin/env python3
"""One-time source rewrite of csrc/dsp_common.hpp's 1-D transforms: every
rounded product sum r12(...) / r11(...) / r8s(...) (with the reference's
'- 4096' overflow-free correction term folded back in, when it follows the
call) gets an exact packed form next to it,

    D2SEL(dr<KA, KB, SH>(a, b), <the original expression>)

where dr is one v_dot2_i32_i16 of the int16 pair (a, b) with the constant
pair (KA, KB) and the rounding constant as accumulator.  D2SEL picks it when
the function's template flag D2 is set: the 8-bit path, where every value a
rotation reads is a transform input (int16 coefficient or a clipped row
output) or a clipped stage output, so it fits int16; 10/12-bit keep the
original expressions (their intermediates exceed int16).

    python tools/gen_itx_d2.py csrc/dsp_common.hpp      (rewrites in place)

Identity of the two forms: r12(P) + s*v == r12(P + 4096*s*v) exactly (4096*v
is a multiple of 4096), likewise r11 with 2048; the sums are exact in int32
for int16 operands and |K| < 2^15.
"""
import ast
import re
import sys

SH = {"r12": (12, 2048), "r11": (11, 1024), "r8s": (8, 128)}


def src(node):
    return ast.unparse(node)


def linear(node):
    """dict atom-source -> int coefficient, or None if not linear."""
    if isinstance(node, ast.BinOp) and isinstance(node.op, (ast.Add, ast.Sub)):
        l, r = linear(node.left), linear(node.right)
        if l is None or r is None:
            return None
        s = 1 if isinstance(node.op, ast.Add) else -1
        out = dict(l)
        for k, v in r.items():
            out[k] = out.get(k, 0) + s * v
        return out
    if isinstance(node, ast.BinOp) and isinstance(node.op, ast.Mult):
        c = const(node.left)
        if c is not None:
            r = linear(node.right)
            return None if r is None else {k: c * v for k, v in r.items()}
        c = const(node.right)
        if c is not None:
            l = linear(node.left)
            return None if l is None else {k: c * v for k, v in l.items()}
        return None
    if isinstance(node, ast.UnaryOp) and isinstance(node.op, ast.USub):
        l = linear(node.operand)
        return None if l is None else {k: -v for k, v in l.items()}
    if const(node) is not None:
        return None   # constants inside the sum: not produced by the sources
    if isinstance(node, (ast.Name, ast.Subscript)):
        return {src(node): 1}
    return None


def const(node):
    try:
        v = eval(compile(ast.Expression(node), "<c>", "eval"), {})
    except Exception:
        return None
    return v if isinstance(v, int) else None


def c_expr(s):   # python unparse -> C (only what these expressions contain)
    return s


def find_call(text, i):
    """text[i:] starts with name( : return the index after the matching )."""
    j = text.index("(", i)
    depth = 0
    for k in range(j, len(text)):
        if text[k] == "(":
            depth += 1
        elif text[k] == ")":
            depth -= 1
            if depth == 0:
                return j, k + 1
    raise ValueError


def rewrite_body(body):
    out = []
    pos = 0
    pat = re.compile(r"\b(r12|r11|r8s)\(")
    n = 0
    while True:
        m = pat.search(body, pos)
        if not m:
            out.append(body[pos:])
            break
        name = m.group(1)
        j, end = find_call(body, m.start())
        arg = body[j + 1:end - 1]
        if "D2SEL" in body[max(0, m.start() - 8):m.start()]:
            out.append(body[pos:end])
            pos = end
            continue
        try:
            tree = ast.parse(arg.replace("->", "."), mode="eval").body
        except SyntaxError:
            out.append(body[pos:end])
            pos = end
            continue
        lin = linear(tree)
        if lin is None or not (1 <= len(lin) <= 4):
            out.append(body[pos:end])
            pos = end
            continue
        sh, rnd = SH[name]
        if name == "r8s":
            lin = {k: 181 * v for k, v in lin.items()}
        # a following ' + atom' / ' - atom' correction that names an atom of the sum
        stop = end
        lin = dict(lin)
        while name in ("r12", "r11"):
            tail = re.match(r"\s*([+-])\s*((?:[A-Za-z_]\w*)(?:\[[^\]]+\])?)(?![\w\[\(*])", body[stop:])
            if not tail or tail.group(2) not in lin:
                break
            nxt = body[stop + tail.end():].lstrip()
            if nxt.startswith(("*", "/", ">>", "<<")):
                break
            lin[tail.group(2)] += (1 if tail.group(1) == "+" else -1) * (1 << sh)
            stop += tail.end()
        lin = {k: v for k, v in lin.items() if v != 0}
        if any(abs(v) >= 32768 for v in lin.values()):
            out.append(body[pos:end])
            pos = end
            continue
        orig = body[m.start():stop]
        atoms = list(lin.items())
        ks = ", ".join(str(v) for _, v in atoms)
        vs = ", ".join(a for a, _ in atoms)
        d2 = f"dr{len(atoms)}<{sh}, {ks}>({vs})"
        out.append(body[pos:m.start()])
        out.append(f"D2SEL(({d2}), ({orig}))")
        pos = stop
        n += 1
    return "".join(out), n


def main():
    path = sys.argv[1]
    text = open(path).read()
    start = text.index("template <int S, bool HALF>\n__device__ __forceinline__ void dct4")
    stop = text.index("// Walsh-Hadamard")
    body, n = rewrite_body(text[start:stop])
    open(path, "w").write(text[:start] + body + text[stop:])
    print(f"{n} sums rewritten")


if __name__ == "__main__":
    main()
