#!/usr/bin/env python3
"""Generates lambdafs_amd/csrc/xor_sched.hpp: common-subexpression XOR
schedules for the compile-time encode matrices.

The static encode kernels evaluate, per 2 KiB window, parity plane (o, q) =
XOR of the data bit-planes (r, i) that the 8x8 bit matrix of G[o][r] selects
(gf::row_mask). Written out plane by plane that is one XOR per selected input
plane (two per v_bitop3 xor3): 1,280 selected planes for RS(10,4), ~650 xor3.
Many triples of input planes recur across the 32 parity planes, so this tool
factors them out greedily (Paar's algorithm with xor3 temporaries): repeatedly
take the triple (or pair) of terms shared by the most parity planes whose
factoring saves the most xor3s, emit it as a temporary, substitute it. Rows are
scheduled in groups of G data rows (the group's 8G planes are the inputs; the
running parity planes carry the earlier groups), so a kernel can trade CSE
depth for registers.

Output (per matrix family, K, P, G), consumed by xor_sched_apply in
hrs_device.hpp:
  ops      temporaries v[8g + j] = v[a] ^ v[b] (^ v[c] unless c == 255), in
           order; v[0 .. 8G) are the group's input planes x[g][i] at 8g + i;
  terms    per parity plane (o, q): the vars XORed into it, flattened with
           offsets.
Deterministic (fixed seeds); tests/test_xor_sched.py regenerates the header
and checks every schedule against the matrix by symbolic evaluation.
"""
import itertools
import os
import random
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "lambdafs_amd", "csrc", "xor_sched.hpp")

# (family, K, P): family 0 = hops RS generator matrix (gf::EncodeMatrix),
# 1 = ISA-L Cauchy rows (gf::CauchyMatrix) -- the kernels' static shapes.
SHAPES = [(0, 3, 2), (0, 6, 3), (0, 10, 4), (0, 12, 4), (1, 10, 4), (1, 6, 3)]
GROUPS = [2, 4]  # + G = K (whole-window schedules)
RESTARTS = 8


def _tables():
    exp = [0] * 512
    log = [0] * 256
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= 0x11D
    for i in range(255, 512):
        exp[i] = exp[i - 255]
    return exp, log


EXP, LOG = _tables()


def mul(a, b):
    return 0 if a == 0 or b == 0 else EXP[LOG[a] + LOG[b]]


def inv(a):
    return EXP[255 - LOG[a]]


def rs_matrix(k, p):
    """gf::encode_matrix: G[r][c] = coefficient r of x^(p+c) mod g(x)."""
    g = [1] + [0] * p
    for i in range(p):
        r = EXP[i]
        for j in range(i + 1, -1, -1):
            hi = g[j - 1] if j > 0 else 0
            g[j] = hi ^ mul(g[j], r)
    rem = g[:p]
    out = [[0] * k for _ in range(p)]
    for c in range(k):
        for r in range(p):
            out[r][c] = rem[r]
        top = rem[p - 1]
        for r in range(p - 1, 0, -1):
            rem[r] = rem[r - 1] ^ mul(top, g[r])
        rem[0] = mul(top, g[0])
    return out


def cauchy_matrix(k, p):
    """gf::CauchyMatrix: m[r][c] = 1 / ((K + r) ^ c)."""
    return [[inv((k + r) ^ c) for c in range(k)] for r in range(p)]


def row_mask(c, q):
    return sum(1 << i for i in range(8) if (mul(c, 1 << i) >> q) & 1)


def plane_sets(mat, k, p, r0, g):
    """Per parity plane (o, q): the group's input vars (8 * (r - r0) + i)."""
    rows = []
    for o in range(p):
        for q in range(8):
            s = set()
            for r in range(r0, min(k, r0 + g)):
                m = row_mask(mat[o][r], q)
                for i in range(8):
                    if (m >> i) & 1:
                        s.add(8 * (r - r0) + i)
            rows.append(s)
    return rows


def final_cost(m, has_acc):
    """xor3 ops to fold m terms into a parity plane (plus its running value)."""
    if has_acc:
        return (m + 1) // 2
    return max(0, m // 2) if m else 0


def schedule(rows, nin, has_acc, seed):
    """Greedy CSE: returns (ops, rows) with ops = [(a, b, c or None)]."""
    rng = random.Random(seed)
    rows = [set(s) for s in rows]
    ops = []
    nxt = nin
    while True:
        # Factoring a triple out of a plane saves exactly one xor3 there; a
        # pair saves one only where the plane's term count has the right
        # parity (odd with a running value, even without). So a candidate's
        # gain is (planes it saves in) - 1 for the temporary itself.
        c3 = Counter()
        c2 = Counter()
        for s in rows:
            ss = sorted(s)
            c3.update(itertools.combinations(ss, 3))
            if (len(s) % 2 == 1) == has_acc:
                c2.update(itertools.combinations(ss, 2))
        best_gain = max(max(c3.values(), default=0), max(c2.values(), default=0)) - 1
        if best_gain <= 0:
            break
        best = [c for c, n in c3.items() if n - 1 == best_gain] + [c for c, n in c2.items() if n - 1 == best_gain]
        cand = rng.choice(sorted(best))
        v = nxt
        nxt += 1
        ops.append((cand[0], cand[1], cand[2] if len(cand) == 3 else None))
        for s in rows:
            if all(x in s for x in cand):
                for x in cand:
                    s.discard(x)
                s.add(v)
    return ops, rows


def best_schedule(rows, nin, has_acc):
    best = None
    for seed in range(RESTARTS):
        ops, fin = schedule(rows, nin, has_acc, seed)
        cost = len(ops) + sum(final_cost(len(s), has_acc) for s in fin)
        if best is None or cost < best[0]:
            best = (cost, ops, fin)
    return best


def evaluate(nin, ops, fin):
    """Symbolic check: each var as the set of input planes it XORs."""
    val = [frozenset([i]) for i in range(nin)]
    for a, b, c in ops:
        x = val[a] ^ val[b]
        if c is not None:
            x = x ^ val[c]
        val.append(x)
    out = []
    for s in fin:
        acc = frozenset()
        for t in s:
            acc = acc ^ val[t]
        out.append(acc)
    return out


def build(k, p, fam, g):
    mat = rs_matrix(k, p) if fam == 0 else cauchy_matrix(k, p)
    groups = []
    naive = 0
    total = 0
    for gi, r0 in enumerate(range(0, k, g)):
        rows = plane_sets(mat, k, p, r0, g)
        nin = 8 * min(g, k - r0)
        has_acc = gi > 0
        naive += sum(final_cost(len(s), has_acc) for s in rows)
        cost, ops, fin = best_schedule(rows, nin, has_acc)
        got = evaluate(nin, ops, [sorted(s) for s in fin])
        assert got == [frozenset(s) for s in rows], (fam, k, p, g, r0)
        total += cost
        groups.append((r0, nin, ops, [sorted(s) for s in fin]))
    return groups, naive, total


def emit(entries):
    lines = [
        "// GENERATED by tools/gen_xor_sched.py -- do not edit. Common-subexpression",
        "// XOR schedules for the compile-time encode matrices (see the tool's",
        "// docstring); applied by xor_sched_apply (hrs_device.hpp).",
        "// clang-format off",
        "#pragma once",
        "#include <cstdint>",
        "",
        "namespace hrs {",
        "namespace xsched {",
        "",
        "struct Op { uint8_t a, b, c; };  // c == 255: two-input XOR",
        "",
        "// Sched<FAMILY, K, P, G>: kGroups groups of G data rows (the last may be",
        "// smaller). Group j: kNin[j] input vars, kOps[kOpOff[j] .. kOpOff[j+1]),",
        "// parity plane (o, q) = its running value ^ XOR of",
        "// kTerms[kTermOff[j][8o+q] .. kTermOff[j][8o+q+1]).",
        "template <int FAMILY, int K, int P, int G> struct Sched;",
        "",
    ]
    for (fam, k, p, g), (groups, naive, total) in entries:
        ng = len(groups)
        nplanes = 8 * p
        opoff = [0]
        allops = []
        termoff = []
        allterms = []
        for r0, nin, ops, fin in groups:
            allops.extend(ops)
            opoff.append(len(allops))
            offs = [len(allterms)]
            for s in fin:
                allterms.extend(s)
                offs.append(len(allterms))
            termoff.append(offs)
        maxvars = max(nin + len(ops) for r0, nin, ops, fin in groups)
        name = "RS" if fam == 0 else "Cauchy"
        lines.append(f"// {name}({k},{p}), groups of {g} rows: {total} xor ops "
                     f"(plane by plane: {naive}).")
        lines.append(f"template <> struct Sched<{fam}, {k}, {p}, {g}> {{")
        lines.append(f"  static constexpr int kGroups = {ng};")
        lines.append(f"  static constexpr int kMaxVars = {maxvars};")
        lines.append(f"  static constexpr int kXorOps = {total};")
        lines.append("  static constexpr int kNin[" + str(ng) + "] = {" +
                     ", ".join(str(nin) for _, nin, _, _ in groups) + "};")
        lines.append("  static constexpr int kOpOff[" + str(ng + 1) + "] = {" +
                     ", ".join(map(str, opoff)) + "};")
        ops_txt = ", ".join("{%d, %d, %d}" % (a, b, 255 if c is None else c) for a, b, c in allops)
        lines.append("  static constexpr Op kOps[" + str(max(1, len(allops))) + "] = {" +
                     (ops_txt if allops else "{0, 0, 255}") + "};")
        lines.append("  static constexpr uint16_t kTermOff[" + str(ng) + "][" + str(nplanes + 1) + "] = {")
        for offs in termoff:
            lines.append("      {" + ", ".join(map(str, offs)) + "},")
        lines.append("  };")
        lines.append("  static constexpr uint8_t kTerms[" + str(max(1, len(allterms))) + "] = {" +
                     ", ".join(map(str, allterms)) + "};")
        lines.append("};")
        lines.append("")
    lines += ["}  // namespace xsched", "}  // namespace hrs", ""]
    return "\n".join(lines)


def generate():
    entries = []
    for fam, k, p in SHAPES:
        for g in GROUPS + [k]:
            if g > k:
                continue
            if any(e[0] == (fam, k, p, g) for e in entries):
                continue
            entries.append(((fam, k, p, g), build(k, p, fam, g)))
    return entries


def main():
    entries = generate()
    text = emit(entries)
    for (fam, k, p, g), (_, naive, total) in entries:
        print(f"family {fam} RS({k},{p}) G={g}: {naive} -> {total} xor ops", file=sys.stderr)
    if "--check" in sys.argv:
        with open(OUT) as f:
            sys.exit(0 if f.read() == text else 1)
    with open(OUT, "w") as f:
        f.write(text)


if __name__ == "__main__":
    main()
