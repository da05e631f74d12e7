"""Combinable output digests of the BASELINE workloads.

Each stripe's outputs (parity rows, or repaired cells) get their own SHA-256;
a block of up to 256 consecutive GLOBAL stripes is then the SHA-256 of its
stripes' 32-byte digests in global order. Ranks hash only their own stripes
and send the per-stripe digests; rank 0 assembles the union and cuts it into
blocks, so any partition of the stripes over the ranks (weak scaling, strong
scaling at any N, a rank range starting mid-block) yields the same block
digests as a 1-rank run and as the oracle (tests/golden/bench_digests.json,
made by tests/golden/make_bench_digests.py with the same two functions).

Keys: "g" for a full block starting at global stripe g (g % 256 == 0), "g+n"
for a run of n < 256 stripes starting at g (a job that ends, or starts, inside
a block).
"""
import hashlib

import numpy as np

BLOCK = 256


def stripe_digests(rows_of, S, g0, fetch=64):
    """{global stripe: sha256 digest (32 bytes)} of this rank's stripes g0 ..
    g0+S-1; rows_of(a, b) returns the bytes of local stripes [a, b) as an
    array (or torch tensor, device or host) whose first axis is the stripe."""
    out = {}
    for a in range(0, S, fetch):
        b = min(S, a + fetch)
        x = rows_of(a, b)
        if not isinstance(x, np.ndarray):  # a torch tensor
            x = x.contiguous().cpu().numpy()
        x = np.ascontiguousarray(x)
        for i in range(b - a):
            out[g0 + a + i] = hashlib.sha256(x[i].tobytes()).digest()
    return out


def combine(per_stripe, block=BLOCK):
    """Block digests of a union of per-stripe digests: maximal runs of
    consecutive global stripes, cut at multiples of `block`."""
    out = {}
    gs = sorted(per_stripe)
    i = 0
    while i < len(gs):
        g = gs[i]
        end = (g // block + 1) * block  # the next block boundary
        j = i
        while j + 1 < len(gs) and gs[j + 1] == gs[j] + 1 and gs[j + 1] < end:
            j += 1
        n = j - i + 1
        h = hashlib.sha256()
        for t in range(i, j + 1):
            h.update(per_stripe[gs[t]])
        out[f"{g}" if (n == block and g % block == 0) else f"{g}+{n}"] = h.hexdigest()
        i = j + 1
    return out


def key_span(key):
    """(first global stripe, count) of a block key."""
    if "+" in key:
        a, n = key.split("+")
        return int(a), int(n)
    return int(key), BLOCK


def compare(got, want, fields, golden_stripes):
    """Checks block digests against the oracle's. got[f] / want[f]: {key:
    hex}. Every block of `got` the oracle holds a digest for must match it; a
    run that covers only part of an oracle block (an ad-hoc --stripes that is
    not a multiple of 256) cannot be checked and is counted in
    `unchecked_stripes`, as are stripes past the oracle's range [0,
    golden_stripes). Raises on any mismatch and when no block at all was
    checked. Returns {"blocks": matched, "match": True, "checked_stripes":
    stripes covered by matched blocks of the first field, "unchecked_stripes":
    the first field's stripes no oracle digest covers, "partial_blocks": runs
    skipped for covering part of a block}."""
    matched = 0
    checked = unchecked = partial = 0
    for fi, f in enumerate(fields):
        ref = want.get(f, {})
        for key, dig in got[f].items():
            a, n = key_span(key)
            inside = max(0, min(a + n, golden_stripes) - a)
            if inside == 0:
                unchecked += n if fi == 0 else 0
                continue
            if key not in ref:  # part of a block: the oracle holds whole blocks only
                partial += 1
                unchecked += n if fi == 0 else 0
                continue
            if ref[key] != dig:
                raise RuntimeError(f"{f} block {key}: digest {dig} != oracle {ref[key]}")
            matched += 1
            if fi == 0:
                checked += n
                unchecked += n - inside
    if matched == 0:
        raise RuntimeError("no block of this run was checked against the oracle (the golden file holds whole "
                           f"blocks of {BLOCK} stripes below {golden_stripes})")
    return {"blocks": matched, "match": True, "checked_stripes": checked, "unchecked_stripes": unchecked,
            "partial_blocks": partial}
