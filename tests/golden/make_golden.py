"""Generates tests/golden/*.json — golden vectors for the RS hot path.

The reference ships no byte-level golden vectors (its RS tests are unseeded
round trips, TestErasureCodes.java:31) and cannot run here (no JDK), so the
expected outputs below come from the pure-Python transcription of the Java
methods (oracle/rs_ref.py) and are cross-checked, case by case, against the
independent C transcription (oracle/rs_oracle.c). Inputs include the exact
bytes of the reference's own deterministic test input generator,
Util.randomBytes(seed) = java.util.Random(seed).nextBytes
(hops-erasure-coding/src/test/java/io/hops/erasure_coding/Util.java:97-106),
with seed 0xDEADBEEF from TestBlockReconstructor.java:52.

Run from the repo root:  python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import rs_oracle as C  # noqa: E402
from oracle import rs_ref as R  # noqa: E402
from oracle.java_random import random_bytes  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def rows_from(buf, nrows, L):
    return [bytes(buf[i * L:(i + 1) * L]) for i in range(nrows)]


def case(name, k, p, data_rows, decodes, source):
    ref = R.ReedSolomonRef(k, p)
    parity = ref.encode_bulk(data_rows)
    c_par = C.encode_bulk(k, p, [np.frombuffer(r, dtype=np.uint8) for r in data_rows])
    assert all(bytes(a) == b for a, b in zip(c_par, parity)), name
    stripe = list(parity) + list(data_rows)  # hops order [parity..., data...]
    dec = []
    for erased in decodes:
        to_read = R.locations_to_read_for_decode(k, p, erased)
        to_read_arr = sorted(to_read)
        ntr = [loc for loc in range(k + p) if loc not in to_read_arr]
        # reads: zeros for erased / not-to-read rows (StripeReader.java:111-120)
        reads = [stripe[i] if i in to_read_arr else bytes(len(stripe[i])) for i in range(k + p)]
        out = ref.decode_bulk5(reads, erased, to_read_arr, ntr)
        c_out = C.decode_bulk5(k, p, [np.frombuffer(r, dtype=np.uint8) for r in reads], erased, to_read_arr, ntr)
        assert all(bytes(a) == b for a, b in zip(c_out, out)), (name, erased)
        for e, o in zip(erased, out):  # a codeword decodes to the erased values
            assert o == stripe[e], (name, erased)
        # 3-arg bulk decode with the erased rows zeroed (TestErasureCodes.java:175-193)
        reads3 = [bytes(len(stripe[i])) if i in erased else stripe[i] for i in range(k + p)]
        out3 = ref.decode_bulk3(reads3, erased) if len(erased) <= p else None
        dec.append({
            "erased": erased,
            "locations_to_read": to_read,
            "locations_to_read_array": to_read_arr,
            "locations_not_to_read_array": ntr,
            "outputs_hex": [o.hex() for o in out],
            "decode3_outputs_hex": [o.hex() for o in out3] if out3 is not None else None,
        })
    return {
        "name": name, "k": k, "p": p, "len": len(data_rows[0]), "source": source,
        "generator": ref.gen,
        "data_hex": [r.hex() for r in data_rows],
        "parity_hex": [r.hex() for r in parity],
        "decodes": dec,
    }


def main():
    cases = []
    L = 64
    buf = random_bytes(0xDEADBEEF, 3 * L)
    cases.append(case("rs_3_2_java_random_deadbeef", 3, 2, rows_from(buf, 3, L),
                      [[3], [0], [1, 4], [2, 3]], "Util.randomBytes(0xDEADBEEF, 192) rows of 64"))
    rng = np.random.default_rng(20261015)
    for k, p, L, decs in [
        (6, 3, 48, [[3], [0, 8], [3, 4, 5]]),
        (10, 4, 97, [[4], [13], [4, 5], [1, 5, 7], [4, 1, 5, 7], [0, 1, 2, 3], [10, 11, 12, 13]]),
        (12, 4, 33, [[4, 9], [15], [0, 5, 10, 15]]),
        (1, 1, 16, [[0], [1]]),
        (17, 7, 21, [[0, 1, 2, 3, 4, 5, 6], [23], [7, 8]]),
    ]:
        rows = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for _ in range(k)]
        cases.append(case(f"rs_{k}_{p}_len{L}", k, p, rows, [sorted(d) for d in decs],
                          "numpy default_rng(20261015) integers"))
    # edge stripes: all-zero, all-0xFF, 0..255 ramp
    for nm, fill in [("zeros", lambda i: bytes(32)), ("ones", lambda i: b"\xff" * 32),
                     ("ramp", lambda i: bytes((i * 32 + j) % 256 for j in range(32)))]:
        cases.append(case(f"rs_10_4_edge_{nm}", 10, 4, [fill(i) for i in range(10)], [[4], [0, 13]], nm))
    # scalar known answers: ReedSolomonCode.encode of unit messages = encode matrix columns
    G = [[C.encode(10, 4, [1 if j == c else 0 for j in range(10)])[r] for c in range(10)] for r in range(4)]
    assert G == [[R.ReedSolomonRef(10, 4).encode([1 if j == c else 0 for j in range(10)])[r] for c in range(10)]
                 for r in range(4)]
    with open(os.path.join(OUT, "rs_vectors.json"), "w") as f:
        json.dump({"cases": cases, "encode_matrix_10_4": G}, f, indent=1)

    # Config 1 of BASELINE.json: RS(3,2) encode of one 1 MiB stripe (C oracle;
    # pinned to the Python transcription on the first 4 KiB).
    L = 1 << 20
    buf = random_bytes(0x5EED0001, 3 * L)
    rows = [np.frombuffer(buf[i * L:(i + 1) * L], dtype=np.uint8) for i in range(3)]
    par = C.encode_bulk(3, 2, rows)
    head = R.ReedSolomonRef(3, 2).encode_bulk([bytes(r[:4096]) for r in rows])
    assert all(bytes(a[:4096]) == b for a, b in zip(par, head))
    cfg1 = {
        "k": 3, "p": 2, "len": L,
        "input": "java.util.Random(0x5EED0001).nextBytes(3 MiB), rows of 1 MiB",
        "input_sha256": hashlib.sha256(buf).hexdigest(),
        "parity_sha256": [hashlib.sha256(bytes(r)).hexdigest() for r in par],
        "parity_head_hex": [bytes(r[:64]).hex() for r in par],
    }
    with open(os.path.join(OUT, "config1_rs_3_2_1mib.json"), "w") as f:
        json.dump(cfg1, f, indent=1)
    print("wrote", len(cases), "cases")


if __name__ == "__main__":
    main()
