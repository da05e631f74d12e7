"""Throughput of the synchronous host-buffer calls (the JNI path):
ReedSolomonCode.encodeBulk / decodeBulk on pageable host rows, one call per
1 MiB-cell stripe, exactly as Encoder.java:442 / Decoder.java:352 issue them;
and the checksummed variants (hrs_encode_crc / hrs_decode_crc) next to the
host zlib CRC pass they replace (Encoder.java:434-447).

Run: python tools/bench_host_api.py [--calls 40]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lambdafs_amd import HipReedSolomonCode  # noqa: E402

GiB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--p", type=int, default=4)
    ap.add_argument("--cell", type=int, default=1 << 20)
    ap.add_argument("--calls", type=int, default=40)
    args = ap.parse_args()
    k, p, L = args.k, args.p, args.cell
    n = k + p
    code = HipReedSolomonCode(k, p, device=0, zero_inputs_after_encode=False)
    rng = np.random.default_rng(0)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    par = [np.zeros(L, np.uint8) for _ in range(p)]
    code.encodeBulk(data, par)  # warm
    t0 = time.perf_counter()
    for _ in range(args.calls):
        code.encodeBulk(data, par)
    te = (time.perf_counter() - t0) / args.calls
    crcs = code.encodeBulkCrc(data, par)  # warm
    t0 = time.perf_counter()
    for _ in range(args.calls):
        crcs = code.encodeBulkCrc(data, par, crcs)
    tec = (time.perf_counter() - t0) / args.calls
    # the Java Encoder's checksum pass on the host (zlib = java.util.zip.CRC32), 1 thread
    import zlib
    t0 = time.perf_counter()
    for r in data + par:
        zlib.crc32(r)
    tz = time.perf_counter() - t0
    stripe = par + data
    erased = [p]
    to_read = sorted(code.locationsToReadForDecode(erased))
    ntr = [x for x in range(n) if x not in to_read]
    reads = [stripe[i] if i in to_read else None for i in range(n)]
    out = [np.zeros(L, np.uint8)]
    code.decodeBulk(reads, out, erased, to_read, ntr)
    assert (out[0] == data[0]).all()
    t0 = time.perf_counter()
    for _ in range(args.calls):
        code.decodeBulk(reads, out, erased, to_read, ntr)
    td = (time.perf_counter() - t0) / args.calls
    code.decodeBulkCrc(reads, out, erased, to_read, ntr)
    t0 = time.perf_counter()
    for _ in range(args.calls):
        code.decodeBulkCrc(reads, out, erased, to_read, ntr)
    tdc = (time.perf_counter() - t0) / args.calls
    print(json.dumps({
        "path": "synchronous host-buffer calls (hrs_encode / hrs_decode), pageable rows, 1 call per stripe",
        "copy_threads": os.environ.get("HRS_HOST_THREADS", "2 (default)"),
        "chunk_bytes": os.environ.get("HRS_HOST_CHUNK", "524288 (default)"),
        "encodeBulk_ms_per_call": round(te * 1e3, 3),
        "encodeBulk_GiBps_user_data": round(k * L / GiB / te, 2),
        "encodeBulk_GBps_pcie": round((k + p) * L / te / 1e9, 2),
        "encodeBulkCrc_ms_per_call": round(tec * 1e3, 3),
        "encodeBulkCrc_GiBps_user_data": round(k * L / GiB / tec, 2),
        "host_zlib_crc_of_stripe_ms_1thread": round(tz * 1e3, 3),
        "decodeBulk_ms_per_call": round(td * 1e3, 3),
        "decodeBulkCrc_ms_per_call": round(tdc * 1e3, 3),
        "decodeBulk_GiBps_user_data": round(k * L / GiB / td, 2),
    }), flush=True)


if __name__ == "__main__":
    main()
