"""Can the CRC pass read the cells back from the Infinity Cache (MALL)?

The fused encode + CRC kernel (3.1 ms for RS(10,4) 1,024 x 1 MiB) is issue-
bound at 4 waves/SIMD; the two-pass form (encode, then CRC of every cell) reads
HBM twice. If a CRC pass over a chunk of stripes that was just encoded is
served from the 256 MiB Infinity Cache, chunked encode -> CRC (on one stream,
or pipelined over two) might beat the fused kernel. This probe times, median of
5 (ms), interleaved:
  fused              encode_stripes_crc over all stripes
  two-pass           encode_stripes, then crc32_rows over all stripes
  crc cold / warm    crc32_rows over one chunk after a 2 GiB flush / right after itself
  chunked C          per chunk of C stripes: encode, then CRC (one stream)
  pipelined C        encode chunk i on stream A, CRC chunk i on stream B (event)
and checks that every variant's CRCs equal the fused kernel's.
Usage: python tools/mall_probe.py   (GPU box; dev tool, not part of the product)
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lambdafs_amd import HipReedSolomonCode, device  # noqa: E402


def med(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return round(float(np.median(ts)), 4)


def main():
    k, p, L, S = 10, 4, 1 << 20, 1024
    code = HipReedSolomonCode(k, p, device=0)
    st = torch.randint(0, 256, (S, k + p, L), dtype=torch.uint8, device="cuda")
    flush = torch.empty(2 << 30, dtype=torch.uint8, device="cuda")

    def cells(a, b):
        return [st[a:b, p + c, :] for c in range(k)] + [st[a:b, r, :] for r in range(p)]

    ref = device.encode_stripes_crc(code, st)
    out = {"fused": med(lambda: device.encode_stripes_crc(code, st))}
    all_cells = cells(0, S)
    out["two_pass"] = med(lambda: (device.encode_stripes(code, st), device.crc32_rows(code, all_cells)))
    sA, sB = torch.cuda.Stream(), torch.cuda.Stream()
    for C in (4, 8, 16, 32):
        chunks = [(a, a + C) for a in range(0, S, C)]
        views = [cells(a, b) for a, b in chunks]
        crc = torch.empty((S, k + p), dtype=torch.int32, device="cuda")

        def chunked():
            for (a, b), v in zip(chunks, views):
                device.encode_stripes(code, st[a:b])
                crc[a:b] = device.crc32_rows(code, v)

        def pipelined():
            ev = []
            cur = torch.cuda.current_stream()
            sA.wait_stream(cur)
            sB.wait_stream(cur)
            for (a, b), v in zip(chunks, views):
                with torch.cuda.stream(sA):
                    device.encode_stripes(code, st[a:b])
                    e = torch.cuda.Event()
                    e.record(sA)
                with torch.cuda.stream(sB):
                    sB.wait_event(e)
                    crc[a:b] = device.crc32_rows(code, v)
                ev.append(e)
            cur.wait_stream(sA)
            cur.wait_stream(sB)

        out[f"chunked_{C}"] = med(chunked)
        if not torch.equal(crc, ref):
            raise RuntimeError(f"chunked {C}: CRCs differ from the fused kernel's")
        crc.zero_()
        out[f"pipelined_{C}"] = med(pipelined)
        if not torch.equal(crc, ref):
            raise RuntimeError(f"pipelined {C}: CRCs differ from the fused kernel's")
        v0 = views[1]
        out[f"crc_cold_{C}"] = med(lambda: (flush.fill_(1), device.crc32_rows(code, v0)))
        out[f"flush_only"] = med(lambda: flush.fill_(1))
        out[f"crc_warm_{C}"] = med(lambda: device.crc32_rows(code, v0))
        out[f"crc_chunk_MiB_{C}"] = C * (k + p)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
