"""Is the host link full duplex? (VERDICT r3 "overlap D2H with H2D").

Config 5's repair moves 12 survivor cells H2D and 2 repaired cells D2H per
stripe (512 x 256 KiB stripes: 1.61 GB in, 0.27 GB out); the host batch
encode moves 12 cells in and 4 out (0.54 GB). This probe times, on pinned
host memory and one GPU:
  h2d alone, d2h alone, h2d then d2h on one stream (serial), and h2d and
  d2h on two streams at once (duplex), each as one copy and as the chunked
  form the pipelines use (12-stripe chunks: 36 MiB in, 6 or 12 MiB out).
If duplex < serial, the link carries both directions at once and the host
pipelines should put H2D and D2H on separate streams.

Run: python tools/duplex_probe.py [--reps 5]  (one JSON line)
"""
import argparse
import json

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    L, S = 256 << 10, 512
    h2d_bytes = 12 * L * S
    out = {"what": "pinned host <-> device copies, one GPU", "h2d_bytes": h2d_bytes}
    dev = torch.device("cuda", 0)
    hin = torch.empty(h2d_bytes, dtype=torch.uint8, pin_memory=True)
    hin.fill_(7)
    din = torch.empty(h2d_bytes, dtype=torch.uint8, device=dev)
    s_in, s_out = torch.cuda.Stream(), torch.cuda.Stream()

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ms = []
        for _ in range(args.reps):
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record()
            fn()
            # join both side streams into the current one before the end event
            torch.cuda.current_stream().wait_stream(s_in)
            torch.cuda.current_stream().wait_stream(s_out)
            b.record()
            b.synchronize()
            ms.append(a.elapsed_time(b))
        return round(float(np.median(ms)), 3)

    for name, nout in (("decode_2_of_16", 2), ("encode_4_of_16", 4)):
        d2h_bytes = nout * L * S
        hout = torch.empty(d2h_bytes, dtype=torch.uint8, pin_memory=True)
        dout = torch.full((d2h_bytes,), 3, dtype=torch.uint8, device=dev)
        chunk = 12  # stripes per chunk, as hrs_decode_batch_host
        ci, co = 12 * L * chunk, nout * L * chunk
        nch = S // chunk

        def h2d(st=s_in, chunked=False):
            torch.cuda.current_stream().synchronize()
            with torch.cuda.stream(st):
                if not chunked:
                    din.copy_(hin, non_blocking=True)
                else:
                    for j in range(nch):
                        din[j * ci:(j + 1) * ci].copy_(hin[j * ci:(j + 1) * ci], non_blocking=True)

        def d2h(st=s_out, chunked=False):
            with torch.cuda.stream(st):
                if not chunked:
                    hout.copy_(dout, non_blocking=True)
                else:
                    for j in range(nch):
                        hout[j * co:(j + 1) * co].copy_(dout[j * co:(j + 1) * co], non_blocking=True)

        r = {"d2h_bytes": d2h_bytes}
        for chunked in (False, True):
            tag = "chunked" if chunked else "one_copy"
            r[f"h2d_alone_ms_{tag}"] = timed(lambda: h2d(chunked=chunked))
            r[f"d2h_alone_ms_{tag}"] = timed(lambda: d2h(chunked=chunked))
            r[f"serial_ms_{tag}"] = timed(lambda: (h2d(s_in, chunked), d2h(s_in, chunked)))
            r[f"duplex_ms_{tag}"] = timed(lambda: (h2d(s_in, chunked), d2h(s_out, chunked)))
            r[f"duplex_gain_{tag}"] = round(r[f"serial_ms_{tag}"] / r[f"duplex_ms_{tag}"], 3)
        r["h2d_GBps"] = round(h2d_bytes / 1e9 / (r["h2d_alone_ms_one_copy"] * 1e-3), 2)
        r["d2h_GBps"] = round(d2h_bytes / 1e9 / (r["d2h_alone_ms_one_copy"] * 1e-3), 2)
        r["duplex_GBps_both"] = round((h2d_bytes + d2h_bytes) / 1e9 / (r["duplex_ms_one_copy"] * 1e-3), 2)
        assert int(hout[::4096].to(torch.int32).sum()) == 3 * hout[::4096].numel()
        out[name] = r
    assert bool((din[::4096] == 7).all())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
