"""Asynchronous rounds from several threads at once, one codec per thread —
the shape of raid.encoder.parallelism Encoders in one JVM (Encoder.java:77-80,
one codec each) calling encodeBulkAsync / collect (Encoder.java:421-453).
Every round's parity is compared with the oracle's encodeBulk
(ReedSolomonCode.java:103-125), under both transfer modes and with the timing
diagnostic (hrs_set_timing) on and off. Bit-exact."""
import ctypes
import threading

import numpy as np
import pytest

from lambdafs_amd import HipReedSolomonCode, _lib
from oracle import rs_oracle as C

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["zero_copy", "copy_engine"])
def transfer_mode(request, monkeypatch):
    if request.param == "copy_engine":
        monkeypatch.setenv("HRS_ZEROCOPY", "0")
    else:
        monkeypatch.delenv("HRS_ZEROCOPY", raising=False)
    return request.param


def _run(threads, depth, rounds, L, timing, seed):
    k, p = 10, 4
    lib = _lib.lib()
    errs = []

    def body(t):
        try:
            code = HipReedSolomonCode(k, p, device=0, zero_inputs_after_encode=False)
            h = code._handle()
            if timing:
                code._check(lib.hrs_set_timing(h, 1))
            rng = np.random.default_rng([seed, t])
            data = [[rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)] for _ in range(rounds)]
            keep = [[x.copy() for x in d] for d in data]
            q = []
            for r in range(rounds + depth):
                if r < rounds:
                    q.append((code.encodeBulkAsync(data[r]), r))
                    for x in data[r]:  # the caller may reuse its rows as soon as submit returns
                        x[:] = 0xC3
                if len(q) == depth or (r >= rounds and q):
                    tk, rr = q.pop(0)
                    if timing:
                        code.wait(tk)
                        ms = ctypes.c_float(-1)
                        code._check(lib.hrs_ticket_gpu_ms(h, tk, ctypes.byref(ms)))
                        assert ms.value > 0
                    out = [np.full(L, 0xEE, np.uint8) for _ in range(p)]
                    code.collect(tk, out)
                    ref = C.encode_bulk(k, p, [x.copy() for x in keep[rr]])
                    for o in range(p):
                        if not np.array_equal(out[o], ref[o]):
                            bad = np.flatnonzero(out[o] != ref[o])
                            raise AssertionError(f"thread {t} round {rr} parity {o}: {bad.size} bytes differ, "
                                                 f"first at {bad[0]}")
        except Exception as e:  # noqa: BLE001 - reported after the join
            errs.append(e)

    ths = [threading.Thread(target=body, args=(t,)) for t in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    if errs:
        raise errs[0]


@pytest.mark.parametrize("timing", [False, True])
@pytest.mark.parametrize("threads,depth", [(1, 2), (4, 1), (4, 4)])
def test_concurrent_async_encoders(cuda, transfer_mode, timing, threads, depth):
    _run(threads, depth, rounds=6, L=256 << 10, timing=timing, seed=threads * 10 + depth)


def test_concurrent_async_encoders_1mib(cuda):
    """bench.py's async_rounds shape: 4 codecs, 1 MiB cells, timing on."""
    _run(4, 2, rounds=4, L=1 << 20, timing=True, seed=99)
