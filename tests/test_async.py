"""Asynchronous Encoder / Decoder rounds (hrs_encode_submit /
hrs_decode_submit / hrs_collect): round r + 1 is read and
submitted while round r runs on the GPU.

Reference behaviour followed: each round is one ReedSolomonCode.encodeBulk
(ReedSolomonCode.java:103-125) as Encoder.encodeStripe calls it per stripe
(Encoder.java:397-464) or one 5-arg decodeBulk (ReedSolomonCode.java:191-211)
as Decoder.fixErasedBlockImpl calls it (Decoder.java:232-401), with the block
CRC32s continued across rounds the way the Encoder's / Decoder's
java.util.zip.CRC32.update calls chain them (Encoder.java:421-453,
Decoder.java:371-382). Parity vs the oracle, CRCs vs zlib, bit-exact."""
import zlib

import numpy as np
import pytest

from lambdafs_amd import HipReedSolomonCode, HrsError
from oracle import rs_oracle as C

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["zero_copy", "copy_engine"])
def transfer_mode(request, monkeypatch):
    """Every test runs both ways the asynchronous rounds can move bytes: zero copy (the
    default: kernels read and write pinned host memory across the link) and
    the copy engine (HRS_ZEROCOPY=0: pinned staging, H2D, kernel, D2H)."""
    if request.param == "copy_engine":
        monkeypatch.setenv("HRS_ZEROCOPY", "0")
    else:
        monkeypatch.delenv("HRS_ZEROCOPY", raising=False)
    return request.param


def _decoder_sets(k, p, erased):
    n = k + p
    tr = C.locations_to_read(k, p, erased)
    return sorted(tr), [x for x in range(n) if x not in tr or x in erased]


@pytest.mark.parametrize("depth", [1, 2, 4])
def test_encode_rounds_pipelined_vs_oracle_and_zlib(cuda, depth):
    """`depth` rounds in flight; ragged row length; the running CRC32s of all
    14 blocks chained over 6 rounds vs zlib.crc32 over the concatenation."""
    k, p, R, L = 10, 4, 6, (1 << 20) + 24
    code = HipReedSolomonCode(k, p, device=0)
    rng = np.random.default_rng(depth)
    rounds = [[rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)] for _ in range(R)]
    keep = [[r.copy() for r in rnd] for rnd in rounds]
    tickets, crcs, want = {}, [0] * (k + p), [0] * (k + p)
    for r in range(R + depth - 1):
        if r < R:
            tickets[r] = code.encodeBulkAsync(rounds[r], checksums=True)
            assert all((x == 0).all() for x in rounds[r])  # encodeBulk zeroes its inputs (GaloisField.java:326-338)
        q = r - depth + 1
        if q >= 0:
            out = [np.full(L, 0xEE, np.uint8) for _ in range(p)]
            crcs = code.collect(tickets[q], out, crcs)
            ref = C.encode_bulk(k, p, [x.copy() for x in keep[q]])
            for o in range(p):
                assert np.array_equal(out[o], ref[o]), (q, o)
            for i, b in enumerate(keep[q] + list(ref)):
                want[i] = zlib.crc32(b.tobytes(), want[i])
    assert crcs == want
    assert code.pending() == 0


def test_decode_rounds_out_of_order_vs_oracle(cuda):
    """RS(12,4): four decode rounds in flight, each with its own erasure
    pattern on NON-codeword rows (every coefficient counts), collected in
    reverse order; the repaired blocks' CRC32s vs zlib."""
    k, p, L = 12, 4, (256 << 10) + 3
    n = k + p
    code = HipReedSolomonCode(k, p, device=0)
    rng = np.random.default_rng(5)
    pats = [[3], [0, 15], [1, 5, 9], [2, 6, 10, 14]]
    subs = []
    for lost in pats:
        tr, ntr = _decoder_sets(k, p, lost)
        rows = [None if x in ntr else rng.integers(0, 256, L, dtype=np.uint8) for x in range(n)]
        reads = [np.zeros(L, np.uint8) if r is None else r.copy() for r in rows]
        want = C.decode_bulk5(k, p, reads, lost, tr, ntr)
        t = code.decodeBulkAsync(rows, lost, tr, ntr, checksums=True)
        for r in rows:  # the rows may be reused as soon as submit returns
            if r is not None:
                r[:] = 0x77
        subs.append((t, lost, want))
    with pytest.raises(HrsError):  # all 4 slots hold uncollected rounds
        code.decodeBulkAsync([np.zeros(L, np.uint8)] * n, [0], list(range(1, k + 1)), [0] + list(range(k + 1, n)))
    assert code.pending() == 4
    for t, lost, want in reversed(subs):
        out = [np.zeros(L, np.uint8) for _ in lost]
        crcs = code.collect(t, out)
        for i in range(len(lost)):
            assert np.array_equal(out[i], want[i]), (lost, i)
        assert crcs == [zlib.crc32(w.tobytes()) for w in want]
        with pytest.raises(HrsError):  # a ticket collects once
            code.collect(t, out)


def test_async_argument_errors(cuda):
    torch = cuda
    k, p, L = 10, 4, 4096
    code = HipReedSolomonCode(k, p, device=0, zero_inputs_after_encode=False)
    ins = [np.full(L, i, np.uint8) for i in range(k)]
    with pytest.raises(ValueError):
        code.encodeBulkAsync(ins[:9])
    dev = [torch.zeros(L, dtype=torch.uint8, device="cuda") for _ in range(k)]
    with pytest.raises(ValueError):  # device rows go through the synchronous calls
        code.encodeBulkAsync(dev)
    t = code.encodeBulkAsync(ins)
    with pytest.raises(ValueError):
        code.collect(t, [np.zeros(L, np.uint8)] * 3)
    with pytest.raises(ValueError):
        code.collect(t, [np.zeros(L - 1, np.uint8)] * 4)
    with pytest.raises(HrsError):
        code.collect(t + 1000, [np.zeros(L, np.uint8)] * 4)
    out = [np.zeros(L, np.uint8) for _ in range(p)]
    assert code.collect(t, out) is None  # not checksummed
    ref = C.encode_bulk(k, p, [x.copy() for x in ins])
    assert all(np.array_equal(out[o], ref[o]) for o in range(p))
    # nothing erased: a decode round with no outputs
    t = code.decodeBulkAsync(ins + [np.zeros(L, np.uint8)] * p, [], list(range(k)), [])
    assert code.collect(t, []) is None


def test_wait_then_collect(cuda):
    """hrs_wait blocks until a round's GPU work is done without collecting it
    (the JNI shim calls it before pinning the output rows); collect then only
    copies. Unknown tickets and double waits are handled."""
    k, p, L = 10, 4, 1 << 20
    code = HipReedSolomonCode(k, p, device=0, zero_inputs_after_encode=False)
    rng = np.random.default_rng(5)
    rows = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    t = code.encodeBulkAsync(rows)
    code.wait(t)
    code.wait(t)  # still uncollected: waiting again is a no-op
    assert code.pending() == 1
    out = [np.zeros(L, np.uint8) for _ in range(p)]
    assert code.collect(t, out) is None
    ref = C.encode_bulk(k, p, rows)
    assert all(np.array_equal(a, b) for a, b in zip(out, ref))
    with pytest.raises(HrsError):
        code.wait(t)  # collected: the ticket is gone


def test_sync_calls_between_pending_rounds(cuda):
    """Synchronous calls on the same handle while asynchronous rounds are in
    flight (an Encoder that mixes encodeBulk and encodeBulkAsync): the
    synchronous call runs over the caller's rows (its own streams and staging,
    pages registered for the call) and leaves the pending rounds untouched;
    every result vs the oracle."""
    k, p, L = 10, 4, 1 << 20
    code = HipReedSolomonCode(k, p, device=0, zero_inputs_after_encode=False)
    rng = np.random.default_rng(77)
    rounds = [[rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)] for _ in range(3)]
    keep = [[r.copy() for r in rnd] for rnd in rounds]
    tickets = [code.encodeBulkAsync(r) for r in rounds]
    sync_data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    sync_par = [np.zeros(L, np.uint8) for _ in range(p)]
    crcs = code.encodeBulkCrc(sync_data, sync_par)
    ref = C.encode_bulk(k, p, sync_data)
    assert all(np.array_equal(a, b) for a, b in zip(sync_par, ref))
    assert crcs == [zlib.crc32(b.tobytes()) for b in sync_data + list(ref)]
    for t, kept in reversed(list(zip(tickets, keep))):
        out = [np.full(L, 0xEE, np.uint8) for _ in range(p)]
        code.collect(t, out)
        want = C.encode_bulk(k, p, kept)
        assert all(np.array_equal(a, b) for a, b in zip(out, want))
    assert code.pending() == 0
