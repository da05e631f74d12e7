"""HBM ceiling probes (include/hrs_probe.h): argument checks on CPU, and on
the GPU that every shape moves exactly the bytes it claims (the figures
bench.py quotes as copy / read / write / pattern ceilings are only ceilings
if the probes do the work)."""
import ctypes

import numpy as np
import pytest

from lambdafs_amd import _lib, device


def test_stream_argument_checks():
    L = _lib.probe_lib()
    buf = ctypes.create_string_buffer(4096)
    p = ctypes.addressof(buf)
    p16 = (p + 15) & ~15
    ok = 0
    # (op, schedule, depth, block threads, blocks per CU)
    for args in ((3, 0, 1, 256, 1), (-1, 0, 1, 256, 1), (0, 3, 1, 256, 1), (0, -1, 1, 256, 1), (0, 0, 3, 256, 1),
                 (0, 0, 16, 256, 1), (0, 0, 1, 128, 1), (0, 0, 1, 768, 1), (0, 0, 1, 256, 0), (0, 0, 1, 256, 33),
                 (0, 2, 8, 1024, 9)):
        op, sc, d, blk, bpc = args
        assert L.hrs_probe_stream(op, p16, p16, 1024, sc, d, 1, blk, bpc, None) != ok, args
    assert L.hrs_probe_stream(0, None, p16, 1024, 0, 1, 1, 256, 1, None) != ok  # copy without a source
    assert L.hrs_probe_stream(2, None, None, 1024, 0, 1, 1, 256, 1, None) != ok  # write without a destination
    einval = L.hrs_probe_stream(0, p16, p16, 1024, 0, 3, 1, 256, 1, None)
    ealign = L.hrs_probe_stream(0, p16 + 1, p16, 1024, 0, 1, 1, 256, 1, None)
    assert ealign not in (ok, einval)
    assert L.hrs_probe_stream(0, p16, p16, 1000, 0, 1, 1, 256, 1, None) == ealign  # bytes % 16
    assert L.hrs_probe_stream(1, p16, p16, 0, 2, 8, 0, 1024, 1, None) == ok  # nothing to move: no launch


def test_rows_argument_checks():
    L = _lib.probe_lib()
    buf = ctypes.create_string_buffer(4096)
    p16 = (ctypes.addressof(buf) + 15) & ~15
    einval = L.hrs_probe_rows(p16, 1, 14, 2048, 11, 4, 0, 2, None)  # 11 + 4 > 14
    assert einval != 0
    assert L.hrs_probe_rows(p16, 1, 14, 2048, 10, 4, 0, 0, None) == einval  # blocks per CU
    assert L.hrs_probe_rows(p16, 1, 14, 2048, 0, 1, 0, 2, None) == einval
    assert L.hrs_probe_rows(p16, 1, 20, 2048, 9, 4, 0, 2, None) == einval  # pair not instantiated
    ealign = L.hrs_probe_rows(p16, 1, 14, 1000, 10, 4, 0, 2, None)
    assert ealign not in (0, einval)
    assert L.hrs_probe_rows(p16 + 1, 1, 14, 2048, 10, 4, 0, 2, None) == ealign
    assert L.hrs_probe_rows(p16, 1, 14, 2048, 10, 4, 4, 2, None) == einval  # schedule
    assert L.hrs_probe_rows(p16, 1, 14, 2048, 10, 4, -1, 2, None) == einval
    assert L.hrs_probe_rows(p16, 0, 14, 2048, 10, 4, 0, 2, None) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("schedule", [device.WAVE_TASKS, device.GRID_STRIDE, device.BLOCK_RANGE])
@pytest.mark.parametrize("depth", [1, 2, 4, 8])
@pytest.mark.parametrize("nt", [True, False])
@pytest.mark.parametrize("block,bpc", [(256, 2), (1024, 1)])
def test_stream_shapes_move_every_byte(cuda, schedule, depth, nt, block, bpc):
    torch = cuda
    nbytes = (5 << 20) + 48 * 16  # not a whole number of tasks / groups: the tail paths run too
    src = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda")
    dst = torch.zeros_like(src)
    kw = dict(schedule=schedule, depth=depth, nontemporal=nt, block_threads=block, blocks_per_cu=bpc)
    device.probe_copy(src, dst, **kw)
    assert torch.equal(dst, src)
    sink = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    device.probe_read(src, sink, **kw)
    dst.zero_()
    device.probe_write(dst, **kw)
    torch.cuda.synchronize()
    assert int(sink.sum().item()) == 0
    w = dst.view(torch.int32).view(-1, 4)  # 16-byte elements as 4 words
    assert (w[:, 1] == 0x5A5A5A5A).all()  # every element written, body and tail


@pytest.mark.gpu
@pytest.mark.parametrize("schedule", [0, 1, 2, 3])
@pytest.mark.parametrize("nr,nw,n", [(10, 4, 14), (10, 1, 14), (6, 3, 9), (12, 2, 16), (3, 2, 5)])
def test_rows_pattern_reads_and_writes_the_claimed_rows(cuda, nr, nw, n, schedule):
    """Schedules 0 and 3 write the plain XOR of the read rows (+ o); 1 and 2
    pass each loaded word through their VALU filler first, so there only the
    rows touched and the + o between written rows are checked."""
    torch = cuda
    S, L = 5, 3 * 2048
    st = torch.randint(0, 256, (S, n, L), dtype=torch.uint8, device="cuda")
    before = st.cpu().numpy()
    device.probe_rows(st, nr, nw, 2, schedule)
    after = st.cpu().numpy()
    x = np.bitwise_xor.reduce(before[:, n - nr:, :], axis=1).view(np.uint32)  # [S, L/4]
    w0 = after[:, 0, :].view(np.uint32) if nw else None
    for o in range(nw):
        got = after[:, o, :].view(np.uint32)
        base = x if schedule in (0, 3) else w0
        assert np.array_equal(got, (base.astype(np.uint64) + o).astype(np.uint32)), o
    assert np.array_equal(after[:, nw:, :], before[:, nw:, :])  # nothing else touched
