"""Window -> wave orders (hrs_device.hpp wave_tasks; HRS_TASK_ORDER 1 =
grid-stride, 0 = block range, C > 1 = block-cyclic chunks of C windows per
wave) against the oracle on task counts that do not divide evenly: fewer
tasks than one block's waves, a last block with a short range, ranges that are not a multiple of the block's waves, and
row tails (the byte-granular kernel) beside whole windows. Every streaming
kernel family: static encode, fused encode + CRC, the pipelined and plain
repairs, fused repair + CRC, the heterogeneous repair batch, CRC-32 windows.
Bar: bit-exact. EVERY stripe is checked (a window an order misses or
runs twice in the middle of the task range must not slip through): coded
bytes against the byte-granular kernel (kernel mode 2, one byte column per
lane, no window order at all) over the whole tensor plus the oracle on sampled
stripes, CRCs against zlib for every cell."""
import zlib

import numpy as np
import pytest

from lambdafs_amd import HipReedSolomonCode, device
from oracle import rs_oracle as C

pytestmark = pytest.mark.gpu

# (stripes, cell bytes): 1 task; 3 x 3; 7 x 5 + tail; 513 x 2 (257 blocks, the
# last with 2 of 4); 300 x 32 (9,600 tasks over 512 blocks: 19 per block)
SHAPES = [(1, 2048), (3, 6144), (7, 2048 * 5 + 100), (513, 4096), (300, 65536)]


@pytest.fixture(params=[1, 0, 2, 32], ids=["grid_stride", "block_range", "cyclic2", "cyclic32"])
def order(request, monkeypatch):
    monkeypatch.setenv("HRS_TASK_ORDER", str(request.param))
    return request.param


def _stripes(torch, S, n, L, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    return torch.randint(0, 256, (S, n, L), dtype=torch.uint8, device="cuda", generator=g)


def _sample(S):
    return sorted({0, S // 2, S - 1})


def _crc(b):
    return zlib.crc32(np.ascontiguousarray(b).tobytes()) & 0xFFFFFFFF


def _bytewise(code, fn):
    """fn() run on the byte-granular kernel (kernel mode 2: no windows, no
    window order), the reference every stripe is compared with."""
    code.setKernelMode(2)
    try:
        return fn()
    finally:
        code.setKernelMode(0)


@pytest.mark.parametrize("S,L", SHAPES)
def test_encode_and_encode_crc(cuda, order, S, L):
    torch = cuda
    k, p = 10, 4
    code = HipReedSolomonCode(k, p)
    st = _stripes(torch, S, k + p, L, seed=S + L)
    st[:, :p] = 0xA5
    ref_dev = st.clone()
    _bytewise(code, lambda: device.encode_stripes(code, ref_dev))
    device.encode_stripes(code, st)
    st2 = st.clone()
    st2[:, :p] = 0x5A
    crc = device.encode_stripes_crc(code, st2)
    torch.cuda.synchronize()
    host, host2, crcs = st.cpu().numpy(), st2.cpu().numpy(), crc.cpu().numpy().view(np.uint32)
    assert np.array_equal(host, ref_dev.cpu().numpy()), (order, S, L)  # every stripe
    assert np.array_equal(host, host2)
    for s in _sample(S):
        ref = np.stack(C.encode_bulk(k, p, [host[s, p + c] for c in range(k)]))
        assert np.array_equal(host[s, :p], ref), (order, S, L, s)
    for s in range(S):
        want = [_crc(host[s, p + c]) for c in range(k)] + [_crc(host[s, r]) for r in range(p)]
        assert list(crcs[s]) == want, (order, S, L, s)


@pytest.mark.parametrize("S,L", SHAPES)
@pytest.mark.parametrize("erased", [[4], [0, 5], [1, 6, 11]])
def test_repairs(cuda, order, S, L, erased):
    torch = cuda
    k, p = 10, 4
    n = k + p
    code = HipReedSolomonCode(k, p)
    st = _stripes(torch, S, n, L, seed=3 * S + L)
    to_read = sorted(C.locations_to_read(k, p, erased))
    ntr = [x for x in range(n) if x not in to_read]
    out = torch.full((S, len(erased), L), 0x5A, dtype=torch.uint8, device="cuda")
    device.decode_stripes(code, st, erased, ntr, out)
    out2 = torch.full_like(out, 0xA5)
    crc = device.decode_stripes_crc(code, st, erased, ntr, out2)
    ref_dev = torch.full_like(out, 0x33)
    _bytewise(code, lambda: device.decode_stripes(code, st, erased, ntr, ref_dev))
    torch.cuda.synchronize()
    host, got, got2 = st.cpu().numpy(), out.cpu().numpy(), out2.cpu().numpy()
    crcs = crc.cpu().numpy().view(np.uint32)
    assert np.array_equal(got, ref_dev.cpu().numpy()), (order, S, L, erased)  # every stripe
    assert np.array_equal(got, got2)
    for s in _sample(S):
        reads = [host[s, i] if i in to_read else np.zeros(L, np.uint8) for i in range(n)]
        ref = C.decode_bulk5(k, p, reads, erased, to_read, ntr)
        for i in range(len(erased)):
            assert np.array_equal(got[s, i], ref[i]), (order, S, L, erased, s, i)
    for s in range(S):
        for i in range(len(erased)):
            assert crcs[s, i] == _crc(got[s, i]), (order, S, L, erased, s, i)


@pytest.mark.parametrize("S,L", SHAPES)
def test_repair_batch(cuda, order, S, L):
    torch = cuda
    k, p = 10, 4
    n = k + p
    code = HipReedSolomonCode(k, p)
    st = _stripes(torch, S, n, L, seed=5 * S + L)
    device.encode_stripes(code, st)
    rng = np.random.default_rng(S * 31 + L)
    er = np.full((S, 2), -1, np.int32)
    for s in range(S):
        e = int(rng.integers(0, 3))  # 0, 1 or 2 losses per stripe
        er[s, :e] = np.sort(rng.choice(n, e, replace=False))
    out = torch.full((S, 2, L), 0x5A, dtype=torch.uint8, device="cuda")
    device.decode_batch(code, st, er, out)
    torch.cuda.synchronize()
    host, got = st.cpu().numpy(), out.cpu().numpy()
    for s in range(S):
        for i, loc in enumerate(er[s]):
            if loc >= 0:
                assert np.array_equal(got[s, i], host[s, loc]), (order, S, L, s, list(er[s]))


@pytest.mark.parametrize("S,L", SHAPES)
def test_crc32_rows(cuda, order, S, L):
    torch = cuda
    code = HipReedSolomonCode(10, 4)
    st = _stripes(torch, S, 3, L, seed=7 * S + L)
    crc = device.crc32_rows(code, [st[:, r] for r in range(3)])
    torch.cuda.synchronize()
    host, crcs = st.cpu().numpy(), crc.cpu().numpy().view(np.uint32)
    for s in range(S):
        assert [int(x) for x in crcs[s]] == [_crc(host[s, r]) for r in range(3)], (order, S, L, s)
