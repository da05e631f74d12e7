"""Device-resident stripe batches on MI355X (the hot path of bench.py).

HBM layout: a batch of S stripes is one uint8 tensor `stripes[S, n, L]` in
hops location order — rows [0, p) parity, [p, p+k) data — i.e. exactly the
`data` array ReedSolomonCode.encodeBulk assembles per call
(ReedSolomonCode.java:114-121), with S stripes stacked. A row view
`stripes[:, loc, :]` is handed to libhrs as (pointer of stripe 0, stride n*L).
Decode outputs go to a separate `out[S, e, L]` tensor.

All calls are asynchronous on the current torch stream of the tensors' device.
"""
import numpy as np

from . import _lib
from ._lib import int_array, ptr_array


def _rows(views):
    """[S, L] row views -> (pointer array, stride bytes, L, S)."""
    if not views:
        raise ValueError("no rows")
    strides, shapes = set(), set()
    for v in views:
        if v is None:
            continue
        if v.dtype != _lib.torch.uint8 or v.dim() != 2 or v.stride(1) != 1 or not v.is_cuda:
            raise ValueError("row views must be [S, L] uint8 device tensors with unit byte stride")
        strides.add(v.stride(0) if v.shape[0] > 1 else None)
        shapes.add(tuple(v.shape))
    if len(shapes) != 1:
        raise ValueError("row views differ in shape")
    strides.discard(None)
    if len(strides) > 1:
        raise ValueError("row views differ in stripe stride")
    S, L = shapes.pop()
    stride = strides.pop() if strides else L
    ptrs = ptr_array([None if v is None else v.data_ptr() for v in views])
    return ptrs, stride, L, S


def _stripe_rows(t, locs):
    """Rows `locs` (None = not passed) of a [S, m, L] uint8 device tensor ->
    (pointer array, stride bytes, L, S), the same as _rows over the views
    t[:, loc, :] but computed from t's own pointer and strides: building m
    tensor views costs ~3 us each in Python, more than a small launch."""
    torch = _lib.torch
    if t.dtype != torch.uint8 or t.dim() != 3 or t.stride(2) != 1 or not t.is_cuda:
        raise ValueError("stripes must be a [S, m, L] uint8 device tensor with unit byte stride")
    S, m, L = t.shape
    base, s_stripe, s_row = t.data_ptr(), t.stride(0), t.stride(1)
    for loc in locs:
        if loc is not None and not 0 <= loc < m:
            raise ValueError(f"row {loc} outside [0, {m})")
    ptrs = ptr_array([None if loc is None else base + loc * s_row for loc in locs])
    return ptrs, (s_stripe if S > 1 else L), L, S


def _stream(t):
    return _lib.torch.cuda.current_stream(t.device).cuda_stream


def encode_stripes(code, stripes):
    """Parity rows of every stripe from its data rows (encodeBulk over S stripes)."""
    k, p = code.stripeSize(), code.paritySize()
    if stripes.dim() != 3 or stripes.shape[1] != k + p:
        raise ValueError(f"stripes must be [S, {k + p}, L]")
    ins, s_in, L, S = _stripe_rows(stripes, range(p, p + k))
    outs, s_out, _, _ = _stripe_rows(stripes, range(p))
    code._check(_lib.lib().hrs_encode_dev(code._handle(), ins, s_in, outs, s_out, L, S, _stream(stripes)))


def encode_stripes_crc(code, stripes, crc_in=None):
    """Encode every stripe and return the CRC-32 (java.util.zip.CRC32) of its
    cells in one pass, as Encoder.encodeStripe keeps them with
    computeBlockChecksum (Encoder.java:408-450): an int32 tensor [S, k + p],
    columns [source 0..k-1, parity 0..p-1] holding the uint32 CRC bits.
    crc_in ([S, k + p] int32, same layout) continues running CRCs across
    successive cells (CRC32.update chaining)."""
    torch = _lib.torch
    k, p = code.stripeSize(), code.paritySize()
    if stripes.dim() != 3 or stripes.shape[1] != k + p:
        raise ValueError(f"stripes must be [S, {k + p}, L]")
    ins, s_in, L, S = _stripe_rows(stripes, range(p, p + k))
    outs, s_out, _, _ = _stripe_rows(stripes, range(p))
    crc = torch.empty((S, k + p), dtype=torch.int32, device=stripes.device)
    cin = None
    if crc_in is not None:
        if crc_in.shape != crc.shape or crc_in.dtype != torch.int32 or not crc_in.is_contiguous():
            raise ValueError(f"crc_in must be a contiguous int32 tensor [S, {k + p}]")
        cin = crc_in.data_ptr()
    code._check(_lib.lib().hrs_encode_crc_dev(code._handle(), ins, s_in, outs, s_out, L, S, cin, crc.data_ptr(),
                                              _stream(stripes)))
    return crc


def encode_rows(code, data_rows, parity_rows):
    """encodeBulk with explicit [S, L] row views (k data, p parity)."""
    ins, s_in, L, S = _rows(data_rows)
    outs, s_out, L2, S2 = _rows(parity_rows)
    if (L, S) != (L2, S2):
        raise ValueError("data and parity views differ in shape")
    code._check(_lib.lib().hrs_encode_dev(code._handle(), ins, s_in, outs, s_out, L, S, _stream(data_rows[0])))


def decode_stripes(code, stripes, erased, not_to_read, out):
    """decodeBulk 5-arg over S stripes: out[S, e, L] <- the erased locations.
    Rows of `stripes` at not_to_read locations are never read."""
    n = code.stripeSize() + code.paritySize()
    if stripes.dim() != 3 or stripes.shape[1] != n:
        raise ValueError(f"stripes must be [S, {n}, L]")
    ntr = set(not_to_read)
    rows, s_in, L, S = _stripe_rows(stripes, [None if loc in ntr else loc for loc in range(n)])
    outs, s_out, L2, S2 = _stripe_rows(out, range(len(erased)))
    if (L, S) != (L2, S2):
        raise ValueError("out must be [S, e, L]")
    code._check(_lib.lib().hrs_decode_dev(
        code._handle(), rows, s_in, outs, s_out, int_array(erased), len(erased),
        int_array(not_to_read), len(not_to_read), L, S, _stream(stripes)))


def decode_stripes_crc(code, stripes, erased, not_to_read, out, crc_in=None):
    """decode_stripes plus the CRC-32 (java.util.zip.CRC32) of every repaired
    cell in one pass, as the Decoder checks a repaired block against the
    NameNode's checksum (Decoder.java:222-229, :645-655): returns an int32
    tensor [S, e] of the uint32 CRC bits; crc_in (same layout) continues
    running CRCs across successive cells."""
    torch = _lib.torch
    n = code.stripeSize() + code.paritySize()
    if stripes.dim() != 3 or stripes.shape[1] != n:
        raise ValueError(f"stripes must be [S, {n}, L]")
    ntr = set(not_to_read)
    rows, s_in, L, S = _stripe_rows(stripes, [None if loc in ntr else loc for loc in range(n)])
    outs, s_out, L2, S2 = _stripe_rows(out, range(len(erased)))
    if (L, S) != (L2, S2):
        raise ValueError("out must be [S, e, L]")
    crc = torch.empty((S, len(erased)), dtype=torch.int32, device=stripes.device)
    cin = None
    if crc_in is not None:
        if crc_in.shape != crc.shape or crc_in.dtype != torch.int32 or not crc_in.is_contiguous():
            raise ValueError(f"crc_in must be a contiguous int32 tensor [S, {len(erased)}]")
        cin = crc_in.data_ptr()
    code._check(_lib.lib().hrs_decode_crc_dev(
        code._handle(), rows, s_in, outs, s_out, int_array(erased), len(erased),
        int_array(not_to_read), len(not_to_read), L, S, cin, crc.data_ptr(), _stream(stripes)))
    return crc


def decode_batch(code, stripes, erased, out):
    """Repair every stripe of stripes[S, n, L] from its own erasure list, in one
    launch (hrs_decode_batch_dev): erased is an int array [S, E] of hops
    locations (ascending per stripe, -1 padded; a row of -1 = nothing lost);
    out[S, E, L] receives stripe s's repaired rows in that order. Survivors are
    the ones locationsToReadForDecode picks, as Decoder.fixErasedBlockImpl does."""
    n = code.stripeSize() + code.paritySize()
    if stripes.dim() != 3 or stripes.shape[1] != n or stripes.stride(2) != 1:
        raise ValueError(f"stripes must be [S, {n}, L] with unit byte stride")
    e = np.ascontiguousarray(np.asarray(erased, dtype=np.int32))
    S, L = stripes.shape[0], stripes.shape[2]
    if e.ndim != 2 or e.shape[0] != S:
        raise ValueError("erased must be [S, E]")
    if out.dim() != 3 or tuple(out.shape) != (S, e.shape[1], L) or out.stride(2) != 1 or out.device != stripes.device:
        raise ValueError("out must be [S, E, L] on the stripes' device")
    code._check(_lib.lib().hrs_decode_batch_dev(
        code._handle(), stripes.data_ptr(), stripes.stride(1), stripes.stride(0), e.ctypes.data, e.shape[1],
        out.data_ptr(), out.stride(1), out.stride(0), L, S, _stream(stripes)))


def _host_ptr(a, name, writable=False):
    """Base address of a host batch (numpy array or CPU tensor, pinned or not)."""
    torch = _lib.torch
    if torch is not None and isinstance(a, torch.Tensor):
        if a.is_cuda or a.dtype != torch.uint8:
            raise ValueError(f"{name} must be a host uint8 tensor")
        return a.data_ptr(), tuple(a.shape), tuple(a.stride())
    a = np.asarray(a)
    if a.dtype != np.uint8 or (writable and not a.flags["WRITEABLE"]):
        raise ValueError(f"{name} must be a {'writable ' if writable else ''}uint8 array")
    return a.ctypes.data, a.shape, tuple(x // a.itemsize for x in a.strides)


def decode_batch_host(code, stripes, erased, out):
    """hrs_decode_batch_host: decode_batch for stripes[S, n, L] and out[S, E, L]
    in HOST memory (numpy arrays or CPU tensors; pinned ones are DMA'd
    directly). Only each stripe's survivors go over PCIe, only the repaired
    cells come back; chunks of stripes pipeline through the device."""
    n = code.stripeSize() + code.paritySize()
    sp, sshape, sstr = _host_ptr(stripes, "stripes")
    op, oshape, ostr = _host_ptr(out, "out", writable=True)
    e = np.ascontiguousarray(np.asarray(erased, dtype=np.int32))
    if len(sshape) != 3 or sshape[1] != n or sstr[2] != 1:
        raise ValueError(f"stripes must be [S, {n}, L] with unit byte stride")
    S, L = sshape[0], sshape[2]
    if e.ndim != 2 or e.shape[0] != S:
        raise ValueError("erased must be [S, E]")
    if len(oshape) != 3 or tuple(oshape) != (S, e.shape[1], L) or ostr[2] != 1:
        raise ValueError("out must be [S, E, L]")
    code._check(_lib.lib().hrs_decode_batch_host(
        code._handle(), sp, sstr[1], sstr[0], e.ctypes.data, e.shape[1], op, ostr[1], ostr[0], L, S))


def encode_batch_host(code, stripes):
    """hrs_encode_batch_host: parity rows of every stripe of a HOST batch
    stripes[S, n, L] (hops order) from its data rows, in place."""
    n = code.stripeSize() + code.paritySize()
    sp, sshape, sstr = _host_ptr(stripes, "stripes", writable=True)
    if len(sshape) != 3 or sshape[1] != n or sstr[2] != 1:
        raise ValueError(f"stripes must be [S, {n}, L] with unit byte stride")
    code._check(_lib.lib().hrs_encode_batch_host(code._handle(), sp, sstr[1], sstr[0], sshape[2], sshape[0]))


def _codec_array(codes):
    codes = list(codes)
    if not codes:
        raise ValueError("a device set needs at least one codec")
    return codes, ptr_array([c._handle().value for c in codes])


def decode_batch_host_multi(codes, stripes, erased, out):
    """hrs_decode_batch_host_multi: decode_batch_host over a device set. `codes`
    are distinct codecs of one code, each on the device it should use; the
    stripes split into len(codes) contiguous ranges, one per codec, run on
    their own host threads (one host link per device)."""
    codes, arr = _codec_array(codes)
    n = codes[0].stripeSize() + codes[0].paritySize()
    sp, sshape, sstr = _host_ptr(stripes, "stripes")
    op, oshape, ostr = _host_ptr(out, "out", writable=True)
    e = np.ascontiguousarray(np.asarray(erased, dtype=np.int32))
    if len(sshape) != 3 or sshape[1] != n or sstr[2] != 1:
        raise ValueError(f"stripes must be [S, {n}, L] with unit byte stride")
    S, L = sshape[0], sshape[2]
    if e.ndim != 2 or e.shape[0] != S:
        raise ValueError("erased must be [S, E]")
    if len(oshape) != 3 or tuple(oshape) != (S, e.shape[1], L) or ostr[2] != 1:
        raise ValueError("out must be [S, E, L]")
    _lib.check(_lib.lib().hrs_decode_batch_host_multi(
        arr, len(codes), sp, sstr[1], sstr[0], e.ctypes.data, e.shape[1], op, ostr[1], ostr[0], L, S),
        codes[0]._h)


def encode_batch_host_multi(codes, stripes):
    """hrs_encode_batch_host_multi: encode_batch_host over a device set
    (contiguous stripe ranges, one per codec, each on its own host thread)."""
    codes, arr = _codec_array(codes)
    n = codes[0].stripeSize() + codes[0].paritySize()
    sp, sshape, sstr = _host_ptr(stripes, "stripes", writable=True)
    if len(sshape) != 3 or sshape[1] != n or sstr[2] != 1:
        raise ValueError(f"stripes must be [S, {n}, L] with unit byte stride")
    _lib.check(_lib.lib().hrs_encode_batch_host_multi(arr, len(codes), sp, sstr[1], sstr[0], sshape[2], sshape[0]),
               codes[0]._h)


def apply_rows(code, matrix, in_rows, out_rows):
    """out_o = XOR_i matrix[o, i] * in_i over S stripes (matrix: host uint8 [nout, nin]).
    Used with coding matrices broadcast over RCCL (bench.py --gpus N)."""
    m = np.ascontiguousarray(np.asarray(matrix, dtype=np.uint8))
    ins, s_in, L, S = _rows(in_rows)
    outs, s_out, L2, S2 = _rows(out_rows)
    if m.shape != (len(out_rows), len(in_rows)) or (L, S) != (L2, S2):
        raise ValueError("shape mismatch")
    code._check(_lib.lib().hrs_apply_dev(code._handle(), m.ctypes.data, m.shape[0], m.shape[1], ins, s_in, outs,
                                         s_out, L, S, _stream(in_rows[0])))


def crc32_rows(code, row_views, crc_in=None):
    """CRC-32 (java.util.zip.CRC32) of every [S, L] row view, per stripe:
    returns an int32 tensor [S, nrows] holding the uint32 CRC bits
    (`& 0xFFFFFFFF` for the Java long value). crc_in, if given, is an int32
    tensor [S, nrows] of running CRCs to continue (CRC32.update chaining)."""
    torch = _lib.torch
    rows, stride, L, S = _rows(row_views)
    ref = next(v for v in row_views if v is not None)
    out = torch.empty((S, len(row_views)), dtype=torch.int32, device=ref.device)
    cin = None
    if crc_in is not None:
        if crc_in.shape != out.shape or crc_in.dtype != torch.int32 or not crc_in.is_contiguous():
            raise ValueError("crc_in must be a contiguous int32 tensor [S, nrows]")
        cin = crc_in.data_ptr()
    code._check(_lib.lib().hrs_crc32_dev(code._handle(), rows, len(row_views), stride, L, S, cin, out.data_ptr(),
                                         _stream(ref)))
    return out


PROBE_COPY, PROBE_READ, PROBE_WRITE = 0, 1, 2
WAVE_TASKS, GRID_STRIDE, BLOCK_RANGE = 0, 1, 2  # hrs_probe_stream schedules


def _nbytes(t):
    return t.numel() * t.element_size()


def _probe_check(status):
    if status != _lib.HRS_OK:
        raise _lib.HrsError(status, "hrs_probe call rejected its arguments")


def _probe_stream(op, src, dst, schedule, depth, nontemporal, block_threads, blocks_per_cu, nbytes, stream):
    _probe_check(_lib.probe_lib().hrs_probe_stream(op, src, dst, nbytes, int(schedule), int(depth),
                                                   int(bool(nontemporal)), int(block_threads), int(blocks_per_cu),
                                                   stream))


def probe_copy(src, dst, schedule=BLOCK_RANGE, depth=8, nontemporal=True, block_threads=1024, blocks_per_cu=1):
    """HBM ceiling probe (libhrs_probe.so, hrs_probe_stream COPY): dst <- src,
    both contiguous device tensors of the same byte size, on the current
    stream. Diagnostic: bench.py's copy_peak. Default = the fastest copy
    schedule of tools/copy_lab.hip (block ranges, 8 in flight, nontemporal,
    one 1024-thread block per CU)."""
    if (not src.is_cuda or not dst.is_cuda or not src.is_contiguous() or not dst.is_contiguous()
            or _nbytes(dst) != _nbytes(src)):
        raise ValueError("probe_copy needs two contiguous device tensors of equal size")
    _probe_stream(PROBE_COPY, src.data_ptr(), dst.data_ptr(), schedule, depth, nontemporal, block_threads,
                  blocks_per_cu, _nbytes(src), _stream(src))


def probe_read(src, sink, schedule=BLOCK_RANGE, depth=8, nontemporal=True, block_threads=1024, blocks_per_cu=1):
    """HBM read-only probe (hrs_probe_stream READ): reads the contiguous
    device tensor `src` once; `sink` is a device tensor of >= 4 KiB (never
    written in practice)."""
    if not src.is_cuda or not src.is_contiguous() or not sink.is_cuda or _nbytes(sink) < 4096:
        raise ValueError("probe_read needs a contiguous device tensor and a 4 KiB device sink")
    _probe_stream(PROBE_READ, src.data_ptr(), sink.data_ptr(), schedule, depth, nontemporal, block_threads,
                  blocks_per_cu, _nbytes(src), _stream(src))


def probe_write(dst, schedule=BLOCK_RANGE, depth=8, nontemporal=True, block_threads=1024, blocks_per_cu=1):
    """HBM write-only probe (hrs_probe_stream WRITE): writes the contiguous
    device tensor `dst` once."""
    if not dst.is_cuda or not dst.is_contiguous():
        raise ValueError("probe_write needs a contiguous device tensor")
    _probe_stream(PROBE_WRITE, None, dst.data_ptr(), schedule, depth, nontemporal, block_threads, blocks_per_cu,
                  _nbytes(dst), _stream(dst))


def probe_rows(stripes, nread, nwrite, blocks_per_cu=2, schedule=0):
    """The coding kernels' access pattern without the math (hrs_probe_rows):
    `stripes` is a contiguous uint8 device tensor [S, nrows, L]; per 2 KiB
    column window rows [nrows - nread, nrows) are read and rows [0, nwrite)
    overwritten with their XOR (+ the row index); `schedule` 0-3 spaces the
    loads (include/hrs_probe.h)."""
    if (not stripes.is_cuda or stripes.dtype != _lib.torch.uint8 or stripes.dim() != 3
            or not stripes.is_contiguous()):
        raise ValueError("probe_rows needs a contiguous uint8 device tensor [S, nrows, L]")
    S, n, L = stripes.shape
    _probe_check(_lib.probe_lib().hrs_probe_rows(stripes.data_ptr(), S, n, L, int(nread), int(nwrite),
                                                 int(schedule), int(blocks_per_cu), _stream(stripes)))
