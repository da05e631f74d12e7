"""Host-side mirror of the hops codec plugin surface, backed by the HIP engine.

`ErasureCode` mirrors io.hops.erasure_coding.ErasureCode
(hadoop-hdfs-project/hadoop-hdfs/src/main/java/io/hops/erasure_coding/
ErasureCode.java:25-182) — same method names, argument meaning and error
behaviour — and `HipReedSolomonCode` is the drop-in for the `rs` codec's
ReedSolomonCode (hops-erasure-coding/src/main/java/io/hops/erasure_coding/
ReedSolomonCode.java), computing every byte on the GPU through libhrs.so.

Rows ("byte[][]") may be host buffers (bytearray, writable memoryview,
contiguous numpy uint8 arrays; read-only `bytes` for inputs) or 1-D uint8
torch tensors on a HIP device (then the device-resident entry points run).
"""
import abc
import ctypes

import numpy as np

from . import _lib
from ._lib import check, int_array, ptr_array


class TooManyErasedLocations(IOError):
    """io.hops.erasure_coding.TooManyErasedLocations (TooManyErasedLocations.java:26-31)."""


class ErasureCode(abc.ABC):
    """io.hops.erasure_coding.ErasureCode (ErasureCode.java:25-182)."""

    @abc.abstractmethod
    def encode(self, message, parity):
        """ErasureCode.java:38 — message: k ints, parity (out): p ints."""

    @abc.abstractmethod
    def decode(self, data, erasedLocations, erasedValues, locationsToRead=None, locationsNotToRead=None):
        """ErasureCode.java:55 (3-arg) and :75 (5-arg)."""

    def locationsToReadForDecode(self, erasedLocations):
        """ErasureCode.java:89-113: the k highest-index locations not erased,
        highest first; TooManyErasedLocations if fewer than k survive."""
        locationsToRead = []
        limit = self.stripeSize() + self.paritySize()
        for loc in range(limit - 1, -1, -1):
            if loc not in erasedLocations:
                locationsToRead.append(loc)
                if self.stripeSize() == len(locationsToRead):
                    break
        if len(locationsToRead) != self.stripeSize():
            raise TooManyErasedLocations(
                "Locations " + "".join(" " + str(e) for e in erasedLocations))
        return locationsToRead

    @abc.abstractmethod
    def stripeSize(self):
        ...

    @abc.abstractmethod
    def paritySize(self):
        ...

    @abc.abstractmethod
    def init(self, codec):
        ...

    @abc.abstractmethod
    def symbolSize(self):
        ...

    @abc.abstractmethod
    def encodeBulk(self, inputs, outputs):
        """ErasureCode.java:136-156."""

    @abc.abstractmethod
    def decodeBulk(self, readBufs, writeBufs, erasedLocations, locationsToRead=None, locationsNotToRead=None):
        """ErasureCode.java:162-181."""


# ------------------------------------------------------------------ buffers

def _is_device_tensor(x):
    t = _lib.torch
    return t is not None and isinstance(x, t.Tensor) and x.is_cuda


def _host_view(buf, writable):
    if isinstance(buf, np.ndarray):
        arr = buf
        if arr.dtype != np.uint8 or arr.ndim != 1 or not arr.flags["C_CONTIGUOUS"]:
            raise ValueError("host rows must be 1-D contiguous uint8 arrays")
        if writable and not arr.flags["WRITEABLE"]:
            raise ValueError("output row is read-only")
        return arr
    if isinstance(buf, bytes):
        if writable:
            raise ValueError("output row is immutable bytes")
        return np.frombuffer(buf, dtype=np.uint8)
    arr = np.frombuffer(buf, dtype=np.uint8)
    if writable and not arr.flags["WRITEABLE"]:
        raise ValueError("output row is read-only")
    return arr


class _Rows:
    """Pointers to a byte[][] argument; keeps views alive for the call."""

    def __init__(self, rows, writable, allow_none=False):
        self.views = []
        self.device = None
        ptrs, lens = [], set()
        for r in rows:
            if r is None:
                if not allow_none:
                    raise ValueError("row is None")
                ptrs.append(None)
                self.views.append(None)
                continue
            if _is_device_tensor(r):
                if r.dtype != _lib.torch.uint8 or r.dim() != 1 or not r.is_contiguous():
                    raise ValueError("device rows must be 1-D contiguous uint8 tensors")
                dev = r.device.index if r.device.index is not None else 0
                if self.device not in (None, dev):
                    raise ValueError("rows span several devices")
                if self.device is None and len([v for v in self.views if v is not None]) > 0:
                    raise ValueError("mixed host and device rows")
                self.device = dev
                ptrs.append(r.data_ptr())
                self.views.append(r)
                lens.add(r.numel())
            else:
                if self.device is not None:
                    raise ValueError("mixed host and device rows")
                v = _host_view(r, writable)
                ptrs.append(v.ctypes.data)
                self.views.append(v)
                lens.add(v.size)
        if len(lens) > 1:
            raise ValueError("rows of different lengths")
        self.len = lens.pop() if lens else 0
        self.ptrs = ptr_array(ptrs)


# ------------------------------------------------------------ the RS codec

class _HipErasureCode(ErasureCode):
    """Common HIP-backed implementation: bulk paths, matrices, lifecycle."""

    CODE_KIND = _lib.HRS_CODE_RS
    JAVA_CLASS = None

    def __init__(self, stripeSize=None, paritySize=None, device=None, zero_inputs_after_encode=False):
        self._h = None
        self._k = self._p = 0
        self._device = device
        self._conf = None
        self.zero_inputs_after_encode = zero_inputs_after_encode
        if stripeSize is not None:
            self._init(stripeSize, paritySize)

    # -- lifecycle
    def setConf(self, conf):
        """Configurable.setConf: Codec.createErasureCode hands the conf to the
        new instance before init (ReflectionUtils.newInstance, Codec.java:209-211).
        Unless the instance was built for an explicit device, init then takes
        the next device of `hdfs.raid.hip.devices` (devset.py)."""
        self._conf = conf

    def getConf(self):
        return self._conf

    def device(self):
        """Device ordinal the handle runs on (hrs_codec_device)."""
        return int(_lib.lib().hrs_codec_device(self._handle()))

    def init(self, codec):
        """ReedSolomonCode.init(Codec), ReedSolomonCode.java:48-54."""
        self._init(codec.stripeLength, codec.parityLength)

    def _opts(self):
        opts = _lib.HipOpts()
        if self._device is None and self._conf is not None:
            from .devset import pick_device
            self._device = pick_device(self._conf)
        opts.device = -1 if self._device is None else int(self._device)
        return opts

    def _init(self, k, p):
        L = _lib.lib()
        self.close()
        opts = self._opts()
        h = ctypes.c_void_p()
        check(L.hrs_create_code(self.CODE_KIND, int(k), int(p), ctypes.byref(opts), ctypes.byref(h)))
        self._h = h
        self._k, self._p = int(k), int(p)

    def close(self):
        if self._h is not None:
            _lib.lib().hrs_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _handle(self):
        if self._h is None:
            raise IOError("HipReedSolomonCode used before init()")
        return self._h

    def _check(self, st):
        check(st, self._h)

    def _placement(self, *row_sets):
        """Where a bulk call runs: None (host rows) or the device ordinal.
        Every row set must agree (a kernel storing to host addresses faults
        the GPU; a host memcpy into device pointers segfaults), and device
        rows must sit on the codec's device when it names one."""
        devs = {r.device for r in row_sets if r.len > 0 or r.device is not None}
        if len(devs) > 1:
            raise ValueError("bulk rows must all be host buffers or all on one device")
        dev = devs.pop() if devs else None
        if dev is not None and self._device is not None and int(self._device) != dev:
            raise ValueError(f"rows are on cuda:{dev} but the codec is on cuda:{int(self._device)}")
        return dev

    # -- geometry
    def stripeSize(self):
        return self._k

    def paritySize(self):
        return self._p

    def symbolSize(self):
        return _lib.lib().hrs_symbol_size(self._handle())

    def locationsToReadForDecode(self, erasedLocations):
        """The product's locationsToReadForDecode (hrs_locations_to_read_list):
        ErasureCode.java:89-113, or SimpleRegeneratingCode.java:300-366."""
        n = self._k + self._p
        buf = (ctypes.c_int * max(1, n))()
        cnt = ctypes.c_int(0)
        erased = [int(e) for e in erasedLocations]
        self._check(_lib.lib().hrs_locations_to_read_list(self._handle(), int_array(erased), len(erased), buf,
                                                           ctypes.byref(cnt)))
        return list(buf[: cnt.value])

    def setKernelMode(self, mode):
        """0 auto, 1 runtime-matrix bit-sliced kernel, 2 byte-granular kernel,
        3 auto but the fused encode+CRC kernel on every eligible shape."""
        self._check(_lib.lib().hrs_set_kernel_mode(self._handle(), int(mode)))

    # -- matrices (host)
    def lastKernel(self):
        """Main kernel of this handle's latest coding call, as rocprofv3 names
        it (hrs_last_kernel); "" before any device work."""
        return _lib.lib().hrs_last_kernel(self._handle()).decode()

    def lastHostPath(self):
        """How the latest synchronous host-buffer call moved its bytes
        (hrs_last_host_path): "pinned" (runtime-pinned rows, zero copy in place),
        "staged", "copy_engine" or ""."""
        return _lib.lib().hrs_last_host_path(self._handle()).decode()

    def encodeMatrix(self):
        g = np.zeros((self._p, self._k), dtype=np.uint8)
        self._check(_lib.lib().hrs_encode_matrix(self._handle(), g.ctypes.data))
        return g

    def decodeMatrix(self, erasedLocations, locationsNotToRead, zero_not_to_read=True):
        n = self._k + self._p
        d = np.zeros((max(1, len(erasedLocations)), n), dtype=np.uint8)
        self._check(_lib.lib().hrs_decode_matrix(
            self._handle(), int_array(erasedLocations), len(erasedLocations),
            int_array(locationsNotToRead), len(locationsNotToRead), int(bool(zero_not_to_read)),
            d.ctypes.data))
        return d[: len(erasedLocations)]

    # -- bulk (the hot path)
    def encodeBulk(self, inputs, outputs):
        """ReedSolomonCode.encodeBulk (ReedSolomonCode.java:103-125)."""
        if len(inputs) != self._k or len(outputs) != self._p:
            raise ValueError(f"encodeBulk needs {self._k} inputs and {self._p} outputs")
        ins = _Rows(inputs, writable=False)
        outs = _Rows(outputs, writable=True)
        if ins.len != outs.len:
            raise ValueError("input and output rows differ in length")
        L = _lib.lib()
        if self._placement(ins, outs) is not None:
            stream = _lib.torch.cuda.current_stream(ins.device).cuda_stream
            self._check(L.hrs_encode_dev(self._handle(), ins.ptrs, 0, outs.ptrs, 0, ins.len, 1, stream))
            return
        self._check(L.hrs_encode(self._handle(), ins.ptrs, outs.ptrs, ins.len))
        if self.zero_inputs_after_encode:
            for v in ins.views:
                if v.flags["WRITEABLE"]:
                    v[:] = 0

    def decodeBulk(self, readBufs, writeBufs, erasedLocations, locationsToRead=None, locationsNotToRead=None):
        """5-arg: ReedSolomonCode.decodeBulk (ReedSolomonCode.java:191-211).
        3-arg (locationsToRead and locationsNotToRead omitted): the RS-specific
        decodeBulk(readBufs, writeBufs, erasedLocation), :168-185."""
        n = self._k + self._p
        if len(readBufs) != n:
            raise ValueError(f"decodeBulk needs {n} read buffers")
        if len(writeBufs) != len(erasedLocations):
            raise ValueError("one write buffer per erased location")
        L = _lib.lib()
        three = locationsNotToRead is None
        if three:
            if not erasedLocations and self.CODE_KIND == _lib.HRS_CODE_RS:
                return
            reads = _Rows(readBufs, writable=False)
            writes = _Rows(writeBufs, writable=True)
            if self._placement(reads, writes) is not None:
                if self.CODE_KIND == _lib.HRS_CODE_XOR:
                    m = self.decodeMatrix(erasedLocations, [])
                else:
                    m = self.decodeMatrix(erasedLocations, erasedLocations, zero_not_to_read=False)
                self._apply_dev(m, reads, writes)
                return
            self._check(L.hrs_decode3(self._handle(), reads.ptrs, writes.ptrs, int_array(erasedLocations),
                                      len(erasedLocations), reads.len))
            return
        if locationsToRead is None:
            locationsToRead = []
        ntr = set(locationsNotToRead)
        reads = _Rows([None if (i in ntr and r is None) else r for i, r in enumerate(readBufs)],
                      writable=False, allow_none=True)
        writes = _Rows(writeBufs, writable=True)
        where = self._placement(reads, writes)
        if not erasedLocations and self.CODE_KIND == _lib.HRS_CODE_RS:
            return
        if where is not None:
            stream = _lib.torch.cuda.current_stream(reads.device).cuda_stream
            self._check(L.hrs_decode_dev(
                self._handle(), reads.ptrs, 0, writes.ptrs, 0, int_array(erasedLocations), len(erasedLocations),
                int_array(locationsNotToRead), len(locationsNotToRead), reads.len, 1, stream))
            return
        self._check(L.hrs_decode(
            self._handle(), reads.ptrs, writes.ptrs, int_array(erasedLocations), len(erasedLocations),
            int_array(locationsToRead), len(locationsToRead), int_array(locationsNotToRead),
            len(locationsNotToRead), reads.len))

    # -- bulk with block checksums (host rows: the JNI path)
    @staticmethod
    def _crc_arrays(crcs, n):
        out = np.zeros(n, dtype=np.uint32)
        if crcs is None:
            return None, out
        crc_in = np.ascontiguousarray(np.asarray(crcs, dtype=np.uint64).astype(np.uint32))
        if crc_in.shape != (n,):
            raise ValueError(f"need {n} running CRC values")
        return crc_in, out

    def encodeBulkCrc(self, inputs, outputs, crcs=None):
        """encodeBulk plus Encoder.encodeStripe's block checksums
        (Encoder.java:408-450): returns k + p CRC32 values, sources then
        parities, each continued from `crcs` (CRC32.update chaining across
        successive cells of a block; None = fresh CRC32 objects). Host rows go
        through the pinned pipeline (hrs_encode_crc), device rows through the
        fused kernel (hrs_encode_crc_dev; inputs are not zeroed there, as in
        encodeBulk's device path)."""
        if len(inputs) != self._k or len(outputs) != self._p:
            raise ValueError(f"encodeBulk needs {self._k} inputs and {self._p} outputs")
        ins = _Rows(inputs, writable=False)
        outs = _Rows(outputs, writable=True)
        if ins.len != outs.len:
            raise ValueError("input and output rows differ in length")
        crc_in, crc_out = self._crc_arrays(crcs, self._k + self._p)
        dev = self._placement(ins, outs)
        if dev is not None:  # device rows: one fused pass (hrs_encode_crc_dev)
            return self._crc_dev(lambda cin, cout, stream: _lib.lib().hrs_encode_crc_dev(
                self._handle(), ins.ptrs, 0, outs.ptrs, 0, ins.len, 1, cin, cout, stream), dev, crc_in, crc_out.size)
        self._check(_lib.lib().hrs_encode_crc(self._handle(), ins.ptrs, outs.ptrs, ins.len,
                                              None if crc_in is None else crc_in.ctypes.data, crc_out.ctypes.data))
        if self.zero_inputs_after_encode:
            for v in ins.views:
                if v.flags["WRITEABLE"]:
                    v[:] = 0
        return [int(x) for x in crc_out]

    def decodeBulkCrc(self, readBufs, writeBufs, erasedLocations, locationsToRead, locationsNotToRead, crcs=None):
        """5-arg decodeBulk plus the CRC32 of every repaired buffer, the value
        Decoder compares with the stored block checksum (Decoder.java:222-229,
        :645-655); continued from `crcs` (None = fresh). Host rows: hrs_decode_crc;
        device rows: hrs_decode_crc_dev (one fused pass)."""
        n = self._k + self._p
        if len(readBufs) != n:
            raise ValueError(f"decodeBulk needs {n} read buffers")
        if len(writeBufs) != len(erasedLocations):
            raise ValueError("one write buffer per erased location")
        ntr = set(locationsNotToRead)
        reads = _Rows([None if (i in ntr and r is None) else r for i, r in enumerate(readBufs)],
                      writable=False, allow_none=True)
        writes = _Rows(writeBufs, writable=True)
        dev = self._placement(reads, writes)
        crc_in, crc_out = self._crc_arrays(crcs, len(erasedLocations))
        if not erasedLocations:
            return []
        if dev is not None:  # device rows: repair + CRC in one pass (hrs_decode_crc_dev)
            return self._crc_dev(lambda cin, cout, stream: _lib.lib().hrs_decode_crc_dev(
                self._handle(), reads.ptrs, 0, writes.ptrs, 0, int_array(erasedLocations), len(erasedLocations),
                int_array(locationsNotToRead), len(locationsNotToRead), reads.len, 1, cin, cout, stream),
                dev, crc_in, crc_out.size)
        locationsToRead = locationsToRead or []
        self._check(_lib.lib().hrs_decode_crc(
            self._handle(), reads.ptrs, writes.ptrs, int_array(erasedLocations), len(erasedLocations),
            int_array(locationsToRead), len(locationsToRead), int_array(locationsNotToRead),
            len(locationsNotToRead), reads.len, None if crc_in is None else crc_in.ctypes.data,
            crc_out.ctypes.data))
        return [int(x) for x in crc_out]

    def _crc_dev(self, call, dev, crc_in, n):
        """Runs a device checksum call on the current stream of cuda:dev with
        device CRC arrays; returns the n CRC32 values (synchronizes)."""
        torch = _lib.torch
        out = torch.empty(n, dtype=torch.int32, device=f"cuda:{dev}")
        cin = None
        if crc_in is not None:
            cin = torch.from_numpy(crc_in.view(np.int32).copy()).to(out.device)
        stream = torch.cuda.current_stream(out.device).cuda_stream
        self._check(call(None if cin is None else cin.data_ptr(), out.data_ptr(), stream))
        return [int(x) & 0xFFFFFFFF for x in out.cpu().tolist()]

    # -- asynchronous rounds (hrs_*_submit / hrs_collect): round r computes on
    #    the GPU while the caller reads round r + 1; host rows only
    def encodeBulkAsync(self, inputs, checksums=False):
        """Submit an encodeBulk (plus the Encoder's block checksums when
        `checksums`); returns a ticket for collect(). The input rows may be
        reused as soon as this returns."""
        if len(inputs) != self._k:
            raise ValueError(f"encodeBulk needs {self._k} inputs")
        ins = _Rows(inputs, writable=False)
        if self._placement(ins) is not None:
            raise ValueError("asynchronous calls take host rows")
        t = ctypes.c_uint64(0)
        self._check(_lib.lib().hrs_encode_submit(self._handle(), ins.ptrs, ins.len, int(bool(checksums)),
                                                 ctypes.byref(t)))
        if self.zero_inputs_after_encode:
            for v in ins.views:
                if v.flags["WRITEABLE"]:
                    v[:] = 0
        return t.value

    def decodeBulkAsync(self, readBufs, erasedLocations, locationsToRead, locationsNotToRead, checksums=False):
        """Submit a 5-arg decodeBulk (plus the repaired blocks' CRC32s when
        `checksums`); returns a ticket for collect()."""
        n = self._k + self._p
        if len(readBufs) != n:
            raise ValueError(f"decodeBulk needs {n} read buffers")
        ntr = set(locationsNotToRead)
        reads = _Rows([None if (i in ntr and r is None) else r for i, r in enumerate(readBufs)],
                      writable=False, allow_none=True)
        if self._placement(reads) is not None:
            raise ValueError("asynchronous calls take host rows")
        locationsToRead = locationsToRead or []
        t = ctypes.c_uint64(0)
        self._check(_lib.lib().hrs_decode_submit(
            self._handle(), reads.ptrs, int_array(erasedLocations), len(erasedLocations), int_array(locationsToRead),
            len(locationsToRead), int_array(locationsNotToRead), len(locationsNotToRead), reads.len,
            int(bool(checksums)), ctypes.byref(t)))
        return t.value

    def collect(self, ticket, outputs, crcs=None):
        """Wait for a submitted operation and copy its output rows into
        `outputs` (p rows for encode, one per erased location for decode).
        A checksummed operation returns its CRC32 values continued from
        `crcs` (the running values; None = fresh CRC32 objects), else None."""
        nout, ln, ncrc = ctypes.c_int(0), ctypes.c_size_t(0), ctypes.c_int(0)
        self._check(_lib.lib().hrs_ticket_shape(self._handle(), int(ticket), ctypes.byref(nout), ctypes.byref(ln),
                                                ctypes.byref(ncrc)))
        if len(outputs) != nout.value:
            raise ValueError(f"this operation has {nout.value} output rows")
        outs = _Rows(outputs, writable=True)
        if outputs and outs.len < ln.value:
            raise ValueError("output rows shorter than the operation's rows")
        crc = np.zeros(max(1, ncrc.value), dtype=np.uint32)
        if ncrc.value and crcs is not None:
            crc[: ncrc.value] = np.asarray(crcs, dtype=np.uint64).astype(np.uint32)
        self._check(_lib.lib().hrs_collect(self._handle(), int(ticket), outs.ptrs,
                                           crc.ctypes.data if ncrc.value else None))
        return [int(x) for x in crc[: ncrc.value]] if ncrc.value else None

    def wait(self, ticket):
        """Block until a submitted operation's GPU work has completed, without
        collecting it (hrs_wait; collect then returns without blocking)."""
        self._check(_lib.lib().hrs_wait(self._handle(), int(ticket)))

    def release(self, ticket):
        """Drop a submitted operation without collecting it (hrs_release): its
        slot is drained and freed."""
        self._check(_lib.lib().hrs_release(self._handle(), int(ticket)))

    def pending(self):
        """Submitted operations not yet collected (at most 4 per codec)."""
        return int(_lib.lib().hrs_pending(self._handle()))

    def _apply_dev(self, m, reads, writes):
        stream = _lib.torch.cuda.current_stream(reads.device).cuda_stream
        m = np.ascontiguousarray(m, dtype=np.uint8)
        self._check(_lib.lib().hrs_apply_dev(self._handle(), m.ctypes.data, m.shape[0], m.shape[1], reads.ptrs, 0,
                                             writes.ptrs, 0, reads.len, 1, stream))

class HipReedSolomonCode(_HipErasureCode):
    """Drop-in for ReedSolomonCode (ReedSolomonCode.java:27-308) on MI355X.

    zero_inputs_after_encode: the reference encodeBulk zeroes its `inputs`
    (the bulk remainder of GaloisField.java:326-338 runs in place);
    True (default) restores that side effect for host rows.
    """

    CODE_KIND = _lib.HRS_CODE_RS
    JAVA_CLASS = "io.hops.erasure_coding.HipReedSolomonCode"

    def __init__(self, stripeSize=None, paritySize=None, device=None, zero_inputs_after_encode=True):
        super().__init__(stripeSize, paritySize, device, zero_inputs_after_encode)

    # -- scalar (one symbol column; still computed by the GPU engine)
    def encode(self, message, parity):
        """ReedSolomonCode.encode (ReedSolomonCode.java:84-97)."""
        if len(message) != self._k or len(parity) != self._p:
            raise ValueError("message/parity length mismatch")
        ins = [np.array([_symbol(v)], dtype=np.uint8) for v in message]
        outs = [np.zeros(1, dtype=np.uint8) for _ in range(self._p)]
        saved = self.zero_inputs_after_encode
        self.zero_inputs_after_encode = False
        try:
            self.encodeBulk(ins, outs)
        finally:
            self.zero_inputs_after_encode = saved
        for i in range(self._p):
            parity[i] = int(outs[i][0])

    def decode(self, data, erasedLocations, erasedValues, locationsToRead=None, locationsNotToRead=None):
        """3-arg ReedSolomonCode.decode (:127-142) or 5-arg (:144-166).
        Like the Java, zeroes data at the locations treated as erased, and
        writes erasedValues[i] only when erasedLocations[i] is one of the
        locations decoded (locationsNotToRead): the Java copies recovered
        values by matching locations (:158-165) and leaves any other entry as
        the caller passed it."""
        n = self._k + self._p
        if len(data) != n or len(erasedValues) != len(erasedLocations):
            raise ValueError("data/erasedValues length mismatch")
        if locationsNotToRead is None:
            # 3-arg (:127-142): zero data[erased], then the bulk 3-arg decode of
            # the zeroed column, erasedValues[i] = solution i (with a repeated
            # location the 5-arg matching would copy the first one's value)
            if not erasedLocations:
                return
            for loc in erasedLocations:
                data[loc] = 0
            rows = [np.array([_symbol(v)], dtype=np.uint8) for v in data]
            outs = [np.zeros(1, dtype=np.uint8) for _ in erasedLocations]
            self.decodeBulk(rows, outs, list(erasedLocations))
            for i in range(len(erasedLocations)):
                erasedValues[i] = int(outs[i][0])
            return
        else:
            ntr = list(locationsNotToRead)
            toread = list(locationsToRead or [])
        for loc in ntr:
            data[loc] = 0
        rows = [np.array([_symbol(v)], dtype=np.uint8) for v in data]
        outs = [np.zeros(1, dtype=np.uint8) for _ in erasedLocations]
        if not erasedLocations:
            return
        self.decodeBulk(rows, outs, list(erasedLocations), toread, ntr)
        decoded = set(ntr)
        for i in range(len(erasedLocations)):
            if erasedLocations[i] in decoded:
                erasedValues[i] = int(outs[i][0])



class HipXORCode(_HipErasureCode):
    """Drop-in for XORCode (hops-erasure-coding/.../XORCode.java:24-146):
    one parity row = XOR of the data rows; repair of one location = XOR of
    all other rows. Inputs are left untouched, as in the Java."""

    CODE_KIND = _lib.HRS_CODE_XOR
    JAVA_CLASS = "io.hops.erasure_coding.HipXORCode"

    def encode(self, message, parity):
        """XORCode.encode (XORCode.java:54-61)."""
        if len(message) != self._k or len(parity) != 1:
            raise ValueError("message/parity length mismatch")
        ins = [np.array([_symbol(v)], dtype=np.uint8) for v in message]
        out = [np.zeros(1, dtype=np.uint8)]
        self.encodeBulk(ins, out)
        parity[0] = int(out[0][0])

    def decode(self, data, erasedLocations, erasedValues, locationsToRead=None, locationsNotToRead=None):
        """XORCode.decode (XORCode.java:63-83): a no-op unless exactly one
        location is erased; data is not modified."""
        if len(erasedLocations) != 1:
            return
        rows = [np.array([_symbol(v)], dtype=np.uint8) for v in data]
        out = [np.zeros(1, dtype=np.uint8)]
        self.decodeBulk(rows, out, list(erasedLocations))
        erasedValues[0] = int(out[0][0])


class HipNativeReedSolomonCode(_HipErasureCode):
    """Drop-in for NativeReedSolomonCode (the `nrs` codec,
    hops-erasure-coding/.../NativeReedSolomonCode.java:32-196), which runs
    libhadoop's ISA-L coder (erasure_coder.c): a Cauchy RS code
    (gf_gen_cauchy1_matrix) in Apache [data, parity] order behind the hops
    [parity, data] locations. Bulk calls only; the scalar methods and
    symbolSize throw in the Java (UnsupportedOperationException), and so
    do they here (NotImplementedError).

    decodeBulk keeps the Java's output ordering: writeBufs[t] receives the
    t-th not-to-read location in Apache order (NativeReedSolomonCode.java:
    138-149), which is erasedLocations[t] whenever the erased locations are
    the not-to-read ones, in that order. Inputs are left untouched.
    """

    CODE_KIND = _lib.HRS_CODE_NRS
    JAVA_CLASS = "io.hops.erasure_coding.HipNativeReedSolomonCode"

    def encode(self, message, parity):
        raise NotImplementedError("Not supported yet.")

    def decode(self, data, erasedLocations, erasedValues, locationsToRead=None, locationsNotToRead=None):
        raise NotImplementedError("Not supported yet.")

    def symbolSize(self):
        raise NotImplementedError("Not supported yet.")

    def decodeBulk(self, readBufs, writeBufs, erasedLocations, locationsToRead=None, locationsNotToRead=None):
        """NativeReedSolomonCode.decodeBulk (NativeReedSolomonCode.java:90-152)."""
        if locationsNotToRead is None:
            raise NotImplementedError("NativeReedSolomonCode has no 3-argument decodeBulk")
        if len(writeBufs) > len(locationsNotToRead):
            # bwriteBufs holds |locationsNotToRead| buffers (NativeReedSolomonCode.java:96, :145-149)
            raise IndexError("more write buffers than not-to-read locations")
        super().decodeBulk(readBufs, writeBufs, erasedLocations, locationsToRead, locationsNotToRead)


class HipSimpleRegeneratingCode(_HipErasureCode):
    """Drop-in for SimpleRegeneratingCode (the `src` codec,
    hops-erasure-coding/.../SimpleRegeneratingCode.java:28-482): RS(k, r)
    plus s stored local XOR parities ("parity_length_src" in the codec JSON;
    init's adjustment loop may lower it, see srcLayout()). Bulk calls follow
    ErasureCode's default per-column loops (ErasureCode.java:136-181) over the
    Java's scalar encode/decode, computed here as matrices on the GPU.

    Not mirrored: the 3-argument scalar decode (an RS decode over the whole
    stripe, SimpleRegeneratingCode.java:188-191, which indexes past its tables
    for locations >= k + r) and the scalar decode's side effects on `data`
    (ErasureCode.decodeBulk hands it a scratch copy, so bulk callers never see
    them)."""

    CODE_KIND = _lib.HRS_CODE_SRC
    JAVA_CLASS = "io.hops.erasure_coding.HipSimpleRegeneratingCode"

    def __init__(self, stripeSize=None, paritySize=None, paritySizeSRC=0, device=None):
        self._src_in = int(paritySizeSRC)
        super().__init__(stripeSize, paritySize, device)

    def init(self, codec):
        """SimpleRegeneratingCode.init(Codec), :52-64."""
        self._src_in = int(codec.json.get("parity_length_src", 0))
        self._init(codec.stripeLength, codec.parityLength)

    def _init(self, k, p):
        L = _lib.lib()
        self.close()
        opts = self._opts()
        h = ctypes.c_void_p()
        check(L.hrs_create_src(int(k), int(p), self._src_in, ctypes.byref(opts), ctypes.byref(h)))
        self._h = h
        self._k, self._p = int(k), int(p)

    def srcLayout(self):
        """(stored SRC parities s, RS parities r, group degree d) after init."""
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self._check(_lib.lib().hrs_src_layout(self._handle(), ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value

    def encode(self, message, parity):
        """SimpleRegeneratingCode.encode, :116-157."""
        if len(message) != self._k or len(parity) != self._p:
            raise ValueError("message/parity length mismatch")
        ins = [np.array([_symbol(v)], dtype=np.uint8) for v in message]
        outs = [np.zeros(1, dtype=np.uint8) for _ in range(self._p)]
        self.encodeBulk(ins, outs)
        for i in range(self._p):
            parity[i] = int(outs[i][0])

    def decode(self, data, erasedLocations, erasedValues, locationsToRead=None, locationsNotToRead=None):
        """5-arg SimpleRegeneratingCode.decode, :194-277."""
        if locationsNotToRead is None:
            raise NotImplementedError("3-argument SimpleRegeneratingCode.decode is not provided")
        n = self._k + self._p
        if len(data) != n or len(erasedValues) != len(erasedLocations):
            raise ValueError("data/erasedValues length mismatch")
        if not erasedLocations:
            return
        rows = [np.array([_symbol(v)], dtype=np.uint8) for v in data]
        outs = [np.zeros(1, dtype=np.uint8) for _ in erasedLocations]
        self.decodeBulk(rows, outs, list(erasedLocations), list(locationsToRead or []), list(locationsNotToRead))
        for i in range(len(erasedLocations)):
            erasedValues[i] = int(outs[i][0])

    def decodeBulk(self, readBufs, writeBufs, erasedLocations, locationsToRead=None, locationsNotToRead=None):
        """ErasureCode.decodeBulk (ErasureCode.java:162-181) over the 5-arg decode."""
        if locationsNotToRead is None:
            raise NotImplementedError("SimpleRegeneratingCode has no 3-argument decodeBulk")
        super().decodeBulk(readBufs, writeBufs, erasedLocations, locationsToRead, locationsNotToRead)


def _symbol(v):
    v = int(v)
    if not 0 <= v < 256:
        raise ValueError(f"symbol {v} outside GF(2^8)")
    return v
