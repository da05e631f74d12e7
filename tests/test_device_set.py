"""Device set of the drop-in (SURVEY §5 "engine env/config
for device set", §8(e)): which GPU each codec instance runs on, and host
batches split over several devices in one process.

Reference hook: Codec.createErasureCode -> ReflectionUtils.newInstance(class,
conf) (a Configurable codec receives conf) -> init(codec)
(hadoop-hdfs/.../io/hops/erasure_coding/Codec.java:200-213); one codec per
Encoder / Decoder (Encoder.java:80, Decoder.java:90).

CPU: the device-set syntax and round robin, the registry's setConf wiring,
and the C ABI's argument checks of the multi-device batches (host-only
handles). GPU: codecs created on explicit devices, an invalid ordinal, and the
multi-device batches with device set {0, 0} and {0, 0, 0} against the
oracle's full-size digests of BASELINE configs 5 and 2.
"""
import ctypes
import json
import os
import sys

import numpy as np
import pytest

from lambdafs_amd import Codec, HipReedSolomonCode, HrsError, _lib, device, devset
from lambdafs_amd import codec as codec_mod

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import synth  # noqa: E402

NONE = -2  # HRS_DEVICE_NONE


# ------------------------------------------------------------------- CPU

def test_parse_device_set():
    assert devset.parse_device_set(None, 4) == [0, 1, 2, 3]
    assert devset.parse_device_set("", 2) == [0, 1]
    assert devset.parse_device_set("all", 3) == [0, 1, 2]
    assert devset.parse_device_set("3", 8) == [3]
    assert devset.parse_device_set("0,2,4-7", 8) == [0, 2, 4, 5, 6, 7]
    assert devset.parse_device_set(" 1 , 1 ,0 ", 2) == [1, 1, 0]  # duplicates weight a device
    assert devset.parse_device_set("9", 1) == [9]  # ordinals are checked by hrs_create, not here
    for bad in ("0,,1", "a", "3-1", "-1", "1-x"):
        with pytest.raises(ValueError):
            devset.parse_device_set(bad, 8)
    with pytest.raises(IOError):
        devset.parse_device_set(None, 0)


def test_pick_device_round_robin(monkeypatch):
    monkeypatch.setattr(devset, "device_count", lambda: 3)
    conf = {}
    got = [devset.pick_device(conf) for _ in range(7)]
    start = got[0]
    assert got == [(start + i) % 3 for i in range(7)]
    conf = {devset.HIP_DEVICES_KEY: "4-5"}
    got = [devset.pick_device(conf) for _ in range(4)]
    assert sorted(got) == [4, 4, 5, 5] and got[0] != got[1]


def test_registry_hands_conf_to_the_codec(monkeypatch):
    """Codec.createErasureCode calls setConf before init (Codec.java:209-211),
    and init asks the device set for its device: here the pick is a host-only
    handle, so the wiring is visible without a GPU."""
    picks = []

    def fake_pick(conf):
        picks.append(conf)
        return NONE

    monkeypatch.setattr(devset, "pick_device", fake_pick)
    conf = {codec_mod.ERASURE_CODING_CODECS_KEY: codec_mod.DEFAULT_CODECS_JSON,
            "hdfs.raid.erasure.code.rs": HipReedSolomonCode.JAVA_CLASS,
            devset.HIP_DEVICES_KEY: "0"}
    Codec.initializeCodecs(conf)
    code = Codec.getCodec("rs").createErasureCode(conf)
    assert picks == [conf] and code.getConf() is conf
    assert code.device() == NONE
    assert (code.stripeSize(), code.paritySize()) == (10, 4)
    # an explicit device wins over the conf
    c2 = HipReedSolomonCode(device=NONE)
    c2.setConf(conf)
    c2.init(Codec.getCodec("rs"))
    assert len(picks) == 1 and c2.device() == NONE


def test_device_queries_without_a_gpu():
    L = _lib.lib()
    assert L.hrs_device_count() >= 0
    assert L.hrs_codec_device(None) == -1
    opts = _lib.HipOpts()
    h = ctypes.c_void_p()
    for bad in (-7, 4096):
        opts.device = bad
        assert L.hrs_create_code(0, 10, 4, ctypes.byref(opts), ctypes.byref(h)) == _lib.HRS_EDEVICE
        assert b"no HIP device" in L.hrs_last_error(None)


def _host_only(k=10, p=4, code=_lib.HRS_CODE_RS):
    opts = _lib.HipOpts()
    opts.device = NONE
    h = ctypes.c_void_p()
    assert _lib.lib().hrs_create_code(code, k, p, ctypes.byref(opts), ctypes.byref(h)) == 0
    return h


def test_multi_batch_rejects_bad_sets():
    """hrs_*_batch_host_multi argument rules (include/hrs.h), checked before any
    range runs."""
    L = _lib.lib()
    buf = np.zeros((4, 14, 64), dtype=np.uint8)
    out = np.zeros((4, 1, 64), dtype=np.uint8)
    er = np.full((4, 1), 4, dtype=np.int32)
    a, b = _host_only(), _host_only()
    x = _host_only(6, 3)
    try:
        def enc(hs, n=None):
            arr = _lib.ptr_array([h.value for h in hs]) if hs is not None else None
            return L.hrs_encode_batch_host_multi(arr, len(hs) if n is None else n, buf.ctypes.data, 64, 14 * 64, 64, 4)

        def dec(hs):
            arr = _lib.ptr_array([h.value for h in hs])
            return L.hrs_decode_batch_host_multi(arr, len(hs), buf.ctypes.data, 64, 14 * 64, er.ctypes.data, 1,
                                                 out.ctypes.data, 64, 64, 64, 4)

        assert enc(None, 0) == _lib.HRS_EINVAL
        assert enc([a], 0) == _lib.HRS_EINVAL
        assert enc([a, a]) == _lib.HRS_EINVAL and b"one handle" in L.hrs_last_error(a)
        assert enc([a, x]) == _lib.HRS_EINVAL and b"another code" in L.hrs_last_error(a)
        assert enc([a, b]) == _lib.HRS_EDEVICE and b"host-only" in L.hrs_last_error(a)
        assert dec([a, b]) == _lib.HRS_EDEVICE
        assert dec([b, a, a]) == _lib.HRS_EINVAL
        with pytest.raises(ValueError):
            device.encode_batch_host_multi([], buf)
    finally:
        for h in (a, b, x):
            L.hrs_destroy(h)


# ------------------------------------------------------------------- GPU

@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")) as f:
        return json.load(f)


def _digests(rows_of, S, g0=0):
    import stripe_digests as SD
    return SD.combine(SD.stripe_digests(rows_of, S, g0))


def _check(got, want):
    assert got, "nothing hashed"
    for key, d in got.items():
        assert want[key] == d, f"block {key}"


@pytest.fixture(params=["zero_copy", "copy_engine"])
def transfer_mode(request, monkeypatch):
    if request.param == "copy_engine":
        monkeypatch.setenv("HRS_ZEROCOPY", "0")
    else:
        monkeypatch.delenv("HRS_ZEROCOPY", raising=False)
    return request.param


@pytest.mark.gpu
def test_codecs_on_explicit_devices(cuda):
    ndev = devset.device_count()
    assert ndev == cuda.cuda.device_count() >= 1
    for d in range(min(ndev, 8)):
        assert HipReedSolomonCode(10, 4, device=d).device() == d
    with pytest.raises(HrsError) as e:
        HipReedSolomonCode(10, 4, device=ndev)
    assert e.value.status == _lib.HRS_EDEVICE
    conf = {codec_mod.ERASURE_CODING_CODECS_KEY: codec_mod.DEFAULT_CODECS_JSON,
            "hdfs.raid.erasure.code.rs": HipReedSolomonCode.JAVA_CLASS}
    Codec.initializeCodecs(conf)
    # default set = every visible device, round robin
    devs = [Codec.getCodec("rs").createErasureCode(conf).device() for _ in range(2 * ndev)]
    assert sorted(devs) == sorted(list(range(ndev)) * 2)
    conf[devset.HIP_DEVICES_KEY] = "0,0"
    assert {Codec.getCodec("rs").createErasureCode(conf).device() for _ in range(3)} == {0}
    conf[devset.HIP_DEVICES_KEY] = str(ndev)  # not a visible device
    with pytest.raises(HrsError) as e:
        Codec.getCodec("rs").createErasureCode(conf)
    assert e.value.status == _lib.HRS_EDEVICE


@pytest.mark.gpu
@pytest.mark.parametrize("members", [2, 3])
@pytest.mark.parametrize("pinned", [True, False])
def test_decode_batch_host_multi_config5_digests(cuda, golden, transfer_mode, members, pinned):
    """BASELINE config 5's per-GPU share (RS(12,4), 256 KiB, 512 stripes, a
    seeded lost pair per stripe) through a device set of `members` codecs on
    device 0 — the call an 8-GPU node makes with {0..7} — against the
    oracle's digests of the repaired cells."""
    torch = cuda
    k, p, L, S = 12, 4, 256 << 10, 512
    n = k + p
    gen = HipReedSolomonCode(k, p)
    dst = torch.zeros((S, n, L), dtype=torch.uint8, device="cuda")
    synth.fill_data_rows(torch, dst, 5, 0, k, p)
    device.encode_stripes(gen, dst)
    er = np.array([sorted(np.random.default_rng([0x5EED0005, g]).choice(n, 2, replace=False)) for g in range(S)],
                  dtype=np.int32)
    if pinned:
        st = torch.empty((S, n, L), dtype=torch.uint8, pin_memory=True)
        out = torch.zeros((S, 2, L), dtype=torch.uint8, pin_memory=True)
        st.copy_(dst)
        st, out = st.numpy(), out.numpy()
    else:
        st = dst.cpu().numpy()
        out = np.zeros((S, 2, L), dtype=np.uint8)
    del dst
    codes = [HipReedSolomonCode(k, p, device=0) for _ in range(members)]
    device.decode_batch_host_multi(codes, st, er, out)
    _check(_digests(lambda a, b: out[a:b], S), golden["config5"]["repaired"])


@pytest.mark.gpu
@pytest.mark.parametrize("members", [2, 3])
def test_encode_batch_host_multi_config2_digests(cuda, golden, transfer_mode, members):
    """BASELINE config 2 (RS(6,3), 64 KiB cells), its first 2,048 stripes,
    encoded in place in pinned host memory by a device set on device 0;
    ranges of 1,024 / 682-683 stripes cut across the 256-stripe digest blocks."""
    torch = cuda
    k, p, L, S = 6, 3, 64 << 10, 2048
    dst = torch.zeros((S, k + p, L), dtype=torch.uint8, device="cuda")
    synth.fill_data_rows(torch, dst, 2, 0, k, p)
    st = torch.empty((S, k + p, L), dtype=torch.uint8, pin_memory=True)
    st.copy_(dst)
    del dst
    codes = [HipReedSolomonCode(k, p, device=0) for _ in range(members)]
    device.encode_batch_host_multi(codes, st.numpy())
    got = _digests(lambda a, b: st[a:b, :p], S)
    assert len(got) == 8
    _check(got, golden["config2"]["parity"])


@pytest.mark.gpu
def test_multi_batch_error_names_the_member(cuda):
    """A range that fails reports its member, device and stripes on codecs[0]."""
    k, p, L, S = 10, 4, 4096, 6
    st = np.zeros((S, k + p, L), dtype=np.uint8)
    out = np.zeros((S, 1, L), dtype=np.uint8)
    er = np.full((S, 1), 4, dtype=np.int32)
    er[5, 0] = 99  # out of range, in member 1's range [3, 6)
    codes = [HipReedSolomonCode(k, p, device=0) for _ in range(2)]
    with pytest.raises(HrsError) as e:
        device.decode_batch_host_multi(codes, st, er, out)
    assert e.value.status == _lib.HRS_EINVAL
    assert "member 1" in str(e.value) and "stripes [3, 6)" in str(e.value)
