"""Many threads creating codecs at once, as TestCodec.java:124-147 does with
100 threads (one codec per Encoder / Decoder, Encoder.java:80, Decoder.java:90,
all through Codec.createErasureCode, Codec.java:200-213).

CPU: 100 threads through the registry with host-only handles: every codec is
initialised with its codec's (k, p) and the reference's survivor choice
(ErasureCode.locationsToReadForDecode, ErasureCode.java:89-113), and the
device-set round robin (hdfs.raid.hip.devices) hands every device the same
number of turns. GPU: 32 threads each create an `rs` codec on device 0 and
immediately run a synchronous host encode and repair on their own stripe,
checked against the oracle (ReedSolomonCode.encodeBulk / decodeBulk 5-arg,
ReedSolomonCode.java:103-125, :191-211)."""
import collections
import threading

import numpy as np
import pytest

from lambdafs_amd import Codec, HipReedSolomonCode, devset
from lambdafs_amd import codec as codec_mod
from oracle import rs_oracle as C

NONE = -2  # HRS_DEVICE_NONE: a host-only handle


def _run(n, body):
    errs = []

    def wrap(i):
        try:
            body(i)
        except Exception as e:  # noqa: BLE001 - reported after the join
            errs.append(e)

    ths = [threading.Thread(target=wrap, args=(i,)) for i in range(n)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    if errs:
        raise errs[0]


def test_registry_init_race_host_only(monkeypatch):
    monkeypatch.setattr(devset, "pick_device", lambda conf: NONE)
    conf = {codec_mod.ERASURE_CODING_CODECS_KEY: codec_mod.DEFAULT_CODECS_JSON,
            "hdfs.raid.erasure.code.rs": HipReedSolomonCode.JAVA_CLASS}
    Codec.initializeCodecs(conf)
    got = [None] * 100

    def body(i):
        code = Codec.getCodec("rs").createErasureCode(conf)
        erased = [i % 14]
        got[i] = (code.stripeSize(), code.paritySize(), code.device(),
                  sorted(code.locationsToReadForDecode(erased)), erased)

    _run(100, body)
    for k, p, dev, tr, erased in got:
        assert (k, p, dev) == (10, 4, NONE)
        assert tr == sorted(C.locations_to_read(10, 4, erased))


def test_device_round_robin_under_threads():
    conf = {devset.HIP_DEVICES_KEY: "0-3"}
    picks = []
    lock = threading.Lock()

    def body(_):
        d = devset.pick_device(conf)
        with lock:
            picks.append(d)

    _run(100, body)
    assert collections.Counter(picks) == {0: 25, 1: 25, 2: 25, 3: 25}


@pytest.mark.gpu
def test_create_and_code_race(cuda):
    k, p, L = 10, 4, 256 << 10
    n = k + p
    conf = {codec_mod.ERASURE_CODING_CODECS_KEY: codec_mod.DEFAULT_CODECS_JSON,
            "hdfs.raid.erasure.code.rs": HipReedSolomonCode.JAVA_CLASS, devset.HIP_DEVICES_KEY: "0"}
    Codec.initializeCodecs(conf)

    def body(i):
        code = Codec.getCodec("rs").createErasureCode(conf)
        code.zero_inputs_after_encode = False
        rng = np.random.default_rng(i)
        data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
        par = [np.zeros(L, np.uint8) for _ in range(p)]
        code.encodeBulk(data, par)
        ref = C.encode_bulk(k, p, data)
        assert all(np.array_equal(a, b) for a, b in zip(par, ref)), i
        stripe = list(ref) + data
        erased = [i % n]
        tr = sorted(code.locationsToReadForDecode(erased))
        ntr = [x for x in range(n) if x not in tr]
        out = [np.zeros(L, np.uint8)]
        code.decodeBulk([stripe[x] if x in tr else None for x in range(n)], out, erased, tr, ntr)
        assert np.array_equal(out[0], stripe[erased[0]]), i
        code.close()

    _run(32, body)
