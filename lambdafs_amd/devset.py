"""Device set of the HIP codecs: which GPUs one process's codec instances use.

The reference builds one codec per Encoder / Decoder (Encoder.java:80,
Decoder.java:90) through Codec.createErasureCode, which instantiates the class
with ReflectionUtils.newInstance(class, conf) — handing `conf` to a
Configurable codec — and then calls init(codec)
(hadoop-hdfs/.../io/hops/erasure_coding/Codec.java:200-213). The HIP codecs
are Configurable: `hdfs.raid.hip.devices` lists the device ordinals a process
may use (default: every visible device), and each new codec instance takes
the next one, round robin, so the mapper threads of a JVM (one Encoder each)
spread over the node's GPUs. Java: HipDevices.java, same rules.

Spec syntax: comma-separated ordinals or ranges ("0,2,4-7"); "" or "all" =
every visible device. Ordinals are not range-checked here: creating a codec
on a device that does not exist fails in hrs_create (HRS_EDEVICE ->
IOException), as the Java binding's create does.
"""
import itertools
import threading

from . import _lib

HIP_DEVICES_KEY = "hdfs.raid.hip.devices"

_next = itertools.count()
_lock = threading.Lock()


def device_count():
    """HIP devices visible to this process (hrs_device_count)."""
    return int(_lib.lib().hrs_device_count())


def parse_device_set(spec, visible):
    """Ordinals named by a hdfs.raid.hip.devices value, in order (duplicates
    kept: "0,0,1" gives device 0 two turns of three)."""
    if spec is None or str(spec).strip().lower() in ("", "all"):
        if visible <= 0:
            raise IOError("no HIP device visible for the device set")
        return list(range(visible))
    out = []
    for part in str(spec).split(","):
        part = part.strip()
        if not part:
            raise ValueError(f"{HIP_DEVICES_KEY}: empty entry in {spec!r}")
        lo, sep, hi = part.partition("-")
        try:
            a = int(lo)
            b = int(hi) if sep else a
        except ValueError:
            raise ValueError(f"{HIP_DEVICES_KEY}: bad entry {part!r}") from None
        if a < 0 or b < a:
            raise ValueError(f"{HIP_DEVICES_KEY}: bad entry {part!r}")
        out.extend(range(a, b + 1))
    return out


def next_turn():
    with _lock:
        return next(_next)


def pick_device(conf, visible=None):
    """The device of the next codec instance under `conf` (a mapping of
    configuration keys): round robin over the device set."""
    spec = conf.get(HIP_DEVICES_KEY) if conf is not None else None
    if visible is None and (spec is None or str(spec).strip().lower() in ("", "all")):
        visible = device_count()
    devs = parse_device_set(spec, visible or 0)
    return devs[next_turn() % len(devs)]
