"""Codec registry: the plug-in point of the hops EC stack, mirrored.

io.hops.erasure_coding.Codec (hadoop-hdfs/src/main/java/io/hops/erasure_coding/
Codec.java:48-243) parses `dfs.erasure_coding.codecs.json`, sorts codecs by
priority and instantiates a codec's ErasureCode class by name, overridable per
codec id with `hdfs.raid.erasure.code.<id>` (Codec.java:52-53, :200-213). The
MI355X engine plugs in exactly there: set
`hdfs.raid.erasure.code.rs = io.hops.erasure_coding.HipReedSolomonCode`.
"""
import json

from .erasure_code import HipNativeReedSolomonCode, HipReedSolomonCode, HipSimpleRegeneratingCode, HipXORCode

ERASURE_CODE_KEY_PREFIX = "hdfs.raid.erasure.code."  # Codec.java:52-53
ERASURE_CODING_CODECS_KEY = "dfs.erasure_coding.codecs.json"  # DFSConfigKeys.java:558

# The codec table of hadoop-hdfs/src/main/resources/erasure-coding-default.xml:13-56.
DEFAULT_CODECS_JSON = json.dumps([
    {"id": "xor", "parity_dir": "/raid", "stripe_length": 10, "parity_length": 1, "priority": 100,
     "erasure_code": "io.hops.erasure_coding.XORCode", "description": "XOR code"},
    {"id": "rs", "parity_dir": "/raidrs", "stripe_length": 10, "parity_length": 4, "priority": 300,
     "erasure_code": "io.hops.erasure_coding.ReedSolomonCode", "description": "ReedSolomonCode code"},
    {"id": "src", "parity_dir": "/raidsrc", "stripe_length": 10, "parity_length": 6, "parity_length_src": 2,
     "erasure_code": "io.hops.erasure_coding.SimpleRegeneratingCode", "priority": 200,
     "description": "SimpleRegeneratingCode code"},
    {"id": "nrs", "parity_dir": "/raidnrs", "stripe_length": 10, "parity_length": 4, "priority": 50,
     "erasure_code": "io.hops.erasure_coding.NativeReedSolomonCode", "description": "Native ReedSolomonCode code"},
])

# Java class name -> implementation available in this engine (the RS hot path
# and its XOR and ISA-L-compatible siblings); any other class resolves to ClassNotFound, as a
# Java conf naming a missing class would (Codec.java:206-208).
ERASURE_CODE_CLASSES = {
    HipReedSolomonCode.JAVA_CLASS: HipReedSolomonCode,
    HipXORCode.JAVA_CLASS: HipXORCode,
    HipNativeReedSolomonCode.JAVA_CLASS: HipNativeReedSolomonCode,
    HipSimpleRegeneratingCode.JAVA_CLASS: HipSimpleRegeneratingCode,
}


class ClassNotFoundException(RuntimeError):
    pass


class Codec:
    """One codec entry (Codec.java:148-158)."""

    _codecs = []
    _id_to_codec = {}

    def __init__(self, json_obj):
        self.json = json_obj
        self.id = _get(json_obj, "id", str)
        self.parityLength = _get(json_obj, "parity_length", int)
        self.stripeLength = _get(json_obj, "stripe_length", int)
        self.erasureCodeClass = _get(json_obj, "erasure_code", str)
        self.parityDirectory = _get(json_obj, "parity_dir", str)
        self.priority = _get(json_obj, "priority", int)
        self.description = json_obj.get("description", "") if isinstance(json_obj.get("description", ""), str) else ""
        self._check_directory(self.parityDirectory)

    @staticmethod
    def _check_directory(d):
        """Codec.java:163-173: "/a/b/c" form."""
        if not d.startswith("/"):
            raise ValueError("Bad directory:" + d)
        if d.endswith("/"):
            raise ValueError("Bad directory:" + d)

    @classmethod
    def initializeCodecs(cls, conf):
        """Codec.java:133-164. conf: a mapping of configuration keys."""
        source = conf.get(ERASURE_CODING_CODECS_KEY)
        if source is None:
            cls._codecs, cls._id_to_codec = [], {}
            return
        try:
            arr = json.loads(source)
        except json.JSONDecodeError as e:  # JSONException -> IOException
            raise IOError(e) from e
        codecs = [Codec(o) for o in arr]
        cls._id_to_codec = {c.id: c for c in codecs}
        cls._codecs = sorted(codecs, key=lambda c: -c.priority)  # higher priority first (stable)

    @classmethod
    def getCodecs(cls):
        return list(cls._codecs)

    @classmethod
    def getCodec(cls, codec_id):
        return cls._id_to_codec.get(codec_id)

    def createErasureCode(self, conf):
        """Codec.java:200-213: class from conf override or JSON, then init(this)."""
        name = conf.get(ERASURE_CODE_KEY_PREFIX + self.id, self.erasureCodeClass)
        impl = ERASURE_CODE_CLASSES.get(name)
        if impl is None:
            raise ClassNotFoundException(name)
        code = impl()
        code.setConf(conf)  # ReflectionUtils.newInstance(erasureCode, conf): Configurable codecs get conf
        code.init(self)
        return code

    def getParityPrefix(self):
        p = self.parityDirectory
        return p if p.endswith("/") else p + "/"

    def getStripeLength(self):
        return self.stripeLength

    def getParityLength(self):
        return self.parityLength

    def getId(self):
        return self.id

    def __repr__(self):
        return json.dumps(self.json) if self.json is not None else f"Test codec {self.id}"


def _get(obj, key, typ):
    if key not in obj:
        raise KeyError(f'JSONObject["{key}"] not found.')
    v = obj[key]
    if typ is int:
        if isinstance(v, bool) or not isinstance(v, (int, str)):
            raise ValueError(f'JSONObject["{key}"] is not a number.')
        return int(v)
    return str(v)
