"""TEST INFRASTRUCTURE ONLY — java.util.Random, restated.

The reference's deterministic test inputs come from
`Util.randomBytes(seed, size)` = `new java.util.Random(seed).nextBytes(b)`
(hops-erasure-coding/src/test/java/io/hops/erasure_coding/Util.java:97-106),
e.g. seed 0xDEADBEEF in TestBlockReconstructor.java:52. java.util.Random is a
documented 48-bit LCG (multiplier 0x5DEECE66D, addend 0xB), so the same bytes
can be regenerated here without a JVM.
"""

_MULT = 0x5DEECE66D
_ADD = 0xB
_MASK = (1 << 48) - 1


def _to_int32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x & 0x80000000 else x


class JavaRandom:
    def __init__(self, seed):
        self._seed = (seed ^ _MULT) & _MASK

    def _next(self, bits):
        self._seed = (self._seed * _MULT + _ADD) & _MASK
        return _to_int32(self._seed >> (48 - bits))

    def nextInt(self, bound=None):
        if bound is None:
            return self._next(32)
        if bound <= 0:
            raise ValueError("bound must be positive")
        if (bound & -bound) == bound:  # power of two
            return _to_int32((bound * self._next(31)) >> 31)
        while True:
            bits = self._next(31)
            val = bits % bound
            if _to_int32(bits - val + (bound - 1)) >= 0:
                return val

    def nextBytes(self, n):
        out = bytearray(n)
        i = 0
        while i < n:
            rnd = self._next(32)
            for _ in range(min(n - i, 4)):
                out[i] = rnd & 0xFF
                rnd >>= 8
                i += 1
        return bytes(out)


def random_bytes(seed, size):
    """Util.randomBytes(long seed, int size), Util.java:101-106."""
    return JavaRandom(seed).nextBytes(size)
