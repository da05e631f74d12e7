"""TEST INFRASTRUCTURE ONLY — pure-Python restatement of the reference RS code.

A second, independent transcription of the same Java methods the C oracle
(rs_oracle.c) restates, for small inputs only (it runs per byte in Python).
It exists to pin the C oracle (two transcriptions must agree byte for byte)
and to generate the committed golden fixtures (tests/golden/make_golden.py).

Reference (under /root/reference/hops-erasure-coding-project/hops-erasure-coding/
src/main/java/io/hops/erasure_coding/):
  GaloisField.java:76-119 tables; :190-204 power; :232-246 Vandermonde;
  :286-298 poly multiply; :310-320 remainder; :375-383 substitute.
  ReedSolomonCode.java:56-82 init; :84-97 encode; :127-166 decode;
  :168-185 decodeBulk 3-arg.
  hadoop-hdfs/.../ErasureCode.java:89-113 locationsToReadForDecode.
"""

FIELD = 256
PERIOD = 255
PRIM_POLY = 285


def _tables():
    log = [0] * FIELD
    pw = [0] * FIELD
    value = 1
    for p in range(FIELD - 1):
        pw[p] = value
        log[value] = p
        value *= 2
        if value >= FIELD:
            value ^= PRIM_POLY
    mul = [[0] * FIELD for _ in range(FIELD)]
    div = [[0] * FIELD for _ in range(FIELD)]
    for i in range(1, FIELD):
        for j in range(1, FIELD):
            z = log[i] + log[j]
            mul[i][j] = pw[z - PERIOD if z >= PERIOD else z]
            z = log[i] - log[j]
            div[i][j] = pw[z + PERIOD if z < 0 else z]
    return log, pw, mul, div


LOG, POW, MUL, DIV = _tables()


def power(x, n):
    if n == 0:
        return 1
    if x == 0:
        return 0
    x = LOG[x] * n
    return POW[x] if x < PERIOD else POW[x % PERIOD]


def poly_mul(p, q):
    r = [0] * (len(p) + len(q) - 1)
    for i, a in enumerate(p):
        for j, b in enumerate(q):
            r[i + j] ^= MUL[a][b]
    return r


def remainder(dividend, divisor):
    """In place, GaloisField.java:310-320."""
    nv = len(divisor)
    for i in range(len(dividend) - nv, -1, -1):
        ratio = DIV[dividend[i + nv - 1]][divisor[nv - 1]]
        for j in range(nv):
            dividend[i + j] ^= MUL[ratio][divisor[j]]


def substitute(p, x):
    result, y = 0, 1
    for c in p:
        result ^= MUL[c][y]
        y = MUL[x][y]
    return result


def solve_vandermonde(x, y, n=None):
    """In place on y, GaloisField.java:232-246."""
    n = len(x) if n is None else n
    for i in range(n - 1):
        for j in range(n - 1, i, -1):
            y[j] ^= MUL[x[i]][y[j - 1]]
    for i in range(n - 1, -1, -1):
        for j in range(i + 1, n):
            y[j] = DIV[y[j]][x[j] ^ x[j - i - 1]]
        for j in range(i, n - 1):
            y[j] ^= y[j + 1]


class ReedSolomonRef:
    """ReedSolomonCode(stripeSize, paritySize), scalar paths."""

    def __init__(self, k, p):
        assert k + p < FIELD
        self.k, self.p, self.n = k, p, k + p
        self.primitive_power = [power(2, i) for i in range(self.n)]
        gen = [1]
        for i in range(p):
            gen = poly_mul(gen, [self.primitive_power[i], 1])
        self.gen = gen

    def encode(self, message):
        buf = [0] * self.p + list(message)
        remainder(buf, self.gen)
        return buf[: self.p]

    def decode3(self, data, erased):
        """ReedSolomonCode.java:127-142; zeroes data[erased] like the Java."""
        if not erased:
            return []
        for loc in erased:
            data[loc] = 0
        sig = [self.primitive_power[loc] for loc in erased]
        vals = [substitute(data, self.primitive_power[i]) for i in range(len(erased))]
        solve_vandermonde(sig, vals, len(erased))
        return vals

    def decode5(self, data, erased, to_read, not_to_read, values=None):
        """ReedSolomonCode.java:144-166. `values` = the caller's erasedValues
        (entries whose location is not in not_to_read are left as passed)."""
        recov = self.decode3(data, list(not_to_read))
        out = list(values) if values is not None else [0] * len(erased)
        for i, e in enumerate(erased):
            for j, ntr in enumerate(not_to_read):
                if e == ntr:
                    out[i] = recov[j]
                    break
        return out

    # bulk forms, per byte (slow; small inputs only)
    def encode_bulk(self, inputs):
        L = len(inputs[0])
        out = [bytearray(L) for _ in range(self.p)]
        for col in range(L):
            par = self.encode([row[col] for row in inputs])
            for r in range(self.p):
                out[r][col] = par[r]
        return [bytes(o) for o in out]

    def decode_bulk5(self, read_bufs, erased, to_read, not_to_read):
        L = max(len(r) for r in read_bufs if r is not None)
        out = [bytearray(L) for _ in erased]
        for col in range(L):
            data = [(r[col] if r is not None else 0) for r in read_bufs]
            vals = self.decode5(data, erased, to_read, not_to_read)
            for i, v in enumerate(vals):
                out[i][col] = v
        return [bytes(o) for o in out]

    def decode_bulk3(self, read_bufs, erased):
        """ReedSolomonCode.java:168-185: no zeroing of the erased rows."""
        L = len(read_bufs[0])
        out = [bytearray(L) for _ in erased]
        if not erased:
            return [bytes(o) for o in out]
        sig = [self.primitive_power[loc] for loc in erased]
        for col in range(L):
            data = [r[col] for r in read_bufs]
            vals = [substitute(data, self.primitive_power[i]) for i in range(len(erased))]
            solve_vandermonde(sig, vals, len(erased))
            for i, v in enumerate(vals):
                out[i][col] = v
        return [bytes(o) for o in out]


def locations_to_read_for_decode(k, p, erased):
    """ErasureCode.java:89-113; returns None where the Java throws."""
    out = []
    for loc in range(k + p - 1, -1, -1):
        if loc not in erased:
            out.append(loc)
            if len(out) == k:
                break
    return out if len(out) == k else None
