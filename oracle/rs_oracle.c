/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle for the Reed-Solomon hot path.
 * Restates the reference Java loop for loop (see rs_oracle.h). Used by
 * tests/ as the parity checker and by bench.py as the timed CPU baseline
 * ("restated reference CPU path"); never by the product library.
 *
 * Pinning: RS parity is "parity unpinned" in the strict sense — the reference
 * is Java (no JDK here, so it cannot be run) and holds no RS golden vectors;
 * this restatement is cross-checked by an independent Python transcription
 * (rs_ref.py) and the reference's own property tests. The
 * CRC-32 tables are pinned to the reference's CRC32_T8 tables.
 *
 * Reference files (under /root/reference):
 *   GaloisField.java     hops-erasure-coding-project/hops-erasure-coding/src/main/java/io/hops/erasure_coding/
 *   ReedSolomonCode.java same directory
 *   ErasureCode.java     hadoop-hdfs-project/hadoop-hdfs/src/main/java/io/hops/erasure_coding/
 */
#include "rs_oracle.h"

#include <stdlib.h>
#include <string.h>

#define FIELD 256
#define PERIOD 255
#define PRIM_POLY 285

/* GaloisField.java:30-33: int tables, mul/div 256x256 (divTable[*][0] == 0). */
static int logTable[FIELD];
static int powTable[FIELD];
static int mulTable[FIELD][FIELD];
static int divTable[FIELD][FIELD];

/* GaloisField(int fieldSize, int primitivePolynomial), GaloisField.java:76-119. */
__attribute__((constructor)) static void gf_init(void) {
  int value = 1;
  for (int pow = 0; pow < FIELD - 1; pow++) {
    powTable[pow] = value;
    logTable[value] = pow;
    value = value * 2;
    if (value >= FIELD) value = value ^ PRIM_POLY;
  }
  for (int i = 0; i < FIELD; i++) {
    for (int j = 0; j < FIELD; j++) {
      if (i == 0 || j == 0) {
        mulTable[i][j] = 0;
        continue;
      }
      int z = logTable[i] + logTable[j];
      z = z >= PERIOD ? z - PERIOD : z;
      mulTable[i][j] = powTable[z];
    }
  }
  for (int i = 0; i < FIELD; i++) {
    for (int j = 1; j < FIELD; j++) {
      if (i == 0) {
        divTable[i][j] = 0;
        continue;
      }
      int z = logTable[i] - logTable[j];
      z = z < 0 ? z + PERIOD : z;
      divTable[i][j] = powTable[z];
    }
  }
}

int orc_gf_mul(int x, int y) { return mulTable[x][y]; }          /* :162-165 */
int orc_gf_div(int x, int y) { return divTable[x][y]; }          /* :176-179 */
int orc_gf_log(int x) { return logTable[x]; }
int orc_gf_pow_table(int i) { return powTable[i]; }

int orc_gf_power(int x, int n) { /* GaloisField.java:190-204 */
  if (n == 0) return 1;
  if (x == 0) return 0;
  x = logTable[x] * n;
  if (x < PERIOD) return powTable[x];
  x = x % PERIOD;
  return powTable[x];
}

/* GaloisField.java:286-298 */
void orc_gf_poly_mul(const int* p, int np, const int* q, int nq, int* result) {
  int len = np + nq - 1;
  for (int i = 0; i < len; i++) result[i] = 0;
  for (int i = 0; i < np; i++)
    for (int j = 0; j < nq; j++) result[i + j] = result[i + j] ^ mulTable[p[i]][q[j]];
}

/* GaloisField.java:351-364 */
void orc_gf_poly_add(const int* p, int np, const int* q, int nq, int* result) {
  int len = np > nq ? np : nq;
  for (int i = 0; i < len; i++) {
    if (i < np && i < nq)
      result[i] = p[i] ^ q[i];
    else if (i < np)
      result[i] = p[i];
    else
      result[i] = q[i];
  }
}

/* GaloisField.java:310-320 (scalar remainder) */
void orc_gf_remainder(int* dividend, int nd, const int* divisor, int nv) {
  for (int i = nd - nv; i >= 0; i--) {
    int ratio = divTable[dividend[i + nv - 1]][divisor[nv - 1]];
    for (int j = 0; j < nv; j++) {
      int k = j + i;
      dividend[k] = dividend[k] ^ mulTable[ratio][divisor[j]];
    }
  }
}

/* GaloisField.java:326-338 (bulk remainder over byte rows) */
static void gf_remainder_bulk(uint8_t* const* dividend, int nd, const int* divisor, int nv, size_t len) {
  for (int i = nd - nv; i >= 0; i--) {
    for (int j = 0; j < nv; j++) {
      uint8_t* top = dividend[i + nv - 1];
      uint8_t* dst = dividend[j + i];
      const int dv = divisor[nv - 1];
      for (size_t k = 0; k < len; k++) {
        int ratio = divTable[top[k] & 0x00FF][dv];
        dst[k] = (uint8_t)((dst[k] & 0x00FF) ^ mulTable[ratio][divisor[j]]);
      }
    }
  }
}

/* GaloisField.java:375-383 */
int orc_gf_substitute(const int* p, int np, int x) {
  int result = 0;
  int y = 1;
  for (int i = 0; i < np; i++) {
    result = result ^ mulTable[p[i]][y];
    y = mulTable[x][y];
  }
  return result;
}

/* GaloisField.java:396-406 (bulk substitute) */
static void gf_substitute_bulk(uint8_t* const* p, int np, uint8_t* q, int x, size_t len) {
  int y = 1;
  for (int i = 0; i < np; i++) {
    const uint8_t* pi = p[i];
    for (size_t j = 0; j < len; j++) {
      int pij = pi[j] & 0x000000FF;
      q[j] = (uint8_t)(q[j] ^ mulTable[pij][y]);
    }
    y = mulTable[x][y];
  }
}

/* GaloisField.java:232-246 */
void orc_gf_solve_vandermonde(const int* x, int* y, int len) {
  for (int i = 0; i < len - 1; i++)
    for (int j = len - 1; j > i; j--) y[j] = y[j] ^ mulTable[x[i]][y[j - 1]];
  for (int i = len - 1; i >= 0; i--) {
    for (int j = i + 1; j < len; j++) y[j] = divTable[y[j]][x[j] ^ x[j - i - 1]];
    for (int j = i; j < len - 1; j++) y[j] = y[j] ^ y[j + 1];
  }
}

/* GaloisField.java:251-273 (bulk Vandermonde) */
static void gf_solve_vandermonde_bulk(const int* x, uint8_t* const* y, int len, size_t data_len) {
  for (int i = 0; i < len - 1; i++)
    for (int j = len - 1; j > i; j--)
      for (size_t k = 0; k < data_len; k++)
        y[j][k] = (uint8_t)(y[j][k] ^ mulTable[x[i]][y[j - 1][k] & 0x000000FF]);
  for (int i = len - 1; i >= 0; i--) {
    for (int j = i + 1; j < len; j++)
      for (size_t k = 0; k < data_len; k++) y[j][k] = (uint8_t)(divTable[y[j][k] & 0x000000FF][x[j] ^ x[j - i - 1]]);
    for (int j = i; j < len - 1; j++)
      for (size_t k = 0; k < data_len; k++) y[j][k] = (uint8_t)(y[j][k] ^ y[j + 1][k]);
  }
}

/* GaloisField.java:412-451; matrix row-major height x width */
void orc_gf_gaussian_elimination(int* m, int height, int width) {
  int* tmp = (int*)malloc(sizeof(int) * (size_t)width);
#define M(r, c) m[(r) * width + (c)]
  for (int i = 0; i < height; i++) {
    int pivotFound = 0;
    for (int j = i; j < height; j++) {
      if (M(i, j) != 0) { /* sic: the reference tests matrix[i][j] and swaps rows i, j */
        memcpy(tmp, &M(i, 0), sizeof(int) * (size_t)width);
        memcpy(&M(i, 0), &M(j, 0), sizeof(int) * (size_t)width);
        memcpy(&M(j, 0), tmp, sizeof(int) * (size_t)width);
        pivotFound = 1;
        break;
      }
    }
    if (!pivotFound) continue;
    int pivot = M(i, i);
    for (int j = i; j < width; j++) M(i, j) = divTable[M(i, j)][pivot];
    for (int j = i + 1; j < height; j++) {
      int lead = M(j, i);
      for (int k = i; k < width; k++) M(j, k) = M(j, k) ^ mulTable[lead][M(i, k)];
    }
  }
  for (int i = height - 1; i >= 0; i--) {
    for (int j = 0; j < i; j++) {
      int lead = M(j, i);
      for (int k = i; k < width; k++) M(j, k) = M(j, k) ^ mulTable[lead][M(i, k)];
    }
  }
#undef M
  free(tmp);
}

/* ---------------------------------------------------------------- RS code */

/* ReedSolomonCode.init(int,int), ReedSolomonCode.java:56-82 */
int orc_rs_generator(int k, int p, int* gen_out) {
  if (k + p >= FIELD) return -1;
  int n = k + p;
  int* primitivePower = (int*)malloc(sizeof(int) * (size_t)n);
  for (int i = 0; i < n; i++) primitivePower[i] = orc_gf_power(2, i);
  int* gen = (int*)malloc(sizeof(int) * (size_t)(p + 1));
  int* tmp = (int*)malloc(sizeof(int) * (size_t)(p + 1));
  int glen = 1;
  gen[0] = 1;
  int poly[2];
  for (int i = 0; i < p; i++) {
    poly[0] = primitivePower[i];
    poly[1] = 1;
    orc_gf_poly_mul(gen, glen, poly, 2, tmp);
    glen += 1;
    memcpy(gen, tmp, sizeof(int) * (size_t)glen);
  }
  memcpy(gen_out, gen, sizeof(int) * (size_t)(p + 1));
  free(primitivePower);
  free(gen);
  free(tmp);
  return 0;
}

/* ReedSolomonCode.encode, :84-97 */
void orc_rs_encode(int k, int p, const int* message, int* parity) {
  int gen[FIELD];
  orc_rs_generator(k, p, gen);
  int* dataBuff = (int*)malloc(sizeof(int) * (size_t)(k + p));
  for (int i = 0; i < p; i++) dataBuff[i] = 0;
  for (int i = 0; i < k; i++) dataBuff[i + p] = message[i];
  orc_gf_remainder(dataBuff, k + p, gen, p + 1);
  for (int i = 0; i < p; i++) parity[i] = dataBuff[i];
  free(dataBuff);
}

/* ReedSolomonCode.encodeBulk, :103-125 */
void orc_rs_encode_bulk(int k, int p, uint8_t* const* inputs, uint8_t* const* outputs, size_t len) {
  int gen[FIELD];
  orc_rs_generator(k, p, gen);
  for (int i = 0; i < p; i++) memset(outputs[i], 0, len);
  uint8_t** data = (uint8_t**)malloc(sizeof(uint8_t*) * (size_t)(k + p));
  for (int i = 0; i < p; i++) data[i] = outputs[i];
  for (int i = 0; i < k; i++) data[i + p] = inputs[i];
  gf_remainder_bulk(data, k + p, gen, p + 1, len);
  free(data);
}

/* ReedSolomonCode.decode 3-arg, :127-142 */
void orc_rs_decode3(int k, int p, int* data, const int* erased, int ne, int* values) {
  (void)p;
  if (ne == 0) return;
  int n = k + p;
  int* errSignature = (int*)malloc(sizeof(int) * (size_t)ne);
  for (int i = 0; i < ne; i++) data[erased[i]] = 0;
  for (int i = 0; i < ne; i++) {
    errSignature[i] = orc_gf_power(2, erased[i]);  /* primitivePower[erasedLocations[i]] */
    values[i] = orc_gf_substitute(data, n, orc_gf_power(2, i));
  }
  orc_gf_solve_vandermonde(errSignature, values, ne);
  free(errSignature);
}

/* ReedSolomonCode.decode 5-arg, :144-166 */
void orc_rs_decode5(int k, int p, int* data, const int* erased, int ne, int* values, const int* to_read, int nr,
                    const int* not_to_read, int nn) {
  (void)to_read;
  (void)nr;
  int* recov = (int*)calloc((size_t)(nn > 0 ? nn : 1), sizeof(int));
  orc_rs_decode3(k, p, data, not_to_read, nn, recov);
  for (int i = 0; i < ne; i++) {
    for (int j = 0; j < nn; j++) {
      if (erased[i] == not_to_read[j]) {
        values[i] = recov[j];
        break;
      }
    }
  }
  free(recov);
}

/* ReedSolomonCode.decodeBulk 5-arg, :191-211 */
void orc_rs_decode_bulk5(int k, int p, uint8_t* const* read_bufs, uint8_t* const* write_bufs, const int* erased,
                         int ne, const int* to_read, int nr, const int* not_to_read, int nn, size_t len) {
  int n = k + p;
  int* tmpInput = (int*)malloc(sizeof(int) * (size_t)n);
  int* tmpOutput = (int*)malloc(sizeof(int) * (size_t)(ne > 0 ? ne : 1));
  for (size_t idx = 0; idx < len; idx++) {
    for (int i = 0; i < ne; i++) tmpOutput[i] = 0;
    for (int i = 0; i < n; i++) tmpInput[i] = read_bufs[i] ? (read_bufs[i][idx] & 0x000000FF) : 0;
    orc_rs_decode5(k, p, tmpInput, erased, ne, tmpOutput, to_read, nr, not_to_read, nn);
    for (int i = 0; i < ne; i++) write_bufs[i][idx] = (uint8_t)tmpOutput[i];
  }
  free(tmpInput);
  free(tmpOutput);
}

/* ReedSolomonCode.decodeBulk 3-arg, :168-185 */
void orc_rs_decode_bulk3(int k, int p, uint8_t* const* read_bufs, uint8_t* const* write_bufs, const int* erased,
                         int ne, size_t len) {
  if (ne == 0) return;
  int n = k + p;
  for (int i = 0; i < ne; i++) memset(write_bufs[i], 0, len);
  int* errSignature = (int*)malloc(sizeof(int) * (size_t)ne);
  for (int i = 0; i < ne; i++) {
    errSignature[i] = orc_gf_power(2, erased[i]);
    gf_substitute_bulk(read_bufs, n, write_bufs[i], orc_gf_power(2, i), len);
  }
  gf_solve_vandermonde_bulk(errSignature, write_bufs, ne, len);
  free(errSignature);
}

/* ErasureCode.locationsToReadForDecode, ErasureCode.java:89-113 */
int orc_locations_to_read(int k, int p, const int* erased, int ne, int* out) {
  int limit = k + p;
  int got = 0;
  for (int loc = limit - 1; loc >= 0; loc--) {
    int bad = 0;
    for (int i = 0; i < ne; i++)
      if (erased[i] == loc) bad = 1;
    if (!bad) {
      out[got++] = loc;
      if (got == k) break;
    }
  }
  return got;
}

/* ReedSolomonCode.computeSyndrome, :298-307 */
static int compute_syndrome(int k, int p, const int* data, int* syndrome) {
  int corruption = 0;
  for (int i = 0; i < p; i++) {
    syndrome[i] = orc_gf_substitute(data, k + p, orc_gf_power(2, i));
    if (syndrome[i] != 0) corruption = 1;
  }
  return !corruption;
}

/* ReedSolomonCode.computeErrorLocations, :243-287 */
int orc_rs_compute_error_locations(int k, int p, int* data, int* locations, int* nloc) {
  int n = k + p;
  int maxError = p / 2;
  int* syndrome = (int*)calloc((size_t)p, sizeof(int));
  *nloc = 0;
  if (compute_syndrome(k, p, data, syndrome)) {
    free(syndrome);
    return 1;
  }
  int w = maxError + 1;
  int* sm = (int*)calloc((size_t)(maxError * w + 1), sizeof(int));
  for (int i = 0; i < maxError; ++i)
    for (int j = 0; j < w; ++j) sm[i * w + j] = syndrome[i + j];
  if (maxError > 0) orc_gf_gaussian_elimination(sm, maxError, w);
  int* poly = (int*)calloc((size_t)w, sizeof(int));
  poly[0] = 1;
  for (int i = 0; i < maxError; ++i) poly[i + 1] = sm[(maxError - 1 - i) * w + maxError];
  for (int i = 0; i < n; ++i) {
    int possibleRoot = orc_gf_div(1, orc_gf_power(2, i));
    if (orc_gf_substitute(poly, w, possibleRoot) == 0) locations[(*nloc)++] = i;
  }
  int* vals = (int*)calloc((size_t)(*nloc > 0 ? *nloc : 1), sizeof(int));
  orc_rs_decode3(k, p, data, locations, *nloc, vals);
  for (int i = 0; i < *nloc; ++i) data[locations[i]] = vals[i];
  int ok = compute_syndrome(k, p, data, syndrome);
  free(vals);
  free(poly);
  free(sm);
  free(syndrome);
  return ok;
}

/* ------------------------------------------------------------- XOR code */

/* XORCode.encode, XORCode.java:54-61 */
void orc_xor_encode(int k, const int* message, int* parity) {
  parity[0] = message[0];
  for (int i = 1; i < k; i++) parity[0] ^= message[i];
}

/* XORCode.decode 3-arg, XORCode.java:63-77: no-op unless exactly one erasure */
void orc_xor_decode(int k, const int* data, const int* erased, int ne, int* values) {
  if (ne != 1) return;
  int skipIndex = erased[0];
  int val = 0;
  for (int i = 0; i < k + 1; i++) {
    if (i == skipIndex) continue;
    val ^= data[i];
  }
  values[0] = val;
}

/* XORCode.encodeBulk, XORCode.java:99-113 */
void orc_xor_encode_bulk(int k, uint8_t* const* inputs, uint8_t* output, size_t len) {
  for (size_t j = 0; j < len; j++) output[j] = inputs[0][j];
  for (int i = 1; i < k; i++)
    for (size_t j = 0; j < len; j++) output[j] ^= inputs[i][j];
}

/* XORCode.decodeBulk 3-arg, XORCode.java:115-138 (readBufs has k + 1 rows) */
void orc_xor_decode_bulk(int k, uint8_t* const* read_bufs, uint8_t* output, int erased, size_t len) {
  for (size_t j = 0; j < len; j++) output[j] = 0;
  for (int i = 0; i < k + 1; i++) {
    if (i == erased) continue;
    const uint8_t* input = read_bufs[i];
    for (size_t j = 0; j < len; j++) output[j] ^= input[j];
  }
}

/* ---------------------------- Apache Java RS coder (ported from ISA-L) */
/* hadoop-common .../io/erasurecode/rawcoder/util/GF256.java. The literal
 * tables GF_BASE (:35-88) and GF_LOG_BASE (:94-147) are regenerated here
 * (powers of 2 mod 0x11D; the log table stores log(1) as 0xff and log(0) as
 * 0) and pinned to the reference's numbers by tests/test_nrs_apache.py. */
static uint8_t ap_base[256], ap_log[256];

__attribute__((constructor)) static void ap_init(void) {
  int v = 1;
  for (int i = 0; i < 256; i++) {
    ap_base[i] = (uint8_t)v;
    v <<= 1;
    if (v & 0x100) v ^= 0x11D;
  }
  ap_log[0] = 0;
  for (int i = 0; i < 255; i++) ap_log[ap_base[i]] = (uint8_t)i;
  ap_log[1] = 0xff; /* GF_LOG_BASE[1] */
}

int orc_apache_gf_base(int i) { return ap_base[i & 0xff]; }
int orc_apache_gf_log_base(int i) { return ap_log[i & 0xff]; }

/* GF256.gfMul, :172-184 */
int orc_apache_gf_mul(int a, int b) {
  if (a == 0 || b == 0) return 0;
  int tmp = ap_log[a & 0xff] + ap_log[b & 0xff];
  if (tmp > 254) tmp -= 255;
  return ap_base[tmp];
}

/* GF256.gfInv, :186-192: GF_BASE[255 - GF_LOG_BASE[a] & 0xff] (Java: the
 * subtraction binds first, then & 0xff). */
int orc_apache_gf_inv(int a) {
  if (a == 0) return 0;
  return ap_base[(255 - ap_log[a & 0xff]) & 0xff];
}

/* GF256.gfInvertMatrix, :199-265 (throws "Not invertible": -1 here). */
static int ap_invert(uint8_t* in, uint8_t* out, int n) {
  for (int i = 0; i < n * n; i++) out[i] = 0;
  for (int i = 0; i < n; i++) out[i * n + i] = 1;
  for (int i = 0; i < n; i++) {
    if (in[i * n + i] == 0) {
      int j;
      for (j = i + 1; j < n; j++)
        if (in[j * n + i] != 0) break;
      if (j == n) return -1;
      for (int t = 0; t < n; t++) {
        uint8_t x = in[i * n + t];
        in[i * n + t] = in[j * n + t];
        in[j * n + t] = x;
        x = out[i * n + t];
        out[i * n + t] = out[j * n + t];
        out[j * n + t] = x;
      }
    }
    const int temp = orc_apache_gf_inv(in[i * n + i]);
    for (int j = 0; j < n; j++) {
      in[i * n + j] = (uint8_t)orc_apache_gf_mul(in[i * n + j], temp);
      out[i * n + j] = (uint8_t)orc_apache_gf_mul(out[i * n + j], temp);
    }
    for (int j = 0; j < n; j++) {
      if (j == i) continue;
      const int f = in[j * n + i];
      for (int t = 0; t < n; t++) {
        out[j * n + t] ^= (uint8_t)orc_apache_gf_mul(f, out[i * n + t]);
        in[j * n + t] ^= (uint8_t)orc_apache_gf_mul(f, in[i * n + t]);
      }
    }
  }
  return 0;
}

/* GF256.gfVectMulInit, :267-337: the 32-byte multiply table of c (ISA-L's
 * gf_vect_mul_init); RSUtil.encodeData reads its entry 1 (= c). */
static void ap_vect_mul_init(uint8_t c, uint8_t* tbl) {
#define AP_X2(v) ((uint8_t)(((v) << 1) ^ (((v)&0x80) ? 0x1d : 0)))
  const uint8_t c2 = AP_X2(c), c4 = AP_X2(c2), c8 = AP_X2(c4);
  const uint8_t c3 = c2 ^ c, c5 = c4 ^ c, c6 = c4 ^ c2, c7 = c4 ^ c3;
  const uint8_t lo[16] = {0, c, c2, c3, c4, c5, c6, c7, c8, (uint8_t)(c8 ^ c), (uint8_t)(c8 ^ c2),
                          (uint8_t)(c8 ^ c3), (uint8_t)(c8 ^ c4), (uint8_t)(c8 ^ c5), (uint8_t)(c8 ^ c6),
                          (uint8_t)(c8 ^ c7)};
  const uint8_t c17 = AP_X2(c8), c18 = AP_X2(c17), c19 = c18 ^ c17, c20 = AP_X2(c18);
  const uint8_t c21 = c20 ^ c17, c22 = c20 ^ c18, c23 = c20 ^ c19, c24 = AP_X2(c20);
  const uint8_t hi[16] = {0,   c17, c18, c19, c20, c21, c22, c23, c24, (uint8_t)(c24 ^ c17), (uint8_t)(c24 ^ c18),
                          (uint8_t)(c24 ^ c19), (uint8_t)(c24 ^ c20), (uint8_t)(c24 ^ c21), (uint8_t)(c24 ^ c22),
                          (uint8_t)(c24 ^ c23)};
#undef AP_X2
  memcpy(tbl, lo, 16);
  memcpy(tbl + 16, hi, 16);
}

/* RSUtil.genCauchyMatrix, :63-76: identity on top, then a[i][j] = gfInv(i ^ j). */
void orc_apache_gen_cauchy(uint8_t* a, int m, int k) {
  memset(a, 0, (size_t)m * k);
  for (int i = 0; i < k; i++) a[k * i + i] = 1;
  int pos = k * k;
  for (int i = k; i < m; i++)
    for (int j = 0; j < k; j++) a[pos++] = (uint8_t)orc_apache_gf_inv(i ^ j);
}

/* RSUtil.initTables, :47-58, then RSUtil.encodeData(byte[]...), :86-135:
 * outputs[l] ^= mul(coefficient (tables[j*32 + l*ninputs*32 + 1]), inputs[j])
 * byte by byte; outputs are zeroed first (CoderUtil.resetOutputBuffers). */
static void ap_encode_data(int ninputs, int noutputs, const uint8_t* coding_matrix, uint8_t* const* inputs,
                           uint8_t* const* outputs, size_t len) {
  uint8_t* tables = (uint8_t*)malloc((size_t)ninputs * noutputs * 32);
  int offset = 0, idx = 0;
  for (int i = 0; i < noutputs; i++)
    for (int j = 0; j < ninputs; j++, offset += 32) ap_vect_mul_init(coding_matrix[idx++], tables + offset);
  for (int l = 0; l < noutputs; l++) {
    memset(outputs[l], 0, len);
    for (int j = 0; j < ninputs; j++) {
      const int s = tables[j * 32 + l * ninputs * 32 + 1];
      for (size_t i = 0; i < len; i++) outputs[l][i] ^= (uint8_t)orc_apache_gf_mul(s, inputs[j][i]);
    }
  }
  free(tables);
}

/* RSRawEncoder: constructor :45-60 (encodeMatrix = genCauchyMatrix(k + p, k),
 * tables from its rows k..), doEncode(ByteArrayEncodingState) :71-78. */
void orc_apache_rs_encode(int k, int p, uint8_t* const* inputs, uint8_t* const* outputs, size_t len) {
  uint8_t* a = (uint8_t*)malloc((size_t)(k + p) * k);
  orc_apache_gen_cauchy(a, k + p, k);
  ap_encode_data(k, p, a + (size_t)k * k, inputs, outputs, len);
  free(a);
}

/* RSRawDecoder.doDecode(ByteArrayDecodingState), :87-102: validIndexes =
 * the non-null inputs (CoderUtil.getValidIndexes), the first k of them read;
 * processErasures :120-144 and generateDecodeMatrix :147-176. */
int orc_apache_rs_decode(int k, int p, uint8_t* const* inputs, const int* erased, int ne, uint8_t* const* outputs,
                         size_t len) {
  const int n = k + p;
  int valid[256], nvalid = 0;
  for (int i = 0; i < n; i++)
    if (inputs[i]) valid[nvalid++] = i;
  if (nvalid < k) return -1;
  uint8_t* enc = (uint8_t*)malloc((size_t)n * k);
  orc_apache_gen_cauchy(enc, n, k);
  int nerased_data = 0;
  for (int i = 0; i < ne; i++)
    if (erased[i] < k) nerased_data++;
  uint8_t* tmp = (uint8_t*)calloc((size_t)n * k, 1);
  uint8_t* inv = (uint8_t*)calloc((size_t)n * k, 1);
  uint8_t* dec = (uint8_t*)calloc((size_t)n * k, 1);
  for (int i = 0; i < k; i++)
    for (int j = 0; j < k; j++) tmp[k * i + j] = enc[k * valid[i] + j];
  int rc = ap_invert(tmp, inv, k);
  if (rc == 0) {
    for (int i = 0; i < nerased_data; i++)
      for (int j = 0; j < k; j++) dec[k * i + j] = inv[k * erased[i] + j];
    for (int q = nerased_data; q < ne; q++)
      for (int i = 0; i < k; i++) {
        uint8_t s = 0;
        for (int j = 0; j < k; j++) s ^= (uint8_t)orc_apache_gf_mul(inv[j * k + i], enc[k * erased[q] + j]);
        dec[k * q + i] = s;
      }
    uint8_t* real[256];
    for (int i = 0; i < k; i++) real[i] = inputs[valid[i]];
    ap_encode_data(k, ne, dec, real, outputs, len);
  }
  free(enc);
  free(tmp);
  free(inv);
  free(dec);
  return rc;
}

/* ------------------------------------- hadoop-common's legacy RS coder
 * The reference's second source of the SAME polynomial code as hops'
 * ReedSolomonCode: hadoop-common
 * .../io/erasurecode/rawcoder/RSLegacyRawEncoder.java, RSLegacyRawDecoder.java
 * over its own util/GaloisField.java and util/RSUtil.java — separate files,
 * restated here loop for loop with their own tables (lg_*), so a slip in one
 * transcription of the hops classes cannot hide in both. */

/* rawcoder/util/GaloisField.java: int tables of the byte field (field size
 * 256, primitive polynomial 285: getInstance(), :119-121), built by the
 * constructor :47-93. */
static int lg_log[FIELD], lg_pow[FIELD], lg_mul[FIELD][FIELD], lg_div[FIELD][FIELD];

__attribute__((constructor)) static void lg_init(void) {
  int value = 1;
  for (int pow = 0; pow < FIELD - 1; pow++) { /* :58-66 */
    lg_pow[pow] = value;
    lg_log[value] = pow;
    value = value * 2;
    if (value >= FIELD) value = value ^ PRIM_POLY;
  }
  for (int i = 0; i < FIELD; i++) /* :68-79 */
    for (int j = 0; j < FIELD; j++) {
      if (i == 0 || j == 0) {
        lg_mul[i][j] = 0;
        continue;
      }
      int z = lg_log[i] + lg_log[j];
      z = z >= PERIOD ? z - PERIOD : z;
      lg_mul[i][j] = lg_pow[z];
    }
  for (int i = 0; i < FIELD; i++) /* :81-92 (divTable[*][0] stays 0) */
    for (int j = 1; j < FIELD; j++) {
      if (i == 0) {
        lg_div[i][j] = 0;
        continue;
      }
      int z = lg_log[i] - lg_log[j];
      z = z < 0 ? z + PERIOD : z;
      lg_div[i][j] = lg_pow[z];
    }
}

/* GaloisField.power, :184-198 */
static int lg_power(int x, int n) {
  if (n == 0) return 1;
  if (x == 0) return 0;
  x = lg_log[x] * n;
  if (x < PERIOD) return lg_pow[x];
  x = x % PERIOD;
  return lg_pow[x];
}

/* RSUtil.getPrimitivePower, RSUtil.java:38-45: primitivePower[i] = 2^i. */
static void lg_primitive_power(int k, int p, int* pp) {
  for (int i = 0; i < k + p; i++) pp[i] = lg_power(2, i);
}

/* RSLegacyRawEncoder(ErasureCoderOptions), RSLegacyRawEncoder.java:36-53:
 * gen = prod_{i<p} (x + primitivePower[i]) through GaloisField.multiply(int[],
 * int[]) (:315-328, add = xor :148-151). Returns p + 1 coefficients. */
static void lg_generator(int k, int p, int* gen) {
  int pp[256], tmp[257];
  lg_primitive_power(k, p, pp);
  int glen = 1;
  gen[0] = 1;
  for (int i = 0; i < p; i++) {
    const int poly[2] = {pp[i], 1};
    for (int t = 0; t < glen + 1; t++) tmp[t] = 0;
    for (int a = 0; a < glen; a++)
      for (int b = 0; b < 2; b++) tmp[a + b] = tmp[a + b] ^ lg_mul[gen[a]][poly[b]];
    glen += 1;
    for (int t = 0; t < glen; t++) gen[t] = tmp[t];
  }
}

int orc_legacy_generator(int k, int p, int* gen_out) {
  if (k + p >= FIELD) return -1; /* the constructor's assert, :39 */
  lg_generator(k, p, gen_out);
  return p + 1;
}

/* RSLegacyRawEncoder.doEncode(ByteArrayEncodingState), :91-128, with
 * allowChangeInputs() false (the coder's default): outputs zeroed
 * (CoderUtil.resetOutputBuffers), inputs copied (Arrays.copyOfRange), all =
 * [outputs..., input copies...], then GaloisField.remainder(byte[][], int[]
 * offsets, int len, int[] divisor), util/GaloisField.java:480-495 (every
 * offset 0 here). inputs: the k data units, outputs: the p parity units. */
void orc_legacy_rs_encode(int k, int p, uint8_t* const* inputs, uint8_t* const* outputs, size_t len) {
  int gen[257];
  lg_generator(k, p, gen);
  const int nv = p + 1, nd = k + p;
  uint8_t** all = (uint8_t**)malloc(sizeof(uint8_t*) * (size_t)nd);
  for (int i = 0; i < p; i++) {
    memset(outputs[i], 0, len);
    all[i] = outputs[i];
  }
  for (int i = 0; i < k; i++) {
    all[p + i] = (uint8_t*)malloc(len ? len : 1);
    memcpy(all[p + i], inputs[i], len);
  }
  for (int i = nd - nv; i >= 0; i--)
    for (int j = 0; j < nv; j++)
      for (size_t idx = 0; idx < len; idx++) {
        const int ratio = lg_div[all[i + nv - 1][idx] & 0xFF][gen[nv - 1]];
        all[j + i][idx] = (uint8_t)((all[j + i][idx] & 0xFF) ^ lg_mul[ratio][gen[j]]);
      }
  for (int i = 0; i < k; i++) free(all[p + i]);
  free(all);
}

/* GaloisField.substitute(byte[][] p, int[] offsets, int len, byte[] q, int
 * offset, int x), util/GaloisField.java:422-434: a null unit counts as 0. */
static void lg_substitute(uint8_t* const* pu, int np, size_t len, uint8_t* q, int x) {
  int y = 1;
  for (int i = 0; i < np; i++) {
    const uint8_t* pi = pu[i];
    for (size_t idx = 0; idx < len; idx++) {
      const int pij = pi != NULL ? pi[idx] & 0xFF : 0;
      q[idx] = (uint8_t)(q[idx] ^ lg_mul[pij][y]);
    }
    y = lg_mul[x][y];
  }
}

/* GaloisField.solveVandermondeSystem(int[] x, byte[][] y, int[] outputOffsets,
 * int len, int dataLen), util/GaloisField.java:241-268. */
static void lg_solve_vandermonde(const int* x, uint8_t* const* y, int len, size_t data_len) {
  for (int i = 0; i < len - 1; i++)
    for (int j = len - 1; j > i; j--)
      for (size_t idx = 0; idx < data_len; idx++) y[j][idx] = (uint8_t)(y[j][idx] ^ lg_mul[x[i]][y[j - 1][idx] & 0xFF]);
  for (int i = len - 1; i >= 0; i--) {
    for (int j = i + 1; j < len; j++)
      for (size_t idx = 0; idx < data_len; idx++) y[j][idx] = (uint8_t)lg_div[y[j][idx] & 0xFF][x[j] ^ x[j - i - 1]];
    for (int j = i; j < len - 1; j++)
      for (size_t idx = 0; idx < data_len; idx++) y[j][idx] = (uint8_t)(y[j][idx] ^ y[j + 1][idx]);
  }
}

/* RSLegacyRawDecoder.decode(byte[][] inputs, int[] erasedIndexes, byte[][]
 * outputs), RSLegacyRawDecoder.java:71-83, in the caller's order: inputs =
 * the n units [data 0..k-1, parity 0..p-1], NULL for a unit not read (erased
 * or not to read); outputs[t] receives unit erased[t].
 *   adjustOrder, :222-253: units to [parity..., data...]; erased parity
 *     indexes first (- k), then erased data (+ p); outputs reordered alike;
 *   ByteArrayDecodingState, ByteArrayDecodingState.java:37-52, 95-115:
 *     at least k non-null inputs (else HadoopIllegalArgumentException: -1);
 *   doDecode(ByteArrayDecodingState), :111-165: outputs zeroed; every null
 *     unit (CoderUtil.getNullIndexes, CoderUtil.java:146-156) gets an output
 *     slot — the caller's buffer where it is an erased index (else -2: the
 *     "not fully corresponding" exception), a scratch buffer otherwise; more
 *     null units than p overflow the p-slot arrays (-3: Java's
 *     ArrayIndexOutOfBoundsException);
 *   doDecodeImpl, :98-109: errSignature[i] = primitivePower[null_i], slot i
 *     = substitute(units, primitivePower[i]) for i < #nulls, then the
 *     Vandermonde solve over the #nulls slots. */
int orc_legacy_rs_decode(int k, int p, uint8_t* const* inputs, const int* erased, int ne, uint8_t* const* outputs,
                         size_t len) {
  const int n = k + p;
  uint8_t* units[256];
  int erased2[256];
  uint8_t* outputs2[256];
  for (int i = 0; i < p; i++) units[i] = inputs[k + i]; /* adjustOrder :227-230 */
  for (int i = 0; i < k; i++) units[p + i] = inputs[i];
  int idx = 0, ned = 0, nep = 0;
  for (int i = 0; i < ne; i++)
    if (erased[i] >= k) {
      erased2[idx++] = erased[i] - k;
      nep++;
    }
  for (int i = 0; i < ne; i++)
    if (erased[i] < k) {
      erased2[idx++] = erased[i] + p;
      ned++;
    }
  for (int i = 0; i < nep; i++) outputs2[i] = outputs[ned + i]; /* :248-252 */
  for (int i = 0; i < ned; i++) outputs2[nep + i] = outputs[i];
  if (len == 0) return 0; /* RawErasureDecoder.decode :138-140 */
  int valid = 0;
  for (int i = 0; i < n; i++) valid += units[i] != NULL;
  if (valid < k) return -1;
  for (int t = 0; t < ne; t++) memset(outputs2[t], 0, len);
  int nulls[256], nn = 0;
  for (int i = 0; i < n; i++)
    if (units[i] == NULL) nulls[nn++] = i;
  uint8_t* adjusted[256] = {0};
  uint8_t* scratch[256] = {0};
  int rc = 0;
  for (int out_idx = 0, i = 0; i < ne && rc == 0; i++) {
    int found = 0;
    for (int j = 0; j < nn; j++)
      if (erased2[i] == nulls[j]) {
        found = 1;
        if (j >= p) {
          rc = -3;
          break;
        }
        memset(outputs2[out_idx], 0, len);
        adjusted[j] = outputs2[out_idx];
        out_idx++;
      }
    if (!found && rc == 0) rc = -2;
  }
  for (int buf = 0, i = 0; i < nn && rc == 0; i++)
    if (adjusted[i] == NULL) {
      if (i >= p || buf >= p) {
        rc = -3;
        break;
      }
      scratch[buf] = (uint8_t*)calloc(len, 1);
      adjusted[i] = scratch[buf++];
    }
  if (rc == 0) {
    int pp[256], sig[256];
    lg_primitive_power(k, p, pp);
    for (int i = 0; i < nn; i++) {
      sig[i] = pp[nulls[i]];
      lg_substitute(units, n, len, adjusted[i], pp[i]);
    }
    lg_solve_vandermonde(sig, adjusted, nn, len);
  }
  for (int i = 0; i < p; i++) free(scratch[i]);
  return rc;
}

/* ------------------------------------------------- nrs (ISA-L Cauchy RS) */

/* ISA-L gf_mul / gf_inv over 0x11D: the same field as GaloisField (285). */
static int isal_mul(int a, int b) { return mulTable[a][b]; }
static int isal_inv(int a) { return a == 0 ? 0 : divTable[1][a]; }

/* ISA-L gf_gen_cauchy1_matrix(a, m, k): identity on top, then a[i][j] = 1/(i ^ j). */
void orc_nrs_encode_matrix(int k, int p, uint8_t* a) {
  int m = k + p;
  memset(a, 0, (size_t)k * m);
  for (int i = 0; i < k; i++) a[k * i + i] = 1;
  uint8_t* q = &a[k * k];
  for (int i = k; i < m; i++)
    for (int j = 0; j < k; j++) *q++ = (uint8_t)isal_inv(i ^ j);
}

/* ISA-L gf_invert_matrix(in, out, n): Gauss-Jordan; returns -1 if singular. */
static int isal_invert(uint8_t* in, uint8_t* out, int n) {
  memset(out, 0, (size_t)n * n);
  for (int i = 0; i < n; i++) out[i * n + i] = 1;
  for (int i = 0; i < n; i++) {
    if (in[i * n + i] == 0) {
      int j;
      for (j = i + 1; j < n; j++)
        if (in[j * n + i]) break;
      if (j == n) return -1;
      for (int t = 0; t < n; t++) {
        uint8_t x = in[i * n + t]; in[i * n + t] = in[j * n + t]; in[j * n + t] = x;
        x = out[i * n + t]; out[i * n + t] = out[j * n + t]; out[j * n + t] = x;
      }
    }
    int piv = isal_inv(in[i * n + i]);
    for (int t = 0; t < n; t++) {
      in[i * n + t] = (uint8_t)isal_mul(in[i * n + t], piv);
      out[i * n + t] = (uint8_t)isal_mul(out[i * n + t], piv);
    }
    for (int j = 0; j < n; j++) {
      if (j == i) continue;
      int f = in[j * n + i];
      for (int t = 0; t < n; t++) {
        out[j * n + t] ^= (uint8_t)isal_mul(f, out[i * n + t]);
        in[j * n + t] ^= (uint8_t)isal_mul(f, in[i * n + t]);
      }
    }
  }
  return 0;
}

/* ISA-L ec_encode_data: dest[r][b] = XOR_j rows[r][j] * src[j][b]. */
static void isal_encode(size_t len, int ksrc, int rows, const uint8_t* mat, uint8_t* const* src, uint8_t* const* dst) {
  for (int r = 0; r < rows; r++)
    for (size_t b = 0; b < len; b++) {
      int s = 0;
      for (int j = 0; j < ksrc; j++) s ^= isal_mul(mat[r * ksrc + j], src[j][b]);
      dst[r][b] = (uint8_t)s;
    }
}

/* NativeReedSolomonCode.encodeBulk (NativeReedSolomonCode.java:55-88) ->
 * erasure_coder.c encode (:66-80): parity = Cauchy rows x data. */
void orc_nrs_encode_bulk(int k, int p, uint8_t* const* inputs, uint8_t* const* outputs, size_t len) {
  uint8_t* a = (uint8_t*)malloc((size_t)(k + p) * k);
  orc_nrs_encode_matrix(k, p, a);
  isal_encode(len, k, p, a + k * k, inputs, outputs);
  free(a);
}

static int cmp_int(const void* x, const void* y) { return *(const int*)x - *(const int*)y; }

/* NativeReedSolomonCode.decodeBulk (NativeReedSolomonCode.java:90-152): hops
 * [parity, data] -> Apache [data, parity]; every not-to-read location is NULL
 * and "erased" (sorted Apache order); erasure_coder.c processErasures
 * (:106-156) + generateDecodeMatrix (:189-230) + ec_encode_data; then
 * writeBufs[i] = the i-th decoded output (sorted Apache order), i < ne. */
int orc_nrs_decode_bulk(int k, int p, uint8_t* const* read_bufs, uint8_t* const* write_bufs, const int* erased,
                        int ne, const int* not_to_read, int nn, size_t len) {
  (void)erased;
  int m = k + p;
  uint8_t** in = (uint8_t**)calloc((size_t)m, sizeof(uint8_t*));
  for (int i = 0; i < p; i++) in[i + k] = read_bufs[i];
  for (int i = 0; i < k; i++) in[i] = read_bufs[i + p];
  int* mod = (int*)malloc(sizeof(int) * (size_t)(nn > 0 ? nn : 1));
  for (int i = 0; i < nn; i++) {
    int loc = not_to_read[i];
    if (loc < p) { in[loc + k] = NULL; mod[i] = loc + k; }
    else { in[loc - p] = NULL; mod[i] = loc - p; }
  }
  qsort(mod, (size_t)nn, sizeof(int), cmp_int);
  /* processErasures: decodeIndex = first k non-NULL inputs */
  int* decodeIndex = (int*)malloc(sizeof(int) * (size_t)k);
  int r = 0;
  for (int i = 0; i < k; i++, r++) {
    while (r < m && in[r] == NULL) r++;
    if (r >= m) { free(in); free(mod); free(decodeIndex); return -1; }
    decodeIndex[i] = r;
  }
  uint8_t* enc = (uint8_t*)malloc((size_t)m * k);
  orc_nrs_encode_matrix(k, p, enc);
  uint8_t* tmp = (uint8_t*)malloc((size_t)k * k);
  uint8_t* inv = (uint8_t*)malloc((size_t)k * k);
  for (int i = 0; i < k; i++)
    for (int j = 0; j < k; j++) tmp[k * i + j] = enc[k * decodeIndex[i] + j];
  int st = isal_invert(tmp, inv, k);
  int nErasedData = 0;
  for (int i = 0; i < nn; i++) if (mod[i] < k) nErasedData++;
  uint8_t* dec = (uint8_t*)calloc((size_t)(nn > 0 ? nn : 1) * k, 1);
  for (int i = 0; i < nErasedData; i++)
    for (int j = 0; j < k; j++) dec[k * i + j] = inv[k * mod[i] + j];
  for (int q = nErasedData; q < nn; q++)
    for (int i = 0; i < k; i++) {
      int s = 0;
      for (int j = 0; j < k; j++) s ^= isal_mul(inv[j * k + i], enc[k * mod[q] + j]);
      dec[k * q + i] = (uint8_t)s;
    }
  uint8_t** real = (uint8_t**)malloc(sizeof(uint8_t*) * (size_t)k);
  for (int i = 0; i < k; i++) real[i] = in[decodeIndex[i]];
  uint8_t** outs = (uint8_t**)malloc(sizeof(uint8_t*) * (size_t)(nn > 0 ? nn : 1));
  for (int i = 0; i < nn; i++) outs[i] = (uint8_t*)calloc(len ? len : 1, 1);
  isal_encode(len, k, nn, dec, real, outs);
  for (int i = 0; i < ne && i < nn; i++) memcpy(write_bufs[i], outs[i], len);
  for (int i = 0; i < nn; i++) free(outs[i]);
  free(outs); free(real); free(dec); free(inv); free(tmp); free(enc); free(decodeIndex); free(mod); free(in);
  return st;
}

/* ------------------------------------------- SimpleRegeneratingCode (src) */

typedef struct {
  int k, p, s, r, d, n;
  int gen[256];
  int ngen;
  int pp[256];       /* primitivePower */
  int* groups[256];  /* groupsTable */
  int gsize[256];
} src_code;

static int src_group(const src_code* c, int loc) { /* getSRCGroup, :415-426 */
  if (0 <= loc && loc < c->s) return loc;
  if (c->s <= loc && loc < c->k + c->p) return (loc - c->s) / c->d;
  return -1;
}

static int src_neighbors(const src_code* c, int loc, int* out) { /* getSRCGroupNeighbors, :371-409 */
  int limit = c->k + c->p, m = 0;
  int group = src_group(c, loc);
  if (group < c->s) {
    if (group != loc) out[m++] = group;
    for (int i = c->s + group * c->d; i < c->s + (group + 1) * c->d; i++)
      if (i != loc) out[m++] = i;
  } else {
    for (int i = 0; i < c->s; i++) out[m++] = i;
    for (int i = c->s + group * c->d; i < limit; i++)
      if (i != loc) out[m++] = i;
  }
  return m;
}

int orc_src_params(int k, int p, int s_in, int* s, int* r, int* d) { /* init, :70-114 */
  int ss = s_in, rr = p - s_in;
  int dd = (k + rr + ss) / (ss + 1); /* ceil((k + rr) / (ss + 1)) */
  dd = (int)((k + rr + ss) / (ss + 1));
  while (dd * ss >= k + rr) {
    ss--;
    rr++;
    dd = (k + rr + ss) / (ss + 1);
  }
  *s = ss;
  *r = rr;
  *d = dd;
  return 0;
}

static void src_init(src_code* c, int k, int p, int s_in) {
  c->k = k;
  c->p = p;
  c->n = k + p;
  orc_src_params(k, p, s_in, &c->s, &c->r, &c->d);
  for (int i = 0; i < k + c->r; i++) c->pp[i] = orc_gf_power(2, i);
  int gen[256] = {1}, ng = 1, poly[2], tmp[256];
  for (int i = 0; i < c->r; i++) {
    poly[0] = c->pp[i];
    poly[1] = 1;
    orc_gf_poly_mul(gen, ng, poly, 2, tmp);
    ng += 1;
    memcpy(gen, tmp, sizeof(int) * (size_t)ng);
  }
  memcpy(c->gen, gen, sizeof(int) * (size_t)ng);
  c->ngen = ng;
  for (int i = 0; i < c->n; i++) {
    c->groups[i] = (int*)malloc(sizeof(int) * (size_t)c->n);
    c->gsize[i] = src_neighbors(c, i, c->groups[i]);
  }
}

static void src_free(src_code* c) {
  for (int i = 0; i < c->n; i++) free(c->groups[i]);
}

static void src_encode(const src_code* c, const int* message, int* parity) { /* encode, :116-157 */
  int buf[512];
  for (int i = 0; i < c->r; i++) buf[i] = 0;
  for (int i = 0; i < c->k; i++) buf[i + c->r] = message[i];
  orc_gf_remainder(buf, c->r + c->k, c->gen, c->ngen);
  for (int i = 0; i < c->r; i++) parity[i + c->s] = buf[i];
  for (int i = 0; i < c->k; i++) buf[i + c->r] = message[i];
  for (int i = 0; i < c->s; i++) {
    parity[i] = 0;
    for (int j = c->d * i; j < c->d * (i + 1); j++) parity[i] = buf[j] ^ parity[i];
  }
}

void orc_src_encode(int k, int p, int s_in, const int* message, int* parity) {
  src_code c;
  src_init(&c, k, p, s_in);
  src_encode(&c, message, parity);
  src_free(&c);
}

/* decodeReedSolomon, :162-182; -1 if more erasures than errSignature holds */
static int src_decode_rs(const src_code* c, int* data, const int* erased, int ne, int* values) {
  if (ne == 0) return 0;
  if (ne > c->r) return -1;
  int sig[256];
  for (int i = 0; i < ne; i++) data[erased[i]] = 0;
  for (int i = 0; i < ne; i++) {
    sig[i] = c->pp[erased[i]];
    values[i] = orc_gf_substitute(data, c->r + c->k, c->pp[i]);
  }
  orc_gf_solve_vandermonde(sig, values, ne);
  return 0;
}

static int src_conflict(const src_code* c, const int* locs, int n) { /* groupConflict, :432-453 */
  int groups[257] = {0};
  for (int i = 0; i < n; i++)
    if (locs[i] < c->s) {
      groups[c->s] = 1;
      break;
    }
  for (int i = 0; i < n; i++)
    if (groups[src_group(c, locs[i])]++ > 0) return 1;
  return 0;
}

static int src_decode5(const src_code* c, int* data, const int* erased, int ne, int* values, const int* to_read,
                       int nr, const int* ntr, int nn) { /* decode 5-arg, :194-277 */
  if (ne == 1) {
    values[0] = 0;
    for (int i = 0; i < nr; i++) values[0] = data[to_read[i]] ^ values[0];
    return 0;
  }
  if (!src_conflict(c, erased, ne)) {
    for (int i = 0; i < ne; i++) {
      int one = erased[i], v = 0;
      src_decode5(c, data, &one, 1, &v, c->groups[erased[i]], c->gsize[erased[i]], NULL, 0);
      values[i] = v;
    }
    return 0;
  }
  int dataRS[512], eRS[256], vRS[256], m = 0;
  for (int i = 0; i < c->r + c->k; i++) dataRS[i] = data[i + c->s];
  for (int i = 0; i < nn; i++)
    if (ntr[i] >= c->s) eRS[m++] = ntr[i] - c->s;
  if (src_decode_rs(c, dataRS, eRS, m, vRS) != 0) return -1;
  for (int i = 0; i < m; i++) data[c->s + eRS[i]] = vRS[i];
  for (int i = 0; i < ne; i++)
    if (erased[i] < c->s) {
      int par = erased[i];
      data[par] = 0;
      for (int j = 0; j < c->gsize[par]; j++) data[par] = data[c->groups[par][j]] ^ data[par];
    }
  for (int i = 0; i < ne; i++) values[i] = data[erased[i]];
  return 0;
}

int orc_src_decode5(int k, int p, int s_in, int* data, const int* erased, int ne, int* values, const int* to_read,
                    int nr, const int* ntr, int nn) {
  src_code c;
  src_init(&c, k, p, s_in);
  int st = src_decode5(&c, data, erased, ne, values, to_read, nr, ntr, nn);
  src_free(&c);
  return st;
}

int orc_src_locations_to_read(int k, int p, int s_in, const int* erased, int ne, int* out) { /* :300-366 */
  src_code c;
  src_init(&c, k, p, s_in);
  int m = 0;
  if (ne == 1) {
    for (int i = 0; i < c.gsize[erased[0]]; i++) out[m++] = c.groups[erased[0]][i];
  } else if (!src_conflict(&c, erased, ne)) {
    for (int e = 0; e < ne; e++)
      for (int i = 0; i < c.gsize[erased[e]]; i++) {
        int loc = c.groups[erased[e]][i], dup = 0;
        for (int j = 0; j < m; j++) dup |= out[j] == loc;
        if (!dup) out[m++] = loc;
      }
  } else {
    for (int loc = c.s; loc < c.n; loc++) {
      int bad = 0;
      for (int i = 0; i < ne; i++) bad |= erased[i] == loc;
      if (!bad) {
        out[m++] = loc;
        if (m == k) break;
      }
    }
    if (m != k) m = -1;
  }
  src_free(&c);
  return m;
}

void orc_src_encode_bulk(int k, int p, int s_in, uint8_t* const* inputs, uint8_t* const* outputs, size_t len) {
  src_code c; /* ErasureCode.encodeBulk, :136-156 */
  src_init(&c, k, p, s_in);
  int data[256], code[256];
  for (size_t j = 0; j < len; j++) {
    for (int i = 0; i < p; i++) code[i] = 0;
    for (int i = 0; i < k; i++) data[i] = inputs[i][j];
    src_encode(&c, data, code);
    for (int i = 0; i < p; i++) outputs[i][j] = (uint8_t)code[i];
  }
  src_free(&c);
}

int orc_src_decode_bulk(int k, int p, int s_in, uint8_t* const* read_bufs, uint8_t* const* write_bufs,
                        const int* erased, int ne, const int* to_read, int nr, const int* ntr, int nn, size_t len) {
  src_code c; /* ErasureCode.decodeBulk, :162-181 */
  src_init(&c, k, p, s_in);
  int in[256], out[256], st = 0;
  for (size_t idx = 0; idx < len && st == 0; idx++) {
    for (int i = 0; i < ne; i++) out[i] = 0;
    for (int i = 0; i < k + p; i++) in[i] = read_bufs[i] ? read_bufs[i][idx] : 0;
    st = src_decode5(&c, in, erased, ne, out, to_read, nr, ntr, nn);
    for (int i = 0; i < ne; i++) write_bufs[i][idx] = (uint8_t)out[i];
  }
  src_free(&c);
  return st;
}
