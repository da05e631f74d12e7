/*
 * TEST INFRASTRUCTURE ONLY — the CPU oracle. Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library, and only as the
 * checker / the timed CPU baseline. The product (lambdafs_amd/libhrs.so)
 * never links or calls it.
 *
 * A C restatement of the reference's Java algorithms, loop for loop:
 *   GaloisField.java      (hops-erasure-coding/src/main/java/io/hops/erasure_coding/)
 *   ReedSolomonCode.java  (same directory)
 *   ErasureCode.java      (hadoop-hdfs/src/main/java/io/hops/erasure_coding/)
 * Parity pinning: the reference ships no golden vectors and cannot run here
 * (no JDK); see oracle/README.md for how this restatement is pinned.
 */
#ifndef RS_ORACLE_H_
#define RS_ORACLE_H_
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* GaloisField(256, 285) tables and scalar ops, GaloisField.java:76-204. */
int orc_gf_mul(int x, int y);
int orc_gf_div(int x, int y);
int orc_gf_power(int x, int n);
int orc_gf_log(int x);
int orc_gf_pow_table(int i);

/* Polynomial helpers, GaloisField.java:286-320, :351-383. Arrays index = power. */
void orc_gf_poly_mul(const int* p, int np, const int* q, int nq, int* out /* np+nq-1 */);
void orc_gf_poly_add(const int* p, int np, const int* q, int nq, int* out /* max(np,nq) */);
void orc_gf_remainder(int* dividend, int nd, const int* divisor, int nv);
int orc_gf_substitute(const int* p, int np, int x);
void orc_gf_solve_vandermonde(const int* x, int* y, int len);
void orc_gf_gaussian_elimination(int* matrix, int height, int width);

/* ReedSolomonCode.init generating polynomial, ReedSolomonCode.java:56-82.
 * gen has p+1 entries. Returns 0, or -1 if k+p >= 256. */
int orc_rs_generator(int k, int p, int* gen);

/* ReedSolomonCode.encode(int[] message, int[] parity), :84-97. */
void orc_rs_encode(int k, int p, const int* message, int* parity);

/* ReedSolomonCode.encodeBulk(byte[][] inputs, byte[][] outputs), :103-125,
 * via the bulk GaloisField.remainder, GaloisField.java:326-338.
 * Like the Java, this ZEROES the input rows. */
void orc_rs_encode_bulk(int k, int p, uint8_t* const* inputs, uint8_t* const* outputs, size_t len);

/* ReedSolomonCode.decode 3-arg, :127-142 (modifies data at erased). */
void orc_rs_decode3(int k, int p, int* data, const int* erased, int ne, int* values);

/* ReedSolomonCode.decode 5-arg, :144-166. */
void orc_rs_decode5(int k, int p, int* data, const int* erased, int ne, int* values, const int* to_read, int nr,
                    const int* not_to_read, int nn);

/* ReedSolomonCode.decodeBulk 5-arg, :191-211 (per byte). */
void orc_rs_decode_bulk5(int k, int p, uint8_t* const* read_bufs, uint8_t* const* write_bufs, const int* erased,
                         int ne, const int* to_read, int nr, const int* not_to_read, int nn, size_t len);

/* ReedSolomonCode.decodeBulk 3-arg, :168-185 (bulk syndromes + bulk Vandermonde). */
void orc_rs_decode_bulk3(int k, int p, uint8_t* const* read_bufs, uint8_t* const* write_bufs, const int* erased,
                         int ne, size_t len);

/* ErasureCode.locationsToReadForDecode, ErasureCode.java:89-113. Returns the
 * count written (k on success, fewer => TooManyErasedLocations). */
int orc_locations_to_read(int k, int p, const int* erased, int ne, int* out);

/* ReedSolomonCode.computeErrorLocations, :243-287. Returns 1 if resolved;
 * writes up to n locations (ascending) and their count. */
int orc_rs_compute_error_locations(int k, int p, int* data, int* locations, int* nloc);

/* XORCode (hops-erasure-coding/.../XORCode.java): encode :54-61, decode :63-83,
 * encodeBulk :99-113, decodeBulk 3-arg :115-138 (5-arg delegates, :140-145). */
void orc_xor_encode(int k, const int* message, int* parity);
void orc_xor_decode(int k, const int* data, const int* erased, int ne, int* values);
void orc_xor_encode_bulk(int k, uint8_t* const* inputs, uint8_t* output, size_t len);
void orc_xor_decode_bulk(int k, uint8_t* const* read_bufs, uint8_t* output, int erased, size_t len);

/* NativeReedSolomonCode (the `nrs` codec, hops-erasure-coding/.../NativeReedSolomonCode.java)
 * over libhadoop's ISA-L shim (hadoop-common/src/main/native/src/org/apache/hadoop/io/
 * erasurecode/erasure_coder.c) and ISA-L (absent here, version unpinned: restated from its
 * published gf_gen_cauchy1_matrix / gf_invert_matrix / ec_encode_data definitions; checked
 * against orc_apache_* below, the restated Java port of ISA-L the reference itself ships).
 * Rows in hops order [parity, data]; read_bufs entries may be NULL (not read). */
void orc_nrs_encode_matrix(int k, int p, uint8_t* a /* (k+p) x k, ISA-L layout */);
void orc_nrs_encode_bulk(int k, int p, uint8_t* const* inputs, uint8_t* const* outputs, size_t len);
int orc_nrs_decode_bulk(int k, int p, uint8_t* const* read_bufs, uint8_t* const* write_bufs, const int* erased,
                        int ne, const int* not_to_read, int nn, size_t len);

/* The reference's pure-Java port of ISA-L's RS coder (hadoop-common/src/main/java/org/apache/
 * hadoop/io/erasurecode/rawcoder/: RSRawEncoder.java, RSRawDecoder.java, util/RSUtil.java,
 * util/GF256.java), restated loop for loop. The reference's own interop tests
 * (TestRSRawCoderInteroperable1/2: Java encode + native decode and the reverse) hold it equal to
 * the native ISA-L coder behind the `nrs` codec, so it pins orc_nrs_* to reference source.
 * Apache unit order [data 0..k-1, parity k..k+p-1]. */
int orc_apache_gf_base(int i);      /* GF256.GF_BASE[i], regenerated; tests pin it to the literal */
int orc_apache_gf_log_base(int i);  /* GF256.GF_LOG_BASE[i] (log(1) stored as 0xff) */
int orc_apache_gf_mul(int a, int b);
int orc_apache_gf_inv(int a);
void orc_apache_gen_cauchy(uint8_t* a, int m, int k);  /* RSUtil.genCauchyMatrix, m x k */
void orc_apache_rs_encode(int k, int p, uint8_t* const* inputs, uint8_t* const* outputs, size_t len);
/* RSRawDecoder.doDecode(ByteArrayDecodingState): inputs[k + p] with NULL for units not read
 * (erased included), erased = the erased unit indexes (ascending, as the hops wrapper passes
 * them), outputs[ne]. Returns 0, or -1 if fewer than k inputs or the matrix is singular. */
int orc_apache_rs_decode(int k, int p, uint8_t* const* inputs, const int* erased, int ne, uint8_t* const* outputs,
                         size_t len);

/* SimpleRegeneratingCode (the `src` codec, SimpleRegeneratingCode.java:28-482),
 * with ErasureCode's default bulk loops (ErasureCode.java:136-181). s_in is
 * the codec's parity_length_src; the init adjustment loop (:70-90) may lower it.
 * Locations: [SRC parities 0..s-1, RS parities s..p-1, data p..p+k-1]. */
int orc_src_params(int k, int p, int s_in, int* s, int* r, int* d);
void orc_src_encode(int k, int p, int s_in, const int* message, int* parity);
/* 5-arg decode of one symbol column; returns -1 where the Java would throw
 * (ArrayIndexOutOfBounds of errSignature). data is modified as in the Java. */
int orc_src_decode5(int k, int p, int s_in, int* data, const int* erased, int ne, int* values, const int* to_read,
                    int nr, const int* ntr, int nn);
/* locationsToReadForDecode; returns the count written to out (capacity k+p)
 * or -1 for TooManyErasedLocations. */
int orc_src_locations_to_read(int k, int p, int s_in, const int* erased, int ne, int* out);
void orc_src_encode_bulk(int k, int p, int s_in, uint8_t* const* inputs, uint8_t* const* outputs, size_t len);
int orc_src_decode_bulk(int k, int p, int s_in, uint8_t* const* read_bufs, uint8_t* const* write_bufs,
                        const int* erased, int ne, const int* to_read, int nr, const int* ntr, int nn, size_t len);

/* hadoop-common's legacy pure-Java RS coder (io/erasurecode/rawcoder/
 * RSLegacyRawEncoder.java, RSLegacyRawDecoder.java, util/GaloisField.java,
 * util/RSUtil.java): the same polynomial code as hops' ReedSolomonCode, in
 * the Apache unit order [data..., parity...]. Decode: inputs NULL for units
 * not read; outputs[t] = unit erased[t]; 0, or -1 (fewer than k inputs), -2
 * (an erased unit is not NULL), -3 (more NULL units than p). */
int orc_legacy_generator(int k, int p, int* gen_out);
void orc_legacy_rs_encode(int k, int p, uint8_t* const* inputs, uint8_t* const* outputs, size_t len);
int orc_legacy_rs_decode(int k, int p, uint8_t* const* inputs, const int* erased, int ne, uint8_t* const* outputs,
                         size_t len);

#ifdef __cplusplus
}
#endif

#endif
