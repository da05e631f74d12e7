/*
 * hrs.h — C ABI of the MI355X-native Reed-Solomon engine (libhrs.so).
 *
 * This is the drop-in boundary behind the hops codec plugin surface
 * `io.hops.erasure_coding.ErasureCode` (hadoop-hdfs-project/hadoop-hdfs/src/
 * main/java/io/hops/erasure_coding/ErasureCode.java:25-182). A JNI shim
 * (lambdafs_amd/jni/) maps the Java class
 * `io.hops.erasure_coding.HipReedSolomonCode extends ErasureCode` onto these
 * entry points exactly as the existing native precedent
 * `NativeReedSolomonCode` maps onto libhadoop's ISA-L shim
 * (hops-erasure-coding/.../NativeReedSolomonCode.java:55-152 ->
 *  hadoop-common/src/main/native/src/org/apache/hadoop/io/erasurecode/
 *  jni_rs_encoder.c:45-63, jni_rs_decoder.c:35-77).
 *
 * Semantics are those of the Java `rs` codec, `ReedSolomonCode`
 * (hops-erasure-coding/src/main/java/io/hops/erasure_coding/
 * ReedSolomonCode.java), bit-exact:
 *   - GF(2^8), primitive polynomial 0x11D, alpha = 2;
 *   - stripe locations in hops order: [0, p) parity, [p, p+k) data;
 *   - encode  = ReedSolomonCode.encodeBulk   (ReedSolomonCode.java:103-125);
 *   - decode  = ReedSolomonCode.decodeBulk 5-arg (ReedSolomonCode.java:191-211);
 *   - decode3 = ReedSolomonCode.decodeBulk 3-arg (ReedSolomonCode.java:168-185).
 *
 * Conventions: no JNI or torch types; plain pointers and sizes. Every
 * function returns HRS_OK (0) on success and a nonzero hrs_status otherwise;
 * the JNI shim turns a nonzero status into java.io.IOException
 * (HRS_ETOOMANY into io.hops.erasure_coding.TooManyErasedLocations), as
 * jni_rs_encoder.c:51 THROWs. A handle is not thread-safe (like the Java
 * ReedSolomonCode, whose scratch arrays are per instance,
 * ReedSolomonCode.java:36-38); distinct handles are fully concurrent.
 */
#ifndef HRS_H_
#define HRS_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int hrs_status;
enum {
  HRS_OK = 0,
  HRS_EINVAL = 1,    /* bad argument (IllegalArgumentException / assert in Java) */
  HRS_ETOOMANY = 2,  /* ErasureCode.java:105-111 TooManyErasedLocations */
  HRS_EDEVICE = 3,   /* HIP runtime failure (no GPU, launch or copy error) */
  HRS_ENOMEM = 4,    /* device or pinned-host allocation failed */
  HRS_EALIGN = 5     /* device-batch rows not 16-byte aligned (see hrs_*_dev) */
};

typedef struct hrs_codec hrs_codec;

/* Code families behind the same boundary (hops codec table,
 * hadoop-hdfs/src/main/resources/erasure-coding-default.xml:13-56). */
enum {
  HRS_CODE_RS = 0,  /* "rs":  io.hops.erasure_coding.ReedSolomonCode (ReedSolomonCode.java) */
  HRS_CODE_XOR = 1, /* "xor": io.hops.erasure_coding.XORCode (XORCode.java), parity_size == 1 */
  HRS_CODE_SRC = 3, /* "src": io.hops.erasure_coding.SimpleRegeneratingCode (SimpleRegeneratingCode.java):
                     * RS(k, r) plus s local XOR parities; create with hrs_create_src.
                     * Locations [SRC parities 0..s-1, RS parities s..p-1, data p..k+p-1].
                     * Variable-length locationsToReadForDecode (hrs_locations_to_read_list);
                     * a one-erasure decode XORs the locations to read (device calls: every
                     * location outside not_to_read); no 3-arg decode. */
  HRS_CODE_NRS = 2  /* "nrs": io.hops.erasure_coding.NativeReedSolomonCode (NativeReedSolomonCode.java)
                     * over libhadoop's ISA-L shim (erasure_coder.c): Cauchy RS, Apache
                     * [data, parity] coding order behind the hops [parity, data] locations.
                     * Decode outputs follow the Java's ordering: output t is the t-th
                     * not-to-read location in Apache order (needs num_erased <= num_not_to_read
                     * <= parity_size). No 3-arg decode (hrs_decode3 -> HRS_EINVAL). The
                     * reference's native limits (k <= 10, k + p <= 14) are lifted. */
};

#define HRS_DEVICE_NONE (-2)

typedef struct hrs_opts {
  int device;         /* HIP device ordinal; -1 = current device; HRS_DEVICE_NONE =
                         host-only handle (matrix/location queries; coding calls
                         fail with HRS_EDEVICE) */
  int reserved[7];    /* must be zero */
} hrs_opts;

/* ---- lifecycle (ReedSolomonCode() + init(Codec), ReedSolomonCode.java:45-82) ---- */

/* Builds the generator polynomial and encode matrix for RS(stripe_size,
 * parity_size). Requires stripe_size >= 1, parity_size >= 1 and
 * stripe_size + parity_size < 256 (ReedSolomonCode.java:57). opts may be NULL. */
hrs_status hrs_create(int stripe_size, int parity_size, const hrs_opts* opts, hrs_codec** out);
/* Same for any code family: HRS_CODE_RS (== hrs_create), HRS_CODE_XOR
 * (XORCode.init asserts parity_size == 1, XORCode.java:46-51) or HRS_CODE_NRS
 * (NativeReedSolomonCode.init, NativeReedSolomonCode.java:44-51). */
hrs_status hrs_create_code(int code, int stripe_size, int parity_size, const hrs_opts* opts,
                           hrs_codec** out);
int hrs_code_kind(const hrs_codec* codec);
/* SimpleRegeneratingCode.init(Codec) (SimpleRegeneratingCode.java:52-114):
 * src_parity_size = the codec's "parity_length_src" (the adjustment loop of
 * init may lower it; hrs_src_layout reports what it settled on). */
hrs_status hrs_create_src(int stripe_size, int parity_size, int src_parity_size, const hrs_opts* opts,
                          hrs_codec** out);
/* SRC layout after init: stored SRC parities s, RS parities r = p - s, and
 * the group degree d (locations per stored SRC group). */
hrs_status hrs_src_layout(const hrs_codec* codec, int* src_parities, int* rs_parities, int* group_degree);
void hrs_destroy(hrs_codec* codec);
/* Last error message of this handle ("" if none); handle may be NULL for create errors. */
const char* hrs_last_error(const hrs_codec* codec);
/* Name of the main kernel the handle's latest coding call launched, as
 * rocprofv3 prints it without its namespace and parameters (e.g.
 * "encode_static_kernel<10, 4>"); "" before any device work. Lets a
 * benchmark attach the PMC traffic of the kernel it actually ran. */
const char* hrs_last_kernel(const hrs_codec* codec);
/* How the handle's latest synchronous host-buffer call (hrs_encode, hrs_decode,
 * hrs_decode3, hrs_*_crc) or host batch (hrs_*_batch_host) moved its bytes:
 * "pinned" (rows or batch in memory the runtime allocated pinned —
 * hipHostMalloc, torch pin_memory —: the zero-copy kernel in place),
 * "staged" (any other host memory, pageable or registered by the caller with
 * hipHostRegister, copied through the library's pinned staging, the zero-copy
 * kernel on the staging; the default), "copy_engine" (staging, H2D, kernel,
 * D2H), or "" before any such call. The GPU never reads or writes
 * caller-registered pageable memory in place: registration does not pin its
 * pages ("Platform constraint"). Diagnostic, like
 * hrs_last_kernel. */
const char* hrs_last_host_path(const hrs_codec* codec);
const char* hrs_version(void);

/* ---- device set (SURVEY §5 "engine env/config for device set"; §8(e)) ----
 * The reference creates one codec per Encoder / Decoder through
 * Codec.createErasureCode -> ReflectionUtils.newInstance(class, conf) -> init
 * (hadoop-hdfs/.../io/hops/erasure_coding/Codec.java:200-213). A binding picks
 * the GPU of each handle with hrs_opts.device (the Java classes: round robin
 * over the conf key hdfs.raid.hip.devices). */

/* HIP devices visible to this process (HIP_VISIBLE_DEVICES applies); 0 if the
 * HIP runtime finds none. Valid ordinals for hrs_opts.device are [0, count). */
int hrs_device_count(void);
/* Device ordinal a handle runs on (HRS_DEVICE_NONE for a host-only handle,
 * -1 for NULL). */
int hrs_codec_device(const hrs_codec* codec);

/* ErasureCode.stripeSize()/paritySize()/symbolSize() (ReedSolomonCode.java:213-226). */
int hrs_stripe_size(const hrs_codec* codec);
int hrs_parity_size(const hrs_codec* codec);
int hrs_symbol_size(const hrs_codec* codec);

/* ---- host helpers (no device work) ---- */

/* locationsToReadForDecode as a list of variable length, for every code
 * family (SRC returns a local group; the others exactly stripe_size
 * locations, as hrs_locations_to_read): to_read has room for k + p entries,
 * *num_to_read receives the count. SimpleRegeneratingCode.java:300-366,
 * ErasureCode.java:89-113. */
hrs_status hrs_locations_to_read_list(const hrs_codec* codec, const int* erased, int num_erased, int* to_read,
                                      int* num_to_read);

/* ErasureCode.locationsToReadForDecode (ErasureCode.java:89-113): writes the
 * k = stripe_size highest-index locations not in `erased` to to_read, in
 * descending order, as the Java list is built. HRS_ETOOMANY if fewer than k
 * survive. */
hrs_status hrs_locations_to_read(const hrs_codec* codec, const int* erased, int num_erased,
                                 int* to_read);

/* p x k encode matrix G (row-major): parity_r = XOR_c G[r][c] * data_c.
 * XOR code: one row of ones (XORCode.encodeBulk, XORCode.java:99-113). */
hrs_status hrs_encode_matrix(const hrs_codec* codec, uint8_t* g);

/* num_erased x n decode matrix D (row-major, n = k + p, hops order):
 * out_i = XOR_l D[i][l] * in_l.
 * zero_not_to_read = 1: decodeBulk 5-arg semantics (ReedSolomonCode.java:144-166,
 *   191-211): locations in not_to_read are zeroed, m = num_not_to_read
 *   syndromes, erased locations absent from not_to_read decode to 0.
 * zero_not_to_read = 0: decodeBulk 3-arg semantics (ReedSolomonCode.java:168-185):
 *   not_to_read is the erased list itself, nothing is zeroed.
 * RS: D is the reference decode run on unit vectors, so it reproduces the
 * Java on every list the Java accepts: repeated locations (a division by zero
 * in solveVandermondeSystem yields 0, GaloisField.java:107-118) and, in the
 * 5-arg form, erased locations of any value (only compared with not_to_read).
 * not_to_read locations (and 3-arg erased ones) must be in [0, n). */
hrs_status hrs_decode_matrix(const hrs_codec* codec, const int* erased, int num_erased,
                             const int* not_to_read, int num_not_to_read, int zero_not_to_read,
                             uint8_t* d);

/* ---- synchronous host-buffer calls: the JNI path (GetPrimitiveArrayCritical rows) ---- */

/* ReedSolomonCode.encodeBulk(byte[][] inputs, byte[][] outputs):
 * inputs[k] rows and outputs[p] rows, each `len` bytes, host memory.
 * Outputs are fully overwritten. Unlike the Java method (whose bulk
 * remainder zeroes `inputs`, GaloisField.java:326-338) inputs are left
 * untouched; the Java/Python shims restore that side effect when asked. */
hrs_status hrs_encode(hrs_codec* codec, const uint8_t* const* inputs, uint8_t* const* outputs,
                      size_t len);

/* XOR code: decode needs exactly one erased location; the output is the XOR
 * of every other row (XORCode.decodeBulk, XORCode.java:115-145; NULL rows
 * count as the zeros the reference reads there). */

/* ReedSolomonCode.decodeBulk(readBufs, writeBufs, erased, toRead, notToRead)
 * (ReedSolomonCode.java:191-211): read_bufs[n] in hops order (a row may be
 * NULL when its location is in not_to_read — the reference feeds zeros
 * there, StripeReader.java:111-120); write_bufs[num_erased], row i = value at
 * erased[i]. to_read is accepted for interface parity; like the Java code the
 * result depends only on erased and not_to_read. */
hrs_status hrs_decode(hrs_codec* codec, const uint8_t* const* read_bufs, uint8_t* const* write_bufs,
                      const int* erased, int num_erased, const int* to_read, int num_to_read,
                      const int* not_to_read, int num_not_to_read, size_t len);

/* ReedSolomonCode.decodeBulk(readBufs, writeBufs, erasedLocation)
 * (ReedSolomonCode.java:168-185): all n rows are read as given. */
hrs_status hrs_decode3(hrs_codec* codec, const uint8_t* const* read_bufs, uint8_t* const* write_bufs,
                       const int* erased, int num_erased, size_t len);

/* hrs_encode plus the block checksums Encoder.encodeStripe keeps when
 * computeBlockChecksum is set (Encoder.java:408-450: sourceChecksums[i].update
 * over readBufs[i], parityChecksums[i].update over writeBufs[i]):
 * crc_out[r] = java.util.zip.CRC32 continued from crc_in[r] over input row r
 * (r < k) or output row r - k (r >= k). crc_in / crc_out are HOST arrays of
 * k + p uint32 (crc_in NULL = fresh CRC32 objects; crc_out may alias crc_in).
 * Each cell is checksummed on the GPU as it passes through, in the same
 * pipelined copy as the encode; no second host pass. */
hrs_status hrs_encode_crc(hrs_codec* codec, const uint8_t* const* inputs, uint8_t* const* outputs,
                          size_t len, const uint32_t* crc_in, uint32_t* crc_out);

/* hrs_decode plus the CRC-32 of every repaired row (Decoder.java:222-229 and
 * :645-655 compare it with the block checksum the NameNode holds):
 * crc_out[i] = CRC32 continued from crc_in[i] over write_bufs[i]. HOST arrays
 * of num_erased uint32 (crc_in NULL = fresh). */
hrs_status hrs_decode_crc(hrs_codec* codec, const uint8_t* const* read_bufs, uint8_t* const* write_bufs,
                          const int* erased, int num_erased, const int* to_read, int num_to_read,
                          const int* not_to_read, int num_not_to_read, size_t len,
                          const uint32_t* crc_in, uint32_t* crc_out);

/* ---- asynchronous host-buffer calls: successive rounds overlap ----
 * An Encoder / Decoder round (Encoder.java:421-453, Decoder.java:280-372)
 * split in two. *_submit copies the caller's rows into a free slot's pinned
 * staging — the rows may be reused or freed as soon as it returns (the JNI
 * shim pins Java arrays only for the call) — queues H2D -> kernel -> D2H on
 * the slot's stream and returns a ticket; hrs_collect waits for that
 * operation and copies its output rows out. While round r runs on the GPU the
 * caller reads round r + 1 and submits it. A handle holds up to 4 uncollected
 * operations (more -> HRS_EINVAL); tickets may be collected in any order.
 * checksums = 1 adds the block CRC-32s of hrs_encode_crc / hrs_decode_crc:
 * the running values are chained at collect time (rounds are collected in
 * order), so they need not be known when the round is submitted. */
hrs_status hrs_encode_submit(hrs_codec* codec, const uint8_t* const* inputs, size_t len, int checksums,
                             uint64_t* ticket);
hrs_status hrs_decode_submit(hrs_codec* codec, const uint8_t* const* read_bufs, const int* erased,
                             int num_erased, const int* to_read, int num_to_read, const int* not_to_read,
                             int num_not_to_read, size_t len, int checksums, uint64_t* ticket);
/* outputs: p rows (encode) or num_erased rows (decode) of `len` bytes.
 * crc_io (checksummed operations only): k + p (sources, then parities) or
 * num_erased running java.util.zip.CRC32 values (0 = a fresh CRC32), each
 * continued over this operation's cell (CRC32.update chaining). */
hrs_status hrs_collect(hrs_codec* codec, uint64_t ticket, uint8_t* const* outputs, uint32_t* crc_io);
/* Waits until the operation's H2D, kernel and D2H have completed, without
 * copying anything out or releasing it (hrs_collect still must be called;
 * it then returns without blocking). Lets a binding wait before it pins the
 * caller's output rows: the JNI shim calls it outside any
 * GetPrimitiveArrayCritical region. HRS_EINVAL for an unknown ticket. */
hrs_status hrs_wait(hrs_codec* codec, uint64_t ticket);
/* Drops an uncollected operation without copying anything out: its slot's
 * stream is drained (whatever state its GPU work ended in) and the slot
 * freed for the next submit. For a binding that gives up on a round — the
 * JNI shim calls it when hrs_wait fails, before the IOException reaches
 * Java, so a caller that treats the exception as final does not lose one of
 * the handle's 4 slots. HRS_EINVAL for an unknown ticket; the drain's HIP
 * error if it fails (the slot is freed either way). */
hrs_status hrs_release(hrs_codec* codec, uint64_t ticket);
/* Uncollected operations of this handle. */
int hrs_pending(const hrs_codec* codec);
/* Diagnostic: with timing on (hrs_set_timing(codec, 1); off by default), each
 * submitted operation records a timing event before its first GPU operation
 * and one after its last, on its slot's stream; hrs_ticket_gpu_ms then gives
 * the GPU-side launch-to-completion time of a waited-for (hrs_wait) and not
 * yet collected operation. HRS_EINVAL for an unknown ticket or an operation
 * submitted with timing off. Lets a benchmark put the GPU time of small
 * asynchronous rounds beside their wall time. */
hrs_status hrs_set_timing(hrs_codec* codec, int on);
hrs_status hrs_ticket_gpu_ms(const hrs_codec* codec, uint64_t ticket, float* ms);
/* Shape of an uncollected operation: output rows, their length, CRC values
 * (0 if not checksummed). HRS_EINVAL for an unknown ticket. */
hrs_status hrs_ticket_shape(const hrs_codec* codec, uint64_t ticket, int* num_outputs, size_t* len, int* num_crcs);

/* ---- device-resident batches (the MI355X hot path) ----
 * Row pointers are DEVICE pointers for stripe 0; stripe s of row r lives at
 * rows[r] + s * stride. `stream` is a hipStream_t (NULL = the null stream).
 * Calls are asynchronous on `stream`. For the vector path every row pointer
 * and stride must be 16-byte aligned; otherwise a byte-granular kernel runs. */

/* Encode nstripes stripes: in_rows[k] data rows -> out_rows[p] parity rows. */
hrs_status hrs_encode_dev(hrs_codec* codec, const uint8_t* const* in_rows, size_t in_stride,
                          uint8_t* const* out_rows, size_t out_stride, size_t len, size_t nstripes,
                          void* stream);

/* decodeBulk 5-arg over nstripes stripes: rows[n] in hops order (entries for
 * not_to_read locations may be NULL), out_rows[num_erased]. */
hrs_status hrs_decode_dev(hrs_codec* codec, const uint8_t* const* rows, size_t in_stride,
                          uint8_t* const* out_rows, size_t out_stride, const int* erased,
                          int num_erased, const int* not_to_read, int num_not_to_read, size_t len,
                          size_t nstripes, void* stream);

/* Repair of a batch whose stripes lost different locations (a repair job over
 * many stripes: Decoder.fixErasedBlockImpl / recoverBlock per stripe,
 * Decoder.java:291-338), in one launch. Stripe s holds location l at
 * stripes + s * stripe_stride + l * row_stride (hops order). Its erased
 * locations are erased[s * max_erased + t] for t < max_erased up to the first
 * negative entry (zero erasures allowed). Each stripe is decoded like
 * hrs_decode_dev with the survivors locationsToReadForDecode picks and every
 * other location not read (Decoder.java:303-338); output t of stripe s goes to
 * out + s * out_stripe_stride + t * out_row_stride. HRS_ETOOMANY if a stripe
 * lost more than the code repairs. */
hrs_status hrs_decode_batch_dev(hrs_codec* codec, const uint8_t* stripes, size_t row_stride,
                                size_t stripe_stride, const int* erased, int max_erased, uint8_t* out,
                                size_t out_row_stride, size_t out_stripe_stride, size_t len,
                                size_t nstripes, void* stream);

/* ---- host-memory batches: many stripes per call, pipelined ----
 * Stripes start and end in host memory (DataNode sockets / local block files;
 * Encoder.encodeFile over a file's stripes, Encoder.java:289-382; a repair job
 * over many stripes, BlockReconstructor -> Decoder.fixErasedBlockImpl per
 * stripe, Decoder.java:232-401). The stripes flow in chunks through a ring of
 * device slots, each on its own stream: H2D of exactly the rows the chunk's
 * code reads, the kernel, D2H of exactly the rows it writes, successive chunks
 * overlapping. Buffers the runtime allocated pinned (hipHostMalloc, torch
 * pin_memory) are used in place (zero copy; or DMA'd directly with
 * HRS_ZEROCOPY=0) and the whole job is queued at once; any other buffer —
 * pageable, or pageable memory the caller registered with hipHostRegister,
 * whose pages are not pinned — is staged through the handle's pinned slots by
 * the copy pool. Synchronous: outputs are in place when the call returns.
 * Rows need no alignment. */

/* hrs_decode_batch_dev over host memory (same layout, semantics and errors):
 * stripe s holds location l at stripes + s * stripe_stride + l * row_stride;
 * only the survivors each stripe's pattern reads cross PCIe (k of the n for
 * rs; fewer for src local groups), and output t of stripe s lands at
 * out + s * out_stripe_stride + t * out_row_stride. */
hrs_status hrs_decode_batch_host(hrs_codec* codec, const uint8_t* stripes, size_t row_stride,
                                 size_t stripe_stride, const int* erased, int max_erased, uint8_t* out,
                                 size_t out_row_stride, size_t out_stripe_stride, size_t len,
                                 size_t nstripes);

/* encodeBulk of every stripe of a host batch, in place: reads data rows
 * (hops locations p..n-1) and writes parity rows (locations 0..p-1) of stripe
 * s at stripes + s * stripe_stride + l * row_stride. Only the k data rows go
 * H2D and the p parity rows D2H. */
hrs_status hrs_encode_batch_host(hrs_codec* codec, uint8_t* stripes, size_t row_stride, size_t stripe_stride,
                                 size_t len, size_t nstripes);

/* The two host batches above over a device set: codecs[0..ncodecs) are
 * distinct handles of one code (same family, stripe and parity size; SRC:
 * same layout), each created on the device it should use (hrs_opts.device;
 * a device may appear more than once). The stripes are split into ncodecs
 * contiguous ranges of equal size (+-1 stripe), range i = stripes
 * [i * nstripes / ncodecs, (i + 1) * nstripes / ncodecs), and range i runs as
 * one hrs_*_batch_host call of codecs[i] on its own host thread (range 0 on
 * the caller's), so every device moves its own share over its own host link
 * (contiguous stripe ranges, one host thread and stream per
 * device, no data exchange between devices). Same layout, semantics and
 * results as the single-handle call; synchronous. On failure the first
 * failing range's status is returned and its message is recorded on
 * codecs[0] (hrs_last_error(codecs[0]); hrs_last_error(NULL) for a set
 * rejected before any range ran with a NULL codecs array). The handles must
 * not be used by other threads during the call. */
hrs_status hrs_decode_batch_host_multi(hrs_codec* const* codecs, int ncodecs, const uint8_t* stripes,
                                       size_t row_stride, size_t stripe_stride, const int* erased, int max_erased,
                                       uint8_t* out, size_t out_row_stride, size_t out_stripe_stride, size_t len,
                                       size_t nstripes);
hrs_status hrs_encode_batch_host_multi(hrs_codec* const* codecs, int ncodecs, uint8_t* stripes, size_t row_stride,
                                       size_t stripe_stride, size_t len, size_t nstripes);

/* Generic GF(2^8) matrix x rows: out_o = XOR_i m[o * nin + i] * in_i (m on
 * the host, row-major nout x nin). Used with coding matrices broadcast over
 * RCCL, and by the 3-arg decode. nin, nout in [1, 255]. */
hrs_status hrs_apply_dev(hrs_codec* codec, const uint8_t* m, int nout, int nin,
                         const uint8_t* const* in_rows, size_t in_stride, uint8_t* const* out_rows,
                         size_t out_stride, size_t len, size_t nstripes, void* stream);

/* CRC-32 of device-resident cells, as java.util.zip.CRC32 (zlib) computes it
 * for the block checksums the hops drivers keep (Encoder.java:408-450,
 * Decoder.java:222-229): crc_out[s * nrows + r] = CRC32 of `len` bytes at
 * rows[r] + s * stride, continuing from crc_in[s * nrows + r] (CRC32.update
 * chaining across cells; crc_in NULL = a fresh CRC32). crc_in / crc_out are
 * DEVICE arrays of nstripes * nrows uint32. Asynchronous on `stream`. */
hrs_status hrs_crc32_dev(hrs_codec* codec, const uint8_t* const* rows, int nrows, size_t stride, size_t len,
                         size_t nstripes, const uint32_t* crc_in, uint32_t* crc_out, void* stream);

/* Encode + CRC-32 in one pass (Encoder.encodeStripe with computeBlockChecksum:
 * sourceChecksums over the read buffers, then encodeBulk, then parityChecksums
 * over the write buffers; Encoder.java:408-450). Same rows as hrs_encode_dev;
 * crc_out[s * (k + p) + r] = CRC32 of data row r (r < k) or of parity row r - k
 * (r >= k) of stripe s, continuing from crc_in (same layout; NULL = fresh).
 * rs / nrs codes with a compile-time kernel ((10,4), (6,3), (3,2), (12,4) rs;
 * (10,4), (6,3) nrs), len a multiple of 2 KiB and 16-byte-aligned rows take
 * one fused kernel (each cell read once); anything else runs hrs_encode_dev
 * then the CRC pass, with identical results. Asynchronous on `stream`. */
hrs_status hrs_encode_crc_dev(hrs_codec* codec, const uint8_t* const* in_rows, size_t in_stride,
                              uint8_t* const* out_rows, size_t out_stride, size_t len, size_t nstripes,
                              const uint32_t* crc_in, uint32_t* crc_out, void* stream);

/* Repair + CRC-32 of the repaired cells in one pass (Decoder: decodeBulk, then
 * the repaired block's CRC32 compared with the NameNode's checksum;
 * Decoder.java:222-229, :352-353, :645-655). Same rows and semantics as
 * hrs_decode_dev; crc_out[s * num_erased + t] = CRC32 of output t of stripe
 * s, continuing from crc_in (same layout; NULL = fresh). DEVICE crc arrays.
 * Repairs of <= 4 locations from <= 12 live survivors (<= 8 at 4 outputs),
 * len a multiple of 2 KiB and 16-byte-aligned rows take one fused kernel
 * (each repaired cell written once, never read back); anything else runs
 * hrs_decode_dev then the CRC pass, with identical results. Asynchronous on
 * `stream`. */
hrs_status hrs_decode_crc_dev(hrs_codec* codec, const uint8_t* const* rows, size_t in_stride,
                              uint8_t* const* out_rows, size_t out_stride, const int* erased, int num_erased,
                              const int* not_to_read, int num_not_to_read, size_t len, size_t nstripes,
                              const uint32_t* crc_in, uint32_t* crc_out, void* stream);

/* Kernel selection for tests and benchmarks: 0 = auto (default), 1 = force
 * the runtime-matrix bit-sliced kernel, 2 = force the byte-granular kernel,
 * 3 = auto, except that hrs_encode_crc_dev takes the fused kernel whenever the
 * shape allows it. */
hrs_status hrs_set_kernel_mode(hrs_codec* codec, int mode);

#ifdef __cplusplus
}
#endif

#endif /* HRS_H_ */
