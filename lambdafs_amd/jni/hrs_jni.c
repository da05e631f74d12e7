/*
 * JNI shim: io.hops.erasure_coding.HrsNative (used by HipReedSolomonCode,
 * HipXORCode, HipNativeReedSolomonCode, HipSimpleRegeneratingCode) ->
 * libhrs.so (include/hrs.h).
 *
 * Pattern of the existing native codec precedent, libhadoop's ISA-L shim
 * (hadoop-common/src/main/native/src/org/apache/hadoop/io/erasurecode/
 * jni_rs_encoder.c:35-71, jni_common.c:27-114): the Java object owns the
 * buffers, the native side owns the coder (a jlong handle), and a failure
 * becomes a Java exception (jni_rs_encoder.c:51). Differences: rows are heap
 * byte[] (ReedSolomonCode's contract, Encoder.java:442 / Decoder.java:352),
 * pinned with GetPrimitiveArrayCritical for the duration of one synchronous
 * hrs_encode / hrs_decode call, instead of direct ByteBuffers.
 *
 * Argument rules (checked before any row is pinned, so a bad call never
 * reaches the engine and never touches memory past a Java array):
 *  - a NULL byte[][] / int[] / row -> NullPointerException (what the Java
 *    codec's first access would throw); read rows of not-to-read locations
 *    may be NULL (the engine never reads them);
 *  - row counts: inputs.length == k and outputs.length == p (encode),
 *    readBufs.length == k + p (decode), else IllegalArgumentException (the
 *    Java only asserts them); writeBufs.length < erased.length ->
 *    ArrayIndexOutOfBoundsException (ReedSolomonCode.java:206-208 indexes
 *    writeBufs[i] for every erased i);
 *  - every row used must hold at least `len` bytes, else
 *    ArrayIndexOutOfBoundsException, as the Java byte loops would throw
 *    (GaloisField.java:326-338, ReedSolomonCode.java:200-208);
 *  - int[] / byte[][] arguments longer than MAX_ROWS (k + p < 256 always) ->
 *    IllegalArgumentException, never a silent truncation;
 *  - engine status: HRS_EINVAL -> IllegalArgumentException, HRS_ETOOMANY ->
 *    TooManyErasedLocations, anything else -> IOException.
 * Local references: each entry point opens a local frame sized for every row
 * it fetches (JNI guarantees only 16 otherwise) and pops it on the way out.
 * Critical regions: no JNI call runs between the first
 * GetPrimitiveArrayCritical and the last ReleasePrimitiveArrayCritical; the
 * region lasts one engine call (~0.45 ms for an RS(10,4) 1 MiB-cell encode,
 * DESIGN.md §7), during which a JVM without region pinning defers GC. collect
 * waits for its round (hrs_wait) before it pins anything, so its region is
 * only the copy out of pinned staging.
 *
 * Build: make jni (this header set) or, with a JDK,
 *   gcc -O2 -fPIC -shared -DHRS_SYSTEM_JNI -I$JAVA_HOME/include -I$JAVA_HOME/include/linux \
 *       -Iinclude lambdafs_amd/jni/hrs_jni.c -Llambdafs_amd -lhrs -o libhrs_jni.so
 */
#ifdef HRS_SYSTEM_JNI
#include <jni.h>
#else
#include "jni_min.h"
#endif
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hrs.h"

#define MAX_ROWS 256
#define FRAME_REFS (2 * MAX_ROWS + 16)

static const char kNPE[] = "java/lang/NullPointerException";
static const char kIAE[] = "java/lang/IllegalArgumentException";
static const char kAIOOBE[] = "java/lang/ArrayIndexOutOfBoundsException";
static const char kISE[] = "java/lang/IllegalStateException";
static const char kIOE[] = "java/io/IOException";
static const char kTooMany[] = "io/hops/erasure_coding/TooManyErasedLocations";

static void throw_msg(JNIEnv* env, const char* cls, const char* fmt, ...) {
  char buf[256];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  jclass k = (*env)->FindClass(env, cls);
  if (k) (*env)->ThrowNew(env, k, buf);  /* FindClass failing leaves its own error pending */
}

static void throw_status(JNIEnv* env, hrs_status st, const hrs_codec* c) {
  const char* cls = st == HRS_ETOOMANY ? kTooMany : st == HRS_EINVAL ? kIAE : kIOE;
  throw_msg(env, cls, "%s", hrs_last_error(c));
}

static hrs_codec* handle(JNIEnv* env, jlong h) {
  if (h == 0) throw_msg(env, kISE, "codec used after release()");
  return (hrs_codec*)(intptr_t)h;
}

/* Copies an int[] (erased / toRead / notToRead locations). Returns the count,
 * or -1 with an exception pending. A NULL array is 0 entries if `nullable`. */
static int copy_ints(JNIEnv* env, jintArray a, const char* what, int nullable, int* out) {
  if (!a) {
    if (nullable) return 0;
    throw_msg(env, kNPE, "%s is null", what);
    return -1;
  }
  const jsize n = (*env)->GetArrayLength(env, a);
  if (n > MAX_ROWS) {
    throw_msg(env, kIAE, "%s has %d entries (at most %d)", what, (int)n, MAX_ROWS);
    return -1;
  }
  if (n > 0) (*env)->GetIntArrayRegion(env, a, 0, n, (jint*)out);
  return (int)n;
}

typedef struct {
  int n;
  jbyteArray obj[MAX_ROWS];
  uint8_t* ptr[MAX_ROWS];
} Rows;

/* Fetches rows [0, want) of a byte[][] and checks them (see the header). The
 * array must hold exactly `want` rows (exact) or at least `want` (otherwise:
 * the Java indexes only the first `want`). may_be_null[i] != 0 lets row i be
 * NULL. Returns 0, or -1 with an exception pending. */
static int fetch_rows(JNIEnv* env, jobjectArray arr, const char* what, int want, int exact,
                      const unsigned char* may_be_null, jint len, Rows* r) {
  r->n = 0;
  if (!arr) {
    throw_msg(env, kNPE, "%s is null", what);
    return -1;
  }
  const jsize have = (*env)->GetArrayLength(env, arr);
  if (have > MAX_ROWS) {
    throw_msg(env, kIAE, "%s has %d rows (at most %d)", what, (int)have, MAX_ROWS);
    return -1;
  }
  if (exact && have != want) {
    throw_msg(env, kIAE, "%s has %d rows, the code needs %d", what, (int)have, want);
    return -1;
  }
  if (have < want) {
    throw_msg(env, kAIOOBE, "%s has %d rows, %d are written", what, (int)have, want);
    return -1;
  }
  for (int i = 0; i < want; i++) {
    r->obj[i] = (jbyteArray)(*env)->GetObjectArrayElement(env, arr, i);
    r->ptr[i] = NULL;
    r->n = i + 1;
    if (!r->obj[i]) {
      if (may_be_null && may_be_null[i]) continue;
      throw_msg(env, kNPE, "%s[%d] is null", what, i);
      return -1;
    }
    const jsize rl = (*env)->GetArrayLength(env, r->obj[i]);
    if (rl < len) {
      throw_msg(env, kAIOOBE, "%s[%d] has %d bytes, %d are coded", what, i, (int)rl, (int)len);
      return -1;
    }
  }
  return 0;
}

/* Pins every non-NULL row (zero-copy). On a NULL return (the JVM could not
 * pin: OutOfMemoryError pending) releases what it pinned and returns -1. */
static int pin_rows(JNIEnv* env, Rows* r) {
  for (int i = 0; i < r->n; i++) {
    if (!r->obj[i]) continue;
    r->ptr[i] = (uint8_t*)(*env)->GetPrimitiveArrayCritical(env, r->obj[i], NULL);
    if (!r->ptr[i]) return -1;
  }
  return 0;
}

static void unpin_rows(JNIEnv* env, Rows* r, jint mode) {
  for (int i = r->n - 1; i >= 0; i--)
    if (r->obj[i] && r->ptr[i]) {
      (*env)->ReleasePrimitiveArrayCritical(env, r->obj[i], r->ptr[i], mode);
      r->ptr[i] = NULL;
    }
}

/* Pins in, then out; runs fn (the engine call) only if both pinned; releases
 * out (copy back) then in (JNI_ABORT: read-only). Returns the engine status,
 * or -1 if pinning failed (exception pending). */
typedef hrs_status (*engine_fn)(hrs_codec* c, Rows* in, Rows* out, void* arg);

static int run_pinned(JNIEnv* env, hrs_codec* c, Rows* in, Rows* out, engine_fn fn, void* arg) {
  int ok = pin_rows(env, in) == 0 && pin_rows(env, out) == 0;
  hrs_status st = ok ? fn(c, in, out, arg) : HRS_OK;
  unpin_rows(env, out, 0);
  unpin_rows(env, in, JNI_ABORT);
  return ok ? (int)st : -1;
}

static int check_len(JNIEnv* env, jint len) {
  if (len >= 0) return 0;
  throw_msg(env, kIAE, "negative length %d", (int)len);
  return -1;
}

static int open_frame(JNIEnv* env) { return (*env)->PushLocalFrame(env, FRAME_REFS) == JNI_OK ? 0 : -1; }
static void close_frame(JNIEnv* env) { (void)(*env)->PopLocalFrame(env, NULL); }

/* ------------------------------------------------------------ lifecycle */

/* The device a codec instance runs on (HipDevices.pick: round robin over
 * hdfs.raid.hip.devices; -1 = the thread's current device). An ordinal that
 * is not a visible device fails hrs_create with HRS_EDEVICE -> IOException. */
static jlong create_on(JNIEnv* env, int code, jint k, jint p, int src, jint s, jint device) {
  hrs_opts o;
  memset(&o, 0, sizeof o);
  o.device = device;
  hrs_codec* c = NULL;
  const hrs_status st = src ? hrs_create_src(k, p, s, &o, &c) : hrs_create_code(code, k, p, &o, &c);
  if (st != HRS_OK) {
    throw_status(env, st, NULL);
    return 0;
  }
  return (jlong)(intptr_t)c;
}

JNIEXPORT jlong JNICALL Java_io_hops_erasure_1coding_HrsNative_create(JNIEnv* env, jclass cls, jint code, jint k,
                                                                       jint p, jint device) {
  (void)cls;
  return create_on(env, code, k, p, 0, 0, device);
}

JNIEXPORT jlong JNICALL Java_io_hops_erasure_1coding_HrsNative_createSrc(JNIEnv* env, jclass cls, jint k, jint p,
                                                                          jint s, jint device) {
  (void)cls;
  return create_on(env, HRS_CODE_SRC, k, p, 1, s, device);
}

/* hrs_device_count: devices visible to this JVM (HIP_VISIBLE_DEVICES applies). */
JNIEXPORT jint JNICALL Java_io_hops_erasure_1coding_HrsNative_deviceCount(JNIEnv* env, jclass cls) {
  (void)env;
  (void)cls;
  return hrs_device_count();
}

/* hrs_codec_device: the ordinal a handle runs on. */
JNIEXPORT jint JNICALL Java_io_hops_erasure_1coding_HrsNative_device(JNIEnv* env, jclass cls, jlong h) {
  (void)cls;
  hrs_codec* c = handle(env, h);
  return c ? hrs_codec_device(c) : -1;
}

JNIEXPORT void JNICALL Java_io_hops_erasure_1coding_HrsNative_destroy(JNIEnv* env, jclass cls, jlong h) {
  (void)env;
  (void)cls;
  hrs_destroy((hrs_codec*)(intptr_t)h);
}

/* ErasureCode.locationsToReadForDecode (ErasureCode.java:89-113;
 * SimpleRegeneratingCode.java:300-366) -> int[] (highest location first). */
JNIEXPORT jintArray JNICALL Java_io_hops_erasure_1coding_HrsNative_locationsToRead(JNIEnv* env, jclass cls, jlong h,
                                                                                  jintArray erased) {
  (void)cls;
  hrs_codec* c = handle(env, h);
  if (!c) return NULL;
  int e[MAX_ROWS], out[MAX_ROWS];
  const int ne = copy_ints(env, erased, "erasedLocations", 0, e);
  if (ne < 0) return NULL;
  int m = 0;
  hrs_status st = hrs_locations_to_read_list(c, e, ne, out, &m);
  if (st != HRS_OK) {
    throw_status(env, st, c);
    return NULL;
  }
  jintArray r = (*env)->NewIntArray(env, m);
  if (r && m > 0) (*env)->SetIntArrayRegion(env, r, 0, m, (const jint*)out);
  return r;
}

/* --------------------------------------------------------------- coding */

struct enc_arg {
  jint len;
  uint32_t* crc;  /* encodeCrc: k + p running values, updated in place */
};

static hrs_status do_encode(hrs_codec* c, Rows* in, Rows* out, void* p) {
  const struct enc_arg* a = (const struct enc_arg*)p;
  if (a->crc) return hrs_encode_crc(c, (const uint8_t* const*)in->ptr, out->ptr, (size_t)a->len, a->crc, a->crc);
  return hrs_encode(c, (const uint8_t* const*)in->ptr, out->ptr, (size_t)a->len);
}

static void encode_common(JNIEnv* env, jlong h, jobjectArray inputs, jobjectArray outputs, jint len, jintArray crcs) {
  hrs_codec* c = handle(env, h);
  if (!c || check_len(env, len) || open_frame(env)) return;
  const int k = hrs_stripe_size(c), p = hrs_parity_size(c);
  uint32_t crc[MAX_ROWS];
  struct enc_arg a = {len, NULL};
  Rows in, out;
  in.n = out.n = 0;
  if (crcs) {
    const int got = copy_ints(env, crcs, "crcs", 0, (int*)crc);
    if (got < 0) goto done;
    if (got != k + p) {
      throw_msg(env, kIAE, "crcs has %d entries, the code needs %d", got, k + p);
      goto done;
    }
    a.crc = crc;
  }
  if (fetch_rows(env, inputs, "inputs", k, 1, NULL, len, &in) ||
      fetch_rows(env, outputs, "outputs", p, 1, NULL, len, &out))
    goto done;
  const int st = run_pinned(env, c, &in, &out, do_encode, &a);
  if (st > 0) throw_status(env, (hrs_status)st, c);
  if (st == 0 && crcs) (*env)->SetIntArrayRegion(env, crcs, 0, k + p, (const jint*)crc);
done:
  close_frame(env);
}

/* ReedSolomonCode.encodeBulk (ReedSolomonCode.java:103-125). */
JNIEXPORT void JNICALL Java_io_hops_erasure_1coding_HrsNative_encode(JNIEnv* env, jclass cls, jlong h,
                                                                    jobjectArray inputs, jobjectArray outputs,
                                                                    jint len) {
  (void)cls;
  encode_common(env, h, inputs, outputs, len, NULL);
}

/* Encoder.encodeStripe with computeBlockChecksum (Encoder.java:408-450):
 * crcs[k + p] = sourceChecksums then parityChecksums, updated in place. */
JNIEXPORT void JNICALL Java_io_hops_erasure_1coding_HrsNative_encodeCrc(JNIEnv* env, jclass cls, jlong h,
                                                                       jobjectArray inputs, jobjectArray outputs,
                                                                       jint len, jintArray crcs) {
  (void)cls;
  if (!crcs) {
    throw_msg(env, kNPE, "crcs is null");
    return;
  }
  encode_common(env, h, inputs, outputs, len, crcs);
}

struct dec_arg {
  int three;  /* decodeBulk 3-arg */
  int e[MAX_ROWS], r[MAX_ROWS], ntr[MAX_ROWS];
  int ne, nr, nn;
  int has_to_read;
  jint len;
  uint32_t* crc;  /* decodeCrc: ne running values */
};

static hrs_status do_decode(hrs_codec* c, Rows* in, Rows* out, void* p) {
  const struct dec_arg* a = (const struct dec_arg*)p;
  const uint8_t* const* rb = (const uint8_t* const*)in->ptr;
  const int* tr = a->has_to_read ? a->r : NULL;
  if (a->three) return hrs_decode3(c, rb, out->ptr, a->e, a->ne, (size_t)a->len);
  if (a->crc)
    return hrs_decode_crc(c, rb, out->ptr, a->e, a->ne, tr, a->nr, a->ntr, a->nn, (size_t)a->len, a->crc, a->crc);
  return hrs_decode(c, rb, out->ptr, a->e, a->ne, tr, a->nr, a->ntr, a->nn, (size_t)a->len);
}

static void decode_common(JNIEnv* env, jlong h, jobjectArray readBufs, jobjectArray writeBufs, jintArray erased,
                          jintArray toRead, jintArray notToRead, jint len, jintArray crcs, int three) {
  hrs_codec* c = handle(env, h);
  if (!c || check_len(env, len)) return;
  struct dec_arg* a = (struct dec_arg*)calloc(1, sizeof *a);
  if (!a) {
    throw_msg(env, "java/lang/OutOfMemoryError", "decode arguments");
    return;
  }
  if (open_frame(env)) {
    free(a);
    return;
  }
  const int n = hrs_stripe_size(c) + hrs_parity_size(c);
  uint32_t crc[MAX_ROWS];
  unsigned char may_be_null[MAX_ROWS];
  Rows* in = (Rows*)malloc(sizeof(Rows));
  Rows* out = (Rows*)malloc(sizeof(Rows));
  if (!in || !out) {
    throw_msg(env, "java/lang/OutOfMemoryError", "decode rows");
    goto done;
  }
  in->n = out->n = 0;
  a->three = three;
  a->len = len;
  a->ne = copy_ints(env, erased, "erasedLocations", 0, a->e);
  if (a->ne < 0) goto done;
  if (!three) {
    a->has_to_read = toRead != NULL;
    a->nr = copy_ints(env, toRead, "locationsToRead", 1, a->r);
    if (a->nr < 0) goto done;
    a->nn = copy_ints(env, notToRead, "locationsNotToRead", 0, a->ntr);
    if (a->nn < 0) goto done;
  }
  if (crcs) {
    const int got = copy_ints(env, crcs, "crcs", 0, (int*)crc);
    if (got < 0) goto done;
    if (got != a->ne) {
      throw_msg(env, kIAE, "crcs has %d entries, %d locations are erased", got, a->ne);
      goto done;
    }
    a->crc = crc;
  }
  memset(may_be_null, 0, sizeof may_be_null);
  for (int j = 0; j < a->nn; j++)  /* never read: StripeReader feeds zeros there */
    if (a->ntr[j] >= 0 && a->ntr[j] < MAX_ROWS) may_be_null[a->ntr[j]] = 1;
  if (fetch_rows(env, readBufs, "readBufs", n, 1, may_be_null, len, in) ||
      fetch_rows(env, writeBufs, "writeBufs", a->ne, 0, NULL, len, out))
    goto done;
  {
    const int st = run_pinned(env, c, in, out, do_decode, a);
    if (st > 0) throw_status(env, (hrs_status)st, c);
    if (st == 0 && crcs && a->ne > 0) (*env)->SetIntArrayRegion(env, crcs, 0, a->ne, (const jint*)crc);
  }
done:
  close_frame(env);
  free(in);
  free(out);
  free(a);
}

/* ReedSolomonCode.decodeBulk 5-arg (ReedSolomonCode.java:191-211). */
JNIEXPORT void JNICALL Java_io_hops_erasure_1coding_HrsNative_decode(JNIEnv* env, jclass cls, jlong h,
                                                                    jobjectArray readBufs, jobjectArray writeBufs,
                                                                    jintArray erased, jintArray toRead,
                                                                    jintArray notToRead, jint len) {
  (void)cls;
  decode_common(env, h, readBufs, writeBufs, erased, toRead, notToRead, len, NULL, 0);
}

/* ReedSolomonCode.decodeBulk 3-arg (ReedSolomonCode.java:168-185). */
JNIEXPORT void JNICALL Java_io_hops_erasure_1coding_HrsNative_decode3(JNIEnv* env, jclass cls, jlong h,
                                                                     jobjectArray readBufs, jobjectArray writeBufs,
                                                                     jintArray erased, jint len) {
  (void)cls;
  decode_common(env, h, readBufs, writeBufs, erased, NULL, NULL, len, NULL, 1);
}

/* The Decoder's repaired-block check (Decoder.java:222-229, :645-655):
 * crcs[erased.length] continued over writeBufs[i], updated in place. */
JNIEXPORT void JNICALL Java_io_hops_erasure_1coding_HrsNative_decodeCrc(JNIEnv* env, jclass cls, jlong h,
                                                                       jobjectArray readBufs, jobjectArray writeBufs,
                                                                       jintArray erased, jintArray toRead,
                                                                       jintArray notToRead, jint len, jintArray crcs) {
  (void)cls;
  if (!crcs) {
    throw_msg(env, kNPE, "crcs is null");
    return;
  }
  decode_common(env, h, readBufs, writeBufs, erased, toRead, notToRead, len, crcs, 0);
}

/* ------------------------------------------------- asynchronous rounds */

/* hrs_encode_submit: stages the rows (pinned only for this call), queues the
 * round, returns the ticket. checksums != 0 adds the block CRC32s (chained by
 * collect). */
JNIEXPORT jlong JNICALL Java_io_hops_erasure_1coding_HrsNative_encodeSubmit(JNIEnv* env, jclass cls, jlong h,
                                                                           jobjectArray inputs, jint len,
                                                                           jboolean checksums) {
  (void)cls;
  hrs_codec* c = handle(env, h);
  if (!c || check_len(env, len) || open_frame(env)) return 0;
  Rows in;
  in.n = 0;
  uint64_t ticket = 0;
  if (fetch_rows(env, inputs, "inputs", hrs_stripe_size(c), 1, NULL, len, &in) == 0) {
    int ok = pin_rows(env, &in) == 0;
    hrs_status st = ok ? hrs_encode_submit(c, (const uint8_t* const*)in.ptr, (size_t)len, checksums ? 1 : 0, &ticket)
                       : HRS_OK;
    unpin_rows(env, &in, JNI_ABORT);
    if (ok && st != HRS_OK) throw_status(env, st, c);
  }
  close_frame(env);
  return (jlong)ticket;
}

/* hrs_decode_submit (the 5-arg decodeBulk round). */
JNIEXPORT jlong JNICALL Java_io_hops_erasure_1coding_HrsNative_decodeSubmit(JNIEnv* env, jclass cls, jlong h,
                                                                           jobjectArray readBufs, jintArray erased,
                                                                           jintArray toRead, jintArray notToRead,
                                                                           jint len, jboolean checksums) {
  (void)cls;
  hrs_codec* c = handle(env, h);
  if (!c || check_len(env, len)) return 0;
  struct dec_arg* a = (struct dec_arg*)calloc(1, sizeof *a);
  Rows* in = (Rows*)malloc(sizeof(Rows));
  uint64_t ticket = 0;
  if (!a || !in) {
    free(a);
    free(in);
    throw_msg(env, "java/lang/OutOfMemoryError", "decode arguments");
    return 0;
  }
  if (open_frame(env)) {
    free(a);
    free(in);
    return 0;
  }
  in->n = 0;
  unsigned char may_be_null[MAX_ROWS];
  a->ne = copy_ints(env, erased, "erasedLocations", 0, a->e);
  if (a->ne < 0) goto done;
  a->has_to_read = toRead != NULL;
  a->nr = copy_ints(env, toRead, "locationsToRead", 1, a->r);
  if (a->nr < 0) goto done;
  a->nn = copy_ints(env, notToRead, "locationsNotToRead", 0, a->ntr);
  if (a->nn < 0) goto done;
  memset(may_be_null, 0, sizeof may_be_null);
  for (int j = 0; j < a->nn; j++)
    if (a->ntr[j] >= 0 && a->ntr[j] < MAX_ROWS) may_be_null[a->ntr[j]] = 1;
  if (fetch_rows(env, readBufs, "readBufs", hrs_stripe_size(c) + hrs_parity_size(c), 1, may_be_null, len, in))
    goto done;
  {
    int ok = pin_rows(env, in) == 0;
    hrs_status st = ok ? hrs_decode_submit(c, (const uint8_t* const*)in->ptr, a->e, a->ne,
                                           a->has_to_read ? a->r : NULL, a->nr, a->ntr, a->nn, (size_t)len,
                                           checksums ? 1 : 0, &ticket)
                       : HRS_OK;
    unpin_rows(env, in, JNI_ABORT);
    if (ok && st != HRS_OK) throw_status(env, st, c);
  }
done:
  close_frame(env);
  free(in);
  free(a);
  return (jlong)ticket;
}

/* hrs_wait, then hrs_collect: copies the round's output rows into `outputs`
 * (p rows / one per erased location, each at least the round's length); a
 * checksummed round continues the running CRC32s in `crcs` (k + p / one per
 * erased location) in place. */
JNIEXPORT void JNICALL Java_io_hops_erasure_1coding_HrsNative_collect(JNIEnv* env, jclass cls, jlong h, jlong ticket,
                                                                     jobjectArray outputs, jintArray crcs) {
  (void)cls;
  hrs_codec* c = handle(env, h);
  if (!c) return;
  int nout = 0, ncrc = 0;
  size_t len = 0;
  if (hrs_ticket_shape(c, (uint64_t)ticket, &nout, &len, &ncrc) != HRS_OK) {
    throw_msg(env, kIAE, "no uncollected operation with ticket %lld", (long long)ticket);
    return;
  }
  /* wait for the round BEFORE pinning the output rows: the critical region
   * below then covers only the copy out of the slot's staging, not a GPU
   * wait that may queue behind up to three other rounds */
  {
    const hrs_status ws = hrs_wait(c, (uint64_t)ticket);
    if (ws != HRS_OK) {
      /* the round failed: throw, then drain and free its slot (hrs_release),
       * so a caller that treats the IOException as final does not lose one
       * of the handle's 4 slots with its copies possibly still in flight */
      throw_status(env, ws, c);
      (void)hrs_release(c, (uint64_t)ticket);
      return;
    }
  }
  if (open_frame(env)) return;
  uint32_t crc[MAX_ROWS];
  Rows out;
  out.n = 0;
  if (ncrc > 0) {
    const int got = copy_ints(env, crcs, "crcs", 0, (int*)crc);
    if (got < 0) goto done;
    if (got != ncrc) {
      throw_msg(env, kIAE, "crcs has %d entries, the operation keeps %d", got, ncrc);
      goto done;
    }
  }
  if (fetch_rows(env, outputs, "outputs", nout, 0, NULL, (jint)len, &out)) goto done;
  {
    int ok = pin_rows(env, &out) == 0;
    hrs_status st = ok ? hrs_collect(c, (uint64_t)ticket, out.ptr, ncrc > 0 ? crc : NULL) : HRS_OK;
    unpin_rows(env, &out, 0);
    if (ok && st != HRS_OK) {
      throw_status(env, st, c);
      goto done;
    }
    if (ok && ncrc > 0) (*env)->SetIntArrayRegion(env, crcs, 0, ncrc, (const jint*)crc);
  }
done:
  close_frame(env);
}

JNIEXPORT jint JNICALL Java_io_hops_erasure_1coding_HrsNative_pending(JNIEnv* env, jclass cls, jlong h) {
  (void)cls;
  hrs_codec* c = handle(env, h);
  return c ? hrs_pending(c) : 0;
}
