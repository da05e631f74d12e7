/*
 * JNI shim: io.hops.erasure_coding.HrsNative (used by HipReedSolomonCode and
 * HipXORCode) -> libhrs.so (include/hrs.h).
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
 * Build (needs a JDK; not part of this repo's CI):
 *   gcc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux \
 *       -Iinclude lambdafs_amd/jni/hrs_jni.c -Llambdafs_amd -lhrs -o libhrs_jni.so
 */
#include <jni.h>
#include <stdlib.h>
#include <string.h>

#include "hrs.h"

#define MAX_ROWS 256

static void throw_status(JNIEnv* env, hrs_status st, const hrs_codec* c) {
  const char* cls = "java/io/IOException";
  if (st == HRS_ETOOMANY) cls = "io/hops/erasure_coding/TooManyErasedLocations";
  if (st == HRS_EINVAL) cls = "java/lang/IllegalArgumentException";
  jclass k = (*env)->FindClass(env, cls);
  if (k) (*env)->ThrowNew(env, k, hrs_last_error(c));
}

/* Fetches the row objects of a byte[][] (no JNI call may run while rows are
 * held critical, so every array is fetched before any row is pinned).
 * Returns the row count or -1. */
static int fetch_rows(JNIEnv* env, jobjectArray arr, jbyteArray* objs, uint8_t** ptrs) {
  if (!arr) return 0;
  jsize n = (*env)->GetArrayLength(env, arr);
  if (n > MAX_ROWS) return -1;
  for (jsize i = 0; i < n; i++) {
    objs[i] = (jbyteArray)(*env)->GetObjectArrayElement(env, arr, i);
    ptrs[i] = NULL;
  }
  return (int)n;
}

/* Pins fetched rows with GetPrimitiveArrayCritical (zero-copy); NULL rows stay NULL. */
static void pin_rows(JNIEnv* env, int n, jbyteArray* objs, uint8_t** ptrs) {
  for (int i = 0; i < n; i++)
    if (objs[i]) ptrs[i] = (uint8_t*)(*env)->GetPrimitiveArrayCritical(env, objs[i], NULL);
}

static void unpin_rows(JNIEnv* env, int n, jbyteArray* objs, uint8_t** ptrs, jint mode) {
  for (int i = n - 1; i >= 0; i--)
    if (objs[i] && ptrs[i]) (*env)->ReleasePrimitiveArrayCritical(env, objs[i], ptrs[i], mode);
}

JNIEXPORT jlong JNICALL Java_io_hops_erasure_1coding_HrsNative_create(JNIEnv* env, jclass cls, jint code, jint k,
                                                                       jint p) {
  (void)cls;
  hrs_codec* c = NULL;
  hrs_status st = hrs_create_code(code, k, p, NULL, &c);
  if (st != HRS_OK) {
    throw_status(env, st, NULL);
    return 0;
  }
  return (jlong)(intptr_t)c;
}

JNIEXPORT jlong JNICALL Java_io_hops_erasure_1coding_HrsNative_createSrc(JNIEnv* env, jclass cls, jint k, jint p,
                                                                          jint s) {
  (void)cls;
  hrs_codec* c = NULL;
  hrs_status st = hrs_create_src(k, p, s, NULL, &c);
  if (st != HRS_OK) {
    throw_status(env, st, NULL);
    return 0;
  }
  return (jlong)(intptr_t)c;
}

JNIEXPORT jintArray JNICALL Java_io_hops_erasure_1coding_HrsNative_locationsToRead(JNIEnv* env, jclass cls, jlong h,
                                                                                  jintArray erased) {
  (void)cls;
  hrs_codec* c = (hrs_codec*)(intptr_t)h;
  const jsize ne = (*env)->GetArrayLength(env, erased);
  jint* e = (*env)->GetIntArrayElements(env, erased, NULL);
  int out[256];
  int m = 0;
  hrs_status st = hrs_locations_to_read_list(c, (const int*)e, ne, out, &m);
  (*env)->ReleaseIntArrayElements(env, erased, e, JNI_ABORT);
  if (st != HRS_OK) {
    throw_status(env, st, c);
    return NULL;
  }
  jintArray r = (*env)->NewIntArray(env, m);
  if (r) (*env)->SetIntArrayRegion(env, r, 0, m, (const jint*)out);
  return r;
}

JNIEXPORT void JNICALL Java_io_hops_erasure_1coding_HrsNative_destroy(JNIEnv* env, jclass cls,
                                                                                     jlong h) {
  (void)env;
  (void)cls;
  hrs_destroy((hrs_codec*)(intptr_t)h);
}

JNIEXPORT void JNICALL Java_io_hops_erasure_1coding_HrsNative_encode(JNIEnv* env, jclass cls, jlong h,
                                                                                    jobjectArray inputs,
                                                                                    jobjectArray outputs, jint len) {
  (void)cls;
  hrs_codec* c = (hrs_codec*)(intptr_t)h;
  jbyteArray io[MAX_ROWS], oo[MAX_ROWS];
  uint8_t *ip[MAX_ROWS], *op[MAX_ROWS];
  int ni = fetch_rows(env, inputs, io, ip);
  int no = fetch_rows(env, outputs, oo, op);
  if (ni >= 0 && no >= 0) {
    pin_rows(env, ni, io, ip);
    pin_rows(env, no, oo, op);
  }
  hrs_status st = (ni < 0 || no < 0) ? HRS_EINVAL : hrs_encode(c, (const uint8_t* const*)ip, op, (size_t)len);
  unpin_rows(env, no > 0 ? no : 0, oo, op, 0);
  unpin_rows(env, ni > 0 ? ni : 0, io, ip, JNI_ABORT);
  if (st != HRS_OK) throw_status(env, st, c);
}

static int copy_ints(JNIEnv* env, jintArray a, int* out) {
  if (!a) return 0;
  jsize n = (*env)->GetArrayLength(env, a);
  if (n > MAX_ROWS) n = MAX_ROWS;
  (*env)->GetIntArrayRegion(env, a, 0, n, out);
  return (int)n;
}

JNIEXPORT void JNICALL Java_io_hops_erasure_1coding_HrsNative_decode(
    JNIEnv* env, jclass cls, jlong h, jobjectArray readBufs, jobjectArray writeBufs, jintArray erased,
    jintArray toRead, jintArray notToRead, jint len) {
  (void)cls;
  hrs_codec* c = (hrs_codec*)(intptr_t)h;
  int e[MAX_ROWS], r[MAX_ROWS], ntr[MAX_ROWS];
  int ne = copy_ints(env, erased, e), nr = copy_ints(env, toRead, r), nn = copy_ints(env, notToRead, ntr);
  jbyteArray io[MAX_ROWS], oo[MAX_ROWS];
  uint8_t *ip[MAX_ROWS], *op[MAX_ROWS];
  int ni = fetch_rows(env, readBufs, io, ip);
  int no = fetch_rows(env, writeBufs, oo, op);
  if (ni >= 0 && no >= 0) {
    pin_rows(env, ni, io, ip);
    pin_rows(env, no, oo, op);
  }
  hrs_status st = (ni < 0 || no < 0)
                      ? HRS_EINVAL
                      : hrs_decode(c, (const uint8_t* const*)ip, op, e, ne, r, nr, ntr, nn, (size_t)len);
  unpin_rows(env, no > 0 ? no : 0, oo, op, 0);
  unpin_rows(env, ni > 0 ? ni : 0, io, ip, JNI_ABORT);
  if (st != HRS_OK) throw_status(env, st, c);
}

JNIEXPORT void JNICALL Java_io_hops_erasure_1coding_HrsNative_decode3(
    JNIEnv* env, jclass cls, jlong h, jobjectArray readBufs, jobjectArray writeBufs, jintArray erased, jint len) {
  (void)cls;
  hrs_codec* c = (hrs_codec*)(intptr_t)h;
  int e[MAX_ROWS];
  int ne = copy_ints(env, erased, e);
  jbyteArray io[MAX_ROWS], oo[MAX_ROWS];
  uint8_t *ip[MAX_ROWS], *op[MAX_ROWS];
  int ni = fetch_rows(env, readBufs, io, ip);
  int no = fetch_rows(env, writeBufs, oo, op);
  if (ni >= 0 && no >= 0) {
    pin_rows(env, ni, io, ip);
    pin_rows(env, no, oo, op);
  }
  hrs_status st = (ni < 0 || no < 0) ? HRS_EINVAL : hrs_decode3(c, (const uint8_t* const*)ip, op, e, ne, (size_t)len);
  unpin_rows(env, no > 0 ? no : 0, oo, op, 0);
  unpin_rows(env, ni > 0 ? ni : 0, io, ip, JNI_ABORT);
  if (st != HRS_OK) throw_status(env, st, c);
}

/* Running checksums as a Java int[] (CRC32.getValue() & 0xFFFFFFFF):
 * read before the rows are pinned, written back after they are released. */
static int copy_crcs(JNIEnv* env, jintArray a, uint32_t* out, int want) {
  if (!a || (*env)->GetArrayLength(env, a) != want || want > MAX_ROWS) return -1;
  (*env)->GetIntArrayRegion(env, a, 0, want, (jint*)out);
  return want;
}

/* Encoder.encodeStripe with computeBlockChecksum (Encoder.java:408-450):
 * crcs[k + p] = sourceChecksums then parityChecksums, updated in place. */
JNIEXPORT void JNICALL Java_io_hops_erasure_1coding_HrsNative_encodeCrc(JNIEnv* env, jclass cls, jlong h,
                                                                       jobjectArray inputs, jobjectArray outputs,
                                                                       jint len, jintArray crcs) {
  (void)cls;
  hrs_codec* c = (hrs_codec*)(intptr_t)h;
  uint32_t crc[MAX_ROWS];
  int ncrc = copy_crcs(env, crcs, crc, hrs_stripe_size(c) + hrs_parity_size(c));
  jbyteArray io[MAX_ROWS], oo[MAX_ROWS];
  uint8_t *ip[MAX_ROWS], *op[MAX_ROWS];
  int ni = fetch_rows(env, inputs, io, ip);
  int no = fetch_rows(env, outputs, oo, op);
  const int ok = ni >= 0 && no >= 0 && ncrc >= 0;
  if (ok) {
    pin_rows(env, ni, io, ip);
    pin_rows(env, no, oo, op);
  }
  hrs_status st = ok ? hrs_encode_crc(c, (const uint8_t* const*)ip, op, (size_t)len, crc, crc) : HRS_EINVAL;
  if (ok) {
    unpin_rows(env, no, oo, op, 0);
    unpin_rows(env, ni, io, ip, JNI_ABORT);
  }
  if (st != HRS_OK) {
    throw_status(env, st, c);
    return;
  }
  (*env)->SetIntArrayRegion(env, crcs, 0, ncrc, (const jint*)crc);
}

/* Decoder's repaired-block check (Decoder.java:222-229, :645-655):
 * crcs[erased.length] continued over writeBufs[i], updated in place. */
JNIEXPORT void JNICALL Java_io_hops_erasure_1coding_HrsNative_decodeCrc(
    JNIEnv* env, jclass cls, jlong h, jobjectArray readBufs, jobjectArray writeBufs, jintArray erased,
    jintArray toRead, jintArray notToRead, jint len, jintArray crcs) {
  (void)cls;
  hrs_codec* c = (hrs_codec*)(intptr_t)h;
  int e[MAX_ROWS], r[MAX_ROWS], ntr[MAX_ROWS];
  int ne = copy_ints(env, erased, e), nr = copy_ints(env, toRead, r), nn = copy_ints(env, notToRead, ntr);
  uint32_t crc[MAX_ROWS];
  int ncrc = copy_crcs(env, crcs, crc, ne);
  jbyteArray io[MAX_ROWS], oo[MAX_ROWS];
  uint8_t *ip[MAX_ROWS], *op[MAX_ROWS];
  int ni = fetch_rows(env, readBufs, io, ip);
  int no = fetch_rows(env, writeBufs, oo, op);
  const int ok = ni >= 0 && no >= 0 && ncrc >= 0;
  if (ok) {
    pin_rows(env, ni, io, ip);
    pin_rows(env, no, oo, op);
  }
  hrs_status st = ok ? hrs_decode_crc(c, (const uint8_t* const*)ip, op, e, ne, r, nr, ntr, nn, (size_t)len, crc, crc)
                     : HRS_EINVAL;
  if (ok) {
    unpin_rows(env, no, oo, op, 0);
    unpin_rows(env, ni, io, ip, JNI_ABORT);
  }
  if (st != HRS_OK) {
    throw_status(env, st, c);
    return;
  }
  (*env)->SetIntArrayRegion(env, crcs, 0, ncrc, (const jint*)crc);
}
