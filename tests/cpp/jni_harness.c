/*
 * Fake-JVM harness for the JNI shim (lambdafs_amd/jni/hrs_jni.c, built into
 * lambdafs_amd/libhrs_jni.so against the hand-declared jni_min.h).
 *
 * A JNIEnv whose function table implements the calls the shim makes over a
 * toy heap, and enforces the JNI rules a real JVM only checks under
 * -Xcheck:jni:
 *  - no JNI call except Get/ReleasePrimitiveArrayCritical inside a critical
 *    region;
 *  - with an exception pending, only the release / frame / ExceptionCheck
 *    calls the spec allows;
 *  - local references never exceed the current frame's capacity (16 unless
 *    PushLocalFrame / EnsureLocalCapacity raised it), and every frame the shim
 *    pushes is popped;
 *  - every pinned array is released.
 * Every byte[] ends exactly at a PROT_NONE guard page, so an access past a
 * Java array's end faults instead of passing silently.
 *
 * Usage: jni_harness --cpu | --gpu
 *  --cpu : argument / error mapping of every HrsNative entry point, through a
 *          host-only handle (no GPU needed).
 *  --gpu : HrsNative.encode / decode / decode3 / encodeCrc / decodeCrc of
 *          RS(10,4) with 1 MiB cells vs the oracle (and zlib for the CRCs),
 *          bit-exact; short rows on a live handle; asynchronous rounds
 *          (encodeSubmit / decodeSubmit / collect: 2 deep with chained CRCs,
 *          the 4-slot limit, out-of-order collects); xor / nrs / src encodes.
 * Prints one JSON line; exit status 0 iff every check passed.
 */
#define _GNU_SOURCE
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <dlfcn.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>
#include <zlib.h>

#include "../../lambdafs_amd/jni/jni_min.h"
#include "hrs.h"
#include "rs_oracle.h"

/* ------------------------------------------------------------- toy heap */

enum { K_BYTES = 1, K_INTS = 2, K_OBJS = 3, K_CLASS = 4 };

struct _jobject {
  int kind;
  jsize len;
  void* data;
  void* map;
  size_t map_len;
  char name[96];
};

static struct _jobject* heap[65536];
static int nheap;

static jobject track(struct _jobject* o) {
  if (nheap < (int)(sizeof heap / sizeof heap[0])) heap[nheap++] = o;
  return o;
}

static jbyteArray new_bytes(jsize len) {
  struct _jobject* o = calloc(1, sizeof *o);
  const size_t pg = (size_t)sysconf(_SC_PAGESIZE);
  const size_t pages = ((size_t)len + pg - 1) / pg;
  o->map_len = (pages + 1) * pg;
  o->map = mmap(NULL, o->map_len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (o->map == MAP_FAILED) abort();
  uint8_t* guard = (uint8_t*)o->map + pages * pg;
  if (mprotect(guard, pg, PROT_NONE)) abort();
  o->data = guard - len; /* the array's last byte abuts the guard page */
  o->kind = K_BYTES;
  o->len = len;
  return track(o);
}

static jintArray new_ints(jsize len, const int* v) {
  struct _jobject* o = calloc(1, sizeof *o);
  o->kind = K_INTS;
  o->len = len;
  o->data = calloc((size_t)len + 1, sizeof(jint));
  if (v) memcpy(o->data, v, (size_t)len * sizeof(jint));
  return track(o);
}

static jobjectArray new_objs(jsize len) {
  struct _jobject* o = calloc(1, sizeof *o);
  o->kind = K_OBJS;
  o->len = len;
  o->data = calloc((size_t)len + 1, sizeof(jobject));
  return track(o);
}

static void set_obj(jobjectArray a, int i, jobject v) { ((jobject*)a->data)[i] = v; }
static uint8_t* bytes_of(jbyteArray a) { return (uint8_t*)a->data; }
static jint* ints_of(jintArray a) { return (jint*)a->data; }

static void free_heap(void) {
  for (int i = 0; i < nheap; i++) {
    struct _jobject* o = heap[i];
    if (o->kind == K_BYTES)
      munmap(o->map, o->map_len);
    else
      free(o->data);
    free(o);
  }
  nheap = 0;
}

/* ------------------------------------------------------------- fake JVM */

static struct {
  int critical;            /* open critical regions */
  int pinned;              /* pinned arrays not yet released */
  int pending;             /* exception pending */
  char exc_class[96];
  char exc_msg[256];
  int frame_cap[64];       /* local-frame stack: capacity and refs held */
  int frame_refs[64];
  int depth;               /* index of the current frame (0 = the native method's own) */
  int violations;
  char first_violation[256];
  int calls;
} vm;

static void violation(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  if (vm.violations++ == 0) vsnprintf(vm.first_violation, sizeof vm.first_violation, fmt, ap);
  va_end(ap);
}

/* allowed_pending: may run with an exception pending; crit_ok: inside a critical region */
static void enter(const char* fn, int allowed_pending, int crit_ok) {
  vm.calls++;
  if (vm.critical > 0 && !crit_ok) violation("%s called inside a critical region", fn);
  if (vm.pending && !allowed_pending) violation("%s called with %s pending", fn, vm.exc_class);
}

static void new_local_ref(const char* fn) {
  if (++vm.frame_refs[vm.depth] > vm.frame_cap[vm.depth])
    violation("%s: %d local refs in a frame of capacity %d", fn, vm.frame_refs[vm.depth], vm.frame_cap[vm.depth]);
}

static void begin_native_call(void) {
  vm.depth = 0;
  vm.frame_cap[0] = 16; /* JNI guarantees 16 local refs to a native method */
  vm.frame_refs[0] = 0;
  vm.pending = 0;
  vm.exc_class[0] = vm.exc_msg[0] = 0;
}

static int end_native_call(const char* what) {
  int bad = 0;
  if (vm.critical) violation("%s: returned inside a critical region", what), bad = 1;
  if (vm.pinned) violation("%s: returned with %d arrays pinned", what, vm.pinned), bad = 1;
  if (vm.depth != 0) violation("%s: returned with %d local frames pushed", what, vm.depth), bad = 1;
  vm.critical = vm.pinned = 0;
  return bad;
}

static jint JNICALL f_GetVersion(JNIEnv* env) {
  (void)env;
  enter("GetVersion", 0, 0);
  return 0x00010008;
}

static jclass JNICALL f_FindClass(JNIEnv* env, const char* name) {
  (void)env;
  enter("FindClass", 0, 0);
  struct _jobject* o = calloc(1, sizeof *o);
  o->kind = K_CLASS;
  snprintf(o->name, sizeof o->name, "%s", name);
  new_local_ref("FindClass");
  return track(o);
}

static jint JNICALL f_ThrowNew(JNIEnv* env, jclass c, const char* msg) {
  (void)env;
  enter("ThrowNew", 0, 0);
  if (!c || c->kind != K_CLASS) violation("ThrowNew on a non-class");
  vm.pending = 1;
  snprintf(vm.exc_class, sizeof vm.exc_class, "%s", c->name);
  snprintf(vm.exc_msg, sizeof vm.exc_msg, "%s", msg ? msg : "");
  return 0;
}

static jint JNICALL f_PushLocalFrame(JNIEnv* env, jint cap) {
  (void)env;
  enter("PushLocalFrame", 1, 0);
  if (vm.depth + 1 >= 64) {
    violation("local frames nested too deep");
    return JNI_ERR;
  }
  vm.depth++;
  vm.frame_cap[vm.depth] = cap;
  vm.frame_refs[vm.depth] = 0;
  return JNI_OK;
}

static jobject JNICALL f_PopLocalFrame(JNIEnv* env, jobject result) {
  (void)env;
  enter("PopLocalFrame", 1, 0);
  if (vm.depth == 0) {
    violation("PopLocalFrame without PushLocalFrame");
    return result;
  }
  vm.depth--;
  if (result) new_local_ref("PopLocalFrame");
  return result;
}

static void JNICALL f_DeleteLocalRef(JNIEnv* env, jobject o) {
  (void)env;
  (void)o;
  enter("DeleteLocalRef", 1, 0);
  if (vm.frame_refs[vm.depth] > 0) vm.frame_refs[vm.depth]--;
}

static jint JNICALL f_EnsureLocalCapacity(JNIEnv* env, jint cap) {
  (void)env;
  enter("EnsureLocalCapacity", 0, 0);
  if (cap > vm.frame_cap[vm.depth] - vm.frame_refs[vm.depth]) vm.frame_cap[vm.depth] = vm.frame_refs[vm.depth] + cap;
  return JNI_OK;
}

static jsize JNICALL f_GetArrayLength(JNIEnv* env, jarray a) {
  (void)env;
  enter("GetArrayLength", 0, 0);
  if (!a || a->kind == K_CLASS) {
    violation("GetArrayLength on %s", a ? "a class" : "NULL");
    return 0;
  }
  return a->len;
}

static jobject JNICALL f_GetObjectArrayElement(JNIEnv* env, jobjectArray a, jsize i) {
  (void)env;
  enter("GetObjectArrayElement", 0, 0);
  if (!a || a->kind != K_OBJS || i < 0 || i >= a->len) {
    violation("GetObjectArrayElement(%d) out of range", (int)i);
    return NULL;
  }
  jobject v = ((jobject*)a->data)[i];
  if (v) new_local_ref("GetObjectArrayElement");
  return v;
}

static jintArray JNICALL f_NewIntArray(JNIEnv* env, jsize len) {
  (void)env;
  enter("NewIntArray", 0, 0);
  new_local_ref("NewIntArray");
  return new_ints(len, NULL);
}

static jint* JNICALL f_GetIntArrayElements(JNIEnv* env, jintArray a, jboolean* is_copy) {
  (void)env;
  enter("GetIntArrayElements", 0, 0);
  if (is_copy) *is_copy = JNI_FALSE;
  vm.pinned++;
  return ints_of(a);
}

static void JNICALL f_ReleaseIntArrayElements(JNIEnv* env, jintArray a, jint* e, jint mode) {
  (void)env;
  (void)a;
  (void)e;
  (void)mode;
  enter("ReleaseIntArrayElements", 1, 0);
  vm.pinned--;
}

static void JNICALL f_GetIntArrayRegion(JNIEnv* env, jintArray a, jsize start, jsize len, jint* buf) {
  (void)env;
  enter("GetIntArrayRegion", 0, 0);
  if (!a || a->kind != K_INTS || start < 0 || len < 0 || start + len > a->len) {
    violation("GetIntArrayRegion out of bounds");
    return;
  }
  memcpy(buf, ints_of(a) + start, (size_t)len * sizeof(jint));
}

static void JNICALL f_SetIntArrayRegion(JNIEnv* env, jintArray a, jsize start, jsize len, const jint* buf) {
  (void)env;
  enter("SetIntArrayRegion", 0, 0);
  if (!a || a->kind != K_INTS || start < 0 || len < 0 || start + len > a->len) {
    violation("SetIntArrayRegion out of bounds");
    return;
  }
  memcpy(ints_of(a) + start, buf, (size_t)len * sizeof(jint));
}

/* hrs_wait interposed (this executable's definition wins over libhrs's for
 * the shim): records the ticket the shim waited on last, so the fake JVM can
 * check that collect pins its output rows only after its round completed,
 * i.e. that no critical region covers a GPU wait. */
static uint64_t g_waited_ticket = 0;
static uint64_t g_collect_ticket = 0; /* nonzero while a collect call runs */
static int g_fail_wait = 0;           /* the next hrs_wait reports a device error */
hrs_status hrs_wait(hrs_codec* c, uint64_t t) {
  static hrs_status (*real)(hrs_codec*, uint64_t) = NULL;
  if (!real) *(void**)&real = dlsym(RTLD_NEXT, "hrs_wait");
  g_waited_ticket = t;
  if (g_fail_wait) {
    g_fail_wait = 0;
    return HRS_EDEVICE;
  }
  return real ? real(c, t) : HRS_EDEVICE;
}

static void* JNICALL f_GetPrimitiveArrayCritical(JNIEnv* env, jarray a, jboolean* is_copy) {
  (void)env;
  enter("GetPrimitiveArrayCritical", 0, 1);
  if (g_collect_ticket && g_waited_ticket != g_collect_ticket)
    violation("collect pinned a row before waiting for ticket %llu", (unsigned long long)g_collect_ticket);
  if (!a || (a->kind != K_BYTES && a->kind != K_INTS)) {
    violation("GetPrimitiveArrayCritical on a non-primitive array");
    return NULL;
  }
  if (is_copy) *is_copy = JNI_FALSE;
  vm.critical++;
  vm.pinned++;
  return a->data;
}

static void JNICALL f_ReleasePrimitiveArrayCritical(JNIEnv* env, jarray a, void* p, jint mode) {
  (void)env;
  (void)mode;
  enter("ReleasePrimitiveArrayCritical", 1, 1);
  if (!a || p != a->data) violation("ReleasePrimitiveArrayCritical of a pointer it did not hand out");
  vm.critical--;
  vm.pinned--;
}

static jboolean JNICALL f_ExceptionCheck(JNIEnv* env) {
  (void)env;
  enter("ExceptionCheck", 1, 0);
  return vm.pending ? JNI_TRUE : JNI_FALSE;
}

static struct JNINativeInterface_ table;
static JNIEnv env_ptr = &table;
static JNIEnv* env = &env_ptr;

static void init_table(void) {
  memset(&table, 0, sizeof table);
  table.GetVersion = f_GetVersion;
  table.FindClass = f_FindClass;
  table.ThrowNew = f_ThrowNew;
  table.PushLocalFrame = f_PushLocalFrame;
  table.PopLocalFrame = f_PopLocalFrame;
  table.DeleteLocalRef = f_DeleteLocalRef;
  table.EnsureLocalCapacity = f_EnsureLocalCapacity;
  table.GetArrayLength = f_GetArrayLength;
  table.GetObjectArrayElement = f_GetObjectArrayElement;
  table.NewIntArray = f_NewIntArray;
  table.GetIntArrayElements = f_GetIntArrayElements;
  table.ReleaseIntArrayElements = f_ReleaseIntArrayElements;
  table.GetIntArrayRegion = f_GetIntArrayRegion;
  table.SetIntArrayRegion = f_SetIntArrayRegion;
  table.GetPrimitiveArrayCritical = f_GetPrimitiveArrayCritical;
  table.ReleasePrimitiveArrayCritical = f_ReleasePrimitiveArrayCritical;
  table.ExceptionCheck = f_ExceptionCheck;
}

/* ----------------------------------------------- the shim's entry points */

JNIEXPORT jlong JNICALL Java_io_hops_erasure_1coding_HrsNative_create(JNIEnv*, jclass, jint, jint, jint, jint);
JNIEXPORT jlong JNICALL Java_io_hops_erasure_1coding_HrsNative_createSrc(JNIEnv*, jclass, jint, jint, jint, jint);
JNIEXPORT jint JNICALL Java_io_hops_erasure_1coding_HrsNative_deviceCount(JNIEnv*, jclass);
JNIEXPORT jint JNICALL Java_io_hops_erasure_1coding_HrsNative_device(JNIEnv*, jclass, jlong);
JNIEXPORT void JNICALL Java_io_hops_erasure_1coding_HrsNative_destroy(JNIEnv*, jclass, jlong);
JNIEXPORT jintArray JNICALL Java_io_hops_erasure_1coding_HrsNative_locationsToRead(JNIEnv*, jclass, jlong, jintArray);
JNIEXPORT void JNICALL Java_io_hops_erasure_1coding_HrsNative_encode(JNIEnv*, jclass, jlong, jobjectArray,
                                                                    jobjectArray, jint);
JNIEXPORT void JNICALL Java_io_hops_erasure_1coding_HrsNative_decode(JNIEnv*, jclass, jlong, jobjectArray,
                                                                    jobjectArray, jintArray, jintArray, jintArray,
                                                                    jint);
JNIEXPORT void JNICALL Java_io_hops_erasure_1coding_HrsNative_decode3(JNIEnv*, jclass, jlong, jobjectArray,
                                                                     jobjectArray, jintArray, jint);
JNIEXPORT void JNICALL Java_io_hops_erasure_1coding_HrsNative_encodeCrc(JNIEnv*, jclass, jlong, jobjectArray,
                                                                       jobjectArray, jint, jintArray);
JNIEXPORT void JNICALL Java_io_hops_erasure_1coding_HrsNative_decodeCrc(JNIEnv*, jclass, jlong, jobjectArray,
                                                                       jobjectArray, jintArray, jintArray, jintArray,
                                                                       jint, jintArray);

JNIEXPORT jlong JNICALL Java_io_hops_erasure_1coding_HrsNative_encodeSubmit(JNIEnv*, jclass, jlong, jobjectArray, jint,
                                                                           jboolean);
JNIEXPORT jlong JNICALL Java_io_hops_erasure_1coding_HrsNative_decodeSubmit(JNIEnv*, jclass, jlong, jobjectArray,
                                                                           jintArray, jintArray, jintArray, jint,
                                                                           jboolean);
JNIEXPORT void JNICALL Java_io_hops_erasure_1coding_HrsNative_collect(JNIEnv*, jclass, jlong, jlong, jobjectArray,
                                                                     jintArray);
JNIEXPORT jint JNICALL Java_io_hops_erasure_1coding_HrsNative_pending(JNIEnv*, jclass, jlong);

#define NS(f) Java_io_hops_erasure_1coding_HrsNative_##f

/* ---------------------------------------------------------------- checks */

static int checks, failures;
static char first_failure[512];

static void expect(int cond, const char* fmt, ...) {
  checks++;
  if (cond) return;
  va_list ap;
  va_start(ap, fmt);
  if (failures++ == 0) vsnprintf(first_failure, sizeof first_failure, fmt, ap);
  va_end(ap);
}

/* The exception the last native call left pending ("" for none). */
static const char* thrown(void) { return vm.pending ? vm.exc_class : ""; }

#define CALL(label, expr)           \
  do {                              \
    begin_native_call();            \
    expr;                           \
    end_native_call(label);         \
  } while (0)

/* HrsNative.collect with the wait-before-pin check armed (hrs_wait above). */
#define COLLECT(label, ticket, outs, crcs)                              \
  do {                                                                  \
    g_collect_ticket = (uint64_t)(ticket);                              \
    CALL(label, NS(collect)(env, NULL, h, (ticket), (outs), (crcs)));   \
    g_collect_ticket = 0;                                               \
  } while (0)

#define EXPECT_THROWN(label, cls, expr)                                                      \
  do {                                                                                       \
    CALL(label, expr);                                                                       \
    expect(strcmp(thrown(), cls) == 0, "%s: threw '%s' (%s), expected %s", label, thrown(), \
           vm.exc_msg, cls);                                                                 \
  } while (0)

static const char kNPE[] = "java/lang/NullPointerException";
static const char kIAE[] = "java/lang/IllegalArgumentException";
static const char kAIOOBE[] = "java/lang/ArrayIndexOutOfBoundsException";
static const char kISE[] = "java/lang/IllegalStateException";
static const char kIOE[] = "java/io/IOException";
static const char kTooMany[] = "io/hops/erasure_coding/TooManyErasedLocations";

static uint64_t splitmix(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static void fill(uint8_t* p, size_t n, uint64_t seed) {
  for (size_t i = 0; i < n; i += 8) {
    uint64_t x = splitmix(&seed);
    for (size_t j = 0; j < 8 && i + j < n; ++j) p[i + j] = (uint8_t)(x >> (8 * j));
  }
}

/* byte[rows][len], each row filled from seed + r (seed 0: zeros) */
static jobjectArray rows(int nrows, jsize len, uint64_t seed) {
  jobjectArray a = new_objs(nrows);
  for (int r = 0; r < nrows; r++) {
    jbyteArray b = new_bytes(len);
    if (seed) fill(bytes_of(b), (size_t)len, seed * 1000 + (uint64_t)r);
    set_obj(a, r, b);
  }
  return a;
}

static jbyteArray row(jobjectArray a, int i) { return ((jobject*)a->data)[i]; }

static int cpu_checks(void) {
  const int k = 10, p = 4, n = 14;
  const jsize L = 4096;
  hrs_opts o;
  memset(&o, 0, sizeof o);
  o.device = HRS_DEVICE_NONE;
  hrs_codec* c = NULL;
  if (hrs_create_code(HRS_CODE_RS, k, p, &o, &c) != HRS_OK) return 1;
  const jlong h = (jlong)(intptr_t)c;

  /* locationsToRead: ErasureCode.java:89-113 */
  int e7[] = {7};
  jintArray r = NULL;
  CALL("locationsToRead", r = NS(locationsToRead)(env, NULL, h, new_ints(1, e7)));
  const int want[] = {13, 12, 11, 10, 9, 8, 6, 5, 4, 3};
  expect(r && !vm.pending && r->len == 10 && memcmp(ints_of(r), want, sizeof want) == 0, "locationsToRead([7])");
  int e5[] = {0, 1, 2, 3, 4};
  EXPECT_THROWN("locationsToRead too many", kTooMany, NS(locationsToRead)(env, NULL, h, new_ints(5, e5)));
  EXPECT_THROWN("locationsToRead null", kNPE, NS(locationsToRead)(env, NULL, h, NULL));
  EXPECT_THROWN("locationsToRead 300", kIAE, NS(locationsToRead)(env, NULL, h, new_ints(300, NULL)));
  EXPECT_THROWN("released handle", kISE, NS(locationsToRead)(env, NULL, 0, new_ints(1, e7)));

  /* create: engine status -> exception class */
  EXPECT_THROWN("create RS(0,4)", kIAE, NS(create)(env, NULL, HRS_CODE_RS, 0, 4, -1));
  EXPECT_THROWN("create XOR(10,2)", kIAE, NS(create)(env, NULL, HRS_CODE_XOR, 10, 2, -1));
  EXPECT_THROWN("createSrc(10,4,5)", kIAE, NS(createSrc)(env, NULL, 10, 4, 5, -1));
  /* device set: an ordinal that is no visible device -> IOException (here
   * none is visible; on the GPU box gpu_checks tries deviceCount() itself) */
  {
    jint nd = -1;
    CALL("deviceCount", nd = NS(deviceCount)(env, NULL));
    expect(nd >= 0 && !vm.pending, "deviceCount");
    EXPECT_THROWN("create on device 4096", kIOE, NS(create)(env, NULL, HRS_CODE_RS, 10, 4, 4096));
    EXPECT_THROWN("create on device -7", kIOE, NS(create)(env, NULL, HRS_CODE_RS, 10, 4, -7));
    EXPECT_THROWN("createSrc on device 4096", kIOE, NS(createSrc)(env, NULL, 10, 6, 2, 4096));
    jint dv = 0;
    CALL("device of a host-only handle", dv = NS(device)(env, NULL, h));
    expect(dv == HRS_DEVICE_NONE && !vm.pending, "device() of a host-only handle: %d", (int)dv);
    EXPECT_THROWN("device of a released handle", kISE, NS(device)(env, NULL, 0));
  }
  CALL("destroy(0)", NS(destroy)(env, NULL, 0));
  expect(!vm.pending, "destroy(0) threw");

  /* encode: shapes */
  EXPECT_THROWN("encode ok shapes, host-only handle", kIOE, NS(encode)(env, NULL, h, rows(k, L, 1), rows(p, L, 0), L));
  EXPECT_THROWN("encode inputs null", kNPE, NS(encode)(env, NULL, h, NULL, rows(p, L, 0), L));
  EXPECT_THROWN("encode outputs null", kNPE, NS(encode)(env, NULL, h, rows(k, L, 1), NULL, L));
  EXPECT_THROWN("encode 9 inputs", kIAE, NS(encode)(env, NULL, h, rows(k - 1, L, 1), rows(p, L, 0), L));
  EXPECT_THROWN("encode 5 outputs", kIAE, NS(encode)(env, NULL, h, rows(k, L, 1), rows(p + 1, L, 0), L));
  EXPECT_THROWN("encode 300 inputs", kIAE, NS(encode)(env, NULL, h, rows(300, 1, 1), rows(p, 1, 0), 1));
  EXPECT_THROWN("encode negative len", kIAE, NS(encode)(env, NULL, h, rows(k, L, 1), rows(p, L, 0), -1));
  {
    jobjectArray in = rows(k, L, 1);
    set_obj(in, 3, new_bytes(L - 1));
    EXPECT_THROWN("encode short input row", kAIOOBE, NS(encode)(env, NULL, h, in, rows(p, L, 0), L));
    jobjectArray out = rows(p, L, 0);
    set_obj(out, 2, new_bytes(L / 2));
    EXPECT_THROWN("encode short output row", kAIOOBE, NS(encode)(env, NULL, h, rows(k, L, 1), out, L));
    jobjectArray in2 = rows(k, L, 1);
    set_obj(in2, 0, NULL);
    EXPECT_THROWN("encode null input row", kNPE, NS(encode)(env, NULL, h, in2, rows(p, L, 0), L));
    /* rows longer than len are fine: only len bytes are coded */
    EXPECT_THROWN("encode long rows", kIOE, NS(encode)(env, NULL, h, rows(k, L + 5, 1), rows(p, L + 9, 0), L));
  }
  EXPECT_THROWN("encodeCrc null crcs", kNPE, NS(encodeCrc)(env, NULL, h, rows(k, L, 1), rows(p, L, 0), L, NULL));
  EXPECT_THROWN("encodeCrc 13 crcs", kIAE,
                NS(encodeCrc)(env, NULL, h, rows(k, L, 1), rows(p, L, 0), L, new_ints(13, NULL)));
  EXPECT_THROWN("encodeCrc ok shapes", kIOE,
                NS(encodeCrc)(env, NULL, h, rows(k, L, 1), rows(p, L, 0), L, new_ints(14, NULL)));

  /* decode 5-arg: Decoder-style arrays for erased {4} */
  int er[] = {4}, tr[] = {3, 5, 6, 7, 8, 9, 10, 11, 12, 13}, ntr[] = {0, 1, 2, 4};
  jintArray E = new_ints(1, er), TR = new_ints(10, tr), NTR = new_ints(4, ntr);
  EXPECT_THROWN("decode ok shapes, host-only handle", kIOE,
                NS(decode)(env, NULL, h, rows(n, L, 2), rows(1, L, 0), E, TR, NTR, L));
  {
    jobjectArray rb = rows(n, L, 2);
    for (int j = 0; j < 4; j++) set_obj(rb, ntr[j], NULL); /* never read: may be null */
    EXPECT_THROWN("decode null not-to-read rows", kIOE, NS(decode)(env, NULL, h, rb, rows(1, L, 0), E, TR, NTR, L));
    jobjectArray rb2 = rows(n, L, 2);
    set_obj(rb2, 9, NULL); /* a location to read */
    EXPECT_THROWN("decode null read row", kNPE, NS(decode)(env, NULL, h, rb2, rows(1, L, 0), E, TR, NTR, L));
    jobjectArray rb3 = rows(n, L, 2);
    set_obj(rb3, 12, new_bytes(L - 7));
    EXPECT_THROWN("decode short read row", kAIOOBE, NS(decode)(env, NULL, h, rb3, rows(1, L, 0), E, TR, NTR, L));
    jobjectArray wb = rows(1, L, 0);
    set_obj(wb, 0, new_bytes(10));
    EXPECT_THROWN("decode short write row", kAIOOBE, NS(decode)(env, NULL, h, rows(n, L, 2), wb, E, TR, NTR, L));
  }
  int er2[] = {1, 4};
  EXPECT_THROWN("decode fewer writeBufs than erased", kAIOOBE,
                NS(decode)(env, NULL, h, rows(n, L, 2), rows(1, L, 0), new_ints(2, er2), TR, NTR, L));
  EXPECT_THROWN("decode 13 readBufs", kIAE, NS(decode)(env, NULL, h, rows(n - 1, L, 2), rows(1, L, 0), E, TR, NTR, L));
  EXPECT_THROWN("decode erased null", kNPE, NS(decode)(env, NULL, h, rows(n, L, 2), rows(1, L, 0), NULL, TR, NTR, L));
  EXPECT_THROWN("decode notToRead null", kNPE,
                NS(decode)(env, NULL, h, rows(n, L, 2), rows(1, L, 0), E, TR, NULL, L));
  EXPECT_THROWN("decode toRead null", kIOE, NS(decode)(env, NULL, h, rows(n, L, 2), rows(1, L, 0), E, NULL, NTR, L));
  EXPECT_THROWN("decode 300 erased", kIAE,
                NS(decode)(env, NULL, h, rows(n, L, 2), rows(1, L, 0), new_ints(300, NULL), TR, NTR, L));
  int bad_loc[] = {20};
  EXPECT_THROWN("decode notToRead location out of range", kIAE,
                NS(decode)(env, NULL, h, rows(n, L, 2), rows(1, L, 0), E, TR, new_ints(1, bad_loc), L));
  /* ReedSolomonCode only compares erased locations with notToRead ones: any
   * value passes validation (this host-only handle then fails on the device) */
  EXPECT_THROWN("decode erased location of any value", kIOE,
                NS(decode)(env, NULL, h, rows(n, L, 2), rows(1, L, 0), new_ints(1, bad_loc), TR, NTR, L));
  EXPECT_THROWN("decode3 ok shapes", kIOE, NS(decode3)(env, NULL, h, rows(n, L, 2), rows(1, L, 0), E, L));
  {
    jobjectArray rb = rows(n, L, 2);
    set_obj(rb, 0, NULL); /* the 3-arg decode reads every row */
    EXPECT_THROWN("decode3 null row", kNPE, NS(decode3)(env, NULL, h, rb, rows(1, L, 0), E, L));
  }
  EXPECT_THROWN("decodeCrc 2 crcs for 1 erased", kIAE,
                NS(decodeCrc)(env, NULL, h, rows(n, L, 2), rows(1, L, 0), E, TR, NTR, L, new_ints(2, NULL)));
  EXPECT_THROWN("decodeCrc ok shapes", kIOE,
                NS(decodeCrc)(env, NULL, h, rows(n, L, 2), rows(1, L, 0), E, TR, NTR, L, new_ints(1, NULL)));

  /* asynchronous rounds */
  EXPECT_THROWN("encodeSubmit host-only handle", kIOE, NS(encodeSubmit)(env, NULL, h, rows(k, L, 1), L, JNI_TRUE));
  EXPECT_THROWN("encodeSubmit 9 inputs", kIAE, NS(encodeSubmit)(env, NULL, h, rows(k - 1, L, 1), L, JNI_FALSE));
  {
    jobjectArray in = rows(k, L, 1);
    set_obj(in, 5, new_bytes(L - 2));
    EXPECT_THROWN("encodeSubmit short row", kAIOOBE, NS(encodeSubmit)(env, NULL, h, in, L, JNI_FALSE));
  }
  EXPECT_THROWN("decodeSubmit host-only handle", kIOE,
                NS(decodeSubmit)(env, NULL, h, rows(n, L, 2), E, TR, NTR, L, JNI_FALSE));
  EXPECT_THROWN("decodeSubmit erased null", kNPE,
                NS(decodeSubmit)(env, NULL, h, rows(n, L, 2), NULL, TR, NTR, L, JNI_FALSE));
  EXPECT_THROWN("collect unknown ticket", kIAE, NS(collect)(env, NULL, h, 12345, rows(p, L, 0), NULL));
  {
    jint pend = -1;
    CALL("pending", pend = NS(pending)(env, NULL, h));
    expect(pend == 0 && !vm.pending, "pending on an idle handle");
  }
  hrs_destroy(c);
  return 0;
}

static uint32_t zcrc(uint32_t c, const uint8_t* p, size_t n) { return (uint32_t)crc32(c, p, (uInt)n); }

/* HipReedSolomonCode.decode 5-arg (lambdafs_amd/jni/HipReedSolomonCode.java),
 * transcribed: zero data at locationsNotToRead, one-byte rows through
 * HrsNative.decode, then copy out[i] only where erasedLocations[i] is one of
 * locationsNotToRead (ReedSolomonCode.java:158-165). Compared with the
 * oracle's ReedSolomonCode.decode on pre-filled erasedValues. */
static void java_scalar_decode5(jlong h, int* data, int n, const int* erased, int ne, int* values, const int* ntr,
                                int nn) {
  for (int j = 0; j < nn; j++) data[ntr[j]] = 0;
  jobjectArray rb = new_objs(n);
  for (int i = 0; i < n; i++) {
    jbyteArray b = new_bytes(1);
    bytes_of(b)[0] = (uint8_t)data[i];
    set_obj(rb, i, b);
  }
  jobjectArray out = rows(ne, 1, 0);
  CALL("scalar decode5 (HrsNative.decode, 1-byte rows)",
       NS(decode)(env, NULL, h, rb, out, new_ints(ne, erased), new_ints(0, NULL), new_ints(nn, ntr), 1));
  for (int i = 0; i < ne; i++)
    for (int j = 0; j < nn; j++)
      if (erased[i] == ntr[j]) {
        values[i] = bytes_of(row(out, i))[0];
        break;
      }
}

static void scalar_decode5_checks(jlong h, int k, int p) {
  const int n = k + p;
  uint64_t seed = 0x5CA1A7ull;
  for (int it = 0; it < 24; it++) {
    int data[64], dref[64], ntr[16], er[16], v[16], vref[16];
    for (int i = 0; i < n; i++) data[i] = dref[i] = (int)(splitmix(&seed) & 0xFF);
    /* not-to-read: 1..p distinct locations; erased: some of them plus 1-2 outside */
    int nn = 1 + (int)(splitmix(&seed) % (uint64_t)p), ne = 0;
    for (int j = 0; j < nn; j++) {
      int loc, dup;
      do {
        loc = (int)(splitmix(&seed) % (uint64_t)n);
        dup = 0;
        for (int q = 0; q < j; q++) dup |= ntr[q] == loc;
      } while (dup);
      ntr[j] = loc;
      if (splitmix(&seed) & 1) er[ne++] = loc;
    }
    for (int extra = 1 + (int)(splitmix(&seed) & 1), loc = 0; extra > 0 && loc < n; loc++) {
      int in = 0;
      for (int j = 0; j < nn; j++) in |= ntr[j] == loc;
      if (!in && (splitmix(&seed) % 3) == 0) er[ne++] = loc, extra--;
    }
    if (ne == 0) continue;
    for (int i = 0; i < ne; i++) v[i] = vref[i] = 0x40 + it + i; /* pre-filled erasedValues */
    java_scalar_decode5(h, data, n, er, ne, v, ntr, nn);
    orc_rs_decode5(k, p, dref, er, ne, vref, NULL, 0, ntr, nn);
    int same = !vm.pending && memcmp(v, vref, sizeof(int) * (size_t)ne) == 0 &&
               memcmp(data, dref, sizeof(int) * (size_t)n) == 0;
    expect(same, "scalar decode5 round %d: erasedValues or data differ from ReedSolomonCode.decode", it);
  }
}

/* Location lists with repeated entries (and a 5-arg erased value outside the
 * stripe), which ReedSolomonCode accepts: its solve divides by zero there and
 * divTable[y][0] = 0 (GaloisField.java:107-118). Bulk 5-arg and 3-arg through
 * HrsNative vs the oracle's bulk loops on ragged rows; the scalar 5-arg and
 * 3-arg decode as HipReedSolomonCode.decode does them vs ReedSolomonCode.decode. */
static void repeated_location_checks(jlong h, int k, int p) {
  const int n = k + p;
  const jsize L = 4099;
  static const struct { int ne, nn, er[4], ntr[4]; } cases[] = {
      {1, 2, {3}, {3, 3}}, {2, 3, {3, 5}, {3, 5, 5}}, {2, 3, {3, 3}, {3, 5, 5}},
      {1, 4, {4}, {4, 4, 4, 4}}, {3, 2, {99, -1, 4}, {4, 2}}, {2, 3, {0, 13}, {13, 0, 13}}};
  for (size_t c = 0; c < sizeof cases / sizeof cases[0]; c++) {
    const int ne = cases[c].ne, nn = cases[c].nn;
    jobjectArray rb = rows(n, L, 31 + (int)c);
    uint8_t* ref_in[16];
    uint8_t* ref_out[4];
    for (int l = 0; l < n; l++) {
      ref_in[l] = malloc((size_t)L);
      memcpy(ref_in[l], bytes_of(row(rb, l)), (size_t)L);
    }
    for (int t = 0; t < ne; t++) ref_out[t] = calloc(1, (size_t)L);
    orc_rs_decode_bulk5(k, p, ref_in, ref_out, cases[c].er, ne, NULL, 0, cases[c].ntr, nn, (size_t)L);
    jobjectArray wb = rows(ne, L, 0);
    CALL("decode, repeated locations",
         NS(decode)(env, NULL, h, rb, wb, new_ints(ne, cases[c].er), new_ints(0, NULL), new_ints(nn, cases[c].ntr), L));
    expect(!vm.pending, "decode case %d threw %s: %s", (int)c, vm.exc_class, vm.exc_msg);
    for (int t = 0; t < ne; t++)
      expect(memcmp(bytes_of(row(wb, t)), ref_out[t], (size_t)L) == 0, "repeated-location decode case %d output %d", (int)c, t);
    /* scalar 5-arg on column 0 */
    int data[16], dref[16], v[4], vref[4];
    for (int l = 0; l < n; l++) data[l] = dref[l] = ref_in[l][0];
    for (int t = 0; t < ne; t++) v[t] = vref[t] = 0x70 + t;
    java_scalar_decode5(h, data, n, cases[c].er, ne, v, cases[c].ntr, nn);
    orc_rs_decode5(k, p, dref, cases[c].er, ne, vref, NULL, 0, cases[c].ntr, nn);
    expect(!vm.pending && memcmp(v, vref, sizeof(int) * (size_t)ne) == 0, "scalar decode5 repeated case %d", (int)c);
    for (int l = 0; l < n; l++) free(ref_in[l]);
    for (int t = 0; t < ne; t++) free(ref_out[t]);
  }
  static const struct { int ne, er[4]; } cases3[] = {{2, {3, 3}}, {3, {1, 5, 1}}, {4, {2, 2, 2, 2}}, {3, {13, 0, 13}}};
  for (size_t c = 0; c < sizeof cases3 / sizeof cases3[0]; c++) {
    const int ne = cases3[c].ne;
    jobjectArray rb = rows(n, L, 41 + (int)c);
    uint8_t* ref_in[16];
    uint8_t* ref_out[4];
    for (int l = 0; l < n; l++) {
      ref_in[l] = malloc((size_t)L);
      memcpy(ref_in[l], bytes_of(row(rb, l)), (size_t)L);
    }
    for (int t = 0; t < ne; t++) ref_out[t] = calloc(1, (size_t)L);
    orc_rs_decode_bulk3(k, p, ref_in, ref_out, cases3[c].er, ne, (size_t)L);
    jobjectArray wb = rows(ne, L, 0);
    CALL("decode3, repeated locations", NS(decode3)(env, NULL, h, rb, wb, new_ints(ne, cases3[c].er), L));
    expect(!vm.pending, "decode3 case %d threw %s: %s", (int)c, vm.exc_class, vm.exc_msg);
    for (int t = 0; t < ne; t++)
      expect(memcmp(bytes_of(row(wb, t)), ref_out[t], (size_t)L) == 0, "repeated-location decode3 case %d output %d", (int)c, t);
    /* scalar 3-arg as HipReedSolomonCode.decode(data, erased, values): zero
     * data[erased], one-byte rows through HrsNative.decode3, copy every output */
    int data[16], dref[16], vref[4];
    for (int l = 0; l < n; l++) data[l] = dref[l] = ref_in[l][7];
    for (int t = 0; t < ne; t++) data[cases3[c].er[t]] = 0;
    jobjectArray r1 = new_objs(n);
    for (int l = 0; l < n; l++) {
      jbyteArray b = new_bytes(1);
      bytes_of(b)[0] = (uint8_t)data[l];
      set_obj(r1, l, b);
    }
    jobjectArray o1 = rows(ne, 1, 0);
    CALL("scalar decode3 (HrsNative.decode3, 1-byte rows)", NS(decode3)(env, NULL, h, r1, o1, new_ints(ne, cases3[c].er), 1));
    orc_rs_decode3(k, p, dref, cases3[c].er, ne, vref);
    int same = !vm.pending;
    for (int t = 0; t < ne; t++) same &= bytes_of(row(o1, t))[0] == (uint8_t)vref[t];
    expect(same, "scalar decode3 repeated case %d", (int)c);
    for (int l = 0; l < n; l++) free(ref_in[l]);
    for (int t = 0; t < ne; t++) free(ref_out[t]);
  }
}

static int gpu_checks(void) {
  const int k = 10, p = 4, n = 14;
  const jsize L = 1 << 20;
  jlong h = 0;
  /* device set: explicit ordinals as HipDevices.pick hands them out */
  jint ndev = 0;
  CALL("deviceCount", ndev = NS(deviceCount)(env, NULL));
  expect(ndev >= 1 && !vm.pending, "deviceCount on the GPU box: %d", (int)ndev);
  for (jint d = 0; d < ndev && d < 8; ++d) {
    jlong hd = 0;
    jint got = -1;
    CALL("create on device d", hd = NS(create)(env, NULL, HRS_CODE_RS, k, p, d));
    CALL("device()", got = hd ? NS(device)(env, NULL, hd) : -1);
    expect(hd != 0 && got == d && !vm.pending, "create on device %d -> handle on %d", (int)d, (int)got);
    if (hd) CALL("destroy", NS(destroy)(env, NULL, hd));
  }
  EXPECT_THROWN("create on device deviceCount()", kIOE, NS(create)(env, NULL, HRS_CODE_RS, k, p, ndev));
  EXPECT_THROWN("createSrc on device deviceCount()", kIOE, NS(createSrc)(env, NULL, 10, 6, 2, ndev));
  CALL("create RS(10,4)", h = NS(create)(env, NULL, HRS_CODE_RS, k, p, 0));
  expect(h != 0 && !vm.pending, "create RS(10,4) on the GPU: %s", vm.exc_msg);
  if (!h) return 1;
  scalar_decode5_checks(h, k, p);
  repeated_location_checks(h, k, p);

  /* encode vs oracle encodeBulk */
  jobjectArray in = rows(k, L, 7), out = rows(p, L, 0);
  CALL("encode", NS(encode)(env, NULL, h, in, out, L));
  expect(!vm.pending, "encode threw %s: %s", vm.exc_class, vm.exc_msg);
  uint8_t* ref_in[16];
  uint8_t* ref_out[16];
  for (int i = 0; i < k; i++) {
    ref_in[i] = malloc((size_t)L);
    memcpy(ref_in[i], bytes_of(row(in, i)), (size_t)L);
  }
  for (int r = 0; r < p; r++) ref_out[r] = calloc(1, (size_t)L);
  orc_rs_encode_bulk(k, p, ref_in, ref_out, (size_t)L); /* zeroes ref_in, like the Java */
  for (int r = 0; r < p; r++)
    expect(memcmp(bytes_of(row(out, r)), ref_out[r], (size_t)L) == 0, "encode parity %d differs from the oracle", r);

  /* encodeCrc: running CRCs continued (CRC32.update chaining) */
  int crcs0[14];
  for (int i = 0; i < 14; i++) crcs0[i] = (int)(0x1234567u * (unsigned)(i + 1));
  jintArray crcs = new_ints(14, crcs0);
  jobjectArray out2 = rows(p, L, 0);
  CALL("encodeCrc", NS(encodeCrc)(env, NULL, h, in, out2, L, crcs));
  expect(!vm.pending, "encodeCrc threw %s: %s", vm.exc_class, vm.exc_msg);
  for (int r = 0; r < p; r++)
    expect(memcmp(bytes_of(row(out2, r)), ref_out[r], (size_t)L) == 0, "encodeCrc parity %d", r);
  for (int i = 0; i < 14; i++) {
    const uint8_t* b = i < k ? bytes_of(row(in, i)) : ref_out[i - k];
    expect((uint32_t)ints_of(crcs)[i] == zcrc((uint32_t)crcs0[i], b, (size_t)L), "encodeCrc crc %d", i);
  }

  /* decode 5-arg on NON-codeword rows vs the oracle's per-byte decodeBulk:
   * erased {1, 4} (parity 1, data 0), Decoder.java:303-338 arrays */
  int er[] = {1, 4};
  int tr_desc[10];
  const int ntrd = orc_locations_to_read(k, p, er, 2, tr_desc);
  int tr[10];
  for (int i = 0; i < ntrd; i++) tr[i] = tr_desc[ntrd - 1 - i];
  int ntr[4], nn = 0;
  for (int l = 0; l < n; l++) {
    int rd = 0;
    for (int i = 0; i < ntrd; i++) rd |= tr[i] == l;
    if (!rd) ntr[nn++] = l;
  }
  jobjectArray rb = rows(n, L, 9);
  uint8_t* zeros_rows[16];
  for (int l = 0; l < n; l++) {
    int skip = 0;
    for (int j = 0; j < nn; j++) skip |= ntr[j] == l;
    if (skip) {
      memset(bytes_of(row(rb, l)), 0, (size_t)L); /* StripeReader.java:111-120 */
      if (l == 0) set_obj(rb, l, NULL);            /* and one of them not passed at all */
    }
    zeros_rows[l] = malloc((size_t)L);
    if (row(rb, l))
      memcpy(zeros_rows[l], bytes_of(row(rb, l)), (size_t)L);
    else
      memset(zeros_rows[l], 0, (size_t)L);
  }
  jobjectArray wb = rows(2, L, 0);
  CALL("decode", NS(decode)(env, NULL, h, rb, wb, new_ints(2, er), new_ints(ntrd, tr), new_ints(nn, ntr), L));
  expect(!vm.pending, "decode threw %s: %s", vm.exc_class, vm.exc_msg);
  uint8_t* ref_w[2] = {calloc(1, (size_t)L), calloc(1, (size_t)L)};
  orc_rs_decode_bulk5(k, p, zeros_rows, ref_w, er, 2, tr, ntrd, ntr, nn, (size_t)L);
  for (int t = 0; t < 2; t++)
    expect(memcmp(bytes_of(row(wb, t)), ref_w[t], (size_t)L) == 0, "decode output %d differs from the oracle", t);

  /* decodeCrc: same outputs, CRCs continued from running values */
  int dc0[2] = {0, (int)0xdeadbeefu};
  jintArray dcrc = new_ints(2, dc0);
  jobjectArray wb2 = rows(2, L, 0);
  CALL("decodeCrc",
       NS(decodeCrc)(env, NULL, h, rb, wb2, new_ints(2, er), new_ints(ntrd, tr), new_ints(nn, ntr), L, dcrc));
  expect(!vm.pending, "decodeCrc threw %s: %s", vm.exc_class, vm.exc_msg);
  for (int t = 0; t < 2; t++) {
    expect(memcmp(bytes_of(row(wb2, t)), ref_w[t], (size_t)L) == 0, "decodeCrc output %d", t);
    expect((uint32_t)ints_of(dcrc)[t] == zcrc((uint32_t)dc0[t], ref_w[t], (size_t)L), "decodeCrc crc %d", t);
  }

  /* decode3 vs the oracle's bulk 3-arg decode (all rows read as given) */
  int er3[] = {4, 9};
  jobjectArray rb3 = rows(n, L, 11);
  uint8_t* rows3[16];
  for (int l = 0; l < n; l++) {
    rows3[l] = malloc((size_t)L);
    memcpy(rows3[l], bytes_of(row(rb3, l)), (size_t)L);
  }
  jobjectArray wb3 = rows(2, L, 0);
  CALL("decode3", NS(decode3)(env, NULL, h, rb3, wb3, new_ints(2, er3), L));
  expect(!vm.pending, "decode3 threw %s: %s", vm.exc_class, vm.exc_msg);
  uint8_t* ref3[2] = {calloc(1, (size_t)L), calloc(1, (size_t)L)};
  orc_rs_decode_bulk3(k, p, rows3, ref3, er3, 2, (size_t)L);
  for (int t = 0; t < 2; t++)
    expect(memcmp(bytes_of(row(wb3, t)), ref3[t], (size_t)L) == 0, "decode3 output %d differs from the oracle", t);

  /* round trip: the codeword's erased cells come back */
  jobjectArray cw = new_objs(n);
  for (int r = 0; r < p; r++) set_obj(cw, r, row(out, r));
  for (int i = 0; i < k; i++) set_obj(cw, p + i, row(in, i));
  int er1[] = {4};
  int tr1[] = {3, 5, 6, 7, 8, 9, 10, 11, 12, 13}, ntr1[] = {0, 1, 2, 4};
  jobjectArray wb1 = rows(1, L, 0);
  CALL("decode round trip", NS(decode)(env, NULL, h, cw, wb1, new_ints(1, er1), new_ints(10, tr1), new_ints(4, ntr1), L));
  expect(!vm.pending && memcmp(bytes_of(row(wb1, 0)), bytes_of(row(in, 0)), (size_t)L) == 0, "decode round trip");

  /* short rows on a live handle: rejected before anything is pinned or
   * touched (a read or write past the row would hit its guard page) */
  {
    jobjectArray sin = rows(k, L, 7);
    set_obj(sin, 9, new_bytes(L - 1));
    jobjectArray sout = rows(p, L, 0);
    memset(bytes_of(row(sout, 0)), 0xA5, (size_t)L);
    EXPECT_THROWN("live encode short input", kAIOOBE, NS(encode)(env, NULL, h, sin, sout, L));
    int untouched = 1;
    for (jsize i = 0; i < L; i++) untouched &= bytes_of(row(sout, 0))[i] == 0xA5;
    expect(untouched, "outputs written by a rejected encode");
    jobjectArray swb = rows(1, L, 0);
    set_obj(swb, 0, new_bytes(L - 4096));
    EXPECT_THROWN("live decode short write", kAIOOBE,
                  NS(decode)(env, NULL, h, cw, swb, new_ints(1, er1), new_ints(10, tr1), new_ints(4, ntr1), L));
    /* a short length is fine: rows longer than len */
    jobjectArray lo = rows(p, L, 0);
    CALL("encode prefix", NS(encode)(env, NULL, h, in, lo, 4096 + 3));
    int same = !vm.pending;
    for (int r = 0; r < p; r++) same &= memcmp(bytes_of(row(lo, r)), ref_out[r], 4096 + 3) == 0;
    expect(same, "encode of a row prefix");
  }
  /* asynchronous Encoder rounds, depth 2: submit round r, collect round r - 1
   * (parity vs the oracle, CRC32s chained across rounds vs zlib) */
  {
    const int R = 4;
    const jsize Lr = 1 << 20;
    jobjectArray rin[4];
    jlong tk[4];
    uint32_t want[14];
    memset(want, 0, sizeof want);
    jintArray run = new_ints(14, NULL);
    int ok = 1;
    for (int r = 0; r <= R; ++r) {
      if (r < R) {
        rin[r] = rows(k, Lr, 40 + (uint64_t)r);
        for (int i = 0; i < k; i++) want[i] = zcrc(want[i], bytes_of(row(rin[r], i)), (size_t)Lr);
        CALL("encodeSubmit", tk[r] = NS(encodeSubmit)(env, NULL, h, rin[r], Lr, JNI_TRUE));
        ok &= !vm.pending && tk[r] != 0;
      }
      if (r >= 1) {
        const int q = r - 1;
        jobjectArray out = rows(p, Lr, 0);
        COLLECT("collect", tk[q], out, run);
        ok &= !vm.pending;
        uint8_t* ri[10];
        uint8_t* ro[4];
        for (int i = 0; i < k; i++) {
          ri[i] = malloc((size_t)Lr);
          memcpy(ri[i], bytes_of(row(rin[q], i)), (size_t)Lr);
        }
        for (int o = 0; o < p; o++) ro[o] = calloc(1, (size_t)Lr);
        orc_rs_encode_bulk(k, p, ri, ro, (size_t)Lr);
        for (int o = 0; o < p; o++) {
          ok &= memcmp(bytes_of(row(out, o)), ro[o], (size_t)Lr) == 0;
          want[k + o] = zcrc(want[k + o], ro[o], (size_t)Lr);
          free(ro[o]);
        }
        for (int i = 0; i < k; i++) free(ri[i]);
      }
    }
    for (int i = 0; i < 14; i++) ok &= (uint32_t)ints_of(run)[i] == want[i];
    jint pend = -1;
    CALL("pending", pend = NS(pending)(env, NULL, h));
    expect(ok && pend == 0, "async encode rounds (depth 2, chained CRCs) vs the oracle and zlib");
    /* an asynchronous decode round (the 5-arg decodeBulk of a codeword) */
    jlong td = 0;
    CALL("decodeSubmit",
         td = NS(decodeSubmit)(env, NULL, h, cw, new_ints(1, er1), new_ints(10, tr1), new_ints(4, ntr1), L, JNI_TRUE));
    jobjectArray dw = rows(1, L, 0);
    jintArray dc = new_ints(1, NULL);
    COLLECT("collect decode", td, dw, dc);
    expect(!vm.pending && memcmp(bytes_of(row(dw, 0)), bytes_of(row(in, 0)), (size_t)L) == 0 &&
               (uint32_t)ints_of(dc)[0] == zcrc(0, bytes_of(row(in, 0)), (size_t)L),
           "async decode round + repaired CRC");
    /* the slot limit: 4 outstanding rounds, the 5th is refused */
    jlong t5[5];
    for (int r = 0; r < 4; ++r) CALL("encodeSubmit x4", t5[r] = NS(encodeSubmit)(env, NULL, h, in, 4096, JNI_FALSE));
    EXPECT_THROWN("fifth outstanding round", kIAE, t5[4] = NS(encodeSubmit)(env, NULL, h, in, 4096, JNI_FALSE));
    for (int r = 3; r >= 0; --r) COLLECT("collect out of order", t5[r], rows(p, 4096, 0), NULL);
    expect(!vm.pending, "collect in any order");
    /* a collect whose wait fails throws IOException AND frees the
     * round's slot (hrs_release), so the handle keeps its 4 slots */
    jlong tf = 0;
    CALL("encodeSubmit (wait fails)", tf = NS(encodeSubmit)(env, NULL, h, in, 4096, JNI_FALSE));
    g_fail_wait = 1;
    g_collect_ticket = (uint64_t)tf;
    EXPECT_THROWN("collect after a failed wait", kIOE, NS(collect)(env, NULL, h, tf, rows(p, 4096, 0), NULL));
    g_collect_ticket = 0;
    jint pend_f = -1;
    CALL("pending after the failed collect", pend_f = NS(pending)(env, NULL, h));
    expect(pend_f == 0, "a failed collect releases its slot (pending %d)", (int)pend_f);
    for (int r = 0; r < 4; ++r) CALL("encodeSubmit x4 again", t5[r] = NS(encodeSubmit)(env, NULL, h, in, 4096, JNI_FALSE));
    expect(!vm.pending, "all 4 slots usable after the failed collect");
    for (int r = 0; r < 4; ++r) COLLECT("collect x4 again", t5[r], rows(p, 4096, 0), NULL);
  }
  CALL("destroy", NS(destroy)(env, NULL, h));

  /* the other code families through the same shim */
  {
    jlong hx = 0;
    CALL("create XOR", hx = NS(create)(env, NULL, HRS_CODE_XOR, 10, 1, -1));
    jobjectArray xin = rows(10, 70000, 21), xout = rows(1, 70000, 0);
    CALL("xor encode", NS(encode)(env, NULL, hx, xin, xout, 70000));
    uint8_t* xr[10];
    for (int i = 0; i < 10; i++) xr[i] = bytes_of(row(xin, i));
    uint8_t* xo = calloc(1, 70000);
    orc_xor_encode_bulk(10, xr, xo, 70000);
    expect(hx && !vm.pending && memcmp(bytes_of(row(xout, 0)), xo, 70000) == 0, "xor encode");
    free(xo);
    CALL("destroy XOR", NS(destroy)(env, NULL, hx));

    jlong hn = 0;
    CALL("create NRS", hn = NS(create)(env, NULL, HRS_CODE_NRS, 10, 4, 0));
    jobjectArray nin = rows(10, 65536, 23), nout = rows(4, 65536, 0);
    CALL("nrs encode", NS(encode)(env, NULL, hn, nin, nout, 65536));
    uint8_t* ni[10];
    uint8_t* no[4];
    for (int i = 0; i < 10; i++) ni[i] = bytes_of(row(nin, i));
    for (int r = 0; r < 4; r++) no[r] = calloc(1, 65536);
    orc_nrs_encode_bulk(10, 4, ni, no, 65536);
    int ok = hn && !vm.pending;
    for (int r = 0; r < 4; r++) ok &= memcmp(bytes_of(row(nout, r)), no[r], 65536) == 0, free(no[r]);
    expect(ok, "nrs encode");
    CALL("destroy NRS", NS(destroy)(env, NULL, hn));

    jlong hs = 0;
    CALL("createSrc", hs = NS(createSrc)(env, NULL, 10, 6, 2, 0));
    jobjectArray sin = rows(10, 40000, 25), sout = rows(6, 40000, 0);
    CALL("src encode", NS(encode)(env, NULL, hs, sin, sout, 40000));
    uint8_t* si[10];
    uint8_t* so[6];
    for (int i = 0; i < 10; i++) si[i] = bytes_of(row(sin, i));
    for (int r = 0; r < 6; r++) so[r] = calloc(1, 40000);
    orc_src_encode_bulk(10, 6, 2, si, so, 40000);
    ok = hs && !vm.pending;
    for (int r = 0; r < 6; r++) ok &= memcmp(bytes_of(row(sout, r)), so[r], 40000) == 0, free(so[r]);
    expect(ok, "src encode");
    CALL("destroy SRC", NS(destroy)(env, NULL, hs));
  }
  for (int i = 0; i < k; i++) free(ref_in[i]);
  for (int r = 0; r < p; r++) free(ref_out[r]);
  for (int l = 0; l < n; l++) free(zeros_rows[l]), free(rows3[l]);
  free(ref_w[0]), free(ref_w[1]), free(ref3[0]), free(ref3[1]);
  return 0;
}

int main(int argc, char** argv) {
  const int gpu = argc > 1 && strcmp(argv[1], "--gpu") == 0;
  init_table();
  const int rc = gpu ? gpu_checks() : cpu_checks();
  free_heap();
  const int ok = rc == 0 && failures == 0 && vm.violations == 0;
  printf("{\"mode\": \"%s\", \"ok\": %s, \"checks\": %d, \"failures\": %d, \"first_failure\": \"%s\", "
         "\"jni_calls\": %d, \"jni_rule_violations\": %d, \"first_violation\": \"%s\"}\n",
         gpu ? "gpu" : "cpu", ok ? "true" : "false", checks, failures, first_failure, vm.calls, vm.violations,
         vm.first_violation);
  return ok ? 0 : 1;
}
