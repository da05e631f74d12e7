/*
 * jni_min.h — the subset of the JNI ABI that hrs_jni.c uses, declared by
 * hand so the shim compiles (and is tested through a fake JNIEnv) in an image
 * without a JDK. Everything here is the published, frozen JNI binary
 * interface: the primitive types, the reference types as opaque pointers, and
 * the JNIEnv function table with every entry at its specified index (JNI
 * specification, "Interface Function Table"). Slots the shim never calls are
 * padding of the same width; static asserts below pin each used entry's
 * offset to index * sizeof(void*), so a call through this header dispatches
 * to the same slot as one compiled against the JDK's <jni.h>.
 *
 * Build with a real JDK instead: -DHRS_SYSTEM_JNI -I$JAVA_HOME/include
 * -I$JAVA_HOME/include/linux (hrs_jni.c then includes <jni.h>).
 */
#ifndef HRS_JNI_MIN_H_
#define HRS_JNI_MIN_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JNIEXPORT __attribute__((visibility("default")))
#define JNIIMPORT
#define JNICALL

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef uint16_t jchar;
typedef int16_t jshort;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jthrowable;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jobjectArray;
typedef jarray jbyteArray;
typedef jarray jintArray;

#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_OK 0
#define JNI_ERR (-1)
#define JNI_COMMIT 1
#define JNI_ABORT 2

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

/* Index in the JNI function table: comments give the specified index. */
struct JNINativeInterface_ {
  void* reserved0;                                                     /* 0 */
  void* reserved1;                                                     /* 1 */
  void* reserved2;                                                     /* 2 */
  void* reserved3;                                                     /* 3 */
  jint(JNICALL* GetVersion)(JNIEnv* env);                              /* 4 */
  void* DefineClass;                                                   /* 5 */
  jclass(JNICALL* FindClass)(JNIEnv* env, const char* name);           /* 6 */
  void* unused_7_13[7];                                                /* 7-13 */
  jint(JNICALL* ThrowNew)(JNIEnv* env, jclass clazz, const char* msg); /* 14 */
  void* ExceptionOccurred;                                             /* 15 */
  void* ExceptionDescribe;                                             /* 16 */
  void* ExceptionClear;                                                /* 17 */
  void* FatalError;                                                    /* 18 */
  jint(JNICALL* PushLocalFrame)(JNIEnv* env, jint capacity);           /* 19 */
  jobject(JNICALL* PopLocalFrame)(JNIEnv* env, jobject result);        /* 20 */
  void* NewGlobalRef;                                                  /* 21 */
  void* DeleteGlobalRef;                                               /* 22 */
  void(JNICALL* DeleteLocalRef)(JNIEnv* env, jobject obj);             /* 23 */
  void* IsSameObject;                                                  /* 24 */
  void* NewLocalRef;                                                   /* 25 */
  jint(JNICALL* EnsureLocalCapacity)(JNIEnv* env, jint capacity);      /* 26 */
  void* unused_27_170[144];                                            /* 27-170 */
  jsize(JNICALL* GetArrayLength)(JNIEnv* env, jarray array);           /* 171 */
  void* NewObjectArray;                                                /* 172 */
  jobject(JNICALL* GetObjectArrayElement)(JNIEnv* env, jobjectArray array, jsize index); /* 173 */
  void* SetObjectArrayElement;                                         /* 174 */
  void* unused_175_178[4];                                             /* 175-178 */
  jintArray(JNICALL* NewIntArray)(JNIEnv* env, jsize len);             /* 179 */
  void* unused_180_186[7];                                             /* 180-186 */
  jint*(JNICALL* GetIntArrayElements)(JNIEnv* env, jintArray array, jboolean* isCopy); /* 187 */
  void* unused_188_194[7];                                             /* 188-194 */
  void(JNICALL* ReleaseIntArrayElements)(JNIEnv* env, jintArray array, jint* elems, jint mode); /* 195 */
  void* unused_196_202[7];                                             /* 196-202 */
  void(JNICALL* GetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len, jint* buf); /* 203 */
  void* unused_204_210[7];                                             /* 204-210 */
  void(JNICALL* SetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len,
                                   const jint* buf);                   /* 211 */
  void* unused_212_221[10];                                            /* 212-221 */
  void*(JNICALL* GetPrimitiveArrayCritical)(JNIEnv* env, jarray array, jboolean* isCopy); /* 222 */
  void(JNICALL* ReleasePrimitiveArrayCritical)(JNIEnv* env, jarray array, void* carray, jint mode); /* 223 */
  void* unused_224_227[4];                                             /* 224-227 */
  jboolean(JNICALL* ExceptionCheck)(JNIEnv* env);                      /* 228 */
};

#define HRS_JNI_SLOT(f, i) \
  _Static_assert(offsetof(struct JNINativeInterface_, f) == (i) * sizeof(void*), "JNI slot " #f)
HRS_JNI_SLOT(GetVersion, 4);
HRS_JNI_SLOT(FindClass, 6);
HRS_JNI_SLOT(ThrowNew, 14);
HRS_JNI_SLOT(PushLocalFrame, 19);
HRS_JNI_SLOT(PopLocalFrame, 20);
HRS_JNI_SLOT(DeleteLocalRef, 23);
HRS_JNI_SLOT(EnsureLocalCapacity, 26);
HRS_JNI_SLOT(GetArrayLength, 171);
HRS_JNI_SLOT(GetObjectArrayElement, 173);
HRS_JNI_SLOT(NewIntArray, 179);
HRS_JNI_SLOT(GetIntArrayElements, 187);
HRS_JNI_SLOT(ReleaseIntArrayElements, 195);
HRS_JNI_SLOT(GetIntArrayRegion, 203);
HRS_JNI_SLOT(SetIntArrayRegion, 211);
HRS_JNI_SLOT(GetPrimitiveArrayCritical, 222);
HRS_JNI_SLOT(ReleasePrimitiveArrayCritical, 223);
HRS_JNI_SLOT(ExceptionCheck, 228);
#undef HRS_JNI_SLOT

#ifdef __cplusplus
}
#endif

#endif /* HRS_JNI_MIN_H_ */
