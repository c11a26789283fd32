/*
 * Minimal stand-in for a JDK's <jni.h>: only the types, macros and JNINativeInterface members
 * jni/flink_gpu_jni.c uses, with the real header's C shape (JNIEnv is a pointer to a function
 * table; calls read (*env)->Fn(env, ...)). Test infrastructure: it lets tests/test_jni_shim.py
 * compile the JNI glue and drive its exports through a fake JNIEnv (tests/jni_stub/jni_driver.c)
 * in an image without a JDK. The real build (jni/Makefile) uses $JAVA_HOME/include.
 */
#ifndef FG_TEST_JNI_STUB_H
#define FG_TEST_JNI_STUB_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2
#define JNI_FALSE 0
#define JNI_TRUE 1

typedef int32_t jint;
typedef int64_t jlong;
typedef uint8_t jboolean;
typedef jint jsize;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jarray;
typedef jarray jobjectArray;
typedef jarray jlongArray;
typedef jobject jthrowable;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
    jclass (*FindClass)(JNIEnv* env, const char* name);
    jint (*ThrowNew)(JNIEnv* env, jclass cls, const char* msg);
    jboolean (*ExceptionCheck)(JNIEnv* env);
    jsize (*GetArrayLength)(JNIEnv* env, jarray a);
    void (*SetObjectArrayElement)(JNIEnv* env, jobjectArray a, jsize i, jobject v);
    jlong* (*GetLongArrayElements)(JNIEnv* env, jlongArray a, jboolean* isCopy);
    void (*ReleaseLongArrayElements)(JNIEnv* env, jlongArray a, jlong* elems, jint mode);
    void (*SetLongArrayRegion)(JNIEnv* env, jlongArray a, jsize start, jsize len, const jlong* buf);
    jobject (*NewDirectByteBuffer)(JNIEnv* env, void* address, jlong capacity);
    void* (*GetDirectBufferAddress)(JNIEnv* env, jobject buf);
    jlong (*GetDirectBufferCapacity)(JNIEnv* env, jobject buf);
    jlongArray (*NewLongArray)(JNIEnv* env, jsize len);
};

#endif
