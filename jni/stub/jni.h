/* jni.h stand-in for tests only (this image has no JDK): the types and the JNIEnv functions the shim
 * jni/redisson_sketch_jni.c calls, in a table of our own.  tests/test_host.py type-checks the shim against it and
 * jni/jni_drive.c drives the shim through it with a fake JNIEnv.  A real build uses the JDK's jni.h. */
#pragma once
#include <stdint.h>
typedef int32_t jint; typedef int64_t jlong; typedef uint8_t jboolean; typedef int8_t jbyte;
typedef double jdouble; typedef jint jsize;
typedef struct _jobject *jobject; typedef jobject jclass; typedef jobject jstring; typedef jobject jarray;
typedef jarray jbyteArray; typedef jarray jlongArray; typedef jarray jintArray; typedef jarray jdoubleArray;
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2
struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;
struct JNINativeInterface_ {
    jsize (*GetArrayLength)(JNIEnv *, jarray);
    void *(*GetPrimitiveArrayCritical)(JNIEnv *, jarray, jboolean *);
    void (*ReleasePrimitiveArrayCritical)(JNIEnv *, jarray, void *, jint);
    jbyte *(*GetByteArrayElements)(JNIEnv *, jbyteArray, jboolean *);
    void (*ReleaseByteArrayElements)(JNIEnv *, jbyteArray, jbyte *, jint);
    jbyteArray (*NewByteArray)(JNIEnv *, jsize);
    jstring (*NewStringUTF)(JNIEnv *, const char *);
};
