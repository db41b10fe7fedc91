/* Minimal stand-in for <jni.h> (no JDK in this image): just the types and
 * JNIEnv functions tsne_hip_jni.c uses, with the JNI specification's
 * signatures, so that tests/test_jni_shim.py can type-check the shim against
 * include/tsne_hip.h with gcc -fsyntax-only.  Never used to build a library
 * that runs: the real build uses $(JAVA_HOME)/include (jni/Makefile). */
#ifndef TSNE_JNI_STUB_H
#define TSNE_JNI_STUB_H
#include <stdint.h>
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2
typedef int32_t jint;
typedef int64_t jlong;
typedef double jdouble;
typedef jint jsize;
typedef struct _jobject *jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jintArray;
typedef uint8_t jboolean;
struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;
struct JNINativeInterface_ {
    jclass (*FindClass)(JNIEnv *env, const char *name);
    jint (*ThrowNew)(JNIEnv *env, jclass clazz, const char *msg);
    jsize (*GetArrayLength)(JNIEnv *env, jarray array);
    jint *(*GetIntArrayElements)(JNIEnv *env, jintArray array, jboolean *isCopy);
    void (*ReleaseIntArrayElements)(JNIEnv *env, jintArray array, jint *elems, jint mode);
    const char *(*GetStringUTFChars)(JNIEnv *env, jstring str, jboolean *isCopy);
    void (*ReleaseStringUTFChars)(JNIEnv *env, jstring str, const char *chars);
    jstring (*NewStringUTF)(JNIEnv *env, const char *utf);
};
#endif
