/* tests/jni_stub/jni.h -- TEST INFRASTRUCTURE ONLY: the few JNI types and
 * JNIEnv functions jni/gpu_jni.c uses, declared so that gcc -fsyntax-only can
 * type-check the shim against include/bsdb_mi355x.h in an image without a
 * JDK.  The function table's layout is NOT the real one: nothing compiled
 * against this header may ever be linked or run (tests/test_jni_shim.py only
 * runs gcc -fsyntax-only).  A real build uses $JAVA_HOME/include/jni.h. */
#ifndef BSDB_TEST_JNI_STUB_H
#define BSDB_TEST_JNI_STUB_H
#include <stdint.h>
typedef int32_t jint;
typedef int64_t jlong;
typedef uint8_t jboolean;
typedef int8_t jbyte;
typedef jint jsize;
typedef struct _jobject *jobject;
typedef jobject jclass, jstring, jthrowable, jarray;
typedef jarray jbyteArray, jintArray, jlongArray;
#define JNIEXPORT
#define JNICALL
#define JNI_ABORT 2
struct JNINativeInterface_ {
    jclass (*FindClass)(const struct JNINativeInterface_ **, const char *);
    jint (*ThrowNew)(const struct JNINativeInterface_ **, jclass, const char *);
    jsize (*GetArrayLength)(const struct JNINativeInterface_ **, jarray);
    jbyteArray (*NewByteArray)(const struct JNINativeInterface_ **, jsize);
    void (*SetByteArrayRegion)(const struct JNINativeInterface_ **, jbyteArray, jsize, jsize, const jbyte *);
    jbyte *(*GetByteArrayElements)(const struct JNINativeInterface_ **, jbyteArray, jboolean *);
    void (*ReleaseByteArrayElements)(const struct JNINativeInterface_ **, jbyteArray, jbyte *, jint);
    jint *(*GetIntArrayElements)(const struct JNINativeInterface_ **, jintArray, jboolean *);
    void (*ReleaseIntArrayElements)(const struct JNINativeInterface_ **, jintArray, jint *, jint);
    jlongArray (*NewLongArray)(const struct JNINativeInterface_ **, jsize);
    void (*SetLongArrayRegion)(const struct JNINativeInterface_ **, jlongArray, jsize, jsize, const jlong *);
    const char *(*GetStringUTFChars)(const struct JNINativeInterface_ **, jstring, jboolean *);
    void (*ReleaseStringUTFChars)(const struct JNINativeInterface_ **, jstring, const char *);
    void *(*GetPrimitiveArrayCritical)(const struct JNINativeInterface_ **, jarray, jboolean *);
    void (*ReleasePrimitiveArrayCritical)(const struct JNINativeInterface_ **, jarray, void *, jint);
};
typedef const struct JNINativeInterface_ *JNIEnv;
#endif
