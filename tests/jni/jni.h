/*
 * jni.h -- TEST INFRASTRUCTURE ONLY.  This image has no JDK, so the JNI shim
 * (cov-tiles_amd/jni/covt_jni.cc) is compiled for its unit test against this
 * minimal stand-in.  It declares only what the shim uses, but keeps the real
 * interface's shape: JNIEnv is a pointer to a function table whose slots sit at
 * the indices the JNI specification assigns them ("Interface Function Table"),
 * and the C++ JNIEnv_ wrappers call through that table exactly as a JDK's jni.h
 * does.  tests/jni/jni_shim_test.cc fills the table with a fake VM.  A real build
 * uses $JAVA_HOME/include/jni.h (make -C cov-tiles_amd jni).
 */
#ifndef COVT_TEST_JNI_H
#define COVT_TEST_JNI_H

#include <stdarg.h>
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef float jfloat;
typedef jint jsize;

class _jobject {};
class _jclass : public _jobject {};
class _jstring : public _jobject {};
class _jarray : public _jobject {};
class _jbyteArray : public _jarray {};
class _jintArray : public _jarray {};
class _jlongArray : public _jarray {};
class _jfloatArray : public _jarray {};
typedef _jobject* jobject;
typedef _jclass* jclass;
typedef _jstring* jstring;
typedef _jarray* jarray;
typedef _jbyteArray* jbyteArray;
typedef _jintArray* jintArray;
typedef _jlongArray* jlongArray;
typedef _jfloatArray* jfloatArray;
struct _jmethodID;
typedef struct _jmethodID* jmethodID;

struct JNIEnv_;
typedef JNIEnv_ JNIEnv;

/* slot indices of the JNI function table (JNI specification, Interface Function Table) */
enum {
    JNI_SLOT_FindClass = 6,
    JNI_SLOT_ThrowNew = 14,
    JNI_SLOT_GetObjectClass = 31,
    JNI_SLOT_GetMethodID = 33,
    JNI_SLOT_CallIntMethodV = 50,
    JNI_SLOT_CallVoidMethodV = 62,
    JNI_SLOT_GetArrayLength = 171,
    JNI_SLOT_NewByteArray = 176,
    JNI_SLOT_NewIntArray = 179,
    JNI_SLOT_NewLongArray = 180,
    JNI_SLOT_GetByteArrayElements = 184,
    JNI_SLOT_ReleaseByteArrayElements = 192,
    JNI_SLOT_GetLongArrayRegion = 204,
    JNI_SLOT_SetByteArrayRegion = 208,
    JNI_SLOT_SetIntArrayRegion = 211,
    JNI_SLOT_SetLongArrayRegion = 212,
    JNI_SLOT_GetDirectBufferAddress = 230,
    JNI_SLOT_GetDirectBufferCapacity = 231,
    JNI_NUM_SLOTS = 234
};

struct JNINativeInterface_ {
    void* slot[JNI_NUM_SLOTS];
};

struct JNIEnv_ {
    const struct JNINativeInterface_* functions;

    template <class F>
    F fn(int i) { return reinterpret_cast<F>(functions->slot[i]); }

    jclass FindClass(const char* name) { return fn<jclass (*)(JNIEnv*, const char*)>(JNI_SLOT_FindClass)(this, name); }
    jint ThrowNew(jclass c, const char* msg) {
        return fn<jint (*)(JNIEnv*, jclass, const char*)>(JNI_SLOT_ThrowNew)(this, c, msg);
    }
    jclass GetObjectClass(jobject o) { return fn<jclass (*)(JNIEnv*, jobject)>(JNI_SLOT_GetObjectClass)(this, o); }
    jmethodID GetMethodID(jclass c, const char* name, const char* sig) {
        return fn<jmethodID (*)(JNIEnv*, jclass, const char*, const char*)>(JNI_SLOT_GetMethodID)(this, c, name, sig);
    }
    jint CallIntMethod(jobject o, jmethodID m, ...) {
        va_list a;
        va_start(a, m);
        jint r = fn<jint (*)(JNIEnv*, jobject, jmethodID, va_list)>(JNI_SLOT_CallIntMethodV)(this, o, m, a);
        va_end(a);
        return r;
    }
    void CallVoidMethod(jobject o, jmethodID m, ...) {
        va_list a;
        va_start(a, m);
        fn<void (*)(JNIEnv*, jobject, jmethodID, va_list)>(JNI_SLOT_CallVoidMethodV)(this, o, m, a);
        va_end(a);
    }
    jsize GetArrayLength(jarray a) { return fn<jsize (*)(JNIEnv*, jarray)>(JNI_SLOT_GetArrayLength)(this, a); }
    jbyteArray NewByteArray(jsize n) { return fn<jbyteArray (*)(JNIEnv*, jsize)>(JNI_SLOT_NewByteArray)(this, n); }
    jintArray NewIntArray(jsize n) { return fn<jintArray (*)(JNIEnv*, jsize)>(JNI_SLOT_NewIntArray)(this, n); }
    jlongArray NewLongArray(jsize n) { return fn<jlongArray (*)(JNIEnv*, jsize)>(JNI_SLOT_NewLongArray)(this, n); }
    jbyte* GetByteArrayElements(jbyteArray a, jboolean* copy) {
        return fn<jbyte* (*)(JNIEnv*, jbyteArray, jboolean*)>(JNI_SLOT_GetByteArrayElements)(this, a, copy);
    }
    void ReleaseByteArrayElements(jbyteArray a, jbyte* p, jint mode) {
        fn<void (*)(JNIEnv*, jbyteArray, jbyte*, jint)>(JNI_SLOT_ReleaseByteArrayElements)(this, a, p, mode);
    }
    void GetLongArrayRegion(jlongArray a, jsize s, jsize n, jlong* b) {
        fn<void (*)(JNIEnv*, jlongArray, jsize, jsize, jlong*)>(JNI_SLOT_GetLongArrayRegion)(this, a, s, n, b);
    }
    void SetByteArrayRegion(jbyteArray a, jsize s, jsize n, const jbyte* b) {
        fn<void (*)(JNIEnv*, jbyteArray, jsize, jsize, const jbyte*)>(JNI_SLOT_SetByteArrayRegion)(this, a, s, n, b);
    }
    void SetIntArrayRegion(jintArray a, jsize s, jsize n, const jint* b) {
        fn<void (*)(JNIEnv*, jintArray, jsize, jsize, const jint*)>(JNI_SLOT_SetIntArrayRegion)(this, a, s, n, b);
    }
    void SetLongArrayRegion(jlongArray a, jsize s, jsize n, const jlong* b) {
        fn<void (*)(JNIEnv*, jlongArray, jsize, jsize, const jlong*)>(JNI_SLOT_SetLongArrayRegion)(this, a, s, n, b);
    }
    void* GetDirectBufferAddress(jobject b) {
        return fn<void* (*)(JNIEnv*, jobject)>(JNI_SLOT_GetDirectBufferAddress)(this, b);
    }
    jlong GetDirectBufferCapacity(jobject b) {
        return fn<jlong (*)(JNIEnv*, jobject)>(JNI_SLOT_GetDirectBufferCapacity)(this, b);
    }
};

#endif
