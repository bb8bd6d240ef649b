// covt_jni.cc -- JNI binding of libcovt for com.covt.decoder.gpu.GpuDecodingUtils.
//
// Each native method has the signature of the DecodingUtils.java method it replaces
// (evaluation/java/src/main/java/com/covt/decoder/DecodingUtils.java:35-444): byte[] input,
// me.lemire.integercompression.IntWrapper cursor, Java-allocated result array.  Status codes of
// include/covt.h become the exceptions the reference throws.  Built only where <jni.h> exists
// (make -C cov-tiles_amd jni JAVA_HOME=...); this image has no JDK.
#include <jni.h>

#include <vector>

#include "covt.h"

namespace {

int get_pos(JNIEnv* env, jobject iw) {
    jclass c = env->GetObjectClass(iw);
    return env->CallIntMethod(iw, env->GetMethodID(c, "get", "()I"));
}
void set_pos(JNIEnv* env, jobject iw, int v) {
    jclass c = env->GetObjectClass(iw);
    env->CallVoidMethod(iw, env->GetMethodID(c, "set", "(I)V"), v);
}
bool check(JNIEnv* env, int st) {
    if (st == COVT_OK) return true;
    const char* cls = "java/lang/IllegalArgumentException";
    if (st == COVT_ERR_TRUNCATED || st == COVT_ERR_COUNT_MISMATCH) cls = "java/lang/ArrayIndexOutOfBoundsException";
    if (st == COVT_ERR_DEVICE) cls = "java/lang/IllegalStateException";
    env->ThrowNew(env->FindClass(cls), "libcovt decode failed");
    return false;
}

struct Bytes {  // pinned view of a byte[]
    JNIEnv* env;
    jbyteArray a;
    jbyte* p;
    jsize n;
    Bytes(JNIEnv* e, jbyteArray arr) : env(e), a(arr), p(e->GetByteArrayElements(arr, nullptr)), n(e->GetArrayLength(arr)) {}
    ~Bytes() { env->ReleaseByteArrayElements(a, p, JNI_ABORT); }
    const uint8_t* u8() const { return reinterpret_cast<const uint8_t*>(p); }
};

template <class F>
jintArray int_result(JNIEnv* env, jsize n, F&& f) {
    std::vector<int32_t> out((size_t)(n > 0 ? n : 0));
    if (!check(env, f(out.data()))) return nullptr;
    jintArray r = env->NewIntArray(n);
    env->SetIntArrayRegion(r, 0, n, out.data());
    return r;
}

}  // namespace

#define JFN(name) Java_com_covt_decoder_gpu_GpuDecodingUtils_##name

extern "C" {

JNIEXPORT jintArray JNICALL JFN(decodeVarint)(JNIEnv* env, jclass, jbyteArray src, jobject pos, jint n) {
    Bytes b(env, src);
    int32_t p = get_pos(env, pos);
    jintArray r = int_result(env, n, [&](int32_t* o) { return covt_decode_varint(b.u8(), (size_t)b.n, &p, n, o); });
    if (r) set_pos(env, pos, p);
    return r;
}
JNIEXPORT jintArray JNICALL JFN(decodeZigZagVarint)(JNIEnv* env, jclass, jbyteArray src, jobject pos, jint n) {
    Bytes b(env, src);
    int32_t p = get_pos(env, pos);
    jintArray r =
        int_result(env, n, [&](int32_t* o) { return covt_decode_zigzag_varint(b.u8(), (size_t)b.n, &p, n, o); });
    if (r) set_pos(env, pos, p);
    return r;
}
JNIEXPORT jintArray JNICALL JFN(decodeZigZagDeltaVarint)(JNIEnv* env, jclass, jbyteArray src, jobject pos, jint n) {
    Bytes b(env, src);
    int32_t p = get_pos(env, pos);
    jintArray r = int_result(
        env, n, [&](int32_t* o) { return covt_decode_zigzag_delta_varint(b.u8(), (size_t)b.n, &p, n, o); });
    if (r) set_pos(env, pos, p);
    return r;
}
JNIEXPORT jintArray JNICALL JFN(decodeZigZagDeltaVarintCoordinates)(JNIEnv* env, jclass, jbyteArray src,
                                                                    jobject pos, jint n) {
    Bytes b(env, src);
    int32_t p = get_pos(env, pos);
    jintArray r = int_result(env, n, [&](int32_t* o) {
        return covt_decode_zigzag_delta_varint_coordinates(b.u8(), (size_t)b.n, &p, n, o);
    });
    if (r) set_pos(env, pos, p);
    return r;
}
JNIEXPORT jlongArray JNICALL JFN(decodeRle)(JNIEnv* env, jclass, jbyteArray buf, jint n, jobject pos,
                                            jboolean is_signed) {
    Bytes b(env, buf);
    int32_t p = get_pos(env, pos);
    std::vector<int64_t> out((size_t)(n > 0 ? n : 0));
    if (!check(env, covt_decode_rle(b.u8(), (size_t)b.n, n, &p, is_signed ? 1 : 0, out.data()))) return nullptr;
    jlongArray r = env->NewLongArray(n);
    env->SetLongArrayRegion(r, 0, n, reinterpret_cast<const jlong*>(out.data()));
    set_pos(env, pos, p);
    return r;
}
JNIEXPORT jbyteArray JNICALL JFN(decodeByteRle)(JNIEnv* env, jclass, jbyteArray buf, jint n, jobject pos,
                                                jint byte_length) {
    Bytes b(env, buf);
    int32_t p = get_pos(env, pos);
    std::vector<uint8_t> out((size_t)(n > 0 ? n : 0));
    if (!check(env, covt_decode_byte_rle(b.u8(), (size_t)b.n, n, &p, byte_length, out.data()))) return nullptr;
    jbyteArray r = env->NewByteArray(n);
    env->SetByteArrayRegion(r, 0, n, reinterpret_cast<const jbyte*>(out.data()));
    set_pos(env, pos, p);
    return r;
}
JNIEXPORT jintArray JNICALL JFN(decodeFastPfor128ZigZagDelta)(JNIEnv* env, jclass, jbyteArray buf, jint n,
                                                              jint byte_length, jobject pos) {
    Bytes b(env, buf);
    int32_t p = get_pos(env, pos);
    jintArray r = int_result(env, n, [&](int32_t* o) {
        return covt_decode_fastpfor_zigzag_delta(b.u8(), (size_t)b.n, n, byte_length, &p, o);
    });
    if (r) set_pos(env, pos, p);
    return r;
}
JNIEXPORT jintArray JNICALL JFN(decodeFastPfor128DeltaCoordinates)(JNIEnv* env, jclass, jbyteArray buf, jint n,
                                                                   jint byte_length, jobject pos) {
    Bytes b(env, buf);
    int32_t p = get_pos(env, pos);
    jintArray r = int_result(env, n, [&](int32_t* o) {
        return covt_decode_fastpfor_delta_coordinates(b.u8(), (size_t)b.n, n, byte_length, &p, o);
    });
    if (r) set_pos(env, pos, p);
    return r;
}
JNIEXPORT jintArray JNICALL JFN(decodeDeltaVarintMortonCodes)(JNIEnv* env, jclass, jbyteArray buf, jobject pos,
                                                              jint n_vertices, jint num_bits) {
    Bytes b(env, buf);
    int32_t p = get_pos(env, pos);
    jintArray r = int_result(env, 2 * n_vertices, [&](int32_t* o) {
        return covt_decode_delta_varint_morton_codes(b.u8(), (size_t)b.n, &p, n_vertices, num_bits, o);
    });
    if (r) set_pos(env, pos, p);
    return r;
}
JNIEXPORT jintArray JNICALL JFN(decodeFastPfor128DeltaMortonCodes)(JNIEnv* env, jclass, jbyteArray buf,
                                                                   jint n_vertices, jint byte_length, jobject pos,
                                                                   jint num_bits) {
    Bytes b(env, buf);
    int32_t p = get_pos(env, pos);
    jintArray r = int_result(env, 2 * n_vertices, [&](int32_t* o) {
        return covt_decode_fastpfor_delta_morton_codes(b.u8(), (size_t)b.n, n_vertices, byte_length, &p, num_bits,
                                                       o);
    });
    if (r) set_pos(env, pos, p);
    return r;
}

}  // extern "C"
