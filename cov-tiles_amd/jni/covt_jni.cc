// covt_jni.cc -- JNI binding of libcovt for com.covt.decoder.gpu.GpuDecodingUtils.
//
// Each native method has the signature of the DecodingUtils.java method it replaces
// (evaluation/java/src/main/java/com/covt/decoder/DecodingUtils.java:35-444): byte[] input,
// me.lemire.integercompression.IntWrapper cursor, Java-allocated result array.  Status codes of
// include/covt.h become the exceptions the reference throws.  Built only where <jni.h> exists
// (make -C cov-tiles_amd jni JAVA_HOME=...); this image has no JDK.
#include <jni.h>

#include <algorithm>
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
// decodeByteRle(byte[], int, IntWrapper) (DecodingUtils.java:290): GpuDecodingUtils' 3-argument
// overload forwards here (a distinct name keeps the 4-argument native's short JNI symbol unambiguous).
JNIEXPORT jbyteArray JNICALL JFN(decodeByteRleReencode)(JNIEnv* env, jclass, jbyteArray buf, jint n, jobject pos) {
    Bytes b(env, buf);
    int32_t p = get_pos(env, pos);
    std::vector<uint8_t> out((size_t)(n > 0 ? n : 0));
    if (!check(env, covt_decode_byte_rle_reencode(b.u8(), (size_t)b.n, n, &p, out.data()))) return nullptr;
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

// ---- com.covt.decoder.gpu.GpuCovtBatch: whole-tile batches through the plan API -------------------
#define BFN(name) Java_com_covt_decoder_gpu_GpuCovtBatch_##name

static covt_plan* plan_of(jlong h) { return reinterpret_cast<covt_plan*>(h); }
static const uint8_t* direct(JNIEnv* env, jobject buf) {
    return static_cast<const uint8_t*>(env->GetDirectBufferAddress(buf));
}

JNIEXPORT jlong JNICALL BFN(create)(JNIEnv* env, jclass, jobject tiles, jlongArray offsets, jlongArray sizes,
                                    jint format, jint id_mode, jint flags) {
    const jsize n = env->GetArrayLength(offsets);
    std::vector<uint64_t> off((size_t)n), sz((size_t)n);
    env->GetLongArrayRegion(offsets, 0, n, reinterpret_cast<jlong*>(off.data()));
    env->GetLongArrayRegion(sizes, 0, n, reinterpret_cast<jlong*>(sz.data()));
    covt_plan* p = nullptr;
    if (!check(env, covt_plan_create_ex(direct(env, tiles), off.data(), sz.data(), n, format, id_mode,
                                        (uint32_t)flags, &p)))
        return 0;
    return reinterpret_cast<jlong>(p);
}
JNIEXPORT void JNICALL BFN(destroy)(JNIEnv*, jclass, jlong h) { covt_plan_destroy(plan_of(h)); }
JNIEXPORT jlong JNICALL BFN(numStreams)(JNIEnv*, jclass, jlong h) { return covt_plan_num_streams(plan_of(h)); }
JNIEXPORT jlong JNICALL BFN(outputBytes)(JNIEnv*, jclass, jlong h) { return covt_plan_output_bytes(plan_of(h)); }
JNIEXPORT jlong JNICALL BFN(numPropertyColumns)(JNIEnv*, jclass, jlong h) {
    return covt_plan_num_property_columns(plan_of(h));
}
JNIEXPORT jlong JNICALL BFN(propertyBytes)(JNIEnv*, jclass, jlong h) { return covt_plan_property_bytes(plan_of(h)); }

JNIEXPORT jintArray JNICALL BFN(tileStatus)(JNIEnv* env, jclass, jlong h, jint n_tiles) {
    std::vector<int32_t> st((size_t)(n_tiles > 0 ? n_tiles : 0));
    if (!check(env, covt_plan_tile_status(plan_of(h), st.data()))) return nullptr;
    jintArray a = env->NewIntArray(n_tiles);
    env->SetIntArrayRegion(a, 0, n_tiles, st.data());
    return a;
}
JNIEXPORT jlongArray JNICALL BFN(streams)(JNIEnv* env, jclass, jlong h) {
    const int64_t n = covt_plan_num_streams(plan_of(h));
    std::vector<covt_stream_info> info((size_t)n);
    if (!check(env, covt_plan_streams(plan_of(h), info.data()))) return nullptr;
    std::vector<jlong> rows((size_t)n * 15);
    for (int64_t i = 0; i < n; ++i) {
        const covt_stream_info& s = info[(size_t)i];
        const jlong r[15] = {s.tile, s.layer, s.column_kind, s.stream_type, s.encoding, s.column_type, s.num_values,
                             s.byte_length, s.num_bits, s.op, s.elem_bytes, s.desc_index, s.in_off, s.out_off,
                             s.out_elems};
        std::copy(r, r + 15, rows.begin() + 15 * i);
    }
    jlongArray a = env->NewLongArray((jsize)rows.size());
    env->SetLongArrayRegion(a, 0, (jsize)rows.size(), rows.data());
    return a;
}
JNIEXPORT jlongArray JNICALL BFN(propertyColumns)(JNIEnv* env, jclass, jlong h) {
    const int64_t n = covt_plan_num_property_columns(plan_of(h));
    std::vector<covt_prop_info> info((size_t)n);
    if (!check(env, covt_plan_property_columns(plan_of(h), info.data()))) return nullptr;
    std::vector<jlong> rows((size_t)n * 22);
    for (int64_t i = 0; i < n; ++i) {
        const covt_prop_info& q = info[(size_t)i];
        const jlong r[22] = {q.tile, q.layer, q.column, q.type, q.column_type, q.n_features, q.n_data, q.n_dict,
                             q.lang, q.name_len, q.lang_len, q.dict_bytes, q.stream[0], q.stream[1], q.stream[2],
                             q.desc_index, q.name_off, q.lang_off, q.out_off[0], q.out_off[1], q.out_off[2],
                             q.out_off[3]};
        std::copy(r, r + 22, rows.begin() + 22 * i);
    }
    jlongArray a = env->NewLongArray((jsize)rows.size());
    env->SetLongArrayRegion(a, 0, (jsize)rows.size(), rows.data());
    return a;
}
JNIEXPORT jintArray JNICALL BFN(decode)(JNIEnv* env, jclass, jlong h, jobject tiles, jobject out) {
    const int64_t n = covt_plan_num_streams(plan_of(h));
    std::vector<covt_stream_result> res((size_t)n);
    if (!check(env, covt_plan_decode_host(plan_of(h), direct(env, tiles), (uint64_t)env->GetDirectBufferCapacity(tiles),
                                          static_cast<uint8_t*>(env->GetDirectBufferAddress(out)), res.data())))
        return nullptr;
    std::vector<jint> st((size_t)n);
    for (int64_t i = 0; i < n; ++i) st[(size_t)i] = res[(size_t)i].status;
    jintArray a = env->NewIntArray((jsize)n);
    env->SetIntArrayRegion(a, 0, (jsize)n, st.data());
    return a;
}
JNIEXPORT jintArray JNICALL BFN(properties)(JNIEnv* env, jclass, jlong h, jobject tiles, jobject out) {
    const int64_t n = covt_plan_num_property_columns(plan_of(h));
    std::vector<covt_prop_result> res((size_t)n);
    if (!check(env, covt_plan_properties_host(plan_of(h), direct(env, tiles),
                                              (uint64_t)env->GetDirectBufferCapacity(tiles),
                                              static_cast<uint8_t*>(env->GetDirectBufferAddress(out)), res.data())))
        return nullptr;
    jintArray a = env->NewIntArray((jsize)(2 * n));
    env->SetIntArrayRegion(a, 0, (jsize)(2 * n), reinterpret_cast<const jint*>(res.data()));
    return a;
}

}  // extern "C"
