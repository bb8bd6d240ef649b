// jni_shim_test.cc -- TEST INFRASTRUCTURE: drives the JNI shim (cov-tiles_amd/jni/covt_jni.cc) the way
// a JVM would, through a hand-built JNIEnv function table (tests/jni/jni.h), without a JDK.
//
// Reads cases from stdin, one per line:   <method> <int args...> | <hex input bytes>
// and prints one line per case:           ok <pos after> <hex of the returned Java array>
//                                    or:  exc <exception class>   (pos after must be unchanged)
// Methods (argument order of GpuDecodingUtils, pos = the IntWrapper's initial value):
//   varint P N | zigzag P N | zzdelta P N | coords P N | morton P NV NB
//   rle N P SIGNED | byterle N P BL | byterle3 N P | fpf N BL P | fpfcoords N BL P | fpfmorton NV BL P NB
//   batch                 (GpuCovtBatch: one tile, create + decode; prints "ok <n streams> <statuses>")
//   batch2 S1 S2 ...      (GpuCovtBatch over the tiles of sizes S1, S2, ... packed back to back in one direct
//                          buffer: decode twice into the SAME direct output buffer, poisoned between the
//                          calls -- the reuse contract of INTEGRATION.md section 3; prints
//                          "ok <n streams> <statuses> <output hex> <ms first call> <ms second call>")
#include <jni.h>

#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#define JFN(name) Java_com_covt_decoder_gpu_GpuDecodingUtils_##name
#define BFN(name) Java_com_covt_decoder_gpu_GpuCovtBatch_##name
extern "C" {
jintArray JFN(decodeVarint)(JNIEnv*, jclass, jbyteArray, jobject, jint);
jintArray JFN(decodeZigZagVarint)(JNIEnv*, jclass, jbyteArray, jobject, jint);
jintArray JFN(decodeZigZagDeltaVarint)(JNIEnv*, jclass, jbyteArray, jobject, jint);
jintArray JFN(decodeZigZagDeltaVarintCoordinates)(JNIEnv*, jclass, jbyteArray, jobject, jint);
jlongArray JFN(decodeRle)(JNIEnv*, jclass, jbyteArray, jint, jobject, jboolean);
jbyteArray JFN(decodeByteRle)(JNIEnv*, jclass, jbyteArray, jint, jobject, jint);
jbyteArray JFN(decodeByteRleReencode)(JNIEnv*, jclass, jbyteArray, jint, jobject);
jintArray JFN(decodeFastPfor128ZigZagDelta)(JNIEnv*, jclass, jbyteArray, jint, jint, jobject);
jintArray JFN(decodeFastPfor128DeltaCoordinates)(JNIEnv*, jclass, jbyteArray, jint, jint, jobject);
jintArray JFN(decodeDeltaVarintMortonCodes)(JNIEnv*, jclass, jbyteArray, jobject, jint, jint);
jintArray JFN(decodeFastPfor128DeltaMortonCodes)(JNIEnv*, jclass, jbyteArray, jint, jint, jobject, jint);
jlong BFN(create)(JNIEnv*, jclass, jobject, jlongArray, jlongArray, jint, jint, jint);
void BFN(destroy)(JNIEnv*, jclass, jlong);
jlong BFN(numStreams)(JNIEnv*, jclass, jlong);
jlong BFN(outputBytes)(JNIEnv*, jclass, jlong);
jintArray BFN(decode)(JNIEnv*, jclass, jlong, jobject, jobject);
}

namespace {

// ---- the fake VM: every Java object is one of these ------------------------------------------------
struct Obj {
    enum Kind { CLASS, INTWRAPPER, ARRAY, DIRECT } kind;
    std::string cls;            // CLASS: its name
    int32_t iv = 0;             // INTWRAPPER: the value
    int elem = 1;               // ARRAY: element size
    std::vector<uint8_t> data;  // ARRAY / DIRECT bytes
};
std::vector<Obj*> g_heap;
std::string g_exc;  // pending exception class ("" = none)
int g_calls_get = 0, g_calls_set = 0;

Obj* make(Obj::Kind k) {
    g_heap.push_back(new Obj{k});
    return g_heap.back();
}
template <class T> Obj* O(T p) { return reinterpret_cast<Obj*>(p); }
template <class T> T J(Obj* o) { return reinterpret_cast<T>(o); }

jclass FindClass(JNIEnv*, const char* name) {
    Obj* c = make(Obj::CLASS);
    c->cls = name;
    return J<jclass>(c);
}
jint ThrowNew(JNIEnv*, jclass c, const char*) {
    if (g_exc.empty()) g_exc = O(c)->cls;
    return 0;
}
jclass GetObjectClass(JNIEnv*, jobject o) {
    Obj* c = make(Obj::CLASS);
    c->cls = O(o)->kind == Obj::INTWRAPPER ? "me/lemire/integercompression/IntWrapper" : "java/lang/Object";
    return J<jclass>(c);
}
jmethodID GetMethodID(JNIEnv*, jclass c, const char* name, const char* sig) {
    if (O(c)->cls != "me/lemire/integercompression/IntWrapper") return nullptr;
    if (!std::strcmp(name, "get") && !std::strcmp(sig, "()I")) return reinterpret_cast<jmethodID>(1);
    if (!std::strcmp(name, "set") && !std::strcmp(sig, "(I)V")) return reinterpret_cast<jmethodID>(2);
    return nullptr;
}
jint CallIntMethodV(JNIEnv*, jobject o, jmethodID m, va_list) {
    if (m != reinterpret_cast<jmethodID>(1)) std::abort();
    ++g_calls_get;
    return O(o)->iv;
}
void CallVoidMethodV(JNIEnv*, jobject o, jmethodID m, va_list a) {
    if (m != reinterpret_cast<jmethodID>(2)) std::abort();
    ++g_calls_set;
    O(o)->iv = va_arg(a, jint);
}
jsize GetArrayLength(JNIEnv*, jarray a) { return (jsize)(O(a)->data.size() / (size_t)O(a)->elem); }
Obj* new_array(jsize n, int elem) {
    Obj* a = make(Obj::ARRAY);
    a->elem = elem;
    a->data.assign((size_t)n * (size_t)elem, 0);
    return a;
}
jbyteArray NewByteArray(JNIEnv*, jsize n) { return J<jbyteArray>(new_array(n, 1)); }
jintArray NewIntArray(JNIEnv*, jsize n) { return J<jintArray>(new_array(n, 4)); }
jlongArray NewLongArray(JNIEnv*, jsize n) { return J<jlongArray>(new_array(n, 8)); }
jbyte* GetByteArrayElements(JNIEnv*, jbyteArray a, jboolean* copy) {
    if (copy) *copy = 0;
    return reinterpret_cast<jbyte*>(O(a)->data.data());
}
void ReleaseByteArrayElements(JNIEnv*, jbyteArray, jbyte*, jint) {}
void region(Obj* a, jsize s, jsize n, void* dst, const void* src) {
    const size_t e = (size_t)a->elem;
    if (s < 0 || n < 0 || (size_t)(s + n) * e > a->data.size()) {
        g_exc = "java/lang/ArrayIndexOutOfBoundsException";
        return;
    }
    if (dst) std::memcpy(dst, a->data.data() + s * e, n * e);
    else std::memcpy(a->data.data() + s * e, src, n * e);
}
void GetLongArrayRegion(JNIEnv*, jlongArray a, jsize s, jsize n, jlong* b) { region(O(a), s, n, b, nullptr); }
void SetByteArrayRegion(JNIEnv*, jbyteArray a, jsize s, jsize n, const jbyte* b) { region(O(a), s, n, nullptr, b); }
void SetIntArrayRegion(JNIEnv*, jintArray a, jsize s, jsize n, const jint* b) { region(O(a), s, n, nullptr, b); }
void SetLongArrayRegion(JNIEnv*, jlongArray a, jsize s, jsize n, const jlong* b) { region(O(a), s, n, nullptr, b); }
void* GetDirectBufferAddress(JNIEnv*, jobject b) { return O(b)->data.data(); }
jlong GetDirectBufferCapacity(JNIEnv*, jobject b) { return (jlong)O(b)->data.size(); }

JNINativeInterface_ make_table() {
    JNINativeInterface_ t{};
    t.slot[JNI_SLOT_FindClass] = (void*)&FindClass;
    t.slot[JNI_SLOT_ThrowNew] = (void*)&ThrowNew;
    t.slot[JNI_SLOT_GetObjectClass] = (void*)&GetObjectClass;
    t.slot[JNI_SLOT_GetMethodID] = (void*)&GetMethodID;
    t.slot[JNI_SLOT_CallIntMethodV] = (void*)&CallIntMethodV;
    t.slot[JNI_SLOT_CallVoidMethodV] = (void*)&CallVoidMethodV;
    t.slot[JNI_SLOT_GetArrayLength] = (void*)&GetArrayLength;
    t.slot[JNI_SLOT_NewByteArray] = (void*)&NewByteArray;
    t.slot[JNI_SLOT_NewIntArray] = (void*)&NewIntArray;
    t.slot[JNI_SLOT_NewLongArray] = (void*)&NewLongArray;
    t.slot[JNI_SLOT_GetByteArrayElements] = (void*)&GetByteArrayElements;
    t.slot[JNI_SLOT_ReleaseByteArrayElements] = (void*)&ReleaseByteArrayElements;
    t.slot[JNI_SLOT_GetLongArrayRegion] = (void*)&GetLongArrayRegion;
    t.slot[JNI_SLOT_SetByteArrayRegion] = (void*)&SetByteArrayRegion;
    t.slot[JNI_SLOT_SetIntArrayRegion] = (void*)&SetIntArrayRegion;
    t.slot[JNI_SLOT_SetLongArrayRegion] = (void*)&SetLongArrayRegion;
    t.slot[JNI_SLOT_GetDirectBufferAddress] = (void*)&GetDirectBufferAddress;
    t.slot[JNI_SLOT_GetDirectBufferCapacity] = (void*)&GetDirectBufferCapacity;
    return t;
}

std::vector<uint8_t> unhex(const std::string& h) {
    std::vector<uint8_t> v;
    for (size_t i = 0; i + 1 < h.size(); i += 2) v.push_back((uint8_t)std::stoi(h.substr(i, 2), nullptr, 16));
    return v;
}
std::string hex(const std::vector<uint8_t>& v) {
    static const char* d = "0123456789abcdef";
    std::string s;
    for (uint8_t b : v) {
        s += d[b >> 4];
        s += d[b & 15];
    }
    return s;
}

}  // namespace

int main() {
    JNINativeInterface_ table = make_table();
    JNIEnv_ env_s{&table};
    JNIEnv* env = &env_s;
    std::string line;
    while (std::getline(std::cin, line)) {
        if (line.empty()) continue;
        const size_t bar = line.find('|');
        std::istringstream is(line.substr(0, bar));
        std::string m;
        is >> m;
        std::vector<long long> a;
        long long x;
        while (is >> x) a.push_back(x);
        std::string hx = bar == std::string::npos ? "" : line.substr(bar + 1);
        hx.erase(0, hx.find_first_not_of(' '));
        Obj* buf = new_array(0, 1);
        buf->data = unhex(hx);
        const jbyteArray jb = J<jbyteArray>(buf);
        Obj* pos = make(Obj::INTWRAPPER);
        g_exc.clear();
        jarray r = nullptr;
        auto P = [&](size_t i) { pos->iv = (int32_t)a[i]; return J<jobject>(pos); };
        if (m == "varint") r = JFN(decodeVarint)(env, nullptr, jb, P(0), (jint)a[1]);
        else if (m == "zigzag") r = JFN(decodeZigZagVarint)(env, nullptr, jb, P(0), (jint)a[1]);
        else if (m == "zzdelta") r = JFN(decodeZigZagDeltaVarint)(env, nullptr, jb, P(0), (jint)a[1]);
        else if (m == "coords") r = JFN(decodeZigZagDeltaVarintCoordinates)(env, nullptr, jb, P(0), (jint)a[1]);
        else if (m == "morton") r = JFN(decodeDeltaVarintMortonCodes)(env, nullptr, jb, P(0), (jint)a[1], (jint)a[2]);
        else if (m == "rle") r = JFN(decodeRle)(env, nullptr, jb, (jint)a[0], P(1), (jboolean)(a[2] != 0));
        else if (m == "byterle") r = JFN(decodeByteRle)(env, nullptr, jb, (jint)a[0], P(1), (jint)a[2]);
        else if (m == "byterle3") r = JFN(decodeByteRleReencode)(env, nullptr, jb, (jint)a[0], P(1));
        else if (m == "fpf") r = JFN(decodeFastPfor128ZigZagDelta)(env, nullptr, jb, (jint)a[0], (jint)a[1], P(2));
        else if (m == "fpfcoords")
            r = JFN(decodeFastPfor128DeltaCoordinates)(env, nullptr, jb, (jint)a[0], (jint)a[1], P(2));
        else if (m == "fpfmorton")
            r = JFN(decodeFastPfor128DeltaMortonCodes)(env, nullptr, jb, (jint)a[0], (jint)a[1], P(2), (jint)a[3]);
        else if (m == "batch") {  // GpuCovtBatch over one tile held in a direct ByteBuffer
            Obj* tiles = make(Obj::DIRECT);
            tiles->data = buf->data;
            tiles->data.resize(tiles->data.size() + 4096, 0);  // COVT_INPUT_PADDING
            Obj* offs = new_array(1, 8);
            Obj* sizes = new_array(1, 8);
            const int64_t sz = (int64_t)buf->data.size();
            std::memcpy(sizes->data.data(), &sz, 8);
            const jlong h = BFN(create)(env, nullptr, J<jobject>(tiles), J<jlongArray>(offs), J<jlongArray>(sizes), 0, 0, 0);
            if (g_exc.empty()) {
                Obj* out = make(Obj::DIRECT);
                out->data.assign((size_t)BFN(outputBytes)(env, nullptr, h), 0);
                r = BFN(decode)(env, nullptr, h, J<jobject>(tiles), J<jobject>(out));
                if (r) {  // statuses, then the output bytes after them
                    const jlong ns = BFN(numStreams)(env, nullptr, h);
                    std::cout << "ok " << ns << " " << hex(O(r)->data) << " " << hex(out->data) << "\n";
                    BFN(destroy)(env, nullptr, h);
                    continue;
                }
                BFN(destroy)(env, nullptr, h);
            }
        } else if (m == "batch2") {  // several tiles, two decodes into one reused direct output buffer
            Obj* tiles = make(Obj::DIRECT);
            const size_t nt = a.size();
            Obj* offs = new_array((jsize)nt, 8);
            Obj* sizes = new_array((jsize)nt, 8);
            // pack: tile k's bytes (consecutive in the hex input) at a 16-byte aligned offset of the buffer
            size_t src = 0;
            for (size_t k = 0; k < nt; ++k) {
                tiles->data.resize((tiles->data.size() + 15) & ~(size_t)15, 0);
                const int64_t o = (int64_t)tiles->data.size(), sz = (int64_t)a[k];
                std::memcpy(offs->data.data() + 8 * k, &o, 8);
                std::memcpy(sizes->data.data() + 8 * k, &sz, 8);
                tiles->data.insert(tiles->data.end(), buf->data.begin() + (std::ptrdiff_t)src,
                                   buf->data.begin() + (std::ptrdiff_t)(src + (size_t)a[k]));
                src += (size_t)a[k];
            }
            tiles->data.resize(tiles->data.size() + 4096, 0);  // COVT_INPUT_PADDING
            const jlong h = BFN(create)(env, nullptr, J<jobject>(tiles), J<jlongArray>(offs), J<jlongArray>(sizes), 0, 0, 0);
            if (g_exc.empty()) {
                Obj* out = make(Obj::DIRECT);
                out->data.assign((size_t)BFN(outputBytes)(env, nullptr, h), 0);
                double ms[2] = {0, 0};
                for (int call = 0; call < 2 && g_exc.empty(); ++call) {
                    if (call) std::memset(out->data.data(), 0xA5, out->data.size());  // the second call rewrites it all
                    const auto t0 = std::chrono::steady_clock::now();
                    r = BFN(decode)(env, nullptr, h, J<jobject>(tiles), J<jobject>(out));
                    ms[call] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                }
                if (r && g_exc.empty()) {
                    const jlong ns = BFN(numStreams)(env, nullptr, h);
                    std::cout << "ok " << ns << " " << hex(O(r)->data) << " " << hex(out->data) << " " << ms[0] << " "
                              << ms[1] << "\n";
                    BFN(destroy)(env, nullptr, h);
                    continue;
                }
                BFN(destroy)(env, nullptr, h);
            }
        } else {
            std::cerr << "unknown method " << m << "\n";
            return 2;
        }
        if (!g_exc.empty()) {
            if (r) std::cout << "bad returned-with-exception\n";
            else std::cout << "exc " << g_exc << " " << pos->iv << "\n";
        } else if (!r) {
            std::cout << "bad null-without-exception\n";
        } else {
            std::cout << "ok " << pos->iv << " " << hex(O(r)->data) << "\n";
        }
    }
    std::cout.flush();
    for (Obj* o : g_heap) delete o;
    return 0;
}
