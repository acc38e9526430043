// kq_gguf.cpp — GGUF model-file reader (host code), the loader side of the hot path:
// it hands the raw K-quant blocks of a real Q4_K_M file to the kernels unchanged.
//
// Reference: llama-bench loads the model through ggml's gguf_reader::read (fread of
// the header, KV strings and tensor infos; artifacts/perf/out.folded:2-3, 17-22) and
// llama_model_loader (out.folded:39-46). The GGUF layout itself lives in the
// un-vendored ggml (gguf.cpp [U]); restated here from the published format:
//   u32 magic "GGUF" | u32 version (2, 3) | u64 n_tensors | u64 n_kv
//   n_kv x { string key | u32 value type | value }            (string = u64 len + bytes)
//   n_tensors x { string name | u32 n_dims | u64 ne[n_dims] | u32 ggml type | u64 offset }
//   padding to `general.alignment` (default 32) | tensor data (offsets relative to here)
// Values: 0 u8, 1 i8, 2 u16, 3 i16, 4 u32, 5 i32, 6 f32, 7 bool, 8 string,
// 9 array (u32 element type, u64 count, elements), 10 u64, 11 i64, 12 f64.
//
// The file is memory-mapped read-only; every read is bounds-checked (a truncated or
// corrupt file fails mi355x_gguf_open with a message, it never reads past the map).
#include <fcntl.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <string>
#include <unordered_map>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "ggml_mi355x.h"

namespace {

enum : uint32_t {
    T_U8 = 0, T_I8, T_U16, T_I16, T_U32, T_I32, T_F32, T_BOOL, T_STR, T_ARR, T_U64, T_I64, T_F64, T_COUNT
};

// ggml type -> (block elements, block bytes); 0 = not known to this reader
struct TypeSize {
    int blck;
    int bytes;
};
TypeSize ggml_type_size(uint32_t t) {
    switch (t) {
        case 0: return {1, 4};       // F32
        case 1: return {1, 2};       // F16
        case 2: return {32, 18};     // Q4_0
        case 3: return {32, 20};     // Q4_1
        case 6: return {32, 22};     // Q5_0
        case 7: return {32, 24};     // Q5_1
        case 8: return {32, 34};     // Q8_0
        case 9: return {32, 36};     // Q8_1
        case 10: return {256, 84};   // Q2_K
        case 11: return {256, 110};  // Q3_K
        case 12: return {256, 144};  // Q4_K
        case 13: return {256, 176};  // Q5_K
        case 14: return {256, 210};  // Q6_K
        case 15: return {256, 292};  // Q8_K
        case 24: return {1, 1};      // I8
        case 25: return {1, 2};      // I16
        case 26: return {1, 4};      // I32
        case 27: return {1, 8};      // I64
        case 28: return {1, 8};      // F64
        case 30: return {1, 2};      // BF16
        default: return {0, 0};
    }
}

struct KV {
    std::string key;
    uint32_t type = 0;
    uint32_t arr_type = 0;  // T_ARR: element type
    uint64_t arr_n = 0;     // T_ARR: element count
    int64_t i = 0;          // integer / bool scalars
    double f = 0;           // float scalars
    std::string s;          // string scalar
};

struct Tensor {
    std::string name;
    uint32_t type = 0;
    uint32_t n_dims = 0;
    int64_t ne[4] = {1, 1, 1, 1};
    uint64_t offset = 0;  // absolute, in the file
    uint64_t size = 0;
};

struct Reader {
    const uint8_t *p, *end;
    bool ok = true;
    std::string err;
    bool need(uint64_t n) {
        if (!ok) return false;
        if ((uint64_t)(end - p) < n) {
            ok = false;
            err = "truncated file";
        }
        return ok;
    }
    template <typename T>
    T get() {
        T v{};
        if (need(sizeof(T))) {
            memcpy(&v, p, sizeof(T));
            p += sizeof(T);
        }
        return v;
    }
    std::string str() {
        const uint64_t n = get<uint64_t>();
        if (!ok) return {};
        if (n > (1ull << 32)) {
            ok = false;
            err = "string length out of range";
            return {};
        }
        if (!need(n)) return {};
        std::string s((const char *)p, (size_t)n);
        p += n;
        return s;
    }
    void skip(uint64_t n) {
        if (need(n)) p += n;
    }
};

uint64_t scalar_bytes(uint32_t t) {
    switch (t) {
        case T_U8: case T_I8: case T_BOOL: return 1;
        case T_U16: case T_I16: return 2;
        case T_U32: case T_I32: case T_F32: return 4;
        case T_U64: case T_I64: case T_F64: return 8;
        default: return 0;
    }
}

bool read_scalar(Reader &r, uint32_t t, KV &kv) {
    switch (t) {
        case T_U8: kv.i = r.get<uint8_t>(); break;
        case T_I8: kv.i = r.get<int8_t>(); break;
        case T_U16: kv.i = r.get<uint16_t>(); break;
        case T_I16: kv.i = r.get<int16_t>(); break;
        case T_U32: kv.i = r.get<uint32_t>(); break;
        case T_I32: kv.i = r.get<int32_t>(); break;
        case T_BOOL: kv.i = r.get<uint8_t>() != 0; break;
        case T_U64: kv.i = (int64_t)r.get<uint64_t>(); break;
        case T_I64: kv.i = r.get<int64_t>(); break;
        case T_F32: kv.f = r.get<float>(); break;
        case T_F64: kv.f = r.get<double>(); break;
        case T_STR: kv.s = r.str(); break;
        default: r.ok = false; r.err = "unknown value type"; return false;
    }
    if (t == T_F32 || t == T_F64) kv.i = (int64_t)kv.f;
    else if (t != T_STR) kv.f = (double)kv.i;
    return r.ok;
}

}  // namespace

struct mi355x_gguf {
    int fd = -1;
    const uint8_t *map = nullptr;
    size_t map_size = 0;
    uint32_t version = 0;
    uint64_t alignment = 32;
    uint64_t data_offset = 0;
    std::vector<KV> kv;
    std::vector<Tensor> tensors;
    std::unordered_map<std::string, int64_t> tensor_index, kv_index;
};

namespace {

mi355x_gguf *fail(mi355x_gguf *g, const char *path, const std::string &why) {
    fprintf(stderr, "ggml_mi355x: gguf: %s: %s\n", path, why.c_str());
    mi355x_gguf_close(g);
    return nullptr;
}

}  // namespace

extern "C" {

mi355x_gguf_t mi355x_gguf_open(const char *path) {
    if (!path) return nullptr;
    mi355x_gguf *g = new mi355x_gguf();
    g->fd = open(path, O_RDONLY);
    if (g->fd < 0) return fail(g, path, "cannot open");
    struct stat st;
    if (fstat(g->fd, &st) != 0 || st.st_size < 24) return fail(g, path, "not a GGUF file (too small)");
    g->map_size = (size_t)st.st_size;
    void *m = mmap(nullptr, g->map_size, PROT_READ, MAP_PRIVATE, g->fd, 0);
    if (m == MAP_FAILED) return fail(g, path, "mmap failed");
    g->map = (const uint8_t *)m;
    Reader r{g->map, g->map + g->map_size};
    const uint32_t magic = r.get<uint32_t>();
    if (magic != 0x46554747u) return fail(g, path, "bad magic (not GGUF)");
    g->version = r.get<uint32_t>();
    if (g->version < 2 || g->version > 3) return fail(g, path, "unsupported GGUF version " + std::to_string(g->version));
    const uint64_t n_tensors = r.get<uint64_t>();
    const uint64_t n_kv = r.get<uint64_t>();
    // every KV takes >= 12 bytes and every tensor info >= 24: bound the counts by the file
    if (n_kv > g->map_size / 12 || n_tensors > g->map_size / 24) return fail(g, path, "header counts out of range");
    g->kv.resize((size_t)n_kv);
    for (uint64_t i = 0; i < n_kv && r.ok; ++i) {
        KV &kv = g->kv[(size_t)i];
        kv.key = r.str();
        kv.type = r.get<uint32_t>();
        if (!r.ok) break;
        if (kv.type == T_ARR) {
            kv.arr_type = r.get<uint32_t>();
            kv.arr_n = r.get<uint64_t>();
            if (!r.ok) break;
            if (kv.arr_type == T_STR) {
                for (uint64_t j = 0; j < kv.arr_n && r.ok; ++j) r.skip(r.get<uint64_t>());
            } else if (kv.arr_type == T_ARR || scalar_bytes(kv.arr_type) == 0) {
                r.ok = false;
                r.err = "unsupported array element type";
            } else {
                if (kv.arr_n > g->map_size) {
                    r.ok = false;
                    r.err = "array length out of range";
                } else {
                    r.skip(kv.arr_n * scalar_bytes(kv.arr_type));
                }
            }
        } else {
            read_scalar(r, kv.type, kv);
        }
        if (r.ok) g->kv_index[kv.key] = (int64_t)i;
    }
    if (!r.ok) return fail(g, path, "metadata: " + r.err);
    auto ai = g->kv_index.find("general.alignment");
    if (ai != g->kv_index.end()) {
        const KV &kv = g->kv[(size_t)ai->second];
        if (kv.type != T_U32 || kv.i <= 0 || (kv.i & (kv.i - 1))) return fail(g, path, "bad general.alignment");
        g->alignment = (uint64_t)kv.i;
    }
    g->tensors.resize((size_t)n_tensors);
    for (uint64_t i = 0; i < n_tensors && r.ok; ++i) {
        Tensor &t = g->tensors[(size_t)i];
        t.name = r.str();
        t.n_dims = r.get<uint32_t>();
        if (!r.ok) break;
        if (t.n_dims < 1 || t.n_dims > 4) {
            r.ok = false;
            r.err = "tensor '" + t.name + "': n_dims out of range";
            break;
        }
        for (uint32_t d = 0; d < t.n_dims; ++d) {
            const uint64_t ne = r.get<uint64_t>();
            if (ne > (1ull << 40)) {
                r.ok = false;
                r.err = "tensor '" + t.name + "': dimension out of range";
            }
            t.ne[d] = (int64_t)ne;
        }
        t.type = r.get<uint32_t>();
        t.offset = r.get<uint64_t>();
        if (!r.ok) break;
        if (g->tensor_index.count(t.name)) {
            r.ok = false;
            r.err = "duplicate tensor '" + t.name + "'";
            break;
        }
        g->tensor_index[t.name] = (int64_t)i;
    }
    if (!r.ok) return fail(g, path, "tensor infos: " + r.err);
    const uint64_t pos = (uint64_t)(r.p - g->map);
    g->data_offset = (pos + g->alignment - 1) / g->alignment * g->alignment;
    for (Tensor &t : g->tensors) {
        const TypeSize ts = ggml_type_size(t.type);
        if (t.offset % g->alignment) return fail(g, path, "tensor '" + t.name + "': misaligned offset");
        // unknown types are rejected: a caller sizing its reads from ne could not be
        // bounded by t.size otherwise (upstream gguf.cpp rejects them too [U])
        if (!ts.blck) return fail(g, path, "tensor '" + t.name + "': unknown ggml type " + std::to_string(t.type));
        if (t.ne[0] % ts.blck) return fail(g, path, "tensor '" + t.name + "': row not a whole number of blocks");
        // every product checked before it is formed (upstream: INT64_MAX / ne checks)
        uint64_t size = (uint64_t)(t.ne[0] / ts.blck);
        bool ovf = size > UINT64_MAX / (uint64_t)ts.bytes;
        size *= ovf ? 1 : (uint64_t)ts.bytes;
        for (int d = 1; d < 4 && !ovf; ++d) {
            const uint64_t ne = (uint64_t)t.ne[d];
            if (ne && size > UINT64_MAX / ne) ovf = true;
            else size *= ne;
        }
        if (ovf || size > (uint64_t)INT64_MAX) return fail(g, path, "tensor '" + t.name + "': size overflows 64 bits");
        t.size = size;
        t.offset += g->data_offset;
        if (t.offset > g->map_size || t.size > g->map_size - t.offset)
            return fail(g, path, "tensor '" + t.name + "': data beyond the end of the file");
    }
    return g;
}

void mi355x_gguf_close(mi355x_gguf_t g) {
    if (!g) return;
    if (g->map) munmap((void *)g->map, g->map_size);
    if (g->fd >= 0) close(g->fd);
    delete g;
}

uint32_t mi355x_gguf_version(mi355x_gguf_t g) { return g ? g->version : 0; }
uint64_t mi355x_gguf_alignment(mi355x_gguf_t g) { return g ? g->alignment : 0; }
uint64_t mi355x_gguf_data_offset(mi355x_gguf_t g) { return g ? g->data_offset : 0; }
int64_t mi355x_gguf_n_tensors(mi355x_gguf_t g) { return g ? (int64_t)g->tensors.size() : -1; }
int64_t mi355x_gguf_n_kv(mi355x_gguf_t g) { return g ? (int64_t)g->kv.size() : -1; }

int64_t mi355x_gguf_find_tensor(mi355x_gguf_t g, const char *name) {
    if (!g || !name) return -1;
    auto it = g->tensor_index.find(name);
    return it == g->tensor_index.end() ? -1 : it->second;
}

int mi355x_gguf_get_tensor(mi355x_gguf_t g, int64_t i, mi355x_gguf_tensor *out) {
    if (!g || !out || i < 0 || i >= (int64_t)g->tensors.size()) return MI355X_E_INVAL;
    const Tensor &t = g->tensors[(size_t)i];
    out->name = t.name.c_str();
    out->type = (int)t.type;
    out->n_dims = (int)t.n_dims;
    for (int d = 0; d < 4; ++d) out->ne[d] = t.ne[d];
    out->offset = t.offset;
    out->size = t.size;
    return MI355X_OK;
}

const void *mi355x_gguf_tensor_data(mi355x_gguf_t g, int64_t i) {
    if (!g || i < 0 || i >= (int64_t)g->tensors.size()) return nullptr;
    return g->map + g->tensors[(size_t)i].offset;
}

int mi355x_gguf_upload(mi355x_gguf_t g, int64_t i, void *dst, size_t dst_size, void *stream) {
    if (!g || !dst || i < 0 || i >= (int64_t)g->tensors.size()) return MI355X_E_INVAL;
    const Tensor &t = g->tensors[(size_t)i];
    if (t.size == 0 || dst_size < t.size) return MI355X_E_INVAL;
    const hipError_t e = hipMemcpyAsync(dst, g->map + t.offset, (size_t)t.size, hipMemcpyHostToDevice,
                                        (hipStream_t)stream);
    if (e != hipSuccess) return e == hipErrorNoDevice || e == hipErrorInsufficientDriver ? MI355X_E_NODEVICE : (int)e;
    return MI355X_OK;
}

int64_t mi355x_gguf_find_key(mi355x_gguf_t g, const char *key) {
    if (!g || !key) return -1;
    auto it = g->kv_index.find(key);
    return it == g->kv_index.end() ? -1 : it->second;
}

const char *mi355x_gguf_key(mi355x_gguf_t g, int64_t i) {
    if (!g || i < 0 || i >= (int64_t)g->kv.size()) return nullptr;
    return g->kv[(size_t)i].key.c_str();
}

int mi355x_gguf_kv_type(mi355x_gguf_t g, int64_t i) {
    if (!g || i < 0 || i >= (int64_t)g->kv.size()) return MI355X_E_INVAL;
    return (int)g->kv[(size_t)i].type;
}

int mi355x_gguf_get_int(mi355x_gguf_t g, int64_t i, int64_t *out) {
    if (!g || !out || i < 0 || i >= (int64_t)g->kv.size()) return MI355X_E_INVAL;
    const KV &kv = g->kv[(size_t)i];
    if (kv.type == T_STR || kv.type == T_ARR || kv.type == T_F32 || kv.type == T_F64) return MI355X_E_INVAL;
    *out = kv.i;
    return MI355X_OK;
}

int mi355x_gguf_get_float(mi355x_gguf_t g, int64_t i, double *out) {
    if (!g || !out || i < 0 || i >= (int64_t)g->kv.size()) return MI355X_E_INVAL;
    const KV &kv = g->kv[(size_t)i];
    if (kv.type == T_STR || kv.type == T_ARR) return MI355X_E_INVAL;
    *out = kv.f;
    return MI355X_OK;
}

const char *mi355x_gguf_get_str(mi355x_gguf_t g, int64_t i) {
    if (!g || i < 0 || i >= (int64_t)g->kv.size()) return nullptr;
    const KV &kv = g->kv[(size_t)i];
    return kv.type == T_STR ? kv.s.c_str() : nullptr;
}

int64_t mi355x_gguf_arr_n(mi355x_gguf_t g, int64_t i) {
    if (!g || i < 0 || i >= (int64_t)g->kv.size()) return -1;
    const KV &kv = g->kv[(size_t)i];
    return kv.type == T_ARR ? (int64_t)kv.arr_n : -1;
}

}  // extern "C"
