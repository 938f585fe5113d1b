// gguf.cpp — GGUF v2/v3 reader behind ggml's gguf_* API, the loader src/gemma_model.cpp:19-229 and
// 583-648 use (gguf_init_from_file with a weight context, gguf_get_n_kv / gguf_get_key /
// gguf_get_kv_type, gguf_get_val_{u32,f32,str}, gguf_get_arr_{type,n,data,str}, gguf_get_n_tensors /
// gguf_get_tensor_name, then ggml_get_tensor on the context).
//
// File layout (GGUF v3, little endian): "GGUF" u32 version, u64 n_tensors, u64 n_kv; n_kv x
// {string key, u32 type, value}; n_tensors x {string name, u32 n_dims, u64 ne[n_dims], u32 ggml type,
// u64 offset}; pad to general.alignment (default 32); tensor data at data_offset + offset.  A string
// is u64 length + bytes; an array is u32 element type, u64 n, n elements.  v1 files (u32 counts) are
// rejected, as by ggml of this era.
//
// Every read is bounds-checked against the file size, so a truncated or corrupt file fails with a
// message instead of over-allocating or reading past the end.  Tensor data for a ggml context is
// read with one pass over the data section into the context's arena (weights are immutable for the
// program, src/gemma_model.cpp:24-27; the graph executor mirrors them to the GPU once).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <unordered_set>
#include <vector>

#include "common.h"
#include "ggml_impl.h"

struct gguf_kv {
    std::string key;
    gguf_type type = GGUF_TYPE_UINT8;
    gguf_type arr_type = GGUF_TYPE_UINT8;  // element type when type == ARRAY
    uint64_t n = 0;                         // elements (arrays)
    std::vector<uint8_t> data;              // scalar bytes, or packed array elements (non-string)
    std::string str;                        // STRING value
    std::vector<std::string> strs;          // string array elements
};

struct gguf_tensor_info {
    std::string name;
    uint32_t n_dims = 0;
    int64_t ne[GGML_MAX_DIMS] = {1, 1, 1, 1};
    ggml_type type = GGML_TYPE_F32;
    uint64_t offset = 0;
};

struct gguf_context {
    uint32_t version = 0;
    std::vector<gguf_kv> kv;
    std::vector<gguf_tensor_info> infos;
    size_t alignment = 32;
    size_t data_offset = 0;
};

namespace {

constexpr uint32_t kMagic = 0x46554747u;  // "GGUF"

size_t scalar_size(int t) {
    switch (t) {
        case GGUF_TYPE_UINT8: case GGUF_TYPE_INT8: case GGUF_TYPE_BOOL: return 1;
        case GGUF_TYPE_UINT16: case GGUF_TYPE_INT16: return 2;
        case GGUF_TYPE_UINT32: case GGUF_TYPE_INT32: case GGUF_TYPE_FLOAT32: return 4;
        case GGUF_TYPE_UINT64: case GGUF_TYPE_INT64: case GGUF_TYPE_FLOAT64: return 8;
        default: return 0;
    }
}

struct reader {
    FILE *f = nullptr;
    uint64_t size = 0, pos = 0;
    std::string err;

    bool fail(const std::string &m) {
        if (err.empty()) err = m;
        return false;
    }
    bool bytes(void *dst, uint64_t n) {
        if (n > size - pos) return fail("unexpected end of file at byte " + std::to_string(pos));
        if (n && fread(dst, 1, n, f) != n) return fail("read error at byte " + std::to_string(pos));
        pos += n;
        return true;
    }
    template <class T> bool get(T &v) { return bytes(&v, sizeof(T)); }
    bool str(std::string &s) {
        uint64_t n;
        if (!get(n)) return false;
        if (n > size - pos) return fail("string length " + std::to_string(n) + " past the end of file");
        s.resize(n);
        return bytes(&s[0], n);
    }
};

bool read_kv(reader &r, gguf_kv &kv) {
    uint32_t t;
    if (!r.str(kv.key) || !r.get(t)) return false;
    kv.type = (gguf_type)t;
    if (t == GGUF_TYPE_STRING) return r.str(kv.str);
    if (t == GGUF_TYPE_ARRAY) {
        uint32_t at;
        if (!r.get(at) || !r.get(kv.n)) return false;
        kv.arr_type = (gguf_type)at;
        if (at == GGUF_TYPE_STRING) {
            if (kv.n > (r.size - r.pos) / 8) return r.fail("key " + kv.key + ": string array longer than the file");
            kv.strs.resize(kv.n);
            for (uint64_t i = 0; i < kv.n; ++i)
                if (!r.str(kv.strs[i])) return false;
            return true;
        }
        const size_t es = scalar_size(at);
        if (!es) return r.fail("key " + kv.key + ": array of unsupported element type " + std::to_string(at));
        if (kv.n > (r.size - r.pos) / es) return r.fail("key " + kv.key + ": array longer than the file");
        kv.data.resize(kv.n * es);
        return r.bytes(kv.data.data(), kv.data.size());
    }
    const size_t es = scalar_size(t);
    if (!es) return r.fail("key " + kv.key + ": unsupported value type " + std::to_string(t));
    kv.data.resize(es);
    return r.bytes(kv.data.data(), es);
}

// SIZE_MAX when the byte count does not fit (a malformed file's dimensions)
size_t tensor_bytes(const gguf_tensor_info &ti) {
    size_t n = ggml_impl::type_size(ti.type);
    if (__builtin_mul_overflow(n, (size_t)(ti.ne[0] / ggml_impl::blck_size(ti.type)), &n)) return SIZE_MAX;
    for (int i = 1; i < GGML_MAX_DIMS; ++i)
        if (__builtin_mul_overflow(n, (size_t)ti.ne[i], &n)) return SIZE_MAX;
    return n;
}

bool read_info(reader &r, gguf_tensor_info &ti) {
    if (!r.str(ti.name) || !r.get(ti.n_dims)) return false;
    if (ti.name.size() >= GGML_MAX_NAME) return r.fail("tensor name too long: " + ti.name);
    if (ti.n_dims == 0 || ti.n_dims > GGML_MAX_DIMS)
        return r.fail("tensor " + ti.name + ": n_dims " + std::to_string(ti.n_dims) + " out of range");
    for (uint32_t i = 0; i < ti.n_dims; ++i) {
        uint64_t v;
        if (!r.get(v)) return false;
        if (v > (uint64_t)INT64_MAX / 2) return r.fail("tensor " + ti.name + ": bad dimension");
        ti.ne[i] = (int64_t)v;
    }
    uint32_t t;
    if (!r.get(t) || !r.get(ti.offset)) return false;
    ti.type = (ggml_type)t;
    if (t >= GGML_TYPE_COUNT || ggml_impl::type_size(t) == 0)
        return r.fail("tensor " + ti.name + ": unsupported ggml type " + std::to_string(t));
    if (ti.ne[0] % ggml_impl::blck_size(t))
        return r.fail("tensor " + ti.name + ": ne[0] not a multiple of the block size");
    // element count must fit (ggml checks INT64_MAX / ne products)
    double ne = 1.0;
    for (int i = 0; i < GGML_MAX_DIMS; ++i) ne *= (double)ti.ne[i];
    if (ne > 9.0e15) return r.fail("tensor " + ti.name + ": too many elements");
    return true;
}

}  // namespace

extern "C" {

struct gguf_context *gguf_init_from_file(const char *fname, struct gguf_init_params params) {
    reader r;
    r.f = fopen(fname, "rb");
    if (!r.f) {
        ghip::set_error(std::string("gguf_init_from_file: cannot open ") + fname);
        fprintf(stderr, "%s\n", ghip::last_error().c_str());
        return nullptr;
    }
    fseeko(r.f, 0, SEEK_END);
    r.size = (uint64_t)ftello(r.f);
    fseeko(r.f, 0, SEEK_SET);
    gguf_context *g = new gguf_context();
    auto bail = [&](const std::string &m) -> gguf_context * {
        ghip::set_error("gguf_init_from_file: " + std::string(fname) + ": " + (r.err.empty() ? m : r.err));
        fprintf(stderr, "%s\n", ghip::last_error().c_str());
        fclose(r.f);
        delete g;
        return nullptr;
    };
    uint32_t magic = 0;
    uint64_t n_tensors = 0, n_kv = 0;
    if (!r.get(magic)) return bail("");
    if (magic != kMagic) return bail("bad magic (not a GGUF file)");
    if (!r.get(g->version)) return bail("");
    if (g->version == 1) return bail("GGUF v1 is not supported");
    if (g->version > 3) return bail("GGUF version " + std::to_string(g->version) + " is newer than supported (3)");
    if (!r.get(n_tensors) || !r.get(n_kv)) return bail("");
    // each kv needs >= 12 bytes, each tensor info >= 28: reject counts the file cannot hold
    if (n_kv > r.size / 12 || n_tensors > r.size / 28) return bail("header counts exceed the file size");
    g->kv.resize(n_kv);
    std::unordered_set<std::string> seen;
    for (uint64_t i = 0; i < n_kv; ++i) {
        if (!read_kv(r, g->kv[i])) return bail("");
        if (!seen.insert(g->kv[i].key).second) return bail("duplicate key " + g->kv[i].key);
    }
    const int ia = gguf_find_key(g, "general.alignment");
    if (ia >= 0) {
        if (g->kv[ia].type != GGUF_TYPE_UINT32) return bail("general.alignment is not u32");
        uint32_t a;
        memcpy(&a, g->kv[ia].data.data(), 4);
        if (a == 0 || (a & (a - 1))) return bail("general.alignment " + std::to_string(a) + " is not a power of two");
        g->alignment = a;
    }
    g->infos.resize(n_tensors);
    seen.clear();
    for (uint64_t i = 0; i < n_tensors; ++i) {
        if (!read_info(r, g->infos[i])) return bail("");
        if (!seen.insert(g->infos[i].name).second) return bail("duplicate tensor " + g->infos[i].name);
    }
    g->data_offset = (r.pos + g->alignment - 1) / g->alignment * g->alignment;
    size_t data_bytes = 0;
    for (const gguf_tensor_info &ti : g->infos) {
        if (ti.offset % g->alignment) return bail("tensor " + ti.name + ": offset not aligned");
        // compared by subtraction: offset + bytes must not wrap for an offset near UINT64_MAX
        const size_t nbytes = tensor_bytes(ti), avail = r.size > g->data_offset ? r.size - g->data_offset : 0;
        if (ti.offset > avail || nbytes > avail - ti.offset)
            return bail("tensor " + ti.name + ": data past the end of file");
        const size_t end = ti.offset + nbytes;
        data_bytes = std::max(data_bytes, end);
    }
    if (params.ctx) {
        ggml_init_params ip = {params.no_alloc ? 0 : data_bytes + 64, nullptr, params.no_alloc};
        ggml_context *c = ggml_init(ip);
        if (!params.no_alloc && data_bytes) {
            if (!c->mem) {
                ggml_free(c);
                return bail("cannot allocate " + std::to_string(data_bytes) + " bytes of tensor data");
            }
            fseeko(r.f, (off_t)g->data_offset, SEEK_SET);
            r.pos = g->data_offset;
            for (size_t done = 0; done < data_bytes;) {
                const size_t n = std::min<size_t>(data_bytes - done, (size_t)64 << 20);
                if (!r.bytes(c->mem + done, n)) {
                    ggml_free(c);
                    return bail("");
                }
                done += n;
            }
        }
        const bool keep = c->no_alloc;
        c->no_alloc = true;  // tensors point into the data section image instead of fresh arena slots
        for (const gguf_tensor_info &ti : g->infos) {
            ggml_tensor *t = ggml_impl::new_tensor_impl(c, ti.type, (int)ti.n_dims, ti.ne, nullptr, 0);
            ggml_set_name(t, ti.name.c_str());
            t->data = params.no_alloc ? nullptr : c->mem + ti.offset;
        }
        c->used = data_bytes;
        c->no_alloc = keep;
        *params.ctx = c;
    }
    fclose(r.f);
    return g;
}

void gguf_free(struct gguf_context *ctx) { delete ctx; }

const char *gguf_type_name(enum gguf_type type) {
    static const char *names[GGUF_TYPE_COUNT] = {"u8", "i8", "u16", "i16", "u32", "i32", "f32",
                                                 "bool", "str", "arr", "u64", "i64", "f64"};
    return (int)type >= 0 && type < GGUF_TYPE_COUNT ? names[type] : nullptr;
}

int gguf_get_version(const struct gguf_context *ctx) { return (int)ctx->version; }
size_t gguf_get_alignment(const struct gguf_context *ctx) { return ctx->alignment; }
size_t gguf_get_data_offset(const struct gguf_context *ctx) { return ctx->data_offset; }
int gguf_get_n_kv(const struct gguf_context *ctx) { return (int)ctx->kv.size(); }

int gguf_find_key(const struct gguf_context *ctx, const char *key) {
    for (size_t i = 0; i < ctx->kv.size(); ++i)
        if (ctx->kv[i].key == key) return (int)i;
    return -1;
}

}  // extern "C"

namespace {
// ggml's GGML_ASSERT on misuse: a wrong key id or type is a programming error, not a file error
const gguf_kv &kv_at(const gguf_context *ctx, int id) {
    if (id < 0 || (size_t)id >= ctx->kv.size()) {
        fprintf(stderr, "[gemma_hip] gguf: key id %d out of range\n", id);
        abort();
    }
    return ctx->kv[id];
}
template <class T> T scalar(const gguf_context *ctx, int id, gguf_type want) {
    const gguf_kv &kv = kv_at(ctx, id);
    if (kv.type != want) {
        fprintf(stderr, "[gemma_hip] gguf: key %s is %s, read as %s\n", kv.key.c_str(), gguf_type_name(kv.type),
                gguf_type_name(want));
        abort();
    }
    T v;
    memcpy(&v, kv.data.data(), sizeof(T));
    return v;
}
const gguf_kv &array_at(const gguf_context *ctx, int id) {
    const gguf_kv &kv = kv_at(ctx, id);
    if (kv.type != GGUF_TYPE_ARRAY) {
        fprintf(stderr, "[gemma_hip] gguf: key %s is not an array\n", kv.key.c_str());
        abort();
    }
    return kv;
}
}  // namespace

extern "C" {

const char *gguf_get_key(const struct gguf_context *ctx, int key_id) { return kv_at(ctx, key_id).key.c_str(); }
enum gguf_type gguf_get_kv_type(const struct gguf_context *ctx, int key_id) { return kv_at(ctx, key_id).type; }
enum gguf_type gguf_get_arr_type(const struct gguf_context *ctx, int key_id) { return array_at(ctx, key_id).arr_type; }

uint8_t gguf_get_val_u8(const struct gguf_context *c, int id) { return scalar<uint8_t>(c, id, GGUF_TYPE_UINT8); }
int8_t gguf_get_val_i8(const struct gguf_context *c, int id) { return scalar<int8_t>(c, id, GGUF_TYPE_INT8); }
uint16_t gguf_get_val_u16(const struct gguf_context *c, int id) { return scalar<uint16_t>(c, id, GGUF_TYPE_UINT16); }
int16_t gguf_get_val_i16(const struct gguf_context *c, int id) { return scalar<int16_t>(c, id, GGUF_TYPE_INT16); }
uint32_t gguf_get_val_u32(const struct gguf_context *c, int id) { return scalar<uint32_t>(c, id, GGUF_TYPE_UINT32); }
int32_t gguf_get_val_i32(const struct gguf_context *c, int id) { return scalar<int32_t>(c, id, GGUF_TYPE_INT32); }
float gguf_get_val_f32(const struct gguf_context *c, int id) { return scalar<float>(c, id, GGUF_TYPE_FLOAT32); }
uint64_t gguf_get_val_u64(const struct gguf_context *c, int id) { return scalar<uint64_t>(c, id, GGUF_TYPE_UINT64); }
int64_t gguf_get_val_i64(const struct gguf_context *c, int id) { return scalar<int64_t>(c, id, GGUF_TYPE_INT64); }
double gguf_get_val_f64(const struct gguf_context *c, int id) { return scalar<double>(c, id, GGUF_TYPE_FLOAT64); }
bool gguf_get_val_bool(const struct gguf_context *c, int id) { return scalar<uint8_t>(c, id, GGUF_TYPE_BOOL) != 0; }

const char *gguf_get_val_str(const struct gguf_context *ctx, int key_id) {
    const gguf_kv &kv = kv_at(ctx, key_id);
    if (kv.type != GGUF_TYPE_STRING) {
        fprintf(stderr, "[gemma_hip] gguf: key %s is not a string\n", kv.key.c_str());
        abort();
    }
    return kv.str.c_str();
}

const void *gguf_get_val_data(const struct gguf_context *ctx, int key_id) {
    const gguf_kv &kv = kv_at(ctx, key_id);
    if (kv.type == GGUF_TYPE_STRING || kv.type == GGUF_TYPE_ARRAY) {
        fprintf(stderr, "[gemma_hip] gguf: key %s has no scalar data\n", kv.key.c_str());
        abort();
    }
    return kv.data.data();
}

int gguf_get_arr_n(const struct gguf_context *ctx, int key_id) { return (int)array_at(ctx, key_id).n; }

const void *gguf_get_arr_data(const struct gguf_context *ctx, int key_id) {
    const gguf_kv &kv = array_at(ctx, key_id);
    if (kv.arr_type == GGUF_TYPE_STRING) {
        fprintf(stderr, "[gemma_hip] gguf: key %s is a string array (use gguf_get_arr_str)\n", kv.key.c_str());
        abort();
    }
    return kv.data.data();
}

const char *gguf_get_arr_str(const struct gguf_context *ctx, int key_id, int i) {
    const gguf_kv &kv = array_at(ctx, key_id);
    if (kv.arr_type != GGUF_TYPE_STRING || i < 0 || (uint64_t)i >= kv.n) {
        fprintf(stderr, "[gemma_hip] gguf: key %s: no string element %d\n", kv.key.c_str(), i);
        abort();
    }
    return kv.strs[i].c_str();
}

int gguf_get_n_tensors(const struct gguf_context *ctx) { return (int)ctx->infos.size(); }

int gguf_find_tensor(const struct gguf_context *ctx, const char *name) {
    for (size_t i = 0; i < ctx->infos.size(); ++i)
        if (ctx->infos[i].name == name) return (int)i;
    return -1;
}

size_t gguf_get_tensor_offset(const struct gguf_context *ctx, int i) { return ctx->infos.at(i).offset; }
const char *gguf_get_tensor_name(const struct gguf_context *ctx, int i) { return ctx->infos.at(i).name.c_str(); }
enum ggml_type gguf_get_tensor_type(const struct gguf_context *ctx, int i) { return ctx->infos.at(i).type; }

}  // extern "C"
