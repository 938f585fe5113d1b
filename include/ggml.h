/*
 * ggml.h — the ggml type/struct subset that the reference's hot-path boundary speaks.
 *
 * The reference links an un-vendored ggml fork (CMakeLists.txt:13,39), so this header
 * restates only what the drop-in needs, with the Feb–Mar 2024 layout as recalled [ext]:
 *   - enum ggml_type numbering (GGUF ids),
 *   - struct ggml_tensor field order (type, backend, buffer, ne[4], nb[4], op, op_params, flags,
 *     grad, src[10], perf counters, view_src, view_offs, data, name[64], extra, padding) so that
 *     `src0->data` / `dst->data` (the only fields src/hpc.cpp:228-229 reads) sit at the same offsets,
 *   - ggml_vec_dot_t, the 8-argument vec_dot pointer type passed at src/hpc.cpp:223 / :35-36.
 * The wider ggml op/graph API used by src/gemma_model.cpp is declared below and
 * implemented by the device graph executor.
 */
#ifndef GGML_AMD_GGML_H
#define GGML_AMD_GGML_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GGML_MAX_DIMS 4
#define GGML_MAX_OP_PARAMS 64
#define GGML_MAX_SRC 10
#define GGML_MAX_NAME 64

typedef uint16_t ggml_fp16_t;

enum ggml_type {
    GGML_TYPE_F32 = 0,
    GGML_TYPE_F16 = 1,
    GGML_TYPE_Q4_0 = 2,
    GGML_TYPE_Q4_1 = 3,
    GGML_TYPE_Q5_0 = 6,
    GGML_TYPE_Q5_1 = 7,
    GGML_TYPE_Q8_0 = 8,
    GGML_TYPE_Q8_1 = 9,
    GGML_TYPE_Q2_K = 10,
    GGML_TYPE_Q3_K = 11,
    GGML_TYPE_Q4_K = 12,
    GGML_TYPE_Q5_K = 13,
    GGML_TYPE_Q6_K = 14,
    GGML_TYPE_Q8_K = 15,
    GGML_TYPE_I8 = 24,
    GGML_TYPE_I16 = 25,
    GGML_TYPE_I32 = 26,
    GGML_TYPE_COUNT
};

enum ggml_backend_type { GGML_BACKEND_TYPE_CPU = 0, GGML_BACKEND_TYPE_GPU = 10, GGML_BACKEND_TYPE_GPU_SPLIT = 20 };

struct ggml_backend_buffer;

struct ggml_tensor {
    enum ggml_type type;
    enum ggml_backend_type backend;
    struct ggml_backend_buffer *buffer;
    int64_t ne[GGML_MAX_DIMS];
    size_t nb[GGML_MAX_DIMS];
    int32_t op; /* enum ggml_op */
    int32_t op_params[GGML_MAX_OP_PARAMS / sizeof(int32_t)];
    int32_t flags;
    struct ggml_tensor *grad;
    struct ggml_tensor *src[GGML_MAX_SRC];
    int perf_runs;
    int64_t perf_cycles;
    int64_t perf_time_us;
    struct ggml_tensor *view_src;
    size_t view_offs;
    void *data;
    char name[GGML_MAX_NAME];
    void *extra;
    char padding[8];
};

/* src/hpc.cpp:35-36 calls vec_dot(n, s, bs, x, bx, y, by, nrc) */
typedef void (*ggml_vec_dot_t)(int n, float *s, size_t bs, const void *x, size_t bx, const void *y, size_t by,
                               int nrc);

/* ==== the ggml context / tensor / graph / op surface src/gemma_model.cpp uses ====
 * Implemented by libgemma_hip.so (gemma.ggml_amd/csrc/ggml_api.cpp): tensors live in host memory
 * exactly as in ggml (a context arena or a "CPU" backend buffer), and ggml_graph_compute_with_ctx
 * runs every node on the GPU with device mirrors of the leaf data — weights uploaded once per
 * pointer, host-written inputs re-uploaded each compute, leaves the graph writes (the KV cache)
 * kept device-authoritative — and copies the LAST node's data back to the host (the one
 * src/gemma_model.cpp:280 reads).  Arithmetic = the ggml CPU ops the oracle restates
 * (bit-identical logits, tests/test_gpu_ggml_graph.py).  GGUF loading is out of scope.        */
enum ggml_op {
    GGML_OP_NONE = 0,
    GGML_OP_GET_ROWS,
    GGML_OP_SCALE,
    GGML_OP_RMS_NORM,
    GGML_OP_MUL,
    GGML_OP_ADD,
    GGML_OP_MUL_MAT,
    GGML_OP_ROPE,
    GGML_OP_SOFT_MAX,
    GGML_OP_GELU,
    GGML_OP_CPY,
    GGML_OP_CONT,
    GGML_OP_VIEW,
    GGML_OP_RESHAPE,
    GGML_OP_PERMUTE,
    GGML_OP_TRANSPOSE,
    GGML_OP_COUNT
};

enum ggml_status { GGML_STATUS_ALLOC_FAILED = -2, GGML_STATUS_FAILED = -1, GGML_STATUS_SUCCESS = 0 };

struct ggml_init_params {
    size_t mem_size;   /* bytes */
    void *mem_buffer;  /* if NULL, memory is allocated internally */
    bool no_alloc;     /* don't allocate memory for the tensor data */
};

struct ggml_context;
struct ggml_cgraph {
    int size;
    int n_nodes;
    int n_leafs;
    struct ggml_tensor **nodes;
    struct ggml_tensor **grads;
    struct ggml_tensor **leafs;
    void *visited; /* the graph's visited-node set (ggml's visited_hash_table role): O(1) per expand */
};

typedef struct ggml_backend_buffer_type *ggml_backend_buffer_type_t;
typedef struct ggml_backend_buffer *ggml_backend_buffer_t;

/* context and sizes */
struct ggml_context *ggml_init(struct ggml_init_params params);
void ggml_free(struct ggml_context *ctx);
size_t ggml_tensor_overhead(void);
size_t ggml_graph_overhead(void);
size_t ggml_get_mem_size(const struct ggml_context *ctx);
size_t ggml_type_size(enum ggml_type type);
int64_t ggml_blck_size(enum ggml_type type);
size_t ggml_row_size(enum ggml_type type, int64_t ne);
size_t ggml_element_size(const struct ggml_tensor *tensor);
int64_t ggml_nelements(const struct ggml_tensor *tensor);
size_t ggml_nbytes(const struct ggml_tensor *tensor);

/* tensors and views */
struct ggml_tensor *ggml_new_tensor(struct ggml_context *ctx, enum ggml_type type, int n_dims, const int64_t *ne);
struct ggml_tensor *ggml_new_tensor_1d(struct ggml_context *ctx, enum ggml_type type, int64_t ne0);
struct ggml_tensor *ggml_new_tensor_2d(struct ggml_context *ctx, enum ggml_type type, int64_t ne0, int64_t ne1);
struct ggml_tensor *ggml_new_tensor_3d(struct ggml_context *ctx, enum ggml_type type, int64_t ne0, int64_t ne1,
                                       int64_t ne2);
struct ggml_tensor *ggml_view_1d(struct ggml_context *ctx, struct ggml_tensor *a, int64_t ne0, size_t offset);
struct ggml_tensor *ggml_view_2d(struct ggml_context *ctx, struct ggml_tensor *a, int64_t ne0, int64_t ne1,
                                 size_t nb1, size_t offset);
struct ggml_tensor *ggml_view_3d(struct ggml_context *ctx, struct ggml_tensor *a, int64_t ne0, int64_t ne1,
                                 int64_t ne2, size_t nb1, size_t nb2, size_t offset);
struct ggml_tensor *ggml_reshape_2d(struct ggml_context *ctx, struct ggml_tensor *a, int64_t ne0, int64_t ne1);
struct ggml_tensor *ggml_reshape_3d(struct ggml_context *ctx, struct ggml_tensor *a, int64_t ne0, int64_t ne1,
                                    int64_t ne2);
struct ggml_tensor *ggml_permute(struct ggml_context *ctx, struct ggml_tensor *a, int axis0, int axis1, int axis2,
                                 int axis3);
struct ggml_tensor *ggml_transpose(struct ggml_context *ctx, struct ggml_tensor *a);
struct ggml_tensor *ggml_cont_2d(struct ggml_context *ctx, struct ggml_tensor *a, int64_t ne0, int64_t ne1);
struct ggml_tensor *ggml_set_name(struct ggml_tensor *tensor, const char *name);
struct ggml_tensor *ggml_format_name(struct ggml_tensor *tensor, const char *fmt, ...);
const char *ggml_get_name(const struct ggml_tensor *tensor);
const char *ggml_op_name(enum ggml_op op); /* "MUL_MAT", "VIEW", ... */
struct ggml_tensor *ggml_get_tensor(struct ggml_context *ctx, const char *name);

/* ops (src/gemma_model.cpp:438-518, 665-747) */
struct ggml_tensor *ggml_get_rows(struct ggml_context *ctx, struct ggml_tensor *a, struct ggml_tensor *b);
struct ggml_tensor *ggml_scale(struct ggml_context *ctx, struct ggml_tensor *a, float s);
struct ggml_tensor *ggml_rms_norm(struct ggml_context *ctx, struct ggml_tensor *a, float eps);
struct ggml_tensor *ggml_mul(struct ggml_context *ctx, struct ggml_tensor *a, struct ggml_tensor *b);
struct ggml_tensor *ggml_add(struct ggml_context *ctx, struct ggml_tensor *a, struct ggml_tensor *b);
struct ggml_tensor *ggml_mul_mat(struct ggml_context *ctx, struct ggml_tensor *a, struct ggml_tensor *b);
struct ggml_tensor *ggml_rope_custom(struct ggml_context *ctx, struct ggml_tensor *a, struct ggml_tensor *b,
                                     int n_dims, int mode, int n_ctx, int n_orig_ctx, float freq_base,
                                     float freq_scale, float ext_factor, float attn_factor, float beta_fast,
                                     float beta_slow);
struct ggml_tensor *ggml_soft_max_ext(struct ggml_context *ctx, struct ggml_tensor *a, struct ggml_tensor *mask,
                                      struct ggml_tensor *pos, float scale, float max_bias);
struct ggml_tensor *ggml_gelu(struct ggml_context *ctx, struct ggml_tensor *a);
struct ggml_tensor *ggml_cpy(struct ggml_context *ctx, struct ggml_tensor *a, struct ggml_tensor *b);

/* graphs */
struct ggml_cgraph *ggml_new_graph(struct ggml_context *ctx);
void ggml_build_forward_expand(struct ggml_cgraph *cgraph, struct ggml_tensor *tensor);
enum ggml_status ggml_graph_compute_with_ctx(struct ggml_context *ctx, struct ggml_cgraph *cgraph, int n_threads);

/* backend ("CPU" buffer type: host memory, mirrored on the device by the graph executor) */
ggml_backend_buffer_type_t ggml_backend_cpu_buffer_type(void);
ggml_backend_buffer_t ggml_backend_alloc_ctx_tensors_from_buft(struct ggml_context *ctx,
                                                               ggml_backend_buffer_type_t buft);
void ggml_backend_buffer_clear(ggml_backend_buffer_t buffer, uint8_t value);
const char *ggml_backend_buffer_name(ggml_backend_buffer_t buffer);
size_t ggml_backend_buffer_get_size(ggml_backend_buffer_t buffer);
void ggml_backend_buffer_free(ggml_backend_buffer_t buffer);
void ggml_backend_tensor_set(struct ggml_tensor *tensor, const void *data, size_t offset, size_t size);
void ggml_backend_tensor_get(const struct ggml_tensor *tensor, void *data, size_t offset, size_t size);

/* ---- GGUF (v2/v3) reader: the gguf_* API src/gemma_model.cpp:19-229, 583-648 loads models with ----
 * gguf_init_from_file reads the header, key/value pairs and tensor infos; with params.ctx != NULL it
 * also creates a ggml context holding every tensor (named as in the file; data read from the file
 * unless params.no_alloc).  Malformed files return NULL with a message (hpc_last_error).
 * gguf_get_val_* / gguf_get_arr_* on a key of another type abort, as ggml's GGML_ASSERT does. */
enum gguf_type {
    GGUF_TYPE_UINT8 = 0,
    GGUF_TYPE_INT8 = 1,
    GGUF_TYPE_UINT16 = 2,
    GGUF_TYPE_INT16 = 3,
    GGUF_TYPE_UINT32 = 4,
    GGUF_TYPE_INT32 = 5,
    GGUF_TYPE_FLOAT32 = 6,
    GGUF_TYPE_BOOL = 7,
    GGUF_TYPE_STRING = 8,
    GGUF_TYPE_ARRAY = 9,
    GGUF_TYPE_UINT64 = 10,
    GGUF_TYPE_INT64 = 11,
    GGUF_TYPE_FLOAT64 = 12,
    GGUF_TYPE_COUNT
};
struct gguf_context;
struct gguf_init_params {
    bool no_alloc;
    struct ggml_context **ctx;  /* if not NULL, receives a context with the file's tensors */
};
struct gguf_context *gguf_init_from_file(const char *fname, struct gguf_init_params params);
void gguf_free(struct gguf_context *ctx);
const char *gguf_type_name(enum gguf_type type);
int gguf_get_version(const struct gguf_context *ctx);
size_t gguf_get_alignment(const struct gguf_context *ctx);
size_t gguf_get_data_offset(const struct gguf_context *ctx);
int gguf_get_n_kv(const struct gguf_context *ctx);
int gguf_find_key(const struct gguf_context *ctx, const char *key); /* -1 if absent */
const char *gguf_get_key(const struct gguf_context *ctx, int key_id);
enum gguf_type gguf_get_kv_type(const struct gguf_context *ctx, int key_id);
enum gguf_type gguf_get_arr_type(const struct gguf_context *ctx, int key_id);
uint8_t gguf_get_val_u8(const struct gguf_context *ctx, int key_id);
int8_t gguf_get_val_i8(const struct gguf_context *ctx, int key_id);
uint16_t gguf_get_val_u16(const struct gguf_context *ctx, int key_id);
int16_t gguf_get_val_i16(const struct gguf_context *ctx, int key_id);
uint32_t gguf_get_val_u32(const struct gguf_context *ctx, int key_id);
int32_t gguf_get_val_i32(const struct gguf_context *ctx, int key_id);
float gguf_get_val_f32(const struct gguf_context *ctx, int key_id);
uint64_t gguf_get_val_u64(const struct gguf_context *ctx, int key_id);
int64_t gguf_get_val_i64(const struct gguf_context *ctx, int key_id);
double gguf_get_val_f64(const struct gguf_context *ctx, int key_id);
bool gguf_get_val_bool(const struct gguf_context *ctx, int key_id);
const char *gguf_get_val_str(const struct gguf_context *ctx, int key_id);
const void *gguf_get_val_data(const struct gguf_context *ctx, int key_id);
int gguf_get_arr_n(const struct gguf_context *ctx, int key_id);
const void *gguf_get_arr_data(const struct gguf_context *ctx, int key_id);
const char *gguf_get_arr_str(const struct gguf_context *ctx, int key_id, int i);
int gguf_get_n_tensors(const struct gguf_context *ctx);
int gguf_find_tensor(const struct gguf_context *ctx, const char *name); /* -1 if absent */
size_t gguf_get_tensor_offset(const struct gguf_context *ctx, int i);
const char *gguf_get_tensor_name(const struct gguf_context *ctx, int i);
enum ggml_type gguf_get_tensor_type(const struct gguf_context *ctx, int i);

#ifdef __cplusplus
}
#endif
#endif
