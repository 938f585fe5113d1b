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
 * The wider ggml op/graph API used by src/gemma_model.cpp is declared in
 * ggml_amd_graph.h and implemented by the device graph executor.
 */
#ifndef GGML_AMD_GGML_H
#define GGML_AMD_GGML_H

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

#ifdef __cplusplus
}
#endif
#endif
