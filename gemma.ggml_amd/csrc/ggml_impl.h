// ggml_impl.h — private layout of the ggml host objects shared by ggml_api.cpp (contexts, tensors,
// graphs, backend buffers, executor) and gguf.cpp (the GGUF reader that fills a weight context).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "../../include/ggml.h"

struct ggml_context {
    char *mem = nullptr;
    size_t mem_size = 0, used = 0;
    bool owns_mem = false, no_alloc = false;
    std::vector<ggml_tensor *> tensors;
    std::vector<ggml_cgraph *> graphs;
    std::vector<ggml_tensor *> slabs;  // tensor objects (ggml_api.cpp slab_take), pooled on free
    size_t slab_used = 0;
};

struct ggml_backend_buffer_type {
    const char *name;
};
struct ggml_backend_buffer {
    char *mem = nullptr;
    size_t size = 0;
    std::vector<ggml_tensor *> tensors;
};

namespace ggml_impl {
// bytes per block and values per block of a ggml type (GGUF ids); 0 bytes = unknown type
size_t type_size(int t);
int64_t blck_size(int t);
// a tensor in ctx: a view of view_src at view_offs, else arena data unless ctx->no_alloc
ggml_tensor *new_tensor_impl(ggml_context *ctx, ggml_type type, int n_dims, const int64_t *ne, ggml_tensor *view_src,
                             size_t view_offs);
}  // namespace ggml_impl

// drops the ggml executor's fast-path engine when it holds a copy of `host` (nullptr: always)
void ggml_fast_drop(const void *host);
