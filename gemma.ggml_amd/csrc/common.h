// common.h — shared host/device definitions for the MI355X (gfx950) hot path.
//
// Numerics contract: every kernel is compiled with -ffp-contract=off, so an
// expression a*b+c is two IEEE roundings; fused multiply-adds appear only where the reference
// (ggml's AVX2 code) uses one, written as __builtin_fmaf.  fp32->fp16 is RNE
// (v_cvt_f16_f32), division and sqrtf are correctly rounded (hipcc default).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <string>

namespace ghip {

// ggml type ids (GGUF numbering)
// diagnostic phase stamps (s_memrealtime per workgroup into mv_args/attn_args::dbg_t): compiled
// out of the product build (the checks and stores cost ~5 % of a decode token); the stamp tools use
// a variant built with -DGHIP_STAMPS=1 (scripts/build_variant.sh stamps ...)
#ifndef GHIP_STAMPS
#define GHIP_STAMPS 0
#endif

enum : int { T_F32 = 0, T_F16 = 1, T_Q4_0 = 2, T_Q8_0 = 8, T_Q4_K = 12, T_Q6_K = 14, T_Q8_K = 15 };

// ggml on-disk/host block formats
struct block_q4_0 { uint16_t d; uint8_t qs[16]; };
struct block_q8_0 { uint16_t d; int8_t qs[32]; };
static_assert(sizeof(block_q4_0) == 18, "q4_0");
static_assert(sizeof(block_q8_0) == 34, "q8_0");

// ---------------------------------------------------------------------------------------------
// Device weight layout ("tiled", DESIGN.md §HBM layout).  A [rows x K] quantized matrix is cut
// into tiles of 8 rows x BT blocks (BT = 8 for Q4_0, 4 for Q8_0).  One tile is exactly one
// wave-instruction's worth of 16-byte loads: thread t = rr*8 + l (row rr of the tile, AVX2
// lane l) owns 16 contiguous bytes, so a wave reads 1 KiB contiguous per tile.
//   Q4_0: dword p of a thread's 16 B holds blocks (2p, 2p+1) of the tile, lane l's 4 elements
//         4l..4l+3: byte k = nib(block 2p, elem 4l+k) | nib(block 2p+1, elem 4l+k) << 4.
//   Q8_0: dword p holds block p's 4 int8 elements 4l..4l+3.
// Scales live in a separate plane: [tile][rr][BT] fp16 (16 B per row for Q4_0, 8 B for Q8_0).
// Algorithmic bytes are unchanged: 18 (Q4_0) / 34 (Q8_0) bytes per 32 weights.
// ---------------------------------------------------------------------------------------------
template <int WT> struct wfmt;
template <> struct wfmt<T_Q4_0> { static constexpr int BT = 8, SCALE_BYTES = 16, BLOCK_BYTES = 18; };
template <> struct wfmt<T_Q8_0> { static constexpr int BT = 4, SCALE_BYTES = 8, BLOCK_BYTES = 34; };

struct tiled_mat {
    int type = T_Q4_0;
    int64_t rows = 0, K = 0;
    int64_t n_rt = 0;   // row tiles (ceil(rows/8))
    int64_t nb = 0;     // real blocks per row (K/32)
    int64_t n_bt = 0;   // block tiles per row (ceil(nb/BT))
    uint8_t *qs = nullptr;   // n_rt * n_bt * 1024 bytes
    uint8_t *sc = nullptr;   // n_rt * n_bt * 8 * SCALE_BYTES bytes
    size_t qs_bytes() const { return (size_t)n_rt * n_bt * 1024; }
    size_t sc_bytes() const { return (size_t)n_rt * n_bt * 8 * (type == T_Q4_0 ? 16 : 8); }
    size_t algo_bytes() const { return (size_t)rows * nb * (type == T_Q4_0 ? 18 : 34); }
};

// error state (thread-local last error, exposed by hpc_last_error)
void set_error(const std::string &msg);
int ghip_debug_level();  // GHIP_GGML_DEBUG (ggml_api.cpp): 0 quiet, 1 fast-path reasons, 2 + host timings
const std::string &last_error();

#define GHIP_CHECK(expr)                                                                        \
    do {                                                                                        \
        hipError_t _e = (expr);                                                                 \
        if (_e != hipSuccess) {                                                                 \
            ::ghip::set_error(std::string(#expr) + ": " + hipGetErrorString(_e) + " @" +          \
                              __FILE__ + ":" + std::to_string(__LINE__));                       \
            return -1;                                                                          \
        }                                                                                       \
    } while (0)

#define GHIP_FATAL(expr)                                                                        \
    do {                                                                                        \
        hipError_t _e = (expr);                                                                 \
        if (_e != hipSuccess) {                                                                 \
            fprintf(stderr, "[gemma_hip] fatal HIP error %s at %s:%d: %s\n", #expr, __FILE__,     \
                    __LINE__, hipGetErrorString(_e));                                           \
            abort();                                                                            \
        }                                                                                       \
    } while (0)

}  // namespace ghip
