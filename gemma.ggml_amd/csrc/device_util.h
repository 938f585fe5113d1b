// device_util.h — bit-exact numeric helpers shared by the gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ghip {

__device__ __forceinline__ float h2f(uint32_t bits) {
    return (float)__builtin_bit_cast(_Float16, (uint16_t)(bits & 0xFFFF));
}

// Opaque to the optimiser: LLVM's AMDGPU backend folds fptrunc(fmul(a, b)) into v_fma_mixlo_f16
// (ONE rounding straight to fp16) even under -ffp-contract=off, while ggml rounds the product to
// fp32 first and then to fp16 (two roundings).  The two differ on fp16 ties, so every computed
// value is pinned in a VGPR before conversion.
__device__ __forceinline__ float pin(float x) {
    asm volatile("" : "+v"(x));
    return x;
}

// fp32 -> fp16 bits, round-to-nearest-even (v_cvt_f16_f32), of an already-rounded fp32 value
__device__ __forceinline__ uint32_t f2h(float f) { return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)pin(f)); }

}  // namespace ghip
