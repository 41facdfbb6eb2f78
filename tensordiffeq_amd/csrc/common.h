// Shared helpers for the gfx950 (CDNA4) kernels of tensordiffeq_amd.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define TDQ_WAVE 64

// 16x16x4 fp32 MFMA: D[16x16] += A[16x4] * B[4x16]
//   lane l supplies A[l&15][l>>4] and B[l>>4][l&15];
//   D/C: lane l, reg r holds D[4*(l>>4)+r][l&15].
__device__ __forceinline__ f32x4 mfma16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// DPP lane permutations inside a 16-lane row (pure VALU, no LDS traffic)
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// sum over the 16 lanes that share (l >> 4); every lane of the row gets the total
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror
  v += dpp<0x140>(v);  // row_mirror
  return v;
}

// sum over the 4 lanes l, l^16, l^32, l^48 (same point, different feature groups)
__device__ __forceinline__ float col4_sum(float v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

#define TDQ_CHECK_LAUNCH() \
  do { hipError_t _e = hipGetLastError(); if (_e != hipSuccess) return (int)_e; } while (0)
