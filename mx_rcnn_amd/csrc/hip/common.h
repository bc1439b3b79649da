// Shared device helpers for the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <cstdint>
#include <cfloat>

#define MXR_WAVE 64

namespace mxr {

__device__ __forceinline__ float bf16_to_f32(uint16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);  // v_cvt_pk_bf16_f32 (RNE, NaN-preserving)
  return *reinterpret_cast<uint16_t*>(&h);
}
__device__ __forceinline__ float f16_to_f32(uint16_t v) { return __half2float(__ushort_as_half(v)); }
__device__ __forceinline__ uint16_t f32_to_f16(float f) { return __half_as_ushort(__float2half(f)); }

// 16-bit storage codes used by the kernels' dtype flags: 0 = fp32, 1 = bf16, 2 = fp16
__device__ __forceinline__ float h16_to_f32(uint16_t v, int code) {
  return code == 2 ? f16_to_f32(v) : bf16_to_f32(v);
}
__device__ __forceinline__ uint16_t f32_to_h16(float f, int code) {
  return code == 2 ? f32_to_f16(f) : f32_to_bf16(f);
}
__device__ __forceinline__ float ld(const void* p, int64_t i, int code) {
  return code ? h16_to_f32(static_cast<const uint16_t*>(p)[i], code) : static_cast<const float*>(p)[i];
}
__device__ __forceinline__ void st(void* p, int64_t i, float v, int code) {
  if (code) static_cast<uint16_t*>(p)[i] = f32_to_h16(v, code);
  else static_cast<float*>(p)[i] = v;
}

// 8 consecutive bf16 <-> fp32 through one 16-B access (p 16-B aligned)
__device__ __forceinline__ void ld8_bf16(const uint16_t* p, float* v) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = __uint_as_float(w[k] << 16);
    v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}
__device__ __forceinline__ void st8_bf16(uint16_t* p, const float* v) {
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) w[k] = (uint32_t)f32_to_bf16(v[2 * k]) | ((uint32_t)f32_to_bf16(v[2 * k + 1]) << 16);
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}

// 8 consecutive 16-bit values (bf16 or fp16 by code) <-> fp32 through one 16-B access
__device__ __forceinline__ void ld8_h16(const uint16_t* p, float* v, int code) {
  if (code != 2) {
    ld8_bf16(p, v);
    return;
  }
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = f16_to_f32((uint16_t)(w[k] & 0xffffu));
    v[2 * k + 1] = f16_to_f32((uint16_t)(w[k] >> 16));
  }
}
__device__ __forceinline__ void st8_h16(uint16_t* p, const float* v, int code) {
  if (code != 2) {
    st8_bf16(p, v);
    return;
  }
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) w[k] = (uint32_t)f32_to_f16(v[2 * k]) | ((uint32_t)f32_to_f16(v[2 * k + 1]) << 16);
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}

// Wave64 reduction (sum) via DPP-backed shuffles.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Box IoU with the +1 pixel convention (reference: bbox_overlaps / nms).
__device__ __forceinline__ float iou_plus1(float ax1, float ay1, float ax2, float ay2, float aarea,
                                           float bx1, float by1, float bx2, float by2, float barea) {
  float iw = fminf(ax2, bx2) - fmaxf(ax1, bx1) + 1.f;
  float ih = fminf(ay2, by2) - fmaxf(ay1, by1) + 1.f;
  if (iw <= 0.f || ih <= 0.f) return 0.f;
  float inter = iw * ih;
  return inter / (aarea + barea - inter);
}

// Philox-4x32-10 (Salmon et al. 2011), the counter-based generator behind the fused dropout:
// key = (seed, 0x9E3779B9), counter = (lo(e), hi(e), lo(step), hi(step)); returns the first
// output word as a uniform in [0, 1) with 24 bits of resolution.  Pure function of its inputs,
// so every epilogue path (vector, scalar, split-K reduce) and the host twin agree bit for bit.
__host__ __device__ __forceinline__ float philox_uniform(uint32_t seed, uint64_t step, uint64_t e) {
  uint32_t c0 = (uint32_t)e, c1 = (uint32_t)(e >> 32), c2 = (uint32_t)step, c3 = (uint32_t)(step >> 32);
  uint32_t k0 = seed, k1 = 0x9E3779B9u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0, h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
    c0 = h1 ^ c1 ^ k0;
    c1 = l1;
    c2 = h0 ^ c3 ^ k1;
    c3 = l0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return (float)(c0 >> 8) * (1.0f / 16777216.0f);
}

inline int div_up(int64_t a, int64_t b) { return static_cast<int>((a + b - 1) / b); }

}  // namespace mxr
