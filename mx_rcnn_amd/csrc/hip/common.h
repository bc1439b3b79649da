// Shared device helpers for the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <cstdint>
#include <cfloat>

#include "../kernels.h"

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
// PostBn (kernels.h): relu(v * s + t) with bn_act.hip's per-channel coefficients, so the fused
// pooling output is bit-identical to pooling followed by bn_relu_fwd
__device__ __forceinline__ float post_bn_relu(const PostBn& p, int c, float v) {
  return fmaxf(v * p.scale[c] + p.shift[c], 0.f);
}
// 8 consecutive channels c0..c0+7 (c0 % 8 == 0): two 16-B loads per coefficient
__device__ __forceinline__ void post_bn_relu8(const PostBn& p, int c0, float* v) {
  const float4 s0 = *reinterpret_cast<const float4*>(p.scale + c0), s1 = *reinterpret_cast<const float4*>(p.scale + c0 + 4);
  const float4 t0 = *reinterpret_cast<const float4*>(p.shift + c0), t1 = *reinterpret_cast<const float4*>(p.shift + c0 + 4);
  const float s[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
  const float t[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = fmaxf(v[k] * s[k] + t[k], 0.f);
}

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

// ---- multi-plane bf16 storage of the fp32 training modes --------------------------------------
// x2 ("bf16x3" mode): every MFMA operand is a PAIR of bf16 planes `plane` elements apart, value =
// hi + lo with hi = RNE(v), lo = RNE(v - hi) -- 16 significant bits -- and a product is
// hi*hi + hi*lo + lo*hi on the bf16 MFMA with fp32 accumulation.  Tensors are (2N, C, H, W), hi
// plane first.
// x3 (the fp32 mode): THREE planes [mid | hi | lo] `plane` apart, hi = RNE(v), mid = RNE(v - hi),
// lo = RNE(v - hi - mid): hi + mid + lo == v exactly (24 significant bits, IEEE fp32 storage), and
// a product is the six terms hh + hm + mh + hl + lh + mm (the dropped ml + lm + ll are below 2^-23
// relative, the size of one fp32 rounding).  Tensors are (3N, C, H, W).  The plane order makes the
// MFMA kernels' two K phases uniform shifts of one operand base: phase (hi, lo) reads planes 1 / 2
// = the pair kernel's (first, second) one plane further on than phase (mid, hi), planes 0 / 1, so a
// pair kernel runs x3 with its K loop twice and a per-phase SGPR offset (hh + hl + lh, then
// mm + mh + hm).  The sign of v is the sign of hi (plane 1).
__device__ __forceinline__ void split_bf16(float v, uint16_t& hi, uint16_t& lo) {
  hi = f32_to_bf16(v);
  lo = f32_to_bf16(v - bf16_to_f32(hi));
}
__device__ __forceinline__ void split3_bf16(float v, uint16_t& hi, uint16_t& mid, uint16_t& lo) {
  hi = f32_to_bf16(v);
  const float r = v - bf16_to_f32(hi);
  mid = f32_to_bf16(r);
  lo = f32_to_bf16(r - bf16_to_f32(mid));
}
// x3 = false: a pair (planes 0, 1); true: a triple (planes 0, 1, 2); the sum is exact either way
__device__ __forceinline__ float ldx(const uint16_t* p, int64_t i, int64_t plane, bool x3 = false) {
  const float v = bf16_to_f32(p[i]) + bf16_to_f32(p[i + plane]);
  return x3 ? v + bf16_to_f32(p[i + 2 * plane]) : v;
}
// stores v in the planes and returns the stored value (what a consumer reading it back sees)
__device__ __forceinline__ float stx(uint16_t* p, int64_t i, int64_t plane, float v, bool x3 = false) {
  if (x3) {
    uint16_t h, m, l;
    split3_bf16(v, h, m, l);
    p[i] = m;
    p[i + plane] = h;
    p[i + 2 * plane] = l;
    return (bf16_to_f32(m) + bf16_to_f32(h)) + bf16_to_f32(l);
  }
  uint16_t h, l;
  split_bf16(v, h, l);
  p[i] = h;
  p[i + plane] = l;
  return bf16_to_f32(h) + bf16_to_f32(l);
}
__device__ __forceinline__ void ld8x(const uint16_t* p, int64_t plane, float* v, bool x3 = false) {
  float t[8];
  ld8_bf16(p, v);
  ld8_bf16(p + plane, t);
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] += t[k];
  if (x3) {
    ld8_bf16(p + 2 * plane, t);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] += t[k];
  }
}
// 8 values -> planes; `stored` (may alias v) receives the stored values
__device__ __forceinline__ void st8x(uint16_t* p, int64_t plane, const float* v, float* stored, bool x3 = false) {
  float h[8], l[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    h[k] = bf16_to_f32(f32_to_bf16(v[k]));
    l[k] = v[k] - h[k];
  }
  if (x3) {
    float m[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      m[k] = bf16_to_f32(f32_to_bf16(l[k]));
      l[k] -= m[k];
    }
    st8_bf16(p, m);  // exact: m and h are already bf16
    st8_bf16(p + plane, h);
    st8_bf16(p + 2 * plane, l);
#pragma unroll
    for (int k = 0; k < 8; ++k) stored[k] = (m[k] + h[k]) + bf16_to_f32(f32_to_bf16(l[k]));
    return;
  }
  st8_bf16(p, h);      // exact: h is already bf16
  st8_bf16(p + plane, l);
#pragma unroll
  for (int k = 0; k < 8; ++k) stored[k] = h[k] + bf16_to_f32(f32_to_bf16(l[k]));
}

// Storage-code access for the elementwise kernels: 0 fp32, 1 bf16, 2 fp16, 3 x2 pair (bf16 hi
// plane + lo plane `plane` elements further; a kernel over an (M, C) activation passes M * C),
// 4 x3 triple (planes mid, hi, lo `plane` apart)
constexpr int kCodeX2 = 3;
constexpr int kCodeX3 = 4;
__device__ __forceinline__ bool code_planes(int code) { return code >= kCodeX2; }
__device__ __forceinline__ float ldc(const void* p, int64_t i, int code, int64_t plane) {
  if (code >= kCodeX2) return ldx(static_cast<const uint16_t*>(p), i, plane, code == kCodeX3);
  return ld(p, i, code);
}
__device__ __forceinline__ void stc(void* p, int64_t i, float v, int code, int64_t plane) {
  if (code >= kCodeX2) stx(static_cast<uint16_t*>(p), i, plane, v, code == kCodeX3);
  else st(p, i, v, code);
}
// 4 consecutive values (i % 4 == 0)
__device__ __forceinline__ void ld4c(const void* p, int64_t i, int code, int64_t plane, float v[4]) {
  if (code == 0) {
    const float4 f = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + i);
    v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
    return;
  }
  const uint16_t* q = static_cast<const uint16_t*>(p);
  const ushort4 u = *reinterpret_cast<const ushort4*>(q + i);
  const int c = code >= kCodeX2 ? 1 : code;
  v[0] = h16_to_f32(u.x, c); v[1] = h16_to_f32(u.y, c); v[2] = h16_to_f32(u.z, c); v[3] = h16_to_f32(u.w, c);
  for (int pl = 1; pl <= code - 2; ++pl) {  // x2: plane 1; x3: planes 1, 2
    const ushort4 l = *reinterpret_cast<const ushort4*>(q + i + pl * plane);
    v[0] += bf16_to_f32(l.x); v[1] += bf16_to_f32(l.y); v[2] += bf16_to_f32(l.z); v[3] += bf16_to_f32(l.w);
  }
}
__device__ __forceinline__ void st4c(void* p, int64_t i, int code, int64_t plane, const float v[4]) {
  if (code == 0) {
    *reinterpret_cast<float4*>(static_cast<float*>(p) + i) = make_float4(v[0], v[1], v[2], v[3]);
    return;
  }
  uint16_t* q = static_cast<uint16_t*>(p);
  if (code == kCodeX3) {
    uint16_t h[4], m[4], l[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) split3_bf16(v[k], h[k], m[k], l[k]);
    *reinterpret_cast<ushort4*>(q + i) = make_ushort4(m[0], m[1], m[2], m[3]);
    *reinterpret_cast<ushort4*>(q + i + plane) = make_ushort4(h[0], h[1], h[2], h[3]);
    *reinterpret_cast<ushort4*>(q + i + 2 * plane) = make_ushort4(l[0], l[1], l[2], l[3]);
    return;
  }
  if (code == kCodeX2) {
    uint16_t h[4], l[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) split_bf16(v[k], h[k], l[k]);
    *reinterpret_cast<ushort4*>(q + i) = make_ushort4(h[0], h[1], h[2], h[3]);
    *reinterpret_cast<ushort4*>(q + i + plane) = make_ushort4(l[0], l[1], l[2], l[3]);
    return;
  }
  *reinterpret_cast<ushort4*>(q + i) =
      make_ushort4(f32_to_h16(v[0], code), f32_to_h16(v[1], code), f32_to_h16(v[2], code), f32_to_h16(v[3], code));
}
// 8 consecutive values (i % 8 == 0)
__device__ __forceinline__ void ld8c(const void* p, int64_t i, int code, int64_t plane, float v[8]) {
  if (code == 0) {
    const float4* f = reinterpret_cast<const float4*>(static_cast<const float*>(p) + i);
    const float4 a = f[0], b = f[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    return;
  }
  const uint16_t* q = static_cast<const uint16_t*>(p) + i;
  if (code >= kCodeX2) ld8x(q, plane, v, code == kCodeX3);
  else ld8_h16(q, v, code);
}
__device__ __forceinline__ void st8c(void* p, int64_t i, int code, int64_t plane, const float v[8]) {
  if (code == 0) {
    float4* f = reinterpret_cast<float4*>(static_cast<float*>(p) + i);
    f[0] = make_float4(v[0], v[1], v[2], v[3]);
    f[1] = make_float4(v[4], v[5], v[6], v[7]);
    return;
  }
  uint16_t* q = static_cast<uint16_t*>(p) + i;
  if (code >= kCodeX2) {
    float s[8];
    st8x(q, plane, v, s, code == kCodeX3);
  } else {
    st8_h16(q, v, code);
  }
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

// One SGD-momentum update (MXNet sgd_mom_update: g = clip(rescale * g); mom = mu * mom - lr * (g +
// wd * w); w += mom): the SGD kernels (sgd.hip) and the fused wgrad + SGD epilogue (wgrad_body.h)
// share it, so both paths round identically.
__device__ __forceinline__ float sgd_one(float w, float& m, float g, float lr, float mu, float wd, float rescale,
                                         float clip) {
  g *= rescale;
  if (clip > 0.f) g = fminf(fmaxf(g, -clip), clip);
  m = mu * m - lr * (g + wd * w);
  return w + m;
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
