// RoI max pooling, forward + backward, on NHWC feature maps (kernel K11;
// MXNet/Caffe ROIPooling semantics: rounded RoI corners, floor/ceil bin edges, strict '>'
// first-max-wins scan in row-major order, empty bin -> 0 with argmax -1).
//
// Layout choice: with channels innermost, the 64 lanes of a wave read 64 (x VEC) consecutive
// channels of the same (h, w) cell, so every bin scan is a fully coalesced 512 B..1 KiB row
// read instead of the NCHW kernel's one-element-per-thread gather.  Forward handles VEC=4
// channels per lane (8 B bf16 / 16 B fp32 loads).  Backward scatters with fp32 atomics shaped
// one channel per lane, i.e. each wave-instruction adds 256 contiguous bytes (Guideline 12);
// 128 RoIs x 49 bins x 1024 ch = 25 MB of adds, ~20 us at the chip-wide atomic rate.
#include "common.h"
#include <cstdlib>
#include "../kernels.h"

namespace mxr {

template <typename T> struct Vec4;
template <> struct Vec4<float> { using type = float4; };
template <> struct Vec4<uint16_t> { using type = ushort4; };

__device__ __forceinline__ float to_f(float v, int) { return v; }
__device__ __forceinline__ float to_f(uint16_t v, int code) { return h16_to_f32(v, code); }

struct Bin {
  int b, hs, he, ws, we;
  bool empty;
};

__device__ __forceinline__ Bin roi_bin(const float* __restrict__ rois, int r, int ph, int pw, int PH, int PW,
                                       int H, int W, float scale) {
  const float* roi = rois + (int64_t)r * 5;
  Bin o;
  o.b = (int)roi[0];
  const int x1 = (int)roundf(roi[1] * scale), y1 = (int)roundf(roi[2] * scale);
  const int x2 = (int)roundf(roi[3] * scale), y2 = (int)roundf(roi[4] * scale);
  const int rw = max(x2 - x1 + 1, 1), rh = max(y2 - y1 + 1, 1);
  const float bh = (float)rh / (float)PH, bw = (float)rw / (float)PW;
  o.hs = min(max((int)floorf(ph * bh) + y1, 0), H);
  o.he = min(max((int)ceilf((ph + 1) * bh) + y1, 0), H);
  o.ws = min(max((int)floorf(pw * bw) + x1, 0), W);
  o.we = min(max((int)ceilf((pw + 1) * bw) + x1, 0), W);
  o.empty = (o.he <= o.hs) || (o.we <= o.ws) || o.b < 0;
  return o;
}

template <typename T>
__global__ void __launch_bounds__(256)
roi_pool_fwd_vec4(const T* __restrict__ feat, int code, int B, int H, int W, int C, const float* __restrict__ rois, int R,
                  int PH, int PW, float scale, T* __restrict__ out, int32_t* __restrict__ argmax, PostBn post) {
  // code 3 / 4 (x2 pairs / x3 triples, T = uint16_t): planes one (B, H, W, C) / (R, PH, PW, C) block apart
  const int64_t fplane = (int64_t)B * H * W * C, oplane = (int64_t)R * PH * PW * C;
  using V = typename Vec4<T>::type;
  const int CV = C >> 2;
  const int64_t total = (int64_t)R * PH * PW * CV;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int cv = (int)(t % CV);
  int64_t rest = t / CV;
  const int pw = (int)(rest % PW); rest /= PW;
  const int ph = (int)(rest % PH);
  const int r = (int)(rest / PH);
  const Bin bin = roi_bin(rois, r, ph, pw, PH, PW, H, W, scale);
  float m0, m1, m2, m3;
  int a0 = -1, a1 = -1, a2 = -1, a3 = -1;
  if (bin.empty || bin.b >= B) {
    m0 = m1 = m2 = m3 = 0.f;
  } else {
    m0 = m1 = m2 = m3 = -FLT_MAX;
    const T* fb = feat + (int64_t)bin.b * H * W * C + (int64_t)cv * 4;
    for (int h = bin.hs; h < bin.he; ++h) {
      for (int w = bin.ws; w < bin.we; ++w) {
        const int idx = h * W + w;
        const V v = *reinterpret_cast<const V*>(fb + (int64_t)idx * C);
        float f0 = to_f(v.x, code >= 3 ? 1 : code), f1 = to_f(v.y, code >= 3 ? 1 : code);
        float f2 = to_f(v.z, code >= 3 ? 1 : code), f3 = to_f(v.w, code >= 3 ? 1 : code);
        if constexpr (sizeof(T) == 2) {
          for (int pl = 1; pl <= code - 2; ++pl) {  // x2: plane 1; x3: planes 1, 2
            const V l = *reinterpret_cast<const V*>(fb + pl * fplane + (int64_t)idx * C);
            f0 += to_f(l.x, 1); f1 += to_f(l.y, 1); f2 += to_f(l.z, 1); f3 += to_f(l.w, 1);
          }
        }
        if (f0 > m0) { m0 = f0; a0 = idx; }
        if (f1 > m1) { m1 = f1; a1 = idx; }
        if (f2 > m2) { m2 = f2; a2 = idx; }
        if (f3 > m3) { m3 = f3; a3 = idx; }
      }
    }
  }
  if (post.scale) {
    m0 = post_bn_relu(post, cv * 4, m0); m1 = post_bn_relu(post, cv * 4 + 1, m1);
    m2 = post_bn_relu(post, cv * 4 + 2, m2); m3 = post_bn_relu(post, cv * 4 + 3, m3);
  }
  const int64_t o = t * 4;
  if constexpr (sizeof(T) == 2) {
    if (code >= 3) {
      const float mv[4] = {m0, m1, m2, m3};
      st4c(out, o, code, oplane, mv);
    } else {
      ushort4 ov = make_ushort4(f32_to_h16(m0, code), f32_to_h16(m1, code), f32_to_h16(m2, code), f32_to_h16(m3, code));
      *reinterpret_cast<ushort4*>(out + o) = ov;
    }
  } else {
    *reinterpret_cast<float4*>(out + o) = make_float4(m0, m1, m2, m3);
  }
  if (argmax) *reinterpret_cast<int4*>(argmax + o) = make_int4(a0, a1, a2, a3);  // null: inference, no backward
}

// 8 channels per lane, single-plane 16-bit maps (bf16 / fp16): 16-B loads, U bin pixels per
// iteration in flight (MXR_ROI_UNROLL, default 2); the batch-8 inference pooling (2400 RoIs x 49 bins x 1024 channels) is a
// latency-bound gather at 4 channels per lane and one load at a time
template <int U>
__global__ void __launch_bounds__(256)
roi_pool_fwd_vec8(const uint16_t* __restrict__ feat, int code, int B, int H, int W, int C,
                  const float* __restrict__ rois, int R, int PH, int PW, float scale, uint16_t* __restrict__ out,
                  int32_t* __restrict__ argmax, PostBn post) {
  const int CV = C >> 3;
  const int64_t total = (int64_t)R * PH * PW * CV;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int cv = (int)(t % CV);
  int64_t rest = t / CV;
  const int pw = (int)(rest % PW); rest /= PW;
  const int ph = (int)(rest % PH);
  const int r = (int)(rest / PH);
  const Bin bin = roi_bin(rois, r, ph, pw, PH, PW, H, W, scale);
  float m[8];
  int a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    m[k] = 0.f;
    a[k] = -1;
  }
  if (!(bin.empty || bin.b >= B)) {
#pragma unroll
    for (int k = 0; k < 8; ++k) m[k] = -FLT_MAX;
    const uint16_t* fb = feat + (int64_t)bin.b * H * W * C + (int64_t)cv * 8;
    const int npx = (bin.he - bin.hs) * (bin.we - bin.ws);
    auto upd = [&](const uint4 v, int idx) {
      const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float f0 = h16_to_f32((uint16_t)(wv[k] & 0xffffu), code), f1 = h16_to_f32((uint16_t)(wv[k] >> 16), code);
        if (f0 > m[2 * k]) { m[2 * k] = f0; a[2 * k] = idx; }
        if (f1 > m[2 * k + 1]) { m[2 * k + 1] = f1; a[2 * k + 1] = idx; }
      }
    };
    // row-major walk with a running (h, w): U loads issued together, compared in order
    int h = bin.hs, w = bin.ws;
    auto next = [&]() {
      const int idx = h * W + w;
      if (++w == bin.we) {
        w = bin.ws;
        ++h;
      }
      return idx;
    };
    int q = 0;
    for (; q + U - 1 < npx; q += U) {
      int ix[U];
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) ix[u] = next();
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const uint4*>(fb + (int64_t)ix[u] * C);
#pragma unroll
      for (int u = 0; u < U; ++u) upd(v[u], ix[u]);
    }
    for (; q < npx; ++q) {
      const int i0 = next();
      upd(*reinterpret_cast<const uint4*>(fb + (int64_t)i0 * C), i0);
    }
  }
  if (post.scale) post_bn_relu8(post, cv * 8, m);
  uint32_t o[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    o[k] = (uint32_t)f32_to_h16(m[2 * k], code) | ((uint32_t)f32_to_h16(m[2 * k + 1], code) << 16);
  *reinterpret_cast<uint4*>(out + t * 8) = make_uint4(o[0], o[1], o[2], o[3]);
  if (argmax) {
    int4* ap = reinterpret_cast<int4*>(argmax + t * 8);
    ap[0] = make_int4(a[0], a[1], a[2], a[3]);
    ap[1] = make_int4(a[4], a[5], a[6], a[7]);
  }
}

template <typename T>
__global__ void __launch_bounds__(256)
roi_pool_fwd_scalar(const T* __restrict__ feat, int code, int B, int H, int W, int C, const float* __restrict__ rois, int R,
                    int PH, int PW, float scale, T* __restrict__ out, int32_t* __restrict__ argmax, PostBn post) {
  const int64_t total = (int64_t)R * PH * PW * C;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int c = (int)(t % C);
  int64_t rest = t / C;
  const int pw = (int)(rest % PW); rest /= PW;
  const int ph = (int)(rest % PH);
  const int r = (int)(rest / PH);
  const Bin bin = roi_bin(rois, r, ph, pw, PH, PW, H, W, scale);
  float m = 0.f;
  int a = -1;
  if (!(bin.empty || bin.b >= B)) {
    m = -FLT_MAX;
    const T* fb = feat + (int64_t)bin.b * H * W * C + c;
    for (int h = bin.hs; h < bin.he; ++h)
      for (int w = bin.ws; w < bin.we; ++w) {
        const int idx = h * W + w;
        const float f = to_f(fb[(int64_t)idx * C], code);
        if (f > m) { m = f; a = idx; }
      }
  }
  if (post.scale) m = post_bn_relu(post, c, m);
  if constexpr (sizeof(T) == 2) out[t] = f32_to_h16(m, code); else out[t] = m;
  if (argmax) argmax[t] = a;
}

template <typename T>
__global__ void __launch_bounds__(256)
roi_pool_bwd_kernel(const T* __restrict__ gout, const int32_t* __restrict__ argmax, const float* __restrict__ rois,
                    int R, int PH, int PW, int B, int HW, int C, float* __restrict__ gin) {
  const int64_t total = (int64_t)R * PH * PW * C;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int a = argmax[t];
  if (a < 0) return;
  const int c = (int)(t % C);
  const int r = (int)(t / ((int64_t)PH * PW * C));
  const int b = (int)rois[(int64_t)r * 5];
  if (b < 0 || b >= B) return;
  const float g = to_f(gout[t], 1);
  if (g != 0.f) atomicAdd(gin + ((int64_t)b * HW + a) * C + c, g);  // no-return global_atomic_add_f32
}

void roi_pool_fwd(const void* feat, int bf16, int B, int H, int W, int C, const float* rois, int R, int PH, int PW,
                  float spatial_scale, void* out, int32_t* argmax, hipStream_t st, PostBn post) {
  if (R == 0 || C == 0) return;
  if (C % 8 == 0 && (bf16 == 1 || bf16 == 2)) {  // single-plane 16-bit: 8 channels per lane
    const int64_t total = (int64_t)R * PH * PW * (C / 8);
    static const int unroll = [] {
      const char* e = getenv("MXR_ROI_UNROLL");
      return e && atoi(e) == 4 ? 4 : 2;
    }();
    if (unroll == 4)
      roi_pool_fwd_vec8<4><<<div_up(total, 256), 256, 0, st>>>((const uint16_t*)feat, bf16, B, H, W, C, rois, R, PH, PW,
                                                               spatial_scale, (uint16_t*)out, argmax, post);
    else
      roi_pool_fwd_vec8<2><<<div_up(total, 256), 256, 0, st>>>((const uint16_t*)feat, bf16, B, H, W, C, rois, R, PH, PW,
                                                               spatial_scale, (uint16_t*)out, argmax, post);
    return;
  }
  if (C % 4 == 0) {
    const int64_t total = (int64_t)R * PH * PW * (C / 4);
    if (bf16)
      roi_pool_fwd_vec4<uint16_t><<<div_up(total, 256), 256, 0, st>>>(
          (const uint16_t*)feat, bf16, B, H, W, C, rois, R, PH, PW, spatial_scale, (uint16_t*)out, argmax, post);
    else
      roi_pool_fwd_vec4<float><<<div_up(total, 256), 256, 0, st>>>(
          (const float*)feat, 0, B, H, W, C, rois, R, PH, PW, spatial_scale, (float*)out, argmax, post);
  } else {
    const int64_t total = (int64_t)R * PH * PW * C;
    if (bf16)
      roi_pool_fwd_scalar<uint16_t><<<div_up(total, 256), 256, 0, st>>>(
          (const uint16_t*)feat, bf16, B, H, W, C, rois, R, PH, PW, spatial_scale, (uint16_t*)out, argmax, post);
    else
      roi_pool_fwd_scalar<float><<<div_up(total, 256), 256, 0, st>>>(
          (const float*)feat, 0, B, H, W, C, rois, R, PH, PW, spatial_scale, (float*)out, argmax, post);
  }
}

// Atomic-free (in global memory) backward: one workgroup per (image, CW-channel slab) accumulates
// the whole H x W x CW gradient slab in LDS, walking every bin of the image's RoIs (argmax + dY:
// 16 + 8 B per bin for CW = 4), then writes its channels of every pixel in the output dtype.  Replaces: a zero fill of an fp32 (B, H, W, C) buffer, 6.4 M global
// fp32 atomics (~120 us at 128 RoIs x 49 bins x 1024 ch) and the cast to bf16.
// CW consecutive channels of one pixel as one vector access (8 B for 4 bf16 / fp16)
template <int CW>
__device__ __forceinline__ void ldv(const uint16_t* p, float* v, int code) {
  if constexpr (CW == 4) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    const uint16_t h[4] = {(uint16_t)(u.x & 0xffff), (uint16_t)(u.x >> 16), (uint16_t)(u.y & 0xffff),
                           (uint16_t)(u.y >> 16)};
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = to_f(h[k], code);
  } else {
#pragma unroll
    for (int k = 0; k < CW; ++k) v[k] = to_f(p[k], code);
  }
}
template <int CW>
__device__ __forceinline__ void ldv(const float* p, float* v, int) {
#pragma unroll
  for (int k = 0; k < CW; ++k) v[k] = p[k];
}
template <int CW>
__device__ __forceinline__ void stv(uint16_t* p, const float* v, int code) {
  if constexpr (CW == 4) {
    uint16_t h[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) h[k] = f32_to_h16(v[k], code);
    *reinterpret_cast<uint2*>(p) = make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16),
                                              (uint32_t)h[2] | ((uint32_t)h[3] << 16));
  } else {
#pragma unroll
    for (int k = 0; k < CW; ++k) p[k] = f32_to_h16(v[k], code);
  }
}
template <int CW>
__device__ __forceinline__ void stv(float* p, const float* v, int) {
#pragma unroll
  for (int k = 0; k < CW; ++k) p[k] = v[k];
}

// Deterministic accumulation: float atomics add in whatever order the waves arrive, so the last bits
// of a pixel's gradient (and of everything below the RoI pooling in the fp32 modes) varied run to
// run.  The slab is instead an exact fixed-point sum: per (image, channel) the largest |dY| over
// the image's bins fixes a power-of-two scale 2^s with max * (bins) < 2^61, every bin's dY is
// added as the 64-bit integer rint(dY * 2^s) (integer addition is associative: any arrival order
// gives the same bits), and the output is float(sum) * 2^-s -- one rounding, more accurate than
// the fp32 atomic chain; a contribution below 2^-27 of the channel's largest keeps its low bits
// only down to 2^-50 of it.  The other gradient of the feature map (gadd: the RPN head's) is added
// once per pixel at the end.  A non-finite dY (a diverging step) has no fixed-point image: its
// channel's gradient for the image is written as NaN, so the trunk gradient stays non-finite and
// the trainer's non-finite guard sees it (a float atomic chain would have propagated it too).
template <int CW, typename T>
__global__ void __launch_bounds__(256)
roi_pool_bwd_lds_kernel(const T* __restrict__ gout, const int32_t* __restrict__ argmax, const float* __restrict__ rois,
                        int R, int PHW, int HW, int C, int code, const T* __restrict__ gadd, T* __restrict__ gin) {
  extern __shared__ long long acc[];  // [HW][CW] fixed-point sums
  __shared__ float red[4][CW];        // per-wave channel maxima
  __shared__ int sh_scale[CW];
  __shared__ int sh_nf[CW];           // channel saw a non-finite dY in this image
  // code 3 / 4 (x2 / x3 planes): gout's planes one (R, PH, PW, C) block apart, gadd's / gin's one (B, H, W, C)
  const int64_t oplane = (int64_t)R * PHW * C, iplane = (int64_t)gridDim.y * HW * C;
  // XCD-aware channel groups: workgroups are dealt round-robin over the 8 XCDs, so consecutive
  // block ids would put neighbouring channel groups -- which read and write the same cache lines
  // of the NHWC argmax / gradient rows -- on different L2s.  Consecutive groups share an XCD.
  const int nx = gridDim.x, bx = blockIdx.x;
  const int q = nx / 8, r8 = nx % 8, xcd = bx % 8;
  const int grp = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + bx / 8;
  const int c0 = grp * CW, b = blockIdx.y;
  const int nb = R * PHW;
  auto load_g = [&](int i, float* g, int* a) {
    const int64_t base = (int64_t)i * C + c0;
    if constexpr (CW == 4) {  // c0 and C are multiples of 4: 16-B argmax / 8-B (per plane) gradient loads
      const int4 av = *reinterpret_cast<const int4*>(argmax + base);
      a[0] = av.x; a[1] = av.y; a[2] = av.z; a[3] = av.w;
      if (code >= 3) ld4c(gout, base, code, oplane, g);
      else
#pragma unroll
        for (int k = 0; k < CW; ++k) g[k] = to_f(gout[base + k], code);
    } else {
#pragma unroll
      for (int k = 0; k < CW; ++k) {
        a[k] = argmax[base + k];
        g[k] = code >= 3 ? ldc(gout, base + k, code, oplane) : to_f(gout[base + k], code);
      }
    }
  };
  // pass 1: zero the slab, and the largest |dY| per channel over this image's bins
  for (int p = threadIdx.x; p < HW * CW; p += blockDim.x) acc[p] = 0;
  float mx[CW];
  int nf[CW];  // fmaxf drops NaN and inf has no usable exponent: track non-finite dY separately
#pragma unroll
  for (int k = 0; k < CW; ++k) {
    mx[k] = 0.f;
    nf[k] = 0;
  }
  if (threadIdx.x < CW) sh_nf[threadIdx.x] = 0;
  // (only a bound is needed: every bin's |dY| regardless of its argmax, and with planes the hi plane
  // alone -- |v| <= |hi| * (1 + 2^-7) -- so this pass reads 8 B per 4 channels, not dY + argmax)
  const int hi_off = code == 4 ? 1 : 0;  // x3 planes (mid, hi, lo); x2 (hi, lo)
  for (int i = threadIdx.x; i < nb; i += blockDim.x) {
    if ((int)rois[(int64_t)(i / PHW) * 5] != b) continue;
    const int64_t base = (int64_t)i * C + c0;
    float g[CW];
    if constexpr (CW == 4 && sizeof(T) == 2) {
      const ushort4 v = *reinterpret_cast<const ushort4*>(gout + base + (code >= 3 ? hi_off * oplane : 0));
      g[0] = to_f(v.x, code >= 3 ? 1 : code); g[1] = to_f(v.y, code >= 3 ? 1 : code);
      g[2] = to_f(v.z, code >= 3 ? 1 : code); g[3] = to_f(v.w, code >= 3 ? 1 : code);
    } else {
#pragma unroll
      for (int k = 0; k < CW; ++k)
        g[k] = to_f(gout[base + k + (code >= 3 ? hi_off * oplane : 0)], code >= 3 ? 1 : code);
    }
#pragma unroll
    for (int k = 0; k < CW; ++k) {
      if (!isfinite(g[k])) nf[k] = 1;  // (a non-finite value has a non-finite hi plane)
      else mx[k] = fmaxf(mx[k], fabsf(g[k]));
    }
  }
  if (code >= 3)
#pragma unroll
    for (int k = 0; k < CW; ++k) mx[k] *= 1.0f + 1.0f / 64.0f;
#pragma unroll
  for (int k = 0; k < CW; ++k) mx[k] = wave_max(mx[k]);
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < CW; ++k) red[threadIdx.x >> 6][k] = mx[k];
#pragma unroll
  for (int k = 0; k < CW; ++k)
    if (nf[k]) atomicOr(&sh_nf[k], 1);  // rare: only on a diverging step
  __syncthreads();
  if (threadIdx.x < CW) {
    const float m = fmaxf(fmaxf(red[0][threadIdx.x], red[1][threadIdx.x]), fmaxf(red[2][threadIdx.x], red[3][threadIdx.x]));
    // max * 2^s * nb < 2^61:  s = 60 - ceil(log2(max)) - ceil(log2(nb))
    int e = 0;
    if (m > 0.f) frexpf(m, &e);  // m < 2^e
    int lb = 0;
    while ((1 << lb) < nb) ++lb;
    sh_scale[threadIdx.x] = m > 0.f ? 60 - e - lb : 0;
  }
  __syncthreads();
  int sc[CW];
#pragma unroll
  for (int k = 0; k < CW; ++k) sc[k] = sh_scale[k];
  // pass 2: exact integer accumulation (any order, same bits)
  for (int i = threadIdx.x; i < nb; i += blockDim.x) {
    if ((int)rois[(int64_t)(i / PHW) * 5] != b) continue;
    float g[CW];
    int a[CW];
    load_g(i, g, a);
#pragma unroll
    for (int k = 0; k < CW; ++k)
      if (a[k] >= 0 && a[k] < HW && g[k] != 0.f && isfinite(g[k]))
        atomicAdd(reinterpret_cast<unsigned long long*>(&acc[a[k] * CW + k]),
                  (unsigned long long)__float2ll_rn(ldexpf(g[k], sc[k])));
  }
  __syncthreads();
  // pass 3: back to float (one rounding), plus the feature map's other gradient, in the output format
#pragma unroll 4
  for (int p = threadIdx.x; p < HW; p += blockDim.x) {
    float v[CW], ga[CW];
#pragma unroll
    for (int k = 0; k < CW; ++k) v[k] = sh_nf[k] ? __builtin_nanf("") : ldexpf((float)acc[p * CW + k], -sc[k]);
    if (gadd) {
      if (code >= 3 && CW == 4) {
        ld4c(gadd, ((int64_t)b * HW + p) * C + c0, code, iplane, ga);  // one 8-B load per plane
      } else if (code >= 3) {
#pragma unroll
        for (int k = 0; k < CW; ++k) ga[k] = ldc(gadd, ((int64_t)b * HW + p) * C + c0 + k, code, iplane);
      } else {
        ldv<CW>(gadd + ((int64_t)b * HW + p) * C + c0, ga, code);
      }
#pragma unroll
      for (int k = 0; k < CW; ++k) v[k] += ga[k];
    }
    if (code >= 3 && CW == 4) {
      st4c(gin, ((int64_t)b * HW + p) * C + c0, code, iplane, v);
    } else if (code >= 3) {
#pragma unroll
      for (int k = 0; k < CW; ++k) stc(gin, ((int64_t)b * HW + p) * C + c0 + k, v[k], code, iplane);
    } else {
      stv<CW>(gin + ((int64_t)b * HW + p) * C + c0, v, code);
    }
  }
}

constexpr int kRoiBwdLds = 150 * 1024;

int roi_pool_bwd_lds(const void* grad_out, int code, const int32_t* argmax, const float* rois, int R, int PH, int PW,
                     int B, int H, int W, int C, void* grad_in, hipStream_t st, const void* grad_add) {
  const int HW = H * W;
  int cw = 0;  // channels per workgroup: the 8-B fixed-point slab of HW x cw must fit the LDS budget
  if (C % 4 == 0 && (int64_t)HW * 4 * 8 <= kRoiBwdLds) cw = 4;
  else if (C % 2 == 0 && (int64_t)HW * 2 * 8 <= kRoiBwdLds) cw = 2;
  else if ((int64_t)HW * 8 <= kRoiBwdLds) cw = 1;
  if (cw == 0 || B <= 0 || (int64_t)R * PH * PW > (1 << 20)) return -1;
  const size_t lds = (size_t)HW * cw * 8;
  const dim3 grid(C / cw, B);
#define MXR_ROI_BWD(CW_, T_)                                                                                   \
  do {                                                                                                        \
    static bool attr = false;                                                                                 \
    if (!attr) {                                                                                              \
      (void)hipFuncSetAttribute((const void*)roi_pool_bwd_lds_kernel<CW_, T_>,                                \
                                hipFuncAttributeMaxDynamicSharedMemorySize, kRoiBwdLds);                      \
      attr = true;                                                                                            \
    }                                                                                                         \
    roi_pool_bwd_lds_kernel<CW_, T_><<<grid, 256, lds, st>>>((const T_*)grad_out, argmax, rois, R, PH * PW, HW, C, \
                                                             code, (const T_*)grad_add, (T_*)grad_in);       \
  } while (0)
  if (code) {
    if (cw == 4) MXR_ROI_BWD(4, uint16_t);
    else if (cw == 2) MXR_ROI_BWD(2, uint16_t);
    else MXR_ROI_BWD(1, uint16_t);
  } else {
    if (cw == 4) MXR_ROI_BWD(4, float);
    else if (cw == 2) MXR_ROI_BWD(2, float);
    else MXR_ROI_BWD(1, float);
  }
#undef MXR_ROI_BWD
  return 0;
}

void roi_pool_bwd(const void* grad_out, int bf16, const int32_t* argmax, const float* rois, int R, int PH, int PW,
                  int B, int H, int W, int C, float* grad_in, hipStream_t st) {
  const int64_t total = (int64_t)R * PH * PW * C;
  if (total == 0) return;
  if (bf16)
    roi_pool_bwd_kernel<uint16_t><<<div_up(total, 256), 256, 0, st>>>((const uint16_t*)grad_out, argmax, rois, R,
                                                                       PH, PW, B, H * W, C, grad_in);
  else
    roi_pool_bwd_kernel<float><<<div_up(total, 256), 256, 0, st>>>((const float*)grad_out, argmax, rois, R, PH, PW,
                                                                    B, H * W, C, grad_in);
}

__global__ void __launch_bounds__(256) cast_f32_bf16_kernel(const float* __restrict__ in, uint16_t* __restrict__ out,
                                                             int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 3 < n) {
    const float4 v = *reinterpret_cast<const float4*>(in + i);
    *reinterpret_cast<ushort4*>(out + i) = make_ushort4(f32_to_bf16(v.x), f32_to_bf16(v.y), f32_to_bf16(v.z),
                                                        f32_to_bf16(v.w));
  } else {
    for (int64_t k = i; k < n; ++k) out[k] = f32_to_bf16(in[k]);
  }
}

void cast_f32(const float* in, void* out, int out_bf16, int64_t n, hipStream_t st) {
  if (n == 0) return;
  if (out_bf16)
    cast_f32_bf16_kernel<<<div_up((n + 3) / 4, 256), 256, 0, st>>>(in, (uint16_t*)out, n);
  else
    (void)hipMemcpyAsync(out, in, n * sizeof(float), hipMemcpyDeviceToDevice, st);
}

}  // namespace mxr
