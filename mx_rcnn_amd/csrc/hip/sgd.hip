// Multi-tensor fused SGD-momentum over flat parameter buffers (SURVEY kernel K20; MXNet
// `sgd_mom_update` semantics: g = clip(rescale*g, +-clip); mom = mu*mom - lr*(g + wd*w);
// w += mom).  One launch per weight-decay group over the whole flat buffer, 4 elements per
// lane with 16-B loads.  The learning rate is read from device memory so the update can be
// captured in a hipGraph and replayed while the schedule changes.  The kernel also writes
// the bf16 shadow of the new weights that the next forward consumes (fusing the cast), and with
// `zero` clears the gradient buffer it consumed (no __restrict__ on either: they may alias, and
// every element is loaded before its zero is stored) (fp32 or bf16, may differ from `grad`: under data
// parallelism the kernel reads the fp32 wire buffer and clears the bf16 one), so the next step's
// gradient writers start from zero without a separate fill pass over every gradient.
#include "common.h"
#include "../kernels.h"
#include <algorithm>
#include <cstdlib>

namespace mxr {

template <bool GBF16>
__global__ void __launch_bounds__(256)
sgd_kernel(float* __restrict__ w, float* __restrict__ mom, const void* grad, int64_t n,
           const float* __restrict__ lr_p, float mu, float wd, float rescale, float clip, uint16_t* __restrict__ wb,
           int64_t x2_plane, int x3, void* zp, int zbf16) {
  const float lr = *lr_p;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
    if (i + 3 < n) {
      float4 wv = *reinterpret_cast<float4*>(w + i);
      float4 mv = *reinterpret_cast<float4*>(mom + i);
      float4 gv;
      if (GBF16) {
        const ushort4 gb = *reinterpret_cast<const ushort4*>(static_cast<const uint16_t*>(grad) + i);
        gv = make_float4(bf16_to_f32(gb.x), bf16_to_f32(gb.y), bf16_to_f32(gb.z), bf16_to_f32(gb.w));
      } else {
        gv = *reinterpret_cast<const float4*>(static_cast<const float*>(grad) + i);
      }
      if (zp) {
        if (zbf16) *reinterpret_cast<ushort4*>(static_cast<uint16_t*>(zp) + i) = make_ushort4(0, 0, 0, 0);
        else *reinterpret_cast<float4*>(static_cast<float*>(zp) + i) = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      wv.x = sgd_one(wv.x, mv.x, gv.x, lr, mu, wd, rescale, clip);
      wv.y = sgd_one(wv.y, mv.y, gv.y, lr, mu, wd, rescale, clip);
      wv.z = sgd_one(wv.z, mv.z, gv.z, lr, mu, wd, rescale, clip);
      wv.w = sgd_one(wv.w, mv.w, gv.w, lr, mu, wd, rescale, clip);
      *reinterpret_cast<float4*>(w + i) = wv;
      *reinterpret_cast<float4*>(mom + i) = mv;
      if (wb && x2_plane) {  // multi-plane shadow: x2 hi / lo pair or x3 (mid, hi, lo) triple (common.h)
        const float v4[4] = {wv.x, wv.y, wv.z, wv.w};
        st4c(wb, i, x3 ? kCodeX3 : kCodeX2, x2_plane, v4);
      } else if (wb) {
        *reinterpret_cast<ushort4*>(wb + i) =
            make_ushort4(f32_to_bf16(wv.x), f32_to_bf16(wv.y), f32_to_bf16(wv.z), f32_to_bf16(wv.w));
      }
    } else {
      for (int64_t k = i; k < n; ++k) {
        const float g = GBF16 ? bf16_to_f32(static_cast<const uint16_t*>(grad)[k]) : static_cast<const float*>(grad)[k];
        if (zp) {
          if (zbf16) static_cast<uint16_t*>(zp)[k] = 0;
          else static_cast<float*>(zp)[k] = 0.f;
        }
        float m = mom[k];
        const float nw = sgd_one(w[k], m, g, lr, mu, wd, rescale, clip);
        w[k] = nw;
        mom[k] = m;
        if (wb && x2_plane) stx(wb, k, x2_plane, nw, x3);
        else if (wb) wb[k] = f32_to_bf16(nw);
      }
    }
  }
}

// 8 elements per lane: two 16-B loads of each fp32 stream issued before any use, the shadow pair
// written as full 16-B rows (8 bf16 per plane).  NT: master / momentum / gradient accesses are
// nontemporal (each byte is touched once per step; keeps the shadow the next forward reads in the
// caches).  Needs x2_plane % 8 == 0 for the aligned lo-plane rows (host checks).
typedef float sgd_f4 __attribute__((ext_vector_type(4)));
typedef unsigned int sgd_u4 __attribute__((ext_vector_type(4)));

template <bool NT, typename T>
__device__ __forceinline__ T sgd_ld(const T* p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT, typename T>
__device__ __forceinline__ void sgd_st(T* p, T v) {
  if (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <bool GBF16, bool NT>
__global__ void __launch_bounds__(256)
sgd8_kernel(float* __restrict__ w, float* __restrict__ mom, const void* grad, int64_t n,
            const float* __restrict__ lr_p, float mu, float wd, float rescale, float clip, uint16_t* __restrict__ wb,
            int64_t x2_plane, int x3, void* zp, int zbf16) {
  const float lr = *lr_p;
  const int64_t n8 = n & ~(int64_t)7;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 8;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8; i < n8; i += stride) {
    const sgd_f4 w0 = sgd_ld<NT>(reinterpret_cast<const sgd_f4*>(w + i));
    const sgd_f4 w1 = sgd_ld<NT>(reinterpret_cast<const sgd_f4*>(w + i + 4));
    const sgd_f4 m0 = sgd_ld<NT>(reinterpret_cast<const sgd_f4*>(mom + i));
    const sgd_f4 m1 = sgd_ld<NT>(reinterpret_cast<const sgd_f4*>(mom + i + 4));
    float g[8];
    if (GBF16) {
      const sgd_u4 u = sgd_ld<NT>(reinterpret_cast<const sgd_u4*>(static_cast<const uint16_t*>(grad) + i));
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        g[2 * k] = __uint_as_float(u[k] << 16);
        g[2 * k + 1] = __uint_as_float(u[k] & 0xffff0000u);
      }
    } else {
      const sgd_f4 g0 = sgd_ld<NT>(reinterpret_cast<const sgd_f4*>(static_cast<const float*>(grad) + i));
      const sgd_f4 g1 = sgd_ld<NT>(reinterpret_cast<const sgd_f4*>(static_cast<const float*>(grad) + i + 4));
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        g[k] = g0[k];
        g[k + 4] = g1[k];
      }
    }
    if (zp) {
      if (zbf16) {
        sgd_st<NT>(reinterpret_cast<sgd_u4*>(static_cast<uint16_t*>(zp) + i), sgd_u4{0u, 0u, 0u, 0u});
      } else {
        sgd_st<NT>(reinterpret_cast<sgd_f4*>(static_cast<float*>(zp) + i), sgd_f4{0.f, 0.f, 0.f, 0.f});
        sgd_st<NT>(reinterpret_cast<sgd_f4*>(static_cast<float*>(zp) + i + 4), sgd_f4{0.f, 0.f, 0.f, 0.f});
      }
    }
    float wv[8], mv[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      wv[k] = w0[k]; wv[k + 4] = w1[k];
      mv[k] = m0[k]; mv[k + 4] = m1[k];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) wv[k] = sgd_one(wv[k], mv[k], g[k], lr, mu, wd, rescale, clip);
    sgd_st<NT>(reinterpret_cast<sgd_f4*>(w + i), sgd_f4{wv[0], wv[1], wv[2], wv[3]});
    sgd_st<NT>(reinterpret_cast<sgd_f4*>(w + i + 4), sgd_f4{wv[4], wv[5], wv[6], wv[7]});
    sgd_st<NT>(reinterpret_cast<sgd_f4*>(mom + i), sgd_f4{mv[0], mv[1], mv[2], mv[3]});
    sgd_st<NT>(reinterpret_cast<sgd_f4*>(mom + i + 4), sgd_f4{mv[4], mv[5], mv[6], mv[7]});
    if (wb && x2_plane) {
      float stored[8];
      st8x(wb + i, x2_plane, wv, stored, x3);
    } else if (wb) {
      st8_bf16(wb + i, wv);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < n - n8) {  // the < 8 trailing elements
    const int64_t k = n8 + threadIdx.x;
    const float gk = GBF16 ? bf16_to_f32(static_cast<const uint16_t*>(grad)[k]) : static_cast<const float*>(grad)[k];
    if (zp) {
      if (zbf16) static_cast<uint16_t*>(zp)[k] = 0;
      else static_cast<float*>(zp)[k] = 0.f;
    }
    float m = mom[k];
    const float nw = sgd_one(w[k], m, gk, lr, mu, wd, rescale, clip);
    w[k] = nw;
    mom[k] = m;
    if (wb && x2_plane) stx(wb, k, x2_plane, nw, x3);
    else if (wb) wb[k] = f32_to_bf16(nw);
  }
}

// MXR_SGD: 0 = the 4-wide kernel (default), 1 = 8-wide, 2 = 8-wide nontemporal
static int sgd_variant() {
  static const int v = [] {
    const char* e = getenv("MXR_SGD");
    return e ? atoi(e) : 0;
  }();
  return v;
}

void sgd_momentum(float* w, float* mom, const void* grad, int grad_bf16, int64_t n, const float* lr, float momentum,
                  float wd, float rescale, float clip, uint16_t* w_bf16, hipStream_t st, int64_t x2_plane,
                  int x3, void* zero, int zero_bf16) {
  if (n == 0) return;
  const int var = sgd_variant();
  const auto a16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (var > 0 && x2_plane % 8 == 0 && a16(w) && a16(mom) && a16(grad) && (w_bf16 == nullptr || a16(w_bf16)) &&
      (zero == nullptr || a16(zero))) {
    const int blocks = (int)std::min<int64_t>(std::max<int64_t>(div_up((n + 7) / 8, 256), 1), 256 * 8);
#define MXR_SGD8(GB, NT) sgd8_kernel<GB, NT><<<blocks, 256, 0, st>>>(w, mom, grad, n, lr, momentum, wd, rescale, clip, w_bf16, x2_plane, x3, zero, zero_bf16)
    if (grad_bf16) { if (var == 2) MXR_SGD8(true, true); else MXR_SGD8(true, false); }
    else { if (var == 2) MXR_SGD8(false, true); else MXR_SGD8(false, false); }
#undef MXR_SGD8
    return;
  }
  static const int64_t max_blocks = [] {  // A/B knob MXR_SGD_BLOCKS: grid cap of the 4-wide kernel
    const char* e = getenv("MXR_SGD_BLOCKS");
    return e != nullptr ? std::max<int64_t>(1, atoll(e)) : (int64_t)256 * 8;
  }();
  const int blocks = (int)std::min<int64_t>(div_up((n + 3) / 4, 256), max_blocks);
  if (grad_bf16)
    sgd_kernel<true><<<blocks, 256, 0, st>>>(w, mom, grad, n, lr, momentum, wd, rescale, clip, w_bf16, x2_plane, x3,
                                                   zero, zero_bf16);
  else
    sgd_kernel<false><<<blocks, 256, 0, st>>>(w, mom, grad, n, lr, momentum, wd, rescale, clip, w_bf16, x2_plane, x3,
                                                   zero, zero_bf16);
}

}  // namespace mxr
