// Multi-tensor fused SGD-momentum over flat parameter buffers (SURVEY kernel K20; MXNet
// `sgd_mom_update` semantics: g = clip(rescale*g, +-clip); mom = mu*mom - lr*(g + wd*w);
// w += mom).  One launch per weight-decay group over the whole flat buffer, 4 elements per
// lane with 16-B loads.  The learning rate is read from device memory so the update can be
// captured in a hipGraph and replayed while the schedule changes.  The kernel also writes
// the bf16 shadow of the new weights that the next forward consumes (fusing the cast).
#include "common.h"
#include "../kernels.h"
#include <algorithm>

namespace mxr {

__device__ __forceinline__ float sgd_one(float w, float& m, float g, float lr, float mu, float wd, float rescale,
                                         float clip) {
  g *= rescale;
  if (clip > 0.f) g = fminf(fmaxf(g, -clip), clip);
  m = mu * m - lr * (g + wd * w);
  return w + m;
}

template <bool GBF16>
__global__ void __launch_bounds__(256)
sgd_kernel(float* __restrict__ w, float* __restrict__ mom, const void* __restrict__ grad, int64_t n,
           const float* __restrict__ lr_p, float mu, float wd, float rescale, float clip, uint16_t* __restrict__ wb,
           int64_t x2_plane) {
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
      wv.x = sgd_one(wv.x, mv.x, gv.x, lr, mu, wd, rescale, clip);
      wv.y = sgd_one(wv.y, mv.y, gv.y, lr, mu, wd, rescale, clip);
      wv.z = sgd_one(wv.z, mv.z, gv.z, lr, mu, wd, rescale, clip);
      wv.w = sgd_one(wv.w, mv.w, gv.w, lr, mu, wd, rescale, clip);
      *reinterpret_cast<float4*>(w + i) = wv;
      *reinterpret_cast<float4*>(mom + i) = mv;
      if (wb && x2_plane) {  // fp32-class shadow: hi / lo pair planes (common.h x2)
        const float v4[4] = {wv.x, wv.y, wv.z, wv.w};
        st4c(wb, i, kCodeX2, x2_plane, v4);
      } else if (wb) {
        *reinterpret_cast<ushort4*>(wb + i) =
            make_ushort4(f32_to_bf16(wv.x), f32_to_bf16(wv.y), f32_to_bf16(wv.z), f32_to_bf16(wv.w));
      }
    } else {
      for (int64_t k = i; k < n; ++k) {
        const float g = GBF16 ? bf16_to_f32(static_cast<const uint16_t*>(grad)[k]) : static_cast<const float*>(grad)[k];
        float m = mom[k];
        const float nw = sgd_one(w[k], m, g, lr, mu, wd, rescale, clip);
        w[k] = nw;
        mom[k] = m;
        if (wb && x2_plane) stx(wb, k, x2_plane, nw);
        else if (wb) wb[k] = f32_to_bf16(nw);
      }
    }
  }
}

void sgd_momentum(float* w, float* mom, const void* grad, int grad_bf16, int64_t n, const float* lr, float momentum,
                  float wd, float rescale, float clip, uint16_t* w_bf16, hipStream_t st, int64_t x2_plane) {
  if (n == 0) return;
  const int blocks = (int)std::min<int64_t>(div_up((n + 3) / 4, 256), 256 * 8);
  if (grad_bf16)
    sgd_kernel<true><<<blocks, 256, 0, st>>>(w, mom, grad, n, lr, momentum, wd, rescale, clip, w_bf16, x2_plane);
  else
    sgd_kernel<false><<<blocks, 256, 0, st>>>(w, mom, grad, n, lr, momentum, wd, rescale, clip, w_bf16, x2_plane);
}

}  // namespace mxr
