// Max-pool forward / backward and global average pool on NHWC bf16 / fp16 maps (SURVEY kernel K14;
// `code` = 1 bf16, 2 fp16, 3 x2 hi / lo pairs: the fp32-class training mode, common.h).
//
// Reference ops: VGG pool1..pool4 2x2/2 (`rcnn/symbol.py:19,28,40,52`), ResNet pool0 3x3/2 pad 1
// (`rcnn/resnet.py:150`), global average pool before the predictors (`rcnn/resnet.py:167`).
// MXNet's default pooling convention is "valid" (floor) with padded taps ignored.
//
// * Forward: one thread per (output pixel, 8 channels): 16-B loads of the window rows, running
//   max in fp32 (exact for bf16), the winning tap index (0..k*k-1, first maximum in row-major
//   window order like MXNet / cuDNN) stored as one byte per output element.
// * Backward is a GATHER, not a scatter: every input element visits the <= ceil(k/s)^2 output
//   windows that cover it and adds dy where that window's recorded winner is itself -- no
//   atomics, deterministic, one 16-B store per 8 channels.
// * Global average pool: one workgroup per (image, 512-channel slab), 64 lanes x 8 channels
//   sum the H*W rows in fp32; the backward broadcasts dy / (H*W).
#include "common.h"
#include "../kernels.h"

namespace mxr {

__global__ void __launch_bounds__(256)
maxpool_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, uint8_t* __restrict__ arg, int N, int H,
                   int W, int C, int Ho, int Wo, int k, int s, int p, int code, PostBn post) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * Ho * Wo * cv;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int c8 = (int)(t % cv);
  const int64_t pix = t / cv;
  const int wo = (int)(pix % Wo), ho = (int)((pix / Wo) % Ho), n = (int)(pix / ((int64_t)Wo * Ho));
  float best[8];
  int bi[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    best[q] = -INFINITY;
    bi[q] = 255;
  }
  const int h0 = ho * s - p, w0 = wo * s - p;
  for (int i = 0; i < k; ++i) {
    const int h = h0 + i;
    if ((unsigned)h >= (unsigned)H) continue;
    for (int j = 0; j < k; ++j) {
      const int w = w0 + j;
      if ((unsigned)w >= (unsigned)W) continue;
      float v[8];
      ld8c(x, (((int64_t)n * H + h) * W + w) * C + c8 * 8, code, (int64_t)N * H * W * C, v);
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (v[q] > best[q] || bi[q] == 255) {  // strict: the first maximum wins
          best[q] = v[q];
          bi[q] = i * k + j;
        }
    }
  }
  if (post.scale) {  // inference: the next unit's bn1 + ReLU on the pooled value
    float a[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) a[q] = best[q];
    post_bn_relu8(post, c8 * 8, a);
    st8c(y, pix * C + c8 * 8, code, (int64_t)N * Ho * Wo * C, a);
  } else {
    st8c(y, pix * C + c8 * 8, code, (int64_t)N * Ho * Wo * C, best);
  }
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    lo |= (uint32_t)bi[q] << (8 * q);
    hi |= (uint32_t)bi[q + 4] << (8 * q);
  }
  if (arg) *reinterpret_cast<uint2*>(arg + pix * C + c8 * 8) = make_uint2(lo, hi);  // null: inference
}

__global__ void __launch_bounds__(256)
maxpool_bwd_kernel(const uint16_t* __restrict__ dy, const uint8_t* __restrict__ arg, uint16_t* __restrict__ dx,
                   int N, int H, int W, int C, int Ho, int Wo, int k, int s, int p, int code) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * H * W * cv;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int c8 = (int)(t % cv);
  const int64_t pix = t / cv;
  const int w = (int)(pix % W), h = (int)((pix / W) % H), n = (int)(pix / ((int64_t)W * H));
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // output windows covering input row h: ho*s - p <= h <= ho*s - p + k - 1
  const int ho_lo = max(0, (h + p - k + s) / s), ho_hi = min(Ho - 1, (h + p) / s);
  const int wo_lo = max(0, (w + p - k + s) / s), wo_hi = min(Wo - 1, (w + p) / s);
  for (int ho = ho_lo; ho <= ho_hi; ++ho) {
    const int i = h - (ho * s - p);
    if (i < 0 || i >= k) continue;
    for (int wo = wo_lo; wo <= wo_hi; ++wo) {
      const int j = w - (wo * s - p);
      if (j < 0 || j >= k) continue;
      const int64_t o = (((int64_t)n * Ho + ho) * Wo + wo) * C + c8 * 8;
      const uint2 a = *reinterpret_cast<const uint2*>(arg + o);
      float g[8];
      ld8c(dy, o, code, (int64_t)N * Ho * Wo * C, g);
      const int tap = i * k + j;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint32_t word = q < 4 ? a.x : a.y;
        if ((int)((word >> (8 * (q & 3))) & 0xff) == tap) acc[q] += g[q];
      }
    }
  }
  st8c(dx, pix * C + c8 * 8, code, (int64_t)N * H * W * C, acc);
}

__global__ void __launch_bounds__(64)
avgpool_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int HW, int C, int code) {
  const int n = blockIdx.y;
  const int64_t N = gridDim.y;
  const int c = (blockIdx.x * 64 + threadIdx.x) * 8;
  if (c >= C) return;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < HW; ++i) {
    float v[8];
    ld8c(x, ((int64_t)n * HW + i) * C + c, code, N * HW * C, v);
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] += v[q];
  }
  const float inv = 1.f / (float)HW;
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] *= inv;
  st8c(y, (int64_t)n * C + c, code, N * C, acc);
}

__global__ void __launch_bounds__(256)
avgpool_bwd_kernel(const uint16_t* __restrict__ dy, uint16_t* __restrict__ dx, int N, int HW, int C, int code) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * HW * cv;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int c8 = (int)(t % cv);
  const int n = (int)(t / ((int64_t)HW * cv));
  float g[8];
  ld8c(dy, (int64_t)n * C + c8 * 8, code, (int64_t)N * C, g);
  const float inv = 1.f / (float)HW;
#pragma unroll
  for (int q = 0; q < 8; ++q) g[q] *= inv;
  st8c(dx, (t / cv) * C + c8 * 8, code, (int64_t)N * HW * C, g);
}

int maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* arg, int N, int H, int W, int C, int Ho, int Wo, int k,
                int s, int p, int code, hipStream_t st, PostBn post) {
  if (C % 8 != 0 || k > 15 || k <= 0 || s <= 0) return -1;
  const int64_t total = (int64_t)N * Ho * Wo * (C / 8);
  if (total == 0) return 0;
  maxpool_fwd_kernel<<<div_up(total, 256), 256, 0, st>>>(x, y, arg, N, H, W, C, Ho, Wo, k, s, p, code, post);
  return 0;
}

int maxpool_bwd(const uint16_t* dy, const uint8_t* arg, uint16_t* dx, int N, int H, int W, int C, int Ho, int Wo,
                int k, int s, int p, int code, hipStream_t st) {
  if (C % 8 != 0 || k > 15 || k <= 0 || s <= 0) return -1;
  const int64_t total = (int64_t)N * H * W * (C / 8);
  if (total == 0) return 0;
  maxpool_bwd_kernel<<<div_up(total, 256), 256, 0, st>>>(dy, arg, dx, N, H, W, C, Ho, Wo, k, s, p, code);
  return 0;
}

int avgpool_fwd(const uint16_t* x, uint16_t* y, int N, int HW, int C, int code, hipStream_t st) {
  if (C % 8 != 0 || N == 0) return -1;
  avgpool_fwd_kernel<<<dim3(div_up(C / 8, 64), N), 64, 0, st>>>(x, y, HW, C, code);
  return 0;
}

int avgpool_bwd(const uint16_t* dy, uint16_t* dx, int N, int HW, int C, int code, hipStream_t st) {
  if (C % 8 != 0) return -1;
  const int64_t total = (int64_t)N * HW * (C / 8);
  if (total == 0) return 0;
  avgpool_bwd_kernel<<<div_up(total, 256), 256, 0, st>>>(dy, dx, N, HW, C, code);
  return 0;
}

}  // namespace mxr
