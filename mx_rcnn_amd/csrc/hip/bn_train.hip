// Training-mode (batch statistics) BatchNorm + optional ReLU for NHWC bf16 activations: the
// stage-4 / bn1 layers of the ResNet C4 head, which normalise over the 128 sampled RoIs
// (`rcnn/resnet.py:152,165`, bn_global=False).  M = N*H*W is small (2 K - 6 K rows) and C large
// (512 - 2048), so one workgroup owns 8 channels (one 16-B load per row) for ALL rows:
// statistics, the running-average update and the normalisation happen in one launch with no
// cross-block reduction, and C/8 = 64-256 workgroups cover the chip.  256 row lanes with 4 rows
// in flight per lane hide the HBM latency; the blocks of neighbouring channel groups read the
// same cache lines, so L2 serves the 16-B-per-row pattern.  The slab stays L2-resident between
// the passes.
// fwd: pass 1 mean, pass 2 centred variance (no E[x^2]-E[x]^2 cancellation), pass 3 y.
// bwd: pass 1 sum(g), sum(g*xhat) with g = dy * relu_mask, pass 2 dx.
// Running stats follow MXNet: moving = mom * moving + (1 - mom) * batch (unbiased variance, as
// the cuDNN path MXNet uses).
#include <type_traits>

#include "common.h"
#include "../kernels.h"

namespace mxr {

constexpr int BT_CB = 8;  // channels per block (one 16-B load per row)

__device__ __forceinline__ void ld8(const uint16_t* p, float* v) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = __uint_as_float(w[k] << 16);
    v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}

__device__ __forceinline__ void st8(uint16_t* p, const float* v) {
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    w[k] = (uint32_t)f32_to_bf16(v[2 * k]) | ((uint32_t)f32_to_bf16(v[2 * k + 1]) << 16);
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}

// block-wide sum of 8 per-thread values (256 threads) -> out[8] visible to all threads
__device__ __forceinline__ void block_sum8(float* v, float (*red)[8], float* out) {
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = wave_sum(v[k]);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < 8; ++k) red[wid][k] = v[k];
  __syncthreads();
  if (threadIdx.x < 8) out[threadIdx.x] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                                          red[3][threadIdx.x];
  __syncthreads();
}

// for each of this thread's rows r = tid + i*256: fn(row_ptr_offset)
template <typename F>
__device__ __forceinline__ void for_rows(int64_t M, F fn) {
  int64_t r = threadIdx.x;
  for (; r + 768 < M; r += 1024) fn(r, std::integral_constant<int, 4>());  // 4 rows in flight
  for (; r < M; r += 256) fn(r, std::integral_constant<int, 1>());
}

__global__ void __launch_bounds__(256)
bn_train_fwd_kernel(const uint16_t* __restrict__ x, int64_t M, int C, const float* __restrict__ gamma,
                    const float* __restrict__ beta, float* __restrict__ rmean, float* __restrict__ rvar,
                    float momentum, float eps, int fix_gamma, int relu, uint16_t* __restrict__ y,
                    float* __restrict__ save_mean, float* __restrict__ save_invstd) {
  __shared__ float red[4][8];
  __shared__ float tot[8];
  const int c0 = blockIdx.x * BT_CB;
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  for_rows(M, [&](int64_t r, auto N) {
    constexpr int n = decltype(N)::value;
    float v[4][8];
#pragma unroll
    for (int u = 0; u < n; ++u) ld8(x + (r + u * 256) * C + c0, v[u]);
#pragma unroll
    for (int u = 0; u < n; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += v[u][k];
  });
  block_sum8(acc, red, tot);
  float mu[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mu[k] = tot[k] / (float)M;
    acc[k] = 0.f;
  }
  __syncthreads();
  for_rows(M, [&](int64_t r, auto N) {
    constexpr int n = decltype(N)::value;
    float v[4][8];
#pragma unroll
    for (int u = 0; u < n; ++u) ld8(x + (r + u * 256) * C + c0, v[u]);
#pragma unroll
    for (int u = 0; u < n; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float d = v[u][k] - mu[k];
        acc[k] += d * d;
      }
  });
  block_sum8(acc, red, tot);
  float sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = c0 + k;
    const float var = tot[k] / (float)M;
    const float inv = rsqrtf(var + eps);
    const float g = fix_gamma ? 1.f : gamma[c];
    sc[k] = g * inv;
    sh[k] = beta[c] - mu[k] * sc[k];
    if (threadIdx.x == 0) {
      save_mean[c] = mu[k];
      save_invstd[c] = inv;
      const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
      rmean[c] = momentum * rmean[c] + (1.f - momentum) * mu[k];
      rvar[c] = momentum * rvar[c] + (1.f - momentum) * unb;
    }
  }
  for_rows(M, [&](int64_t r, auto N) {
    constexpr int n = decltype(N)::value;
    float v[4][8];
#pragma unroll
    for (int u = 0; u < n; ++u) ld8(x + (r + u * 256) * C + c0, v[u]);
#pragma unroll
    for (int u = 0; u < n; ++u) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        v[u][k] = v[u][k] * sc[k] + sh[k];
        if (relu) v[u][k] = fmaxf(v[u][k], 0.f);
      }
      st8(y + (r + u * 256) * C + c0, v[u]);
    }
  });
}

__global__ void __launch_bounds__(256)
bn_train_bwd_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy, int64_t M, int C,
                    const float* __restrict__ gamma, const float* __restrict__ beta,
                    const float* __restrict__ save_mean, const float* __restrict__ save_invstd, int fix_gamma,
                    int relu, uint16_t* __restrict__ dx, float* __restrict__ dgamma, float* __restrict__ dbeta,
                    int accumulate) {
  __shared__ float red[4][8];
  __shared__ float tot_g[8], tot_gx[8];
  const int c0 = blockIdx.x * BT_CB;
  float mu[8], inv[8], g[8], b[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mu[k] = save_mean[c0 + k];
    inv[k] = save_invstd[c0 + k];
    g[k] = fix_gamma ? 1.f : gamma[c0 + k];
    b[k] = beta[c0 + k];
  }
  float sg[8], sgx[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) sg[k] = sgx[k] = 0.f;
  for_rows(M, [&](int64_t r, auto N) {
    constexpr int n = decltype(N)::value;
    float v[4][8], d[4][8];
#pragma unroll
    for (int u = 0; u < n; ++u) {
      ld8(x + (r + u * 256) * C + c0, v[u]);
      ld8(dy + (r + u * 256) * C + c0, d[u]);
    }
#pragma unroll
    for (int u = 0; u < n; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float xh = (v[u][k] - mu[k]) * inv[k];
        const float gm = (!relu || xh * g[k] + b[k] > 0.f) ? d[u][k] : 0.f;
        sg[k] += gm;
        sgx[k] += gm * xh;
      }
  });
  block_sum8(sg, red, tot_g);
  block_sum8(sgx, red, tot_gx);
  float mg[8], mgx[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mg[k] = tot_g[k] / (float)M;
    mgx[k] = tot_gx[k] / (float)M;
    if (threadIdx.x == 0) {
      const int c = c0 + k;
      if (dgamma && !fix_gamma) dgamma[c] = accumulate ? dgamma[c] + tot_gx[k] : tot_gx[k];
      if (dbeta) dbeta[c] = accumulate ? dbeta[c] + tot_g[k] : tot_g[k];
    }
  }
  if (!dx) return;
  for_rows(M, [&](int64_t r, auto N) {
    constexpr int n = decltype(N)::value;
    float v[4][8], d[4][8];
#pragma unroll
    for (int u = 0; u < n; ++u) {
      ld8(x + (r + u * 256) * C + c0, v[u]);
      ld8(dy + (r + u * 256) * C + c0, d[u]);
    }
#pragma unroll
    for (int u = 0; u < n; ++u) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float xh = (v[u][k] - mu[k]) * inv[k];
        const float gm = (!relu || xh * g[k] + b[k] > 0.f) ? d[u][k] : 0.f;
        d[u][k] = g[k] * inv[k] * (gm - mg[k] - xh * mgx[k]);
      }
      st8(dx + (r + u * 256) * C + c0, d[u]);
    }
  });
}

int bn_train_fwd(const uint16_t* x, int64_t M, int C, const float* gamma, const float* beta, float* rmean,
                 float* rvar, float momentum, float eps, int fix_gamma, int relu, uint16_t* y, float* save_mean,
                 float* save_invstd, hipStream_t st) {
  if (C % BT_CB != 0 || M <= 0) return -1;
  bn_train_fwd_kernel<<<C / BT_CB, 256, 0, st>>>(x, M, C, gamma, beta, rmean, rvar, momentum, eps, fix_gamma, relu,
                                                 y, save_mean, save_invstd);
  return 0;
}

int bn_train_bwd(const uint16_t* x, const uint16_t* dy, int64_t M, int C, const float* gamma, const float* beta,
                 const float* save_mean, const float* save_invstd, int fix_gamma, int relu, uint16_t* dx,
                 float* dgamma, float* dbeta, int accumulate, hipStream_t st) {
  if (C % BT_CB != 0 || M <= 0) return -1;
  bn_train_bwd_kernel<<<C / BT_CB, 256, 0, st>>>(x, dy, M, C, gamma, beta, save_mean, save_invstd, fix_gamma, relu,
                                                 dx, dgamma, dbeta, accumulate);
  return 0;
}

}  // namespace mxr
