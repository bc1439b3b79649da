// Frozen ("use_global_stats") BatchNorm + ReLU on channels-last activations (SURVEY K13;
// reference pre-activation units `rcnn/resnet.py:27-54` with bn_global=True: stages 1-3).
// Forward folds mean/var/gamma/beta into one scale+shift per channel on the fly; backward
// recomputes the ReLU mask from x (nothing saved but x) and reduces dgamma/dbeta per channel
// with per-thread register partials (each thread owns a fixed channel quad because the grid
// size is a multiple of C/4), then one atomic per thread.  16-B bf16 loads (8 channels) are
// not used because ResNet C4 channel counts are all multiples of 4 but stage widths start
// at 64, where 4-wide keeps a whole row per 16 lanes.
#include "common.h"
#include "../kernels.h"
#include <algorithm>

namespace mxr {

struct BnQuad {
  float s[4], t[4];
};

__device__ __forceinline__ void bn_coeffs(int c, const float* gamma, const float* beta, const float* mean,
                                          const float* var, float eps, int fix_gamma, float& s, float& t) {
  const float inv = rsqrtf(var[c] + eps);
  const float g = fix_gamma ? 1.f : gamma[c];
  s = g * inv;
  t = beta[c] - mean[c] * s;
}

// `bf16` is the storage code (common.h: 0 fp32, 1 bf16, 2 fp16, 3 x2 pair with plane = M * C)
__device__ __forceinline__ void load4(const void* p, int64_t i, int code, float v[4], int64_t plane) {
  ld4c(p, i, code, plane, v);
}
__device__ __forceinline__ void store4(void* p, int64_t i, int code, const float v[4], int64_t plane) {
  st4c(p, i, code, plane, v);
}

__global__ void __launch_bounds__(256)
bn_relu_fwd_kernel(const void* __restrict__ x, int bf16, int64_t M, int C, const float* __restrict__ gamma,
                   const float* __restrict__ beta, const float* __restrict__ mean, const float* __restrict__ var,
                   float eps, int fix_gamma, int relu, void* __restrict__ y) {
  const int CV = C >> 2;
  const int64_t T = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int cv = (int)(tid % CV);  // fixed per thread: T % CV == 0
  float s[4], t[4];
  for (int k = 0; k < 4; ++k) bn_coeffs(cv * 4 + k, gamma, beta, mean, var, eps, fix_gamma, s[k], t[k]);
  const int64_t total = M * CV;
  // 4 independent 8/16-B loads in flight per thread per trip (latency hiding at low occupancy)
  int64_t e = tid;
  for (; e + 3 * T < total; e += 4 * T) {
    float v[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) load4(x, (e + u * T) * 4, bf16, v[u], (int64_t)M * C);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[u][k] = v[u][k] * s[k] + t[k];
        if (relu) v[u][k] = fmaxf(v[u][k], 0.f);
      }
      store4(y, (e + u * T) * 4, bf16, v[u], (int64_t)M * C);
    }
  }
  for (; e < total; e += T) {
    float v[4];
    load4(x, e * 4, bf16, v, (int64_t)M * C);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[k] = v[k] * s[k] + t[k];
      if (relu) v[k] = fmaxf(v[k], 0.f);
    }
    store4(y, e * 4, bf16, v, (int64_t)M * C);
  }
}

__global__ void __launch_bounds__(256)
bn_relu_bwd_kernel(const void* __restrict__ x, const void* __restrict__ dy, int bf16, int64_t M, int C,
                   const float* __restrict__ gamma, const float* __restrict__ beta, const float* __restrict__ mean,
                   const float* __restrict__ var, float eps, int fix_gamma, int relu, void* __restrict__ dx,
                   const void* __restrict__ dres, float* __restrict__ part) {
  __shared__ float red[256][9];  // per-thread (sum g * xhat, sum g) x 4 channels, padded row
  const int CV = C >> 2;
  const int64_t T = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int cv = (int)(tid % CV);
  float s[4], t[4], inv[4], mu[4];
  for (int k = 0; k < 4; ++k) {
    const int c = cv * 4 + k;
    bn_coeffs(c, gamma, beta, mean, var, eps, fix_gamma, s[k], t[k]);
    inv[k] = rsqrtf(var[c] + eps);
    mu[k] = mean[c];
  }
  float ag[4] = {0.f, 0.f, 0.f, 0.f}, ab[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t total = M * CV;
  auto body = [&](float* xv, float* g, int64_t e) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float pre = xv[k] * s[k] + t[k];
      const float gm = (!relu || pre > 0.f) ? g[k] : 0.f;
      ab[k] += gm;
      ag[k] += gm * (xv[k] - mu[k]) * inv[k];
      g[k] = gm * s[k];
    }
    if (dx) {
      if (dres) {  // fused gradient accumulation: dx = dres + d(bn_relu)
        float rv[4];
        load4(dres, e * 4, bf16, rv, (int64_t)M * C);
#pragma unroll
        for (int k = 0; k < 4; ++k) g[k] += rv[k];
      }
      store4(dx, e * 4, bf16, g, (int64_t)M * C);
    }
  };
  int64_t e = tid;
  for (; e + 3 * T < total; e += 4 * T) {  // 8 independent loads in flight per thread
    float xv[4][4], g[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      load4(x, (e + u * T) * 4, bf16, xv[u], (int64_t)M * C);
      load4(dy, (e + u * T) * 4, bf16, g[u], (int64_t)M * C);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) body(xv[u], g[u], e + u * T);
  }
  for (; e < total; e += T) {
    float xv[4], g[4];
    load4(x, e * 4, bf16, xv, (int64_t)M * C);
    load4(dy, e * 4, bf16, g, (int64_t)M * C);
    body(xv, g, e);
  }
  if (part) {
    // ordered in-block sum (no LDS float atomics: the step is bitwise reproducible): the threads
    // of channel quad q are t0(q), t0(q) + CV, ... (thread t holds quad (block * 256 + t) % CV),
    // summed in increasing t, then one partial row per block, folded in order by bn_part_reduce
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      red[threadIdx.x][k] = ag[k];
      red[threadIdx.x][4 + k] = ab[k];
    }
    __syncthreads();
    float* row = part + (int64_t)blockIdx.x * 2 * C;
    const int base = (int)(((int64_t)blockIdx.x * blockDim.x) % CV);
    for (int i = threadIdx.x; i < 2 * C; i += blockDim.x) {
      const int stat = i >= C, c = i - stat * C, q = c >> 2, k = c & 3;
      float acc = 0.f;
      for (int t = (q - base + CV) % CV; t < (int)blockDim.x; t += CV) acc += red[t][stat * 4 + k];
      row[i] = acc;
    }
  }
}

// Stage 2: 64 columns per block (one per lane), the 4 waves split the partial rows and keep
// 8 independent loads in flight each (a serial per-thread loop over 160 rows was latency
// bound at ~37 us/call), then combine through LDS.
__global__ void __launch_bounds__(256)
bn_part_reduce(const float* __restrict__ part, int nblk, int C, int fix_gamma, float* __restrict__ dgamma,
               float* __restrict__ dbeta, int accumulate) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  float acc = 0.f;
  if (i < 2 * C) {
    int b = wid;
    for (; b + 28 < nblk; b += 32) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(b + 4 * u) * 2 * C + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; b < nblk; b += 4) acc += part[(int64_t)b * 2 * C + i];
  }
  red[wid][lane] = acc;
  __syncthreads();
  if (wid == 0 && i < 2 * C) {
    const float s = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    if (i < C) {
      if (dgamma && !fix_gamma) dgamma[i] = accumulate ? dgamma[i] + s : s;
    } else if (dbeta) {
      dbeta[i - C] = accumulate ? dbeta[i - C] + s : s;
    }
  }
}

// Scalar path for channel counts that are not a multiple of 4 (bn_data on the 3-channel
// image).  Each thread keeps a fixed channel (grid size multiple of C); the backward reduces
// dgamma/dbeta through LDS so each block issues one global atomic per channel.
__global__ void __launch_bounds__(256)
bn_relu_fwd_scalar(const void* __restrict__ x, int bf16, int64_t M, int C, const float* __restrict__ gamma,
                   const float* __restrict__ beta, const float* __restrict__ mean, const float* __restrict__ var,
                   float eps, int fix_gamma, int relu, void* __restrict__ y) {
  const int64_t T = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int c = (int)(tid % C);
  float s, t;
  bn_coeffs(c, gamma, beta, mean, var, eps, fix_gamma, s, t);
  for (int64_t e = tid; e < M * C; e += T) {
    float v = ldc(x, e, bf16, M * C) * s + t;
    if (relu) v = fmaxf(v, 0.f);
    stc(y, e, v, bf16, M * C);
  }
}

__global__ void __launch_bounds__(256)
bn_relu_bwd_scalar(const void* __restrict__ x, const void* __restrict__ dy, int bf16, int64_t M, int C,
                   const float* __restrict__ gamma, const float* __restrict__ beta, const float* __restrict__ mean,
                   const float* __restrict__ var, float eps, int fix_gamma, int relu, void* __restrict__ dx,
                   float* __restrict__ dgamma, float* __restrict__ dbeta) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // 2*C
  const int64_t T = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int c = (int)(tid % C);
  for (int i = threadIdx.x; i < 2 * C; i += blockDim.x) red[i] = 0.f;
  __syncthreads();
  float s, t;
  bn_coeffs(c, gamma, beta, mean, var, eps, fix_gamma, s, t);
  const float inv = rsqrtf(var[c] + eps), mu = mean[c];
  float ag = 0.f, ab = 0.f;
  for (int64_t e = tid; e < M * C; e += T) {
    const float xv = ldc(x, e, bf16, M * C);
    const float g = ldc(dy, e, bf16, M * C);
    const float gm = (!relu || xv * s + t > 0.f) ? g : 0.f;
    ab += gm;
    ag += gm * (xv - mu) * inv;
    if (dx) stc(dx, e, gm * s, bf16, M * C);
  }
  atomicAdd(&red[c], ag);
  atomicAdd(&red[C + c], ab);
  __syncthreads();
  for (int i = threadIdx.x; i < C; i += blockDim.x) {
    if (dgamma && !fix_gamma && red[i] != 0.f) atomicAdd(dgamma + i, red[i]);
    if (dbeta && red[C + i] != 0.f) atomicAdd(dbeta + i, red[C + i]);
  }
}

static int bn_grid_scalar(int64_t M, int C) {
  int64_t blocks = std::max<int64_t>(std::min<int64_t>((M * C + 255) / 256, 1024), 1);
  while ((blocks * 256) % C != 0) ++blocks;
  return (int)blocks;
}

static int bn_grid(int64_t M, int C, int64_t cap = 1024) {
  const int CV = C >> 2;
  // threads must be a multiple of CV so each thread keeps one channel quad
  int64_t want = std::min<int64_t>((M * CV + 255) / 256, cap);
  int64_t blocks = std::max<int64_t>(want, 1);
  while ((blocks * 256) % CV != 0) ++blocks;
  return (int)blocks;
}

__global__ void __launch_bounds__(256)
bn_affine_kernel(const float* __restrict__ gamma, const float* __restrict__ beta, const float* __restrict__ mean,
                 const float* __restrict__ var, float eps, int fix_gamma, int C, float* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s, t;
  bn_coeffs(c, gamma, beta, mean, var, eps, fix_gamma, s, t);
  out[c] = s;
  out[C + c] = t;
}

void bn_affine(const float* gamma, const float* beta, const float* mean, const float* var, float eps, int fix_gamma,
               int C, float* out, hipStream_t st) {
  if (C > 0) bn_affine_kernel<<<(C + 255) / 256, 256, 0, st>>>(gamma, beta, mean, var, eps, fix_gamma, C, out);
}

void bn_relu_fwd(const void* x, int bf16, int64_t M, int C, const float* gamma, const float* beta, const float* mean,
                 const float* var, float eps, int fix_gamma, int relu, void* y, hipStream_t st) {
  if (M == 0 || C == 0) return;
  if (C % 4 != 0) {
    bn_relu_fwd_scalar<<<bn_grid_scalar(M, C), 256, 0, st>>>(x, bf16, M, C, gamma, beta, mean, var, eps, fix_gamma,
                                                             relu, y);
    return;
  }
  bn_relu_fwd_kernel<<<bn_grid(M, C), 256, 0, st>>>(x, bf16, M, C, gamma, beta, mean, var, eps, fix_gamma, relu, y);
}

int bn_bwd_workspace_floats(int64_t M, int C) {
  if (C % 4 != 0) return 0;
  return bn_grid(M, C, 320) * 2 * C;
}

void bn_relu_bwd(const void* x, const void* dy, int bf16, int64_t M, int C, const float* gamma, const float* beta,
                 const float* mean, const float* var, float eps, int fix_gamma, int relu, void* dx, const void* dres,
                 float* dgamma, float* dbeta, float* workspace, int accumulate, hipStream_t st) {
  if (M == 0 || C == 0) return;
  if (C % 4 != 0) {
    if (dres) return;  // not supported on the scalar path (caller checks)
    bn_relu_bwd_scalar<<<bn_grid_scalar(M, C), 256, 2 * C * sizeof(float), st>>>(
        x, dy, bf16, M, C, gamma, beta, mean, var, eps, fix_gamma, relu, dx, dgamma, dbeta);
    return;
  }
  const int nblk = bn_grid(M, C, 320);
  float* part = (dgamma || dbeta) ? workspace : nullptr;
  bn_relu_bwd_kernel<<<nblk, 256, 0, st>>>(x, dy, bf16, M, C, gamma, beta, mean, var, eps, fix_gamma, relu, dx, dres,
                                            part);
  if (part) bn_part_reduce<<<(2 * C + 63) / 64, 256, 0, st>>>(part, nblk, C, fix_gamma, dgamma, dbeta, accumulate);
}

// Many folds in one launch (the deterministic frozen-BN sums of a whole backward pass: one launch
// per up to kMaxFolds BNs instead of one each).  Workgroup b serves the entry whose block range
// holds b; each entry's blocks reduce 64 of its 2C columns like bn_part_reduce.
__global__ void __launch_bounds__(256) bn_part_fold_multi_kernel(FoldBatch fb) {
  __shared__ float red[4][64];
  int e = 0;
  while (e + 1 < fb.n && (int)blockIdx.x >= fb.e[e + 1].blk0) ++e;
  const FoldEntry& f = fb.e[e];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i = ((int)blockIdx.x - f.blk0) * 64 + lane;
  const int C = f.C;
  float acc = 0.f;
  if (i < 2 * C) {
    int b = wid;
    for (; b + 28 < f.nparts; b += 32) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = f.part[(int64_t)(b + 4 * u) * 2 * C + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; b < f.nparts; b += 4) acc += f.part[(int64_t)b * 2 * C + i];
  }
  red[wid][lane] = acc;
  __syncthreads();
  if (wid == 0 && i < 2 * C) {
    const float s = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    if (i < C) {
      if (f.out0) f.out0[i] += s;
    } else if (f.out1) {
      f.out1[i - C] += s;
    }
  }
}

void bn_part_fold_multi(const FoldBatch& fb, hipStream_t st) {
  if (fb.n <= 0) return;
  const FoldEntry& last = fb.e[fb.n - 1];
  const int blocks = last.blk0 + (2 * last.C + 63) / 64;
  bn_part_fold_multi_kernel<<<blocks, 256, 0, st>>>(fb);
}

// Fixed-order fold of nparts partial rows [nparts][2][C] (first half -> out0, second -> out1;
// either may be null), added to the outputs: the deterministic replacement of per-tile fp32
// atomics for the BN-backward column sums of the conv epilogues (ConvEpi::bnb_part).
void col_part_fold(const float* part, int nparts, int C, float* out0, float* out1, hipStream_t st) {
  if (nparts <= 0 || C <= 0 || (!out0 && !out1)) return;
  bn_part_reduce<<<(2 * C + 63) / 64, 256, 0, st>>>(part, nparts, C, 0, out0, out1, 1);
}

// ReLU (+ inverted dropout) backward on its own: out = dy * [y > 0] * scale over n 16-bit elements
// (8 per thread), y the ReLU output (its hi plane with planes); x2 / x3: the mask of element i applies
// to every plane of dy (`np` planes `plane` = n apart).  The VGG trunk's top gradient (ops/vgg_fused.py);
// every other ReLU backward rides in a data-gradient epilogue (ConvEpi::rmask).
__global__ void __launch_bounds__(256)
relu_mask_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ y, uint16_t* __restrict__ out,
                 int64_t n, int64_t plane, int np, float scale) {
  const int64_t e = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (e >= n) return;
  const uint4 yv = *reinterpret_cast<const uint4*>(y + e);
  const uint16_t* yh = reinterpret_cast<const uint16_t*>(&yv);
  for (int q = 0; q < np; ++q) {
    float d[8];
    ld8_bf16(dy + q * plane + e, d);
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = ((yh[k] & 0x8000u) == 0 && (yh[k] & 0x7fffu) != 0) ? d[k] * scale : 0.f;
    st8_bf16(out + q * plane + e, d);
  }
}

void relu_mask(const uint16_t* dy, const uint16_t* y, uint16_t* out, int64_t n, int64_t plane, float scale,
               hipStream_t st, int np) {
  if (n <= 0) return;
  relu_mask_kernel<<<(unsigned)((n / 8 + 255) / 256), 256, 0, st>>>(dy, y, out, n, plane, np < 1 ? 1 : np, scale);
}

}  // namespace mxr
