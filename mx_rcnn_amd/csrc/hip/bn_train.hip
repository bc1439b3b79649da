// Training-mode (batch statistics) BatchNorm + optional ReLU for NHWC bf16 activations: the
// stage-4 / bn1 layers of the ResNet C4 head, which normalise over the 128 sampled RoIs
// (`rcnn/resnet.py:152,165`, bn_global=False).  M = N*H*W = 2 K - 6 K rows, C = 512 - 2048.
//
// Two kernels per direction, both fully coalesced: a workgroup owns 64 channels (one 128-B
// line per row, 8 lanes x 16 B) and a chunk of `rows` rows (32 row lanes).  The chunk height
// (32-256, bn_train_rows) is picked per shape so the grid has >= 512 workgroups: at 128 RoIs
// the stage-4 maps are only 2 K - 6 K rows x 8 - 32 channel blocks, and one 256-row chunk per
// workgroup left most of the 256 CUs idle (64-256 workgroups, 5-12 us per launch).
//   fwd 1: per-chunk partial sum / sum of squares (shifted by the running mean, so the
//          E[x^2] - E[x]^2 form does not cancel) -> workspace [chunks][2][C]
//   fwd 2: every block folds the chunk partials of its 64 channels (a few dozen rows),
//          derives scale/shift, normalises (+ReLU) its chunk; chunk 0 writes the running
//          stats (moving = mom * moving + (1 - mom) * batch, unbiased var, as MXNet's cuDNN
//          path) and the saved mean / invstd.  The stats kernel records the shift it used in
//          the workspace, so no block of this kernel reads the running mean it updates.
//   bwd 1: partial sum(g), sum(g * xhat) with g = dy * relu_mask
//   bwd 2: fold partials -> dgamma / dbeta (chunk 0) and dx for the chunk.
// An earlier one-block-per-8-channels version read every 128-B line 8 times through L2 and
// ran ~37 us per call; this layout touches each line once per pass.
#include "common.h"
#include "../kernels.h"

namespace mxr {

constexpr int BT_C = 64;       // channels per block
constexpr int BT_LANES = 32;   // row lanes per block (8 channel groups x 32 = 256 threads)

int bn_train_rows(int64_t M, int C) {
  int rows = 256;
  while (rows > BT_LANES && (int64_t)(C / BT_C) * ((M + rows - 1) / rows) < 512) rows >>= 1;
  return rows;
}

// fold the per-chunk partials [nchunks][2][C] of this block's 64 channels: 4 threads per channel
// each sum every 4th chunk, combined through LDS -> out_a / out_b [64] (visible after the call)
__device__ __forceinline__ void fold_partials(const float* __restrict__ part, int nchunks, int C, float* red4,
                                              float* out_a, float* out_b) {
  const int tid = threadIdx.x, c = tid & 63, q = tid >> 6;
  const int cc = blockIdx.x * BT_C + c;
  // 8 chunks in flight per thread: the partials sit in L2, and a dependent chain of ~500-cycle
  // loads was most of these kernels' time
  float a8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, b8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int i = q;
  for (; i + 28 < nchunks; i += 32) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      a8[u] += part[(int64_t)(i + 4 * u) * 2 * C + cc];
      b8[u] += part[(int64_t)(i + 4 * u) * 2 * C + C + cc];
    }
  }
  for (; i < nchunks; i += 4) {
    a8[0] += part[(int64_t)i * 2 * C + cc];
    b8[0] += part[(int64_t)i * 2 * C + C + cc];
  }
  float a = 0.f, b = 0.f;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    a += a8[u];
    b += b8[u];
  }
  red4[q * 128 + c] = a;
  red4[q * 128 + 64 + c] = b;
  __syncthreads();
  if (tid < 128) {
    const int k = tid & 63, w = tid >> 6;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) s += red4[j * 128 + w * 64 + k];
    (w ? out_b : out_a)[k] = s;
  }
  __syncthreads();
}

// 8 channels of one row; pl > 0: x2 / x3 planes (common.h) pl elements apart
__device__ __forceinline__ void ld8(const uint16_t* p, float* v, int64_t pl, bool x3) {
  if (pl) ld8x(p, pl, v, x3);
  else ld8_bf16(p, v);
}

__device__ __forceinline__ void st8(uint16_t* p, const float* v, int64_t pl, bool x3) {
  if (pl) {
    float t[8];
    st8x(p, pl, v, t, x3);
  } else {
    st8_bf16(p, v);
  }
}

// sum a[8] / b[8] over the 32 row lanes of each channel group; results for channel
// (cg*8 + k) land in out_a / out_b [64] (visible after the call)
__device__ __forceinline__ void lane_reduce(const float* a, const float* b, float (*red)[BT_LANES][16],
                                            float* out_a, float* out_b) {
  const int cg = threadIdx.x & 7, rl = threadIdx.x >> 3;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[cg][rl][k] = a[k];
    red[cg][rl][8 + k] = b[k];
  }
  __syncthreads();
  if (threadIdx.x < 128) {
    const int c = threadIdx.x & 63, which = threadIdx.x >> 6;
    const int g = c >> 3, k = c & 7;
    float s = 0.f;
    for (int r = 0; r < BT_LANES; ++r) s += red[g][r][which * 8 + k];
    (which ? out_b : out_a)[c] = s;
  }
  __syncthreads();
}

__global__ void __launch_bounds__(256)
bn_train_stats_kernel(const uint16_t* __restrict__ x, int64_t M, int C, int rows, const float* __restrict__ shift,
                      float* __restrict__ part, int x2) {
  const int64_t pl = x2 ? M * C : 0;  // x2 (2) / x3 (3) planes of every (M, C) operand
  __shared__ float red[8][BT_LANES][16];
  __shared__ float sa[64], sb[64];
  const int cg = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c0 = blockIdx.x * BT_C + cg * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rows;
  const int64_t r1 = r0 + rows < M ? r0 + rows : M;
  float sh[8], s1[8], s2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sh[k] = shift[c0 + k];
    s1[k] = s2[k] = 0.f;
  }
#pragma unroll 4
  for (int64_t r = r0 + rl; r < r1; r += BT_LANES) {
    float v[8];
    ld8(x + r * C + c0, v, pl, x2 == 3);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float d = v[k] - sh[k];
      s1[k] += d;
      s2[k] += d * d;
    }
  }
  lane_reduce(s1, s2, red, sa, sb);
  if (threadIdx.x < 64) {
    float* row = part + (int64_t)blockIdx.y * 2 * C;
    row[blockIdx.x * BT_C + threadIdx.x] = sa[threadIdx.x];
    row[C + blockIdx.x * BT_C + threadIdx.x] = sb[threadIdx.x];
    // the shift of these partials, for the norm kernel (which then owns the running stats)
    if (blockIdx.y == 0) part[(int64_t)gridDim.y * 2 * C + blockIdx.x * BT_C + threadIdx.x] = shift[blockIdx.x * BT_C + threadIdx.x];
  }
}

__global__ void __launch_bounds__(256)
bn_train_norm_kernel(const uint16_t* __restrict__ x, int64_t M, int C, int rows, int nchunks, const float* __restrict__ part,
                     const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ rmean,
                     float* __restrict__ rvar, float momentum, float eps, int fix_gamma, int relu,
                     uint16_t* __restrict__ y, float* __restrict__ save_mean, float* __restrict__ save_invstd,
                     float* __restrict__ save_veps, int x2) {
  const int64_t pl = x2 ? M * C : 0;  // x2 (2) / x3 (3) planes of every (M, C) operand
  __shared__ float scale_sh[64], shift_sh[64], red4[512], fa[64], fb[64];
  const int tid = threadIdx.x;
  fold_partials(part, nchunks, C, red4, fa, fb);
  if (tid < 64) {
    const int c = blockIdx.x * BT_C + tid;
    const float sh = part[(int64_t)nchunks * 2 * C + c];  // the shift the stats kernel used
    const float a = fa[tid], b = fb[tid];
    const float dm = a / (float)M;  // mean - shift
    const float var = fmaxf(b / (float)M - dm * dm, 0.f);
    const float mu = sh + dm;
    const float inv = rsqrtf(var + eps);
    const float g = fix_gamma ? 1.f : gamma[c];
    scale_sh[tid] = g * inv;
    shift_sh[tid] = beta[c] - mu * g * inv;
    if (blockIdx.y == 0) {
      save_mean[c] = mu;
      save_invstd[c] = inv;
      // var + eps: a BN-backward conv epilogue given (mean, veps, eps = 0) recomputes exactly inv
      if (save_veps) save_veps[c] = var + eps;
      // running statistics (MXNet cuDNN path: unbiased batch variance); no block reads rmean
      const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
      rmean[c] = momentum * rmean[c] + (1.f - momentum) * mu;
      rvar[c] = momentum * rvar[c] + (1.f - momentum) * unb;
    }
  }
  __syncthreads();
  const int cg = tid & 7, rl = tid >> 3;
  const int c0 = blockIdx.x * BT_C + cg * 8;
  float sc[8], sf[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc[k] = scale_sh[cg * 8 + k];
    sf[k] = shift_sh[cg * 8 + k];
  }
  const int64_t r0 = (int64_t)blockIdx.y * rows;
  const int64_t r1 = r0 + rows < M ? r0 + rows : M;
#pragma unroll 4
  for (int64_t r = r0 + rl; r < r1; r += BT_LANES) {
    float v[8];
    ld8(x + r * C + c0, v, pl, x2 == 3);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      v[k] = v[k] * sc[k] + sf[k];
      if (relu) v[k] = fmaxf(v[k], 0.f);
    }
    st8(y + r * C + c0, v, pl, x2 == 3);
  }
}

__global__ void __launch_bounds__(256)
bn_train_bstats_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy, int64_t M, int C,
                       const float* __restrict__ gamma, const float* __restrict__ beta,
                       const float* __restrict__ save_mean, const float* __restrict__ save_invstd, int fix_gamma,
                       int relu, int rows, float* __restrict__ part, int x2) {
  const int64_t pl = x2 ? M * C : 0;  // x2 (2) / x3 (3) planes of every (M, C) operand
  __shared__ float red[8][BT_LANES][16];
  __shared__ float sa[64], sb[64];
  const int cg = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c0 = blockIdx.x * BT_C + cg * 8;
  float mu[8], inv[8], g[8], b[8], sg[8], sgx[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mu[k] = save_mean[c0 + k];
    inv[k] = save_invstd[c0 + k];
    g[k] = fix_gamma ? 1.f : gamma[c0 + k];
    b[k] = beta[c0 + k];
    sg[k] = sgx[k] = 0.f;
  }
  const int64_t r0 = (int64_t)blockIdx.y * rows;
  const int64_t r1 = r0 + rows < M ? r0 + rows : M;
#pragma unroll 4
  for (int64_t r = r0 + rl; r < r1; r += BT_LANES) {
    float v[8], d[8];
    ld8(x + r * C + c0, v, pl, x2 == 3);
    ld8(dy + r * C + c0, d, pl, x2 == 3);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float xh = (v[k] - mu[k]) * inv[k];
      const float gm = (!relu || xh * g[k] + b[k] > 0.f) ? d[k] : 0.f;
      sg[k] += gm;
      sgx[k] += gm * xh;
    }
  }
  lane_reduce(sg, sgx, red, sa, sb);
  if (threadIdx.x < 64) {
    float* row = part + (int64_t)blockIdx.y * 2 * C;
    row[blockIdx.x * BT_C + threadIdx.x] = sa[threadIdx.x];
    row[C + blockIdx.x * BT_C + threadIdx.x] = sb[threadIdx.x];
  }
}

__global__ void __launch_bounds__(256)
bn_train_dx_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy, int64_t M, int C, int rows, int nchunks,
                   const float* __restrict__ part, const float* __restrict__ gamma, const float* __restrict__ beta,
                   const float* __restrict__ save_mean, const float* __restrict__ save_invstd, int fix_gamma,
                   int relu, uint16_t* __restrict__ dx, float* __restrict__ dgamma, float* __restrict__ dbeta,
                   int accumulate, int x2) {
  const int64_t pl = x2 ? M * C : 0;  // x2 (2) / x3 (3) planes of every (M, C) operand
  __shared__ float mg_sh[64], mgx_sh[64], red4[512], fa[64], fb[64];
  const int tid = threadIdx.x;
  fold_partials(part, nchunks, C, red4, fa, fb);
  if (tid < 64) {
    const int c = blockIdx.x * BT_C + tid;
    const float a = fa[tid], b = fb[tid];
    mg_sh[tid] = a / (float)M;
    mgx_sh[tid] = b / (float)M;
    if (blockIdx.y == 0) {
      if (dgamma && !fix_gamma) dgamma[c] = accumulate ? dgamma[c] + b : b;
      if (dbeta) dbeta[c] = accumulate ? dbeta[c] + a : a;
    }
  }
  __syncthreads();
  if (!dx) return;
  const int cg = tid & 7, rl = tid >> 3;
  const int c0 = blockIdx.x * BT_C + cg * 8;
  float mu[8], inv[8], g[8], b[8], mg[8], mgx[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mu[k] = save_mean[c0 + k];
    inv[k] = save_invstd[c0 + k];
    g[k] = fix_gamma ? 1.f : gamma[c0 + k];
    b[k] = beta[c0 + k];
    mg[k] = mg_sh[cg * 8 + k];
    mgx[k] = mgx_sh[cg * 8 + k];
  }
  const int64_t r0 = (int64_t)blockIdx.y * rows;
  const int64_t r1 = r0 + rows < M ? r0 + rows : M;
#pragma unroll 4
  for (int64_t r = r0 + rl; r < r1; r += BT_LANES) {
    float v[8], d[8];
    ld8(x + r * C + c0, v, pl, x2 == 3);
    ld8(dy + r * C + c0, d, pl, x2 == 3);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float xh = (v[k] - mu[k]) * inv[k];
      const float gm = (!relu || xh * g[k] + b[k] > 0.f) ? d[k] : 0.f;
      d[k] = g[k] * inv[k] * (gm - mg[k] - xh * mgx[k]);
    }
    st8(dx + r * C + c0, d, pl, x2 == 3);
  }
}

int bn_train_workspace_floats(int64_t M, int C) {
  const int rows = bn_train_rows(M, C);
  return (int)(((M + rows - 1) / rows) * 2 * C + C);
}

int bn_train_fwd(const uint16_t* x, int64_t M, int C, const float* gamma, const float* beta, float* rmean,
                 float* rvar, float momentum, float eps, int fix_gamma, int relu, uint16_t* y, float* save_mean,
                 float* save_invstd, float* workspace, hipStream_t st, float* save_veps, int x2) {
  if (C % BT_C != 0 || M <= 0) return -1;
  const int rows = bn_train_rows(M, C);
  const int nchunks = (int)((M + rows - 1) / rows);
  const dim3 grid(C / BT_C, nchunks);
  bn_train_stats_kernel<<<grid, 256, 0, st>>>(x, M, C, rows, rmean, workspace, x2);
  bn_train_norm_kernel<<<grid, 256, 0, st>>>(x, M, C, rows, nchunks, workspace, gamma, beta, rmean, rvar, momentum, eps,
                                             fix_gamma, relu, y, save_mean, save_invstd, save_veps, x2);
  return 0;
}

int bn_train_apply(const uint16_t* x, int64_t M, int C, const float* part, int nparts, const float* gamma,
                   const float* beta, float* rmean, float* rvar, float momentum, float eps, int fix_gamma, int relu,
                   uint16_t* y, float* save, hipStream_t st, int x2) {
  if (C % BT_C != 0 || M <= 0 || nparts <= 0) return -1;
  const int rows = bn_train_rows(M, C);
  const dim3 grid(C / BT_C, (int)((M + rows - 1) / rows));
  bn_train_norm_kernel<<<grid, 256, 0, st>>>(x, M, C, rows, nparts, part, gamma, beta, rmean, rvar, momentum, eps,
                                             fix_gamma, relu, y, save, save + C, save + 2 * C, x2);
  return 0;
}

// dx = s * (g - mean(g) - xhat * mean(g * xhat)) (+ dres), from o = g * s written by a BN-backward
// conv epilogue that left per-row-tile partial rows [nparts][sum g | sum g * xhat][C] (ConvEpi::
// bnb_part; folded here in a fixed order, so the step is deterministic).  o and dx may alias
// (each element is read then written by the same thread).
__global__ void __launch_bounds__(256)
bn_train_dx_apply_kernel(const uint16_t* o, const uint16_t* __restrict__ x, int64_t M, int C, int rows,
                         const float* __restrict__ part, int nparts, const float* __restrict__ gamma,
                         const float* __restrict__ save, const uint16_t* __restrict__ dres, uint16_t* dx,
                         float* __restrict__ dgamma, float* __restrict__ dbeta, int x2) {
  const int64_t pl = x2 ? M * C : 0;  // x2 (2) / x3 (3) planes of every (M, C) operand
  __shared__ float red4[512], fa[64], fb[64];
  const int tid = threadIdx.x, cg = tid & 7, rl = tid >> 3;
  fold_partials(part, nparts, C, red4, fa, fb);
  if (blockIdx.y == 0 && tid < 64) {
    const int c = blockIdx.x * BT_C + tid;
    if (dbeta) dbeta[c] += fa[tid];
    if (dgamma) dgamma[c] += fb[tid];
  }
  const int c0 = blockIdx.x * BT_C + cg * 8;
  const float invM = 1.f / (float)M;
  float a[8], b[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float mu = save[c0 + k], inv = save[C + c0 + k];
    const float s = gamma[c0 + k] * inv;
    // dx = o - s * mg - s * mgx * (x - mu) * inv = o - a - b * x
    const float mg = fa[cg * 8 + k] * invM, mgx = fb[cg * 8 + k] * invM;
    b[k] = s * mgx * inv;
    a[k] = s * mg - b[k] * mu;
  }
  const int64_t r0 = (int64_t)blockIdx.y * rows;
  const int64_t r1 = r0 + rows < M ? r0 + rows : M;
#pragma unroll 4
  for (int64_t r = r0 + rl; r < r1; r += BT_LANES) {
    float v[8], d[8], rr[8];
    ld8(x + r * C + c0, v, pl, x2 == 3);
    ld8(o + r * C + c0, d, pl, x2 == 3);
    if (dres) ld8(dres + r * C + c0, rr, pl, x2 == 3);
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = d[k] - a[k] - b[k] * v[k] + (dres ? rr[k] : 0.f);
    st8(dx + r * C + c0, d, pl, x2 == 3);
  }
}

int bn_train_dx_apply(const uint16_t* o, const uint16_t* x, int64_t M, int C, const float* part, int nparts,
                      const float* gamma, const float* save, const uint16_t* dres, uint16_t* dx, float* dgamma,
                      float* dbeta, hipStream_t st, int x2) {
  if (C % BT_C != 0 || M <= 0 || nparts <= 0) return -1;
  const int rows = bn_train_rows(M, C);
  const dim3 grid(C / BT_C, (int)((M + rows - 1) / rows));
  bn_train_dx_apply_kernel<<<grid, 256, 0, st>>>(o, x, M, C, rows, part, nparts, gamma, save, dres, dx, dgamma, dbeta, x2);
  return 0;
}

int bn_train_bwd(const uint16_t* x, const uint16_t* dy, int64_t M, int C, const float* gamma, const float* beta,
                 const float* save_mean, const float* save_invstd, int fix_gamma, int relu, uint16_t* dx,
                 float* dgamma, float* dbeta, int accumulate, float* workspace, hipStream_t st, int x2) {
  if (C % BT_C != 0 || M <= 0) return -1;
  const int rows = bn_train_rows(M, C);
  const int nchunks = (int)((M + rows - 1) / rows);
  const dim3 grid(C / BT_C, nchunks);
  bn_train_bstats_kernel<<<grid, 256, 0, st>>>(x, dy, M, C, gamma, beta, save_mean, save_invstd, fix_gamma, relu,
                                               rows, workspace, x2);
  bn_train_dx_kernel<<<grid, 256, 0, st>>>(x, dy, M, C, rows, nchunks, workspace, gamma, beta, save_mean, save_invstd,
                                           fix_gamma, relu, dx, dgamma, dbeta, accumulate, x2);
  return 0;
}

}  // namespace mxr
