// Implicit-GEMM convolution on NHWC bf16 activations with MFMA (SURVEY kernels K1/K2/K3).
//
//   out[m][n] = sum_k A[m][k] * W[n][k],   m = (img, ho, wo), n = cout, k = (fr, fc, cin)
//
// A is never materialised: each K-step gathers 64 input channels of ONE filter tap for
// BM output pixels straight from the NHWC map (out-of-image taps read as zero), so both
// operands are K-contiguous in memory and land in LDS as [row][64] bf16 tiles (128 B rows)
// with an XOR swizzle on the 16-B chunk index (chunk ^ ((row >> 1) & 7)), which makes the
// MFMA-operand ds_read_b128 of 16 consecutive rows conflict-free.  256 threads = 4 wave64 in a
// 2x2 arrangement, wave tile (BM/2)x(BN/2) of v_mfma_f32_16x16x32_bf16 (fp32 accumulate); 1-D
// grid with a bijective XCD remap so the column tiles sharing an A row-panel run on one XCD's L2.
//
// Variants (tile codes; conv_igemm_plan picks 22 / 23 with split-K only for small grids):
//   1-3     register-staged loads, double-buffered LDS (the first version; test oracle shapes)
//   11-16   global_load_lds DMA straight into an S-deep LDS ring, counted vmcnt + raw barrier
//   21-25   buffer-resource DMA (buffer_load ... lds).  Per lane a 32-bit row offset and a
//           64-bit tap mask are precomputed once, the per-step offsets are uniform (SGPR),
//           padding comes from the buffer range check returning zeros
//   100+    the tile-balanced ring (any wave layout, 4-16 waves, ring depth per config); the
//           per-shape autotune (bindings.cpp) picks among 22 / 23 / 100+ on first use
// Epilogues (ConvEpi): bias, ReLU, residual add, frozen BN+ReLU of the consumer (second output),
// BN-backward column sums (dgrad fused with the BN backward), fp32 split-K slab + reduce; the
// LDS-transposed epilogue makes every global access a 16-B vector.  Cin % 64 == 0.
//
// The same kernel computes the stride-1 data gradient (dgrad) as a forward convolution of
// dY with the flipped / transposed filter (pad' = k-1-pad); see ops/conv.py.
#include <cstdlib>

#include "igemm_body.h"

namespace mxr {

template <int BM, int BN>
__global__ void __launch_bounds__(256)
conv_igemm_fwd_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, uint16_t* __restrict__ y,
                      int NB, int H, int W, int Cin, int Ho, int Wo, int Cout, int KH, int KW, int stride, int pad,
                      const ConvEpi ep, int tiles_n, int nwg, int ntiles, int splits, float* __restrict__ slab) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int ACH = BM * 8 / 256;  // 16-B chunks of A per thread per K-step
  constexpr int BCH = BN * 8 / 256;
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * (BM + BN) * BK];
  uint16_t* As = lds;                    // [2][BM][BK]
  uint16_t* Bs = lds + 2 * BM * BK;      // [2][BN][BK]

  // bijective XCD-aware block remap (blocks that share an A panel -> same XCD)
  const int bid = blockIdx.x;
  const int q = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
  const int wgid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + bid / 8;
  const int split = wgid / ntiles, tile = wgid % ntiles;
  const int tm_idx = tile / tiles_n, tn_idx = tile % tiles_n;
  const int m0 = tm_idx * BM, n0 = tn_idx * BN;
  const int M = NB * Ho * Wo;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  // per-thread A rows: precompute pixel decomposition
  int a_hi0[ACH], a_wi0[ACH], a_img[ACH], a_row[ACH], a_ch[ACH];
#pragma unroll
  for (int i = 0; i < ACH; ++i) {
    const int qq = tid + i * 256;
    a_row[i] = qq >> 3;
    a_ch[i] = qq & 7;
    const int m = m0 + a_row[i];
    if (m < M) {
      const int img = m / (Ho * Wo), rem = m % (Ho * Wo);
      a_img[i] = img;
      a_hi0[i] = (rem / Wo) * stride - pad;
      a_wi0[i] = (rem % Wo) * stride - pad;
    } else {
      a_img[i] = -1; a_hi0[i] = 0; a_wi0[i] = 0;
    }
  }
  int b_row[BCH], b_ch[BCH];
#pragma unroll
  for (int i = 0; i < BCH; ++i) {
    const int qq = tid + i * 256;
    b_row[i] = qq >> 3;
    b_ch[i] = qq & 7;
  }
  const int K = KH * KW * Cin;
  const int cin_steps = Cin / BK;
  const int nk_all = KH * KW * cin_steps;
  const int per = (nk_all + splits - 1) / splits;
  const int k_begin = split * per;
  const int k_end = min(nk_all, k_begin + per);
  const int nk = max(0, k_end - k_begin);

  uint4 ra[ACH], rb[BCH];
  auto load = [&](int kl) {
    const int ks = k_begin + kl;
    const int tap = ks / cin_steps;
    const int ci0 = (ks % cin_steps) * BK;
    const int fr = tap / KW, fc = tap % KW;
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int hi = a_hi0[i] + fr, wi = a_wi0[i] + fc;
      if (a_img[i] >= 0 && hi >= 0 && hi < H && wi >= 0 && wi < W) {
        const int64_t off = (((int64_t)a_img[i] * H + hi) * W + wi) * Cin + ci0 + a_ch[i] * 8;
        ra[i] = *reinterpret_cast<const uint4*>(x + off);
      } else {
        ra[i] = make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int co = n0 + b_row[i];
      if (co < Cout) {
        const int64_t off = (int64_t)co * K + tap * Cin + ci0 + b_ch[i] * 8;
        rb[i] = *reinterpret_cast<const uint4*>(w + off);
      } else {
        rb[i] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < ACH; ++i)
      *reinterpret_cast<uint4*>(As + (buf * BM + a_row[i]) * BK + swz(a_row[i], a_ch[i]) * 8) = ra[i];
#pragma unroll
    for (int i = 0; i < BCH; ++i)
      *reinterpret_cast<uint4*>(Bs + (buf * BN + b_row[i]) * BK + swz(b_row[i], b_ch[i]) * 8) = rb[i];
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nk) load(ks + 1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[TM], bfr[TN];
      const int chunk = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(As + (buf * BM + row) * BK + swz(row, chunk) * 8);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + j * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + (buf * BN + row) * BK + swz(row, chunk) * 8);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (ks + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }

  igemm_epilogue<TM, TN, WM, WN>(acc, m0, n0, wm, wn, lane, M, Cout, ep, y, split, splits, slab);
}

// split-K reduce for the BN-backward epilogue: column-blocked so the per-column statistics are
// accumulated in registers over 64 rows and leave the block with one atomic per column.
// Block = 16 column quads (64 columns) x 16 row lanes; grid = (Cout/64) x ceil(M/64).
__global__ void __launch_bounds__(256)
splitk_reduce_bnb_kernel(const float* __restrict__ slab, int splits, int M, int Cout, const ConvEpi ep,
                         uint16_t* __restrict__ y) {
  __shared__ float red[2][16][64];
  const int cq = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int n = blockIdx.x * 64 + cq * 4;
  const int r0 = blockIdx.y * 64;
  const int64_t MN = (int64_t)M * Cout;
  float sg[4] = {0.f, 0.f, 0.f, 0.f}, sgx[4] = {0.f, 0.f, 0.f, 0.f};
  EpiCol ec[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) ec[k] = epi_col(ep, min(n + k, Cout - 1));
  if (n < Cout) {
    for (int r = r0 + rl; r < min(M, r0 + 64); r += 16) {
      const int64_t e = (int64_t)r * Cout + n;
      float4 a = *reinterpret_cast<const float4*>(slab + e);
      for (int sidx = 1; sidx < splits; ++sidx) {
        const float4 b = *reinterpret_cast<const float4*>(slab + (int64_t)sidx * MN + e);
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      }
      const float v[4] = {a.x, a.y, a.z, a.w};
      const int64_t drow = dadd_row(ep, r, r);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (ep.x2) epi_bnb<true>(ep, ec[k], y, e + k, v[k], sg[k], sgx[k], drow < 0 ? -1 : drow * Cout + n + k);
        else epi_bnb<false>(ep, ec[k], y, e + k, v[k], sg[k], sgx[k], drow < 0 ? -1 : drow * Cout + n + k);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    red[0][rl][cq * 4 + k] = sg[k];
    red[1][rl][cq * 4 + k] = sgx[k];
  }
  __syncthreads();
  if (threadIdx.x < 128) {
    const int stat = threadIdx.x >> 6, col = threadIdx.x & 63;
    float t = 0.f;
    for (int q = 0; q < 16; ++q) t += red[stat][q][col];
    const int nc = blockIdx.x * 64 + col;
    if (nc < Cout) {
      if (stat == 0 && ep.bnb_dbeta) atomicAdd(ep.bnb_dbeta + nc, t);
      if (stat == 1 && ep.bnb_dgamma && !ep.bn_fix_gamma) atomicAdd(ep.bnb_dgamma + nc, t);
    }
  }
}

// split-K reduce + the fused epilogue, 4 outputs per thread (Cout % 4 == 0)
__global__ void __launch_bounds__(256)
splitk_reduce_kernel(const float* __restrict__ slab, int splits, int64_t MN, int Cout, const ConvEpi ep,
                     uint16_t* __restrict__ y) {
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (e >= MN) return;
  float4 a = *reinterpret_cast<const float4*>(slab + e);
  for (int sidx = 1; sidx < splits; ++sidx) {
    const float4 b = *reinterpret_cast<const float4*>(slab + (int64_t)sidx * MN + e);
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  }
  float v[4] = {a.x, a.y, a.z, a.w};
  const int n = (int)(e % Cout);
  float res[4] = {0.f, 0.f, 0.f, 0.f};
  if (ep.residual) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      res[k] = ep.x2 ? epi_ld1<true>(ep, ep.residual, e + k, ep.x2_py) : epi_ld1<false>(ep, ep.residual, e + k, 0);
  }
  if (ep.x2 || ep.yf) {  // scalar pair / fp32 stores (the packed 16-bit path below is the common one)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const EpiCol c = epi_col(ep, n + k);
      float t = v[k] + c.bias + res[k];
      if (ep.relu) t = fmaxf(t, 0.f);
      t = epi_rmask(ep, e + k, epi_dropout(ep, e + k, t));
      if (ep.yf) {
        ep.yf[e + k] = t;
        continue;
      }
      const float ys = epi_st1<true>(ep, y, e + k, ep.x2_py, t);
      if (ep.y2) {
        float q = ys * c.s + c.t;
        if (ep.act_relu) q = fmaxf(q, 0.f);
        epi_st1<true>(ep, ep.y2, e + k, ep.x2_py, q);
      }
    }
    return;
  }
  uint16_t out[4], out2[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const EpiCol c = epi_col(ep, n + k);
    float t = v[k] + c.bias + res[k];
    if (ep.relu) t = fmaxf(t, 0.f);
    t = epi_rmask(ep, e + k, epi_dropout(ep, e + k, t));
    out[k] = f32_to_h16c(EPC, t);
    float q = h16_to_f32c(EPC, out[k]) * c.s + c.t;
    if (ep.act_relu) q = fmaxf(q, 0.f);
    out2[k] = f32_to_h16c(EPC, q);
  }
  *reinterpret_cast<ushort4*>(y + e) = make_ushort4(out[0], out[1], out[2], out[3]);
  if (ep.y2) *reinterpret_cast<ushort4*>(ep.y2 + e) = make_ushort4(out2[0], out2[1], out2[2], out2[3]);
}

void splitk_reduce_launch(const float* slab, int splits, int M, int Cout, const ConvEpi& ep, uint16_t* y,
                          hipStream_t st) {
  const int64_t MN = (int64_t)M * Cout;
  if (ep.bnb_x)
    splitk_reduce_bnb_kernel<<<dim3(div_up(Cout, 64), div_up(M, 64)), 256, 0, st>>>(slab, splits, M, Cout, ep, y);
  else
    splitk_reduce_kernel<<<div_up((MN + 3) / 4, 256), 256, 0, st>>>(slab, splits, MN, Cout, ep, y);
}

// ---- S-stage LDS-DMA pipeline (the latency-bound 1-image detection regime) -----------------
// One image's stage-3/4 convs give M = 2-6 K output rows: a few hundred workgroups, one per CU,
// 4 waves each.  The register-staged kernel above keeps one K-step in flight, so every K-step
// pays a full L2/MALL round trip (~1 us under load) for ~8-32 MFMAs.  Here every thread issues
// its tile chunks as global_load_lds_dwordx4 (LDS-DMA, no VGPRs) S-1 K-steps ahead into an S-deep
// LDS ring; a counted `s_waitcnt vmcnt` retires exactly the oldest stage and a raw s_barrier
// publishes it (a __syncthreads() fence would drain every DMA in flight).  The LDS image is
// written lane-linearly (DMA destination = wave base + lane * 16 B), so the XOR swizzle of the
// MFMA-operand reads is applied to the per-lane SOURCE chunk instead; out-of-image taps and
// rows past Cout read a 128-B block of zeros.  The MFMA tile, fragment reads and epilogue are
// those of conv_igemm_fwd_kernel.
__device__ __attribute__((aligned(128))) uint16_t g_igemm_zeros[64];

template <int BM, int BN, int S>
__global__ void __launch_bounds__(256)
conv_igemm_glds_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, uint16_t* __restrict__ y,
                       int NB, int H, int W, int Cin, int Ho, int Wo, int Cout, int KH, int KW, int stride, int pad,
                       const ConvEpi ep, int tiles_n, int nwg, int ntiles, int splits, float* __restrict__ slab) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int ACH = BM / 32, BCH = BN / 32;  // DMA instructions per thread per stage (8 rows each)
  constexpr int LPS = ACH + BCH;
  static_assert(S >= 2 && S <= 4, "pipeline depth");
  __shared__ __attribute__((aligned(16))) uint16_t lds[S * (BM + BN) * BK];  // the ONLY __shared__ object
  uint16_t* As = lds;               // [S][BM][BK]
  uint16_t* Bs = lds + S * BM * BK;  // [S][BN][BK]

  const int bid = blockIdx.x;
  const int q = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
  const int wgid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + bid / 8;
  const int split = wgid / ntiles, tile = wgid % ntiles;
  const int tm_idx = tile / tiles_n, tn_idx = tile % tiles_n;
  const int m0 = tm_idx * BM, n0 = tn_idx * BN;
  const int M = NB * Ho * Wo;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  // DMA instruction i of wave wid fills tile rows 32 i + 8 wid .. +8; lane -> row + lane/8, slot lane%8
  const int slot = lane & 7;
  int a_hi0[ACH], a_wi0[ACH], a_img[ACH], a_lc[ACH];
#pragma unroll
  for (int i = 0; i < ACH; ++i) {
    const int row = 32 * i + 8 * wid + (lane >> 3);
    a_lc[i] = slot ^ ((row >> 1) & 7);  // logical 16-B chunk stored in this slot (swizzle)
    const int m = m0 + row;
    if (m < M) {
      const int img = m / (Ho * Wo), rem = m % (Ho * Wo);
      a_img[i] = img;
      a_hi0[i] = (rem / Wo) * stride - pad;
      a_wi0[i] = (rem % Wo) * stride - pad;
    } else {
      a_img[i] = -1; a_hi0[i] = 0; a_wi0[i] = 0;
    }
  }
  const uint16_t* b_src[BCH];
#pragma unroll
  for (int i = 0; i < BCH; ++i) {
    const int row = 32 * i + 8 * wid + (lane >> 3);
    const int co = n0 + row;
    b_src[i] = co < Cout ? w + (int64_t)co * KH * KW * Cin + (slot ^ ((row >> 1) & 7)) * 8 : nullptr;
  }
  const int cin_steps = Cin / BK;
  const int nk_all = KH * KW * cin_steps;
  const int per = (nk_all + splits - 1) / splits;
  const int k_begin = split * per;
  const int k_end = min(nk_all, k_begin + per);
  const int nk = max(0, k_end - k_begin);

  auto issue = [&](int kl, int buf) {
    const int ks = k_begin + kl;
    const int tap = ks / cin_steps;
    const int ci0 = (ks % cin_steps) * BK;
    const int fr = tap / KW, fc = tap % KW;
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int hi = a_hi0[i] + fr, wi = a_wi0[i] + fc;
      const uint16_t* src = g_igemm_zeros;
      if (a_img[i] >= 0 && hi >= 0 && hi < H && wi >= 0 && wi < W)
        src = x + (((int64_t)a_img[i] * H + hi) * W + wi) * Cin + ci0 + a_lc[i] * 8;
      glds16(src, As + (buf * BM + 32 * i + 8 * wid) * BK);
    }
    const int koff = tap * Cin + ci0;
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const uint16_t* src = b_src[i] ? b_src[i] + koff : g_igemm_zeros;
      glds16(src, Bs + (buf * BN + 32 * i + 8 * wid) * BK);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) issue(s, s);
  for (int ks = 0; ks < nk; ++ks) {
    // retire stage ks: the stages issued after it may stay in flight
    const int ahead = min(S - 2, nk - 1 - ks);
    if (ahead >= 2) wait_vmcnt<2 * LPS>();
    else if (ahead == 1) wait_vmcnt<LPS>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();  // every wave's DMA of stage ks landed; stage ks-1 fully read
    if (ks + S - 1 < nk) issue(ks + S - 1, (ks + S - 1) % S);
    const int buf = ks % S;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[TM], bfr[TN];
      const int chunk = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(As + (buf * BM + row) * BK + swz(row, chunk) * 8);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + j * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + (buf * BN + row) * BK + swz(row, chunk) * 8);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  igemm_epilogue<TM, TN, WM, WN>(acc, m0, n0, wm, wn, lane, M, Cout, ep, y, split, splits, slab);
}

template <int BM, int BN, int S, bool F16 = false, bool X2 = false, bool BT = false, bool X3 = false>
__global__ void __launch_bounds__(256)
conv_igemm_buf_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, uint16_t* __restrict__ y,
                      int NB, int H, int W, int Cin, int Ho, int Wo, int Cout, int KH, int KW, int stride, int pad,
                      const ConvEpi ep, int tiles_n, int nwg, int ntiles, int splits, float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[S * igemm_ring_stage<BM, BN, BT, X3>()];
  igemm_buf_body<BM, BN, S, F16, X2, BT, 1, X3>(lds, blockIdx.x, x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride,
                                                pad, ep, tiles_n, nwg, ntiles, splits, slab);
}

// ---- fp32-class pairs, wide stages (tile code 26) ---------------------------------------------
// The x2 buffer kernel above stages 32 channels of both planes per K step (128-B LDS rows): a
// stage-3 conv at batch 1 then runs 32-72 barrier-separated steps of 16 KB, and the per-step DMA
// round trip sets its pace (profiles/r3_conv_study.md: the isolated load + fragment-read + MFMA
// loop at 32 KB stages is 18 % faster than at 16 KB).  Here a stage is 64 channels of BOTH planes:
// 256-B LDS rows, logical 16-B chunks 0-7 the hi plane's channels c..c+63, 8-15 the lo plane's,
// stored at chunk lc ^ (row & 15) (16 rows of one logical chunk -> 16 distinct bank slots, also
// across the ds_read_b128 lane groups, which pair chunk c with c+1 for even c).  Two stages deep
// (64 KB for 64x64: two workgroups fit a CU, so a 264-tile grid runs in one round), one barrier per
// 64 channels, 2 k-halves x 3 products per stage.  Forward (non-BT) convs, plain and BN epilogues
// as the buffer kernel (same epilogue code).
template <int BM, int BN>
__device__ __forceinline__ void igemm_x2w_body(uint16_t* lds, int bid, const uint16_t* __restrict__ x,
                                               const uint16_t* __restrict__ w, uint16_t* __restrict__ y, int NB, int H,
                                               int W, int Cin, int Ho, int Wo, int Cout, int KH, int KW, int stride,
                                               int pad, const ConvEpi& ep, int tiles_n, int nwg, int ntiles) {
  constexpr int S = 2;
  constexpr int RB = 2 * BK;  // LDS row: 64 channels x 2 planes
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int ACH = BM / 16, BCH = BN / 16;  // DMA instructions per wave per stage (4 rows each)
  static_assert(BM % 64 == 0 && BN % 64 == 0, "whole 16-row blocks per wave");
  uint16_t* As = lds;
  uint16_t* Bs = lds + S * BM * RB;

  const int q = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
  const int wgid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + bid / 8;
  const int tm_idx = wgid / tiles_n, tn_idx = wgid % tiles_n;
  const int m0 = tm_idx * BM, n0 = tn_idx * BN;
  const int M = NB * Ho * Wo;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int K = KH * KW * Cin;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)x, (short)0, (int)((int64_t)NB * H * W * Cin * 2 + ep.x2_pa), 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)w, (short)0, (int)((int64_t)Cout * K * 2 + ep.x2_pb), 0x00020000);

  // instruction i of wave w loads rows (BM / 4) * w + 4 * i .. + 3, lane -> row + (lane >> 4),
  // physical chunk lane & 15 = logical chunk (lane & 15) ^ (row & 15)
  constexpr int RPW_A = BM / 4, RPW_B = BN / 4;  // rows per wave
  const int pch = lane & 15;
  uint32_t a_off[ACH];
  uint64_t a_mask[ACH];
#pragma unroll
  for (int i = 0; i < ACH; ++i) {
    const int row = RPW_A * wid + 4 * i + (lane >> 4);
    const int lc = pch ^ (row & 15);
    const int m = m0 + row;
    a_off[i] = 0;
    a_mask[i] = 0;
    if (m < M) {
      const int img = m / (Ho * Wo), rem = m % (Ho * Wo);
      const int hi0 = (rem / Wo) * stride - pad, wi0 = (rem % Wo) * stride - pad;
      a_off[i] = (uint32_t)((((int64_t)img * H + hi0) * W + wi0) * Cin * 2 + (lc & 7) * 16) + (lc >= 8 ? ep.x2_pa : 0u);
      for (int fr = 0; fr < KH; ++fr)
        for (int fc = 0; fc < KW; ++fc)
          if ((unsigned)(hi0 + fr) < (unsigned)H && (unsigned)(wi0 + fc) < (unsigned)W) a_mask[i] |= 1ull << (fr * KW + fc);
    }
  }
  uint32_t b_off[BCH];
#pragma unroll
  for (int i = 0; i < BCH; ++i) {
    const int row = RPW_B * wid + 4 * i + (lane >> 4);
    const int lc = pch ^ (row & 15);
    const int co = n0 + row;
    b_off[i] = co < Cout ? (uint32_t)((int64_t)co * K * 2 + (lc & 7) * 16) + (lc >= 8 ? ep.x2_pb : 0u) : kBufOOB;
  }
  const int cin_steps = Cin / 64;
  const int nk = KH * KW * cin_steps;
  int c_tap = 0, c_ci = 0, c_fr = 0, c_fc = 0;
  auto issue = [&](int buf) {
    const uint32_t tap_a = (uint32_t)((c_fr * W + c_fc) * Cin * 2);
    const uint32_t soff_a = (uint32_t)(c_ci * 2);
    const uint32_t soff_b = (uint32_t)((c_tap * Cin + c_ci) * 2);
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const uint32_t vo = ((a_mask[i] >> c_tap) & 1ull) ? a_off[i] + tap_a : kBufOOB;
      buf_lds16(xr, As + (buf * BM + RPW_A * wid + 4 * i) * RB, vo, soff_a);
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) buf_lds16(wr, Bs + (buf * BN + RPW_B * wid + 4 * i) * RB, b_off[i], soff_b);
    c_ci += 64;
    if (c_ci == Cin) {
      c_ci = 0;
      ++c_tap;
      if (++c_fc == KW) {
        c_fc = 0;
        ++c_fr;
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) issue(0);
  for (int ks = 0; ks < nk; ++ks) {
    wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();  // stage ks landed for every wave; stage ks-1's buffer is free
    if (ks + 1 < nk) issue((ks + 1) & 1);
    const int buf = ks & 1;
    const int g = lane >> 4;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 16 + (lane & 15);
        const uint16_t* r = As + (buf * BM + row) * RB;
        ah[i] = *reinterpret_cast<const bf16x8*>(r + (((kk * 4 + g) ^ (row & 15)) << 3));
        al[i] = *reinterpret_cast<const bf16x8*>(r + (((8 + kk * 4 + g) ^ (row & 15)) << 3));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + j * 16 + (lane & 15);
        const uint16_t* r = Bs + (buf * BN + row) * RB;
        bh[j] = *reinterpret_cast<const bf16x8*>(r + (((kk * 4 + g) ^ (row & 15)) << 3));
        bl[j] = *reinterpret_cast<const bf16x8*>(r + (((8 + kk * 4 + g) ^ (row & 15)) << 3));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
    }
  }
  static_assert((BM * (BN + 4) + 5 * BN) * 4 <= S * (BM + BN) * RB * 2,
                "epilogue tile + column table must fit the operand ring");
  if (Cout % 8 == 0)
    igemm_epilogue_lds<BM, BN, TM, TN, WM, WN, true>(acc, reinterpret_cast<float*>(lds), m0, n0, wm, wn, lane, tid, M,
                                                     Cout, ep, y, 0, 1, nullptr, Ho, Wo);
  else
    igemm_epilogue<TM, TN, WM, WN, true>(acc, m0, n0, wm, wn, lane, M, Cout, ep, y, 0, 1, nullptr, Ho, Wo);
}

template <int BM, int BN>
__global__ void __launch_bounds__(256)
conv_x2w_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, uint16_t* __restrict__ y, int NB,
                int H, int W, int Cin, int Ho, int Wo, int Cout, int KH, int KW, int stride, int pad, const ConvEpi ep,
                int tiles_n, int nwg, int ntiles) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * (BM + BN) * 2 * BK];
  igemm_x2w_body<BM, BN>(lds, blockIdx.x, x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, tiles_n, nwg,
                         ntiles);
}

// ---- tile-balanced LDS-DMA ring (the production path) ----------------------------------------
// Measured on the ResNet-101 C4 stage-3/4 shapes (rocprofv3 --pmc, profiles/r2_conv_pmc.txt): the
// 64x64 ring above is limited by what ONE CU can pull into LDS (~27 GB/s at two 16 KB stages in
// flight, 47 % of wave cycles parked on vmcnt/barrier), and by tile quantisation: 4200 x 256 gives
// 264 tiles for 256 CUs, so 8 CUs carry two tiles and set the kernel time.  This kernel
//   * sizes the tile so the grid is at most one (or an integer number of) tile(s) per CU
//     (BM = 16*TM*WGM rows x BN = 16*TN*WGN columns, any wave layout WGM x WGN),
//   * keeps 5-7 K-steps in flight (S-deep ring, up to ~150 KB of LDS: one workgroup per CU),
//   * spreads the (BM+BN)/8 DMA instructions of a stage over the waves (a wave issues q or
//     q+1, and waits for exactly its own count), 1x1 convs skip the tap mask entirely,
//   * keeps the fragment reads, MFMA and fused epilogues of the kernels above.
template <int TM, int TN, int WGM, int WGN, int SFIX = 0>
struct RingCfg {
  static constexpr int NW = WGM * WGN, NT = 64 * NW;
  static constexpr int BM = 16 * TM * WGM, BN = 16 * TN * WGN;
  static constexpr int RA = BM / 8, RB = BN / 8, RT = RA + RB;  // 8-row DMA pieces per stage
  static constexpr int QL = RT / NW, RL = RT % NW;              // pieces per wave: QL (+1 for wid < RL)
  static constexpr int QMAX = QL + (RL ? 1 : 0);
  static constexpr int STAGE_BYTES = (BM + BN) * BK * 2;
  // deepest ring within ~150 KB of LDS, 3..8 stages, and <= 63 outstanding DMAs per wave
  static constexpr int S0 = (150 * 1024) / STAGE_BYTES;
  static constexpr int S1 = S0 > 8 ? 8 : (S0 < 3 ? 3 : S0);
  static constexpr int S2 = (S1 - 2) * QMAX > 60 ? 60 / QMAX + 2 : S1;
  static constexpr int S = SFIX ? SFIX : S2;
};

// wait until this wave has at most `ahead` stages of its own DMAs (n per stage) in flight
template <int N>
__device__ __forceinline__ void wait_ring(int ahead) {
  switch (ahead) {
    case 6: wait_vmcnt<6 * N>(); break;
    case 5: wait_vmcnt<5 * N>(); break;
    case 4: wait_vmcnt<4 * N>(); break;
    case 3: wait_vmcnt<3 * N>(); break;
    case 2: wait_vmcnt<2 * N>(); break;
    case 1: wait_vmcnt<N>(); break;
    default: wait_vmcnt<0>(); break;
  }
}

// Generic LDS-transposed epilogue for NT threads and any wave layout (see igemm_epilogue_lds).
template <int BM, int BN, int TM, int TN, int NT>
__device__ __forceinline__ void ring_epilogue(f32x4 (&acc)[TM][TN], float* __restrict__ T, int m0, int n0, int wm,
                                              int wn, int lane, int tid, int M, int Cout, const ConvEpi& ep,
                                              uint16_t* __restrict__ y, int split, int splits,
                                              float* __restrict__ slab, int Ho = 1, int Wo = 1) {
  constexpr int LDT = BN + 4;
  constexpr int VPR = BN / 8;
  constexpr int NVEC = BM * VPR;
  constexpr int WM = 16 * TM, WN = 16 * TN;
  constexpr int NW = NT / 64;
  static_assert(64 % VPR == 0 && NT % VPR == 0, "column groups must tile the wave");
  __syncthreads();  // every wave is done reading the operand ring
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        T[(wm * WM + i * 16 + (lane >> 4) * 4 + r) * LDT + wn * WN + j * 16 + (lane & 15)] = acc[i][j][r];
  const bool use_tab = ep.y2 || ep.bnb_x;  // (bias-only: direct loads, see igemm_epilogue_lds)
  float* const tab = T + BM * LDT;  // [5][BN] column constants (igemm_body.h epi_cols_stage)
  if (splits <= 1 && use_tab) epi_cols_stage<BN, NT>(tab, ep, tid, n0, Cout);
  __syncthreads();
  const int cv = tid % VPR;
  const int n = n0 + cv * 8;
  const bool ncol = n < Cout;
  if (splits > 1) {
    float* sp = slab + (int64_t)split * M * Cout;
    for (int q = tid; q < NVEC; q += NT) {
      const int row = q / VPR, m = m0 + row;
      if (m >= M || !ncol) continue;
      const float4* src = reinterpret_cast<const float4*>(T + row * LDT + cv * 8);
      float4* dst = reinterpret_cast<float4*>(sp + (int64_t)m * Cout + n);
      dst[0] = src[0];
      dst[1] = src[1];
    }
    return;
  }
  EpiCol ec[8];
  if (use_tab) {
    epi_cols_load<BN>(tab, cv, ec);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) ec[k] = epi_col(ep, ncol ? n + k : 0);
  }
  if (ep.bnb_x) {
    float sg[8], sgx[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) sg[k] = sgx[k] = 0.f;
    for (int q = tid; q < NVEC; q += NT) {
      const int row = q / VPR, m = m0 + row;
      if (m >= M || !ncol) continue;
      const int64_t e = epi_row(ep, m, Ho, Wo) * Cout + n;
      float a[8], xv[8], d[8], rs[8];
      const float4* src = reinterpret_cast<const float4*>(T + row * LDT + cv * 8);
      const float4 a0 = src[0], a1 = src[1];
      a[0] = a0.x; a[1] = a0.y; a[2] = a0.z; a[3] = a0.w; a[4] = a1.x; a[5] = a1.y; a[6] = a1.z; a[7] = a1.w;
      ld8_h16(ep.bnb_x + e, xv, EPC);
      const int64_t drow = ep.dadd ? dadd_row(ep, m, e / Cout) : -1;
      if (drow >= 0) {
        ld8_h16(ep.dadd + drow * Cout + n, d, EPC);
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] += d[k];
      }
      if (ep.residual) ld8_h16(ep.residual + e, rs, EPC);
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float g = (!ep.act_relu || xv[k] * ec[k].s + ec[k].t > 0.f) ? a[k] : 0.f;
        sg[k] += g;
        sgx[k] += g * (xv[k] - ec[k].mean) * ec[k].inv;
        o[k] = g * ec[k].s + (ep.residual ? rs[k] : 0.f);
      }
      st8_h16(y + e, o, EPC);
    }
    epi_bnb_sums<BM, BN, NT>(sg, sgx, T, tid, m0, n0, Cout, ep);
    return;
  }
  float s1[8], s2[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    s1[k] = s2[k] = 0.f;
    sh[k] = (ep.st_part && ncol) ? ep.st_shift[n + k] : 0.f;
  }
  for (int q = tid; q < NVEC; q += NT) {
    const int row = q / VPR, m = m0 + row;
    if (m >= M || !ncol) continue;
    const int64_t e = epi_row(ep, m, Ho, Wo) * Cout + n;
    const float4* src = reinterpret_cast<const float4*>(T + row * LDT + cv * 8);
    const float4 a0 = src[0], a1 = src[1];
    float a[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    float rs[8];
    if (ep.residual) ld8_h16(ep.residual + e, rs, EPC);
    uint16_t yb[8];
    float y2v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float t = a[k] + ec[k].bias + (ep.residual ? rs[k] : 0.f);
      if (ep.relu) t = fmaxf(t, 0.f);
      t = epi_rmask(ep, e + k, epi_dropout(ep, e + k, t));
      yb[k] = f32_to_h16c(EPC, t);
      const float ys = h16_to_f32c(EPC, yb[k]);
      float qv = ys * ec[k].s + ec[k].t;
      if (ep.act_relu) qv = fmaxf(qv, 0.f);
      y2v[k] = qv;
      const float d = ys - sh[k];
      s1[k] += d;
      s2[k] += d * d;
    }
    *reinterpret_cast<uint4*>(y + e) =
        make_uint4((uint32_t)yb[0] | ((uint32_t)yb[1] << 16), (uint32_t)yb[2] | ((uint32_t)yb[3] << 16),
                   (uint32_t)yb[4] | ((uint32_t)yb[5] << 16), (uint32_t)yb[6] | ((uint32_t)yb[7] << 16));
    if (ep.y2) st8_h16(ep.y2 + e, y2v, EPC);
  }
  if (ep.st_part) epi_bn_stats<BM, BN, NT>(s1, s2, T, tid, m0, n0, M, Cout, ep);
}

template <int TM, int TN, int WGM, int WGN, int SFIX, bool ONE, bool F16 = false>
__global__ void __launch_bounds__(64 * WGM * WGN)
conv_ring_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, uint16_t* __restrict__ y, int NB,
                 int H, int W, int Cin, int Ho, int Wo, int Cout, int KH, int KW, int stride, int pad,
                 const ConvEpi ep, int tiles_n, int nwg, int ntiles, int splits, float* __restrict__ slab) {
  using C = RingCfg<TM, TN, WGM, WGN, SFIX>;
  constexpr int BM = C::BM, BN = C::BN, S = C::S, NT = C::NT, NW = C::NW;
  static_assert((C::BM * (C::BN + 4) + 5 * C::BN) * 4 <= S * (C::BM + C::BN) * BK * 2,
                "epilogue tile + column table must fit the ring");
  __shared__ __attribute__((aligned(16))) uint16_t lds[S * (BM + BN) * BK];
  uint16_t* As = lds;
  uint16_t* Bs = lds + S * BM * BK;

  const int bid = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int split = wgid / ntiles, tile = wgid % ntiles;
  const int tm_idx = tile / tiles_n, tn_idx = tile % tiles_n;
  const int m0 = tm_idx * BM, n0 = tn_idx * BN;
  const int M = NB * Ho * Wo;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WGN, wn = wid % WGN;
  const int K = KH * KW * Cin;

  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, (int)((int64_t)NB * H * W * Cin * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)w, (short)0, (int)((int64_t)Cout * K * 2), 0x00020000);

  // this wave's DMA pieces: d = wid + j * NW (d < RA: A rows 8d.., else B rows 8(d-RA)..)
  const int nmine = C::QL + (wid < C::RL ? 1 : 0);
  const int slot = lane & 7;
  uint32_t off[C::QMAX];
  uint64_t amask[C::QMAX];
#pragma unroll
  for (int j = 0; j < C::QMAX; ++j) {
    const int d = wid + j * NW;
    off[j] = kBufOOB;
    amask[j] = 0;
    if (j >= nmine) continue;
    if (d < C::RA) {
      const int row = 8 * d + (lane >> 3);
      const int lc = slot ^ ((row >> 1) & 7);
      const int m = m0 + row;
      if (m < M) {
        const int img = m / (Ho * Wo), rem = m % (Ho * Wo);
        const int hi0 = (rem / Wo) * stride - pad, wi0 = (rem % Wo) * stride - (ep.pad_w >= 0 ? ep.pad_w : pad);
        off[j] = (uint32_t)(((((int64_t)img * H + hi0) * W + wi0) * Cin + lc * 8) * 2);
        if (!ONE) {
          for (int fr = 0; fr < KH; ++fr)
            for (int fc = 0; fc < KW; ++fc)
              if ((unsigned)(hi0 + fr) < (unsigned)H && (unsigned)(wi0 + fc) < (unsigned)W)
                amask[j] |= 1ull << (fr * KW + fc);
        }
      }
    } else {
      const int row = 8 * (d - C::RA) + (lane >> 3);
      const int co = n0 + row;
      if (co < Cout) off[j] = (uint32_t)(((int64_t)co * K + (slot ^ ((row >> 1) & 7)) * 8) * 2);
    }
  }
  const int cin_steps = Cin / BK;
  const int nk_all = KH * KW * cin_steps;
  const int per = (nk_all + splits - 1) / splits;
  const int k_begin = split * per;
  const int k_end = min(nk_all, k_begin + per);
  const int nk = max(0, k_end - k_begin);

  int c_tap = k_begin / cin_steps, c_ci = (k_begin % cin_steps) * BK;
  int c_fr = c_tap / KW, c_fc = c_tap % KW;
  auto issue = [&](int buf) {
    const uint32_t tap_a = (uint32_t)((c_fr * W + c_fc) * Cin * 2);
    const uint32_t soff_a = (uint32_t)(c_ci * 2);
    const uint32_t soff_b = (uint32_t)((c_tap * Cin + c_ci) * 2);
#pragma unroll
    for (int j = 0; j < C::QMAX; ++j) {
      if (j >= nmine) break;
      const int d = wid + j * NW;
      if (d < C::RA) {
        uint32_t vo;
        if (ONE) vo = off[j];
        else vo = ((amask[j] >> c_tap) & 1ull) ? off[j] + tap_a : kBufOOB;
        buf_lds16(xr, As + (buf * BM + 8 * d) * BK, vo, soff_a);
      } else {
        buf_lds16(wr, Bs + (buf * BN + 8 * (d - C::RA)) * BK, off[j], soff_b);
      }
    }
    c_ci += BK;
    if (c_ci == Cin) {
      c_ci = 0;
      ++c_tap;
      if (++c_fc == KW) {
        c_fc = 0;
        ++c_fr;
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) issue(s);
  for (int ks = 0; ks < nk; ++ks) {
    const int ahead = min(S - 2, nk - 1 - ks);
    if (C::RL == 0 || wid < C::RL) wait_ring<C::QMAX>(ahead);
    else wait_ring<C::QL>(ahead);
    __builtin_amdgcn_s_barrier();
    if (ks + S - 1 < nk) issue((ks + S - 1) % S);
    const int buf = ks % S;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      typename Mfma16<F16>::T af[TM], bfr[TN];
      const int chunk = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * 16 * TM + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const typename Mfma16<F16>::T*>(As + (buf * BM + row) * BK + swz(row, chunk) * 8);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * 16 * TN + j * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const typename Mfma16<F16>::T*>(Bs + (buf * BN + row) * BK + swz(row, chunk) * 8);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = Mfma16<F16>::mma(af[i], bfr[j], acc[i][j]);
    }
  }
  if (Cout % 8 == 0)
    ring_epilogue<BM, BN, TM, TN, NT>(acc, reinterpret_cast<float*>(lds), m0, n0, wm, wn, lane, tid, M, Cout, ep, y,
                                      split, splits, slab, Ho, Wo);
  else
    igemm_epilogue<TM, TN, 16 * TM, 16 * TN>(acc, m0, n0, wm, wn, lane, M, Cout, ep, y, split, splits, slab, Ho, Wo);
}

// ring configurations (tile codes 100 + index)
struct RingShape {
  int bm, bn, nt, stage_bytes, s;
};
template <int TM, int TN, int WGM, int WGN, int SFIX>
constexpr RingShape ring_shape() {
  using C = RingCfg<TM, TN, WGM, WGN, SFIX>;
  return RingShape{C::BM, C::BN, C::NT, C::STAGE_BYTES, C::S};
}
#define MXR_RING_CONFIGS(X)   \
  X(0, 2, 2, 2, 2, 3)   /* 64x64, 4 waves, S3 */ \
  X(1, 2, 1, 2, 4, 3)   /* 64x64, 8 waves, S3 */ \
  X(2, 2, 1, 2, 4, 4)   /* 64x64, 8 waves, S4 */ \
  X(3, 1, 1, 4, 4, 3)   /* 64x64, 16 waves, S3 */ \
  X(4, 1, 2, 2, 2, 3)   /* 32x64, 4 waves, S3 */ \
  X(5, 2, 2, 4, 2, 3)   /* 128x64, 8 waves, S3 */ \
  X(6, 2, 2, 4, 4, 3)   /* 128x128, 16 waves, S3 */ \
  X(7, 4, 4, 2, 2, 3)   /* 128x128, 4 waves, S3 */ \
  X(8, 2, 4, 4, 2, 3)   /* 128x128, 8 waves, S3 */ \
  X(9, 2, 2, 2, 4, 3)   /* 64x128, 8 waves, S3 */ \
  X(10, 1, 2, 4, 2, 3)  /* 64x64, 8 waves (4x2), S3 */ \
  X(11, 2, 2, 2, 2, 2)  /* 64x64, 4 waves, S2 */
static const RingShape kRingShapes[] = {
#define MXR_X(i, a, b, c, d, e) ring_shape<a, b, c, d, e>(),
    MXR_RING_CONFIGS(MXR_X)
#undef MXR_X
};
constexpr int kNumRing = sizeof(kRingShapes) / sizeof(kRingShapes[0]);

template <int TM, int TN, int WGM, int WGN, int SFIX>
static void launch_ring(const uint16_t* x, const uint16_t* w, uint16_t* y, int NB, int H, int W, int Cin, int Ho,
                        int Wo, int Cout, int KH, int KW, int stride, int pad, const ConvEpi& ep, int splits,
                        float* slab, hipStream_t st) {
  using C = RingCfg<TM, TN, WGM, WGN, SFIX>;
  const int M = NB * Ho * Wo;
  const int tiles_m = (M + C::BM - 1) / C::BM, tiles_n = (Cout + C::BN - 1) / C::BN;
  const int ntiles = tiles_m * tiles_n;
  const int nwg = ntiles * splits;
  const bool one = KH == 1 && KW == 1 && pad == 0 && ep.pad_w <= 0;
#define MXR_RING_LAUNCH(ONE_, F16_)                                                                              \
  conv_ring_kernel<TM, TN, WGM, WGN, SFIX, ONE_, F16_><<<nwg, C::NT, 0, st>>>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, \
                                                                             KH, KW, stride, pad, ep, tiles_n, nwg,  \
                                                                             ntiles, splits, slab)
  if (ep.f16) {
    if (one) MXR_RING_LAUNCH(true, true);
    else MXR_RING_LAUNCH(false, true);
  } else {
    if (one) MXR_RING_LAUNCH(true, false);
    else MXR_RING_LAUNCH(false, false);
  }
#undef MXR_RING_LAUNCH
  if (splits > 1) {
    const int64_t MN = (int64_t)M * Cout;
    if (ep.bnb_x)
      splitk_reduce_bnb_kernel<<<dim3(div_up(Cout, 64), div_up(M, 64)), 256, 0, st>>>(slab, splits, M, Cout, ep, y);
    else
      splitk_reduce_kernel<<<div_up((MN + 3) / 4, 256), 256, 0, st>>>(slab, splits, MN, Cout, ep, y);
  }
}

static void launch_ring_code(int idx, const uint16_t* x, const uint16_t* w, uint16_t* y, int NB, int H, int W,
                             int Cin, int Ho, int Wo, int Cout, int KH, int KW, int stride, int pad, const ConvEpi& ep,
                             int splits, float* slab, hipStream_t st) {
  switch (idx) {
#define MXR_X(i, a, b, c, d, e) \
  case i: launch_ring<a, b, c, d, e>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
    MXR_RING_CONFIGS(MXR_X)
#undef MXR_X
    default: break;
  }
}

// Ring plan: the configuration with the least modelled time.  Model: a CU streams its tiles'
// operand bytes at a per-CU rate (LDS-DMA, ~70 GB/s) while the MFMA work proceeds at its own
// rate; the grid takes ceil(tiles / 256) rounds of the slower of the two, plus a per-tile
// prologue/epilogue latency; output columns wider than the tile cost A re-reads (already in bytes).
static int ring_plan(int64_t M, int Cout, int nk, int* splits_out) {
  int best = 0;
  double best_t = 1e30;
  for (int i = 0; i < kNumRing; ++i) {
    const RingShape& r = kRingShapes[i];
    const int64_t tiles = ((M + r.bm - 1) / r.bm) * ((Cout + r.bn - 1) / r.bn);
    const int64_t rounds = (tiles + 255) / 256;
    const double bytes = (double)(r.bm + r.bn) * 128.0 * nk;            // per tile
    const double flops = 2.0 * r.bm * r.bn * 64.0 * nk;                  // per tile
    const double t_mem = bytes / 70e3;                                   // us at 70 GB/s per CU
    const double t_mma = flops / (4.0 * 1024 * 2.1e3);                   // us at 4 SIMDs x 1024 FLOP/clk, 2.1 GHz
    const double t = rounds * ((t_mem > t_mma ? t_mem : t_mma) + 1.0);
    if (t < best_t * 0.999) {
      best_t = t;
      best = i;
    }
  }
  *splits_out = 1;
  return 100 + best;
}

template <int BM, int BN, int S = 0, bool BUF = false>
static void launch_fwd(const uint16_t* x, const uint16_t* w, uint16_t* y, int NB, int H, int W, int Cin, int Ho,
                       int Wo, int Cout, int KH, int KW, int stride, int pad, const ConvEpi& ep, int splits,
                       float* slab, hipStream_t st) {
  const int M = NB * Ho * Wo;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (Cout + BN - 1) / BN;
  const int ntiles = tiles_m * tiles_n;
  const int nwg = ntiles * splits;
  if constexpr (BUF) {
    if (ep.f16)
      conv_igemm_buf_kernel<BM, BN, S, true><<<nwg, 256, 0, st>>>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride,
                                                                 pad, ep, tiles_n, nwg, ntiles, splits, slab);
    else if (ep.x2 && !ep.bt && ((S == 3 && BN == 128) || S == 4)) {
      if constexpr ((S == 3 && BN == 128 && BM == 128) || (S == 4 && BN == 64 && (BM == 64 || BM == 128)))
        conv_igemm_buf_kernel<BM, BN, S, false, true, false><<<nwg, 256, 0, st>>>(
            x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, tiles_n, nwg, ntiles, splits, slab);
    } else if (ep.x2 || ep.bt) {
      if constexpr ((S == 3 && BN == 64 && (BM == 64 || BM == 128)) || (S == 2 && BN == 64 && BM == 64)) {
#define MXR_BUF_LAUNCH(X, B, X3_)                                                                                  \
  conv_igemm_buf_kernel<BM, BN, S, false, X, B, X3_><<<nwg, 256, 0, st>>>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, \
                                                                          KW, stride, pad, ep, tiles_n, nwg, ntiles,  \
                                                                          splits, slab)
        if (ep.x3 && ep.bt) MXR_BUF_LAUNCH(true, true, true);  // fp32 triples: the fused one-pass form
        else if (ep.x3) MXR_BUF_LAUNCH(true, false, true);
        else if (ep.x2 && ep.bt) MXR_BUF_LAUNCH(true, true, false);
        else if (ep.x2) MXR_BUF_LAUNCH(true, false, false);
        else MXR_BUF_LAUNCH(false, true, false);
#undef MXR_BUF_LAUNCH
      }
    } else
      conv_igemm_buf_kernel<BM, BN, S, false><<<nwg, 256, 0, st>>>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride,
                                                                  pad, ep, tiles_n, nwg, ntiles, splits, slab);
  }
  else if constexpr (S > 0)
    conv_igemm_glds_kernel<BM, BN, S><<<nwg, 256, 0, st>>>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad,
                                                          ep, tiles_n, nwg, ntiles, splits, slab);
  else
    conv_igemm_fwd_kernel<BM, BN><<<nwg, 256, 0, st>>>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep,
                                                       tiles_n, nwg, ntiles, splits, slab);
  if (splits > 1) {
    const int64_t MN = (int64_t)M * Cout;
    if (ep.bnb_x)
      splitk_reduce_bnb_kernel<<<dim3(div_up(Cout, 64), div_up(M, 64)), 256, 0, st>>>(slab, splits, M, Cout, ep, y);
    else
      splitk_reduce_kernel<<<div_up((MN + 3) / 4, 256), 256, 0, st>>>(slab, splits, MN, Cout, ep, y);
  }
}

float philox_uniform_host(uint32_t seed, uint64_t step, uint64_t e) { return philox_uniform(seed, step, e); }

int conv_tile_bm(int tile) {
  if (tile == 200 || tile == 201 || tile == 207) return 256;
  if (tile == 202 || tile == 203 || tile == 205 || tile == 206) return 128;
  if (tile == 204) return 160;
  if (tile >= 100 && tile < 100 + kNumRing) return kRingShapes[tile - 100].bm;
  switch (tile) {
    case 1: case 2: case 11: case 12: case 14: case 15: case 21: case 22: case 31: case 32: return 128;
    case 24: return 32;
    default: return 64;
  }
}

int conv_igemm_plan(int NB, int Ho, int Wo, int Cin, int Cout, int KH, int KW, int tile, int* splits_out) {
  const int64_t M = (int64_t)NB * Ho * Wo;
  const int nk = KH * KW * (Cin / BK);
  static const bool ring = [] {
    const char* e = getenv("MXR_CONV_RING");
    return e != nullptr && e[0] == '1';
  }();
  if (tile <= 0 && ring && Cin % BK == 0 && KH * KW <= 64) return ring_plan(M, Cout, nk, splits_out);
  if (tile <= 0) {
    // buffer-resource LDS-DMA kernel, 3-deep (tools/microbench/conv_tiles.py sweep on the
    // ResNet-101 C4 shapes): 64x64 everywhere except many-block, long-K shapes (the 128-RoI
    // stage-4 convs), where 128x64 halves the operand bytes per FLOP -- but not on wide outputs
    // (the RPN 3x3's dgrad, Cout 1024: 64x64 71 us vs 128x64 89 us); split-K only for grids
    // too small to cover the CUs
    const int64_t b64 = ((M + 63) / 64) * ((Cout + 63) / 64);
    static const bool wide22 = getenv("MXR_PLAN_WIDE22") != nullptr;  // A/B switch for the rule below
    const int t = (b64 >= 600 && nk >= 16 && (Cout <= 512 || wide22)) ? 22 : 23;
    const int64_t blocks = t == 22 ? ((M + 127) / 128) * ((Cout + 63) / 64) : b64;
    int splits = 1;
    while (splits < 4 && blocks * splits < 128 && nk / (splits * 2) >= 8 && Cout % 4 == 0) splits *= 2;
    *splits_out = splits;
    return t;
  }
  // explicit tile (A/B runs): tile codes -> (BM, BN); split K until ~4 blocks per CU
  const int code = tile % 10;
  const int bm = code == 3 || code == 5 || code == 6 ? 64 : code == 4 ? 32 : 128,
            bn = code == 1 ? 128 : code == 5 ? 32 : 64;
  const int64_t blocks = ((M + bm - 1) / bm) * ((Cout + bn - 1) / bn);
  int splits = 1;
  while (splits < 8 && blocks * splits * 2 <= 1024 && nk / (splits * 2) >= 6 && Cout % 4 == 0) splits *= 2;
  *splits_out = splits;
  return tile;
}

int conv_igemm_fwd(const uint16_t* x, const uint16_t* w, uint16_t* y, int NB, int H, int W, int Cin, int Ho, int Wo,
                   int Cout, int KH, int KW, int stride, int pad, const ConvEpi& ep, int tile, int splits, float* slab,
                   hipStream_t st) {
  if (tile >= 200 && tile <= 207)  // large-tile kernel (conv_big.hip): whole K per workgroup
    return splits > 1 ? -1 : conv_big_fwd(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, tile, st);
  if (Cin % BK != 0) return -1;
  if (splits > 1 && (slab == nullptr || Cout % 4 != 0)) return -1;
  if ((ep.y2 || ep.bnb_x) && (!ep.bn_beta || !ep.bn_mean || !ep.bn_var || (!ep.bn_fix_gamma && !ep.bn_gamma)))
    return -1;
  if (ep.y2 && ep.bnb_x) return -1;
  if (ep.rmask && (ep.bnb_x || ep.y2 || ep.f16)) return -1;
  const bool kgt = tile >= 27 && tile <= 29;  // K-group tiles (conv_kg.hip)
  if ((ep.omap || ep.pad_w >= 0) && (splits > 1 || !(tile == 22 || tile == 23 || tile == 30 || tile >= 100 || kgt))) return -1;
  if (ep.f16 && !(tile == 21 || tile == 22 || tile == 23 || tile == 30 || tile >= 100)) return -1;
  // BN statistics: LDS-epilogue kernels (buffer / ring), whole K per workgroup
  if (ep.st_part && (splits > 1 || Cout % 8 != 0 || !(tile == 21 || tile == 22 || tile == 23 || tile == 30 || tile >= 100 || kgt)))
    return -1;
  // buffer variants: 32-bit byte offsets below the kBufOOB sentinel, tap mask of 64 bits
  if (tile >= 100 && ((int64_t)NB * H * W * Cin * 2 >= (int64_t)kBufOOB ||
                      (int64_t)Cout * KH * KW * Cin * 2 >= (int64_t)kBufOOB || KH * KW > 64))
    tile = 23;
  if (tile >= 21 && ((int64_t)NB * H * W * Cin * 2 >= (int64_t)kBufOOB ||
                     (int64_t)Cout * KH * KW * Cin * 2 >= (int64_t)kBufOOB || KH * KW > 64))
    tile = 3;
  if ((ep.st_part || ep.bnb_part) && tile < 21) return -1;  // needs the buffer / ring epilogue
  if (ep.bnb_part && (splits > 1 || Cout % 8 != 0)) return -1;
  if (ep.bt && (ep.f16 || Cout % 8 != 0)) return -1;
  if (tile == 26) {  // fp32-class pairs, wide stages: x2 forward only, whole K per workgroup
    if (!ep.x2 || ep.x3 || ep.bt || ep.f16 || splits > 1 || ep.omap || ep.pad_w >= 0 || Cin % 64 != 0 || KH * KW > 64 ||
        (int64_t)NB * H * W * Cin * 2 + ep.x2_pa >= (int64_t)kBufOOB ||
        (int64_t)Cout * KH * KW * Cin * 2 + ep.x2_pb >= (int64_t)kBufOOB)
      return -1;
    const int M = NB * Ho * Wo;
    const int tiles_n = (Cout + 63) / 64, ntiles = ((M + 63) / 64) * tiles_n;
    conv_x2w_kernel<64, 64><<<ntiles, 256, 0, st>>>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep,
                                                    tiles_n, ntiles, ntiles);
    return tile;
  }
  if (ep.x2 || ep.yf || ep.bt) {
    // pairs / fp32 outputs / filter read transposed: the buffer kernels (x2 also at depth 4 and
    // 128x128, A/B tiles 21 / 32 / 33)
    const bool x2_ok = !ep.bt && !ep.x3 && (tile == 21 || tile == 32 || tile == 33);
    // x3: the fused 22 / 23, or the K-group forms 27 / 28 (tile 29's four 144 KB-class rings do not fit)
    if (!(tile == 22 || tile == 23 || tile == 30 || x2_ok || (kgt && !(ep.x3 && tile == 29)))) tile = 23;
    if ((int64_t)NB * H * W * Cin * 2 >= (int64_t)kBufOOB || (int64_t)Cout * KH * KW * Cin * 2 >= (int64_t)kBufOOB ||
        KH * KW > 64 || ep.f16)
      return -1;
    if (ep.x2 && ((int64_t)NB * H * W * Cin * 2 + (ep.x3 ? 2 : 1) * (int64_t)ep.x2_pa >= (int64_t)kBufOOB ||
                  (int64_t)Cout * KH * KW * Cin * 2 + (ep.x3 ? 2 : 1) * (int64_t)ep.x2_pb >= (int64_t)kBufOOB))
      return -1;
    if (ep.yf && (ep.y2 || ep.bnb_x || ep.st_part)) return -1;
  }
  if (tile >= 27 && tile <= 29) return conv_igemm_kg(tile, x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st);
  if (tile >= 100 && tile < 100 + kNumRing) {
    launch_ring_code(tile - 100, x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st);
    return tile;
  }
  switch (tile) {
    case 1: launch_fwd<128, 128>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
    case 2: launch_fwd<128, 64>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
    // LDS-DMA pipelined variants (tile code 10 + x: x = 1 128x128, 2 128x64, 3 64x64, 4/5/6 the same at depth 3)
    case 11: launch_fwd<128, 128, 4>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
    case 12: launch_fwd<128, 64, 4>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
    case 13: launch_fwd<64, 64, 4>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
    case 14: launch_fwd<128, 128, 3>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
    case 15: launch_fwd<128, 64, 3>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
    case 16: launch_fwd<64, 64, 3>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
    // buffer-resource LDS-DMA variants: 2x = depth 3, 3x = depth 4 (x as above).  Depth 6 / 8 were
    // 1.5-2x slower on every ResNet shape (tools/microbench/conv_tiles.py): 3 is the sweet spot
    case 21: launch_fwd<128, 128, 3, true>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
    case 22: launch_fwd<128, 64, 3, true>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
    case 23: launch_fwd<64, 64, 3, true>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
    // tile 23 at ring depth 2: the fp32 triples' 72 KB ring becomes 48 KB, three workgroups per CU
    // instead of two (the batch-1 stage-3 grids are 264 tiles on 256 CUs)
    case 30: launch_fwd<64, 64, 2, true>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
    case 31: launch_fwd<128, 128, 4, true>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
    case 32: launch_fwd<128, 64, 4, true>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
    case 33: launch_fwd<64, 64, 4, true>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
    // small tiles (2-4 workgroups per CU on the ~4K-row stage-3 GEMMs: more waves to hide latency)
    case 24: launch_fwd<32, 64, 3, true>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
    case 25: launch_fwd<64, 32, 3, true>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
    default: launch_fwd<64, 64>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
  }
  return tile;
}

// ---- dgrad filter cache: flip + transpose every registered filter in one launch -------------
// One 256-thread block per (entry, tap, 64-o x 64-i tile).  The tile goes through LDS so both
// the read (rows of i) and the write (rows of o) are 16-B vectorised and coalesced.
__global__ void __launch_bounds__(256)
conv_wt_flip_kernel(const WtFlipEntry* __restrict__ entries, int n_entries) {
  __shared__ uint16_t t[64][64 + 8];
  const int b = blockIdx.x;
  int lo = 0, hi = n_entries - 1;  // last entry with tile_begin <= b
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (entries[mid].tile_begin <= b) lo = mid; else hi = mid - 1;
  }
  const WtFlipEntry e = entries[lo];
  const int local = b - e.tile_begin;
  const int to = (e.O + 63) / 64, ti = (e.I + 63) / 64;
  const int tap = local / (to * ti), rem = local % (to * ti);
  const int o0 = (rem / ti) * 64, i0 = (rem % ti) * 64;
  const int taps = e.KH * e.KW;
  const int ftap = taps - 1 - tap;  // (KH-1-r, KW-1-s) flattened
  const int tid = threadIdx.x;
  // read: src[o][tap][i], 64 rows of o x 8 chunks of 8 i
  for (int q = tid; q < 512; q += 256) {
    const int row = q >> 3, ch = q & 7;
    const int o = o0 + row, i = i0 + ch * 8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (o < e.O && i < e.I) v = *reinterpret_cast<const uint4*>(e.src + ((int64_t)o * taps + ftap) * e.I + i);
    const uint16_t* pv = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
    for (int k = 0; k < 8; ++k) t[ch * 8 + k][row] = pv[k];
  }
  __syncthreads();
  // write: dst[i][tap][o], 64 rows of i x 8 chunks of 8 o (and the tap's parity sub-filter)
  const int tr = tap / e.KW, tc = tap % e.KW;
  uint16_t* sd = nullptr;
  int sub_taps = 0, sub_tap = 0;
  if (tr < 8 && tc < 8) {
    sd = e.sub[2 * e.rcls[tr] + e.ccls[tc]];
    sub_taps = e.rcnt[e.rcls[tr]] * e.ccnt[e.ccls[tc]];
    sub_tap = e.ridx[tr] * e.ccnt[e.ccls[tc]] + e.cidx[tc];
  }
  for (int q = tid; q < 512; q += 256) {
    const int row = q >> 3, ch = q & 7;
    const int i = i0 + row, o = o0 + ch * 8;
    if (i < e.I && o < e.O) {
      const uint4 v = *reinterpret_cast<const uint4*>(&t[row][ch * 8]);
      *reinterpret_cast<uint4*>(e.dst + ((int64_t)i * taps + tap) * e.O + o) = v;
      if (sd) *reinterpret_cast<uint4*>(sd + ((int64_t)i * sub_taps + sub_tap) * e.O + o) = v;
    }
  }
}

void conv_wt_flip_multi(const WtFlipEntry* entries, int n_entries, int total_tiles, hipStream_t st) {
  if (n_entries <= 0 || total_tiles <= 0) return;
  conv_wt_flip_kernel<<<total_tiles, 256, 0, st>>>(entries, n_entries);
}

// ---- grouped data + weight gradient launch -----------------------------------------------------
// The backward of a stride-1 conv inside a fused residual unit as ONE launch: workgroups
// [0, nwg_d) run the data gradient (the 64x64 buffer kernel above over dY with the flipped filter,
// any ConvEpi epilogue -- the BN-ReLU backward of the fused units), workgroups [nwg_d, ...) the
// weight gradient (conv_wgrad.hip's LDS-DMA body, split over pixels into fp32 slabs).  Both roles
// read the same dY and use one 48 KB LDS ring, so a CU holds up to three blocks of either role.
// Replaces the two-stream schedule (wgrad on a side stream, one cross-queue wait per wgrad and a
// join per unit): every cross-queue edge of a replayed graph cost ~10 us of idle time, four per
// unit (profiles/r2_resnet101_stage3_unit_timeline.txt).
//
// KG > 1: both roles in their K-group form (4*KG waves per workgroup, each group of four over a
// contiguous slice of the role's reduction through its own sub-ring, partial tiles summed in the
// LDS epilogue; the reduce role covers 4 * 256 * KG elements per workgroup).
template <int S, bool X2 = false, bool BT = false, int KG = 1, bool X3 = false>
__global__ void __launch_bounds__(256 * KG)
conv_dgrad_wgrad_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, uint16_t* __restrict__ y,
                        int NB, int H, int W, int Cin, int Ho, int Wo, int Cout, int KH, int KW, int pad,
                        const ConvEpi ep, int tiles_n, int nwg_d, int ntiles, WgradParams wp, WgradReduceParams rp) {
  // both roles run an S-deep ring over the same LDS: S * (64 + 64) * 64 bf16 (48 KB at S = 3) per
  // group, plus the lo tiles of the fused fp32 form (72 KB at S = 3)
  static_assert(igemm_ring_stage<64, 64, BT, X3>() == wgrad_ring_stage<X3>(), "both roles use the same ring");
  __shared__ __attribute__((aligned(16))) uint16_t lds[S * KG * igemm_ring_stage<64, 64, BT, X3>()];
  // roles: [0, rp.nwg) the previous grouped launch's deferred split-K reduce (short, dispatched
  // first; rp.nwg is a multiple of 8 so the dgrad role keeps its XCD-aware tile order), then the
  // data gradient, then the weight gradient
  const int b = (int)blockIdx.x;
  if (b < rp.nwg) {
    wgrad_reduce_body(b, rp.slab, rp.splits, rp.n, rp.dw, rp.accumulate, rp.dwf, 256 * KG);
  } else if (b < rp.nwg + nwg_d) {
    igemm_buf_body<64, 64, S, false, X2, BT, KG, X3>(lds, b - rp.nwg, x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, 1,
                                                     pad, ep, tiles_n, nwg_d, ntiles, 1, nullptr);
  } else {
    wgrad_buf_body<S, X2, KG, X3>(lds, b - rp.nwg - nwg_d, wp);
  }
}

int conv_dgrad_wgrad(const uint16_t* x, const uint16_t* w, uint16_t* y, int NB, int H, int W, int Cin, int Ho, int Wo,
                     int Cout, int KH, int KW, int pad, const ConvEpi& ep, const uint16_t* wg_dy,
                     const uint16_t* wg_x, uint16_t* dw, float* slab, int wg_NB, int wg_H, int wg_W, int wg_Cin,
                     int wg_Ho, int wg_Wo, int wg_Cout, int wg_KH, int wg_KW, int wg_stride, int wg_pad, int wg_splits,
                     int accumulate, hipStream_t st, int defer_reduce, const float* prev_slab, int prev_splits,
                     int64_t prev_n, uint16_t* prev_dw, const WgradX2& wx2, float* prev_dwf) {
  if (Cin % BK != 0 || Cout % 8 != 0 || ep.f16 || ep.omap || ep.pad_w >= 0) return -1;
  if ((int64_t)NB * H * W * Cin * 2 >= (int64_t)kBufOOB || (int64_t)Cout * KH * KW * Cin * 2 >= (int64_t)kBufOOB)
    return -1;
  if (wg_Cin % WG_BN != 0 || wg_Cout % 8 != 0 || wg_splits < 1) return -1;
  if ((int64_t)wg_NB * wg_Ho * wg_Wo * wg_Cout * 2 >= (int64_t)kWgOOB ||
      (int64_t)wg_NB * wg_H * wg_W * wg_Cin * 2 >= (int64_t)kWgOOB)
    return -1;
  if (prev_slab != nullptr && (prev_splits < 2 || prev_n % 4 != 0 || (prev_dw == nullptr && prev_dwf == nullptr)))
    return -1;
  if (ep.x2 != wx2.x2 || ep.x3 != wx2.x3) return -1;  // both roles read the same dY: one storage format
  const int M = NB * Ho * Wo;
  const int tiles_n = (Cout + 63) / 64;
  const int ntiles = ((M + 63) / 64) * tiles_n;
  WgradParams wp = wgrad_params(wg_dy, wg_x, dw, slab, wg_NB, wg_H, wg_W, wg_Cin, wg_Ho, wg_Wo, wg_Cout, wg_KH,
                                wg_KW, wg_stride, wg_pad, wg_splits, accumulate);
  wp.x2 = wx2.x2;
  wp.x3 = wx2.x3;
  wp.x2_pdy = wx2.pdy;
  wp.x2_px = wx2.px;
  wp.dwf = wx2.dwf;
  WgradReduceParams rp;
  if (prev_slab != nullptr) {
    rp.slab = prev_slab;
    rp.dw = prev_dw;
    rp.dwf = prev_dwf;
    rp.n = prev_n;
    rp.splits = prev_splits;
    rp.accumulate = 1;
  }
  static const int depth = [] {  // A/B knob MXR_GROUPED_S: ring depth of both roles (3: 48 KB, 4: 64 KB)
    const char* e = getenv("MXR_GROUPED_S");
    return e != nullptr && e[0] == '4' ? 4 : 3;
  }();
  // K groups of both roles (data gradients read the forward filter, bt): MXR_GROUPED_KG = 1 | 2 |
  // 22 (two groups at ring depth 2, 64 KB: two workgroups per CU); default 2 in the fp32 (x3) mode,
  // whose reductions run twice as long, else 1
  static const int kg_env = [] {
    const char* e = getenv("MXR_GROUPED_KG");
    return e != nullptr ? atoi(e) : -1;
  }();
  const int kg = !ep.bt || ep.x3 ? 1 : (kg_env >= 0 ? kg_env : 1);  // (measured: no gain at S = 2, -17 % at S = 3)
  const int nt = kg > 1 ? 512 : 256;
  if (prev_slab != nullptr) rp.nwg = (int)((div_up(prev_n / 4, nt) + 7) / 8 * 8);
  const int nwg_all = rp.nwg + ntiles + wp.nwg;
  if (kg == 2 || kg == 22) {
#define MXR_GROUPED_KG(S_, X) \
  conv_dgrad_wgrad_kernel<S_, X, true, 2><<<nwg_all, 512, 0, st>>>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, pad, \
                                                                   ep, tiles_n, ntiles, ntiles, wp, rp)
    if (kg == 22) {
      if (wx2.x2) MXR_GROUPED_KG(2, true);
      else MXR_GROUPED_KG(2, false);
    } else {
      if (wx2.x2) MXR_GROUPED_KG(3, true);
      else MXR_GROUPED_KG(3, false);
    }
#undef MXR_GROUPED_KG
    if (wg_splits > 1 && !defer_reduce)
      wgrad_reduce(slab, wg_splits, (int64_t)wg_Cout * wg_KH * wg_KW * wg_Cin, dw, accumulate, st, wx2.dwf);
    return 0;
  }
#define MXR_GROUPED(S_, X, B, ...) \
  conv_dgrad_wgrad_kernel<S_, X, B, ##__VA_ARGS__><<<nwg_all, 256, 0, st>>>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, pad, ep, \
                                                            tiles_n, ntiles, ntiles, wp, rp)
  // fp32 triples: the fused one-pass form, at ring depth 2 (48 KB of LDS: three workgroups per CU;
  // measured 73.5 vs 69.1 img/s on the fp32 headline against depth 3's 72 KB, two per CU;
  // MXR_GROUPED_X3S=3 restores depth 3)
  static const int x3_depth = [] {
    const char* e = getenv("MXR_GROUPED_X3S");
    return e != nullptr && e[0] == '3' ? 3 : 2;
  }();
  if (wx2.x3 && ep.bt && x3_depth == 2) MXR_GROUPED(2, true, true, 1, true);
  else if (wx2.x3 && ep.bt) MXR_GROUPED(3, true, true, 1, true);
  else if (wx2.x3) MXR_GROUPED(3, true, false, 1, true);
  else if (wx2.x2 && ep.bt) MXR_GROUPED(3, true, true);
  else if (wx2.x2) MXR_GROUPED(3, true, false);
  else if (ep.bt) MXR_GROUPED(3, false, true);
#undef MXR_GROUPED
  else if (depth == 4)
    conv_dgrad_wgrad_kernel<4><<<rp.nwg + ntiles + wp.nwg, 256, 0, st>>>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW,
                                                                         pad, ep, tiles_n, ntiles, ntiles, wp, rp);
  else
    conv_dgrad_wgrad_kernel<3><<<rp.nwg + ntiles + wp.nwg, 256, 0, st>>>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW,
                                                                         pad, ep, tiles_n, ntiles, ntiles, wp, rp);
  if (wg_splits > 1 && !defer_reduce)
    wgrad_reduce(slab, wg_splits, (int64_t)wg_Cout * wg_KH * wg_KW * wg_Cin, dw, accumulate, st, wx2.dwf);
  return 0;
}

}  // namespace mxr
