// Shared device code of the implicit-GEMM convolution kernels (conv_igemm.hip, conv_kg.hip):
// storage helpers, the fused epilogues and the buffer-resource LDS-DMA main loop body.  See
// conv_igemm.hip for the design notes.
#pragma once
#include <cstdlib>

#include "common.h"
#include "../kernels.h"
#include "wgrad_body.h"

// epilogue storage code: fp16 when the conv runs on fp16 activations (inference), else bf16
#define EPC (ep.f16 ? 2 : 1)

namespace mxr {

__device__ __forceinline__ uint16_t f32_to_h16c(int code, float f) { return f32_to_h16(f, code); }
__device__ __forceinline__ float h16_to_f32c(int code, uint16_t v) { return h16_to_f32(v, code); }

// epilogue element access in the launch's storage format: one 16-bit value (bf16 / fp16), or (X2)
// an x2 hi / lo pair `plane` elements apart (ConvEpi::x2).  Stores return the STORED value, which
// the fused consumers (BN of the next unit, statistics) must read, exactly like the unfused pair.
// X2 is a template flag so the bf16 / fp16 epilogues compile exactly as before (unrolled loops).
template <bool X2>
__device__ __forceinline__ float epi_ld1(const ConvEpi& ep, const uint16_t* p, int64_t i, int64_t plane) {
  if constexpr (X2) return ldx(p, i, plane, ep.x3);
  return h16_to_f32c(ep.f16 ? 2 : 1, p[i]);
}
template <bool X2>
__device__ __forceinline__ float epi_st1(const ConvEpi& ep, uint16_t* p, int64_t i, int64_t plane, float v) {
  if constexpr (X2) return stx(p, i, plane, v, ep.x3);
  const uint16_t h = f32_to_h16c(ep.f16 ? 2 : 1, v);
  p[i] = h;
  return h16_to_f32c(ep.f16 ? 2 : 1, h);
}
template <bool X2>
__device__ __forceinline__ void epi_ld8(const ConvEpi& ep, const uint16_t* p, int64_t i, int64_t plane, float* v) {
  if constexpr (X2) ld8x(p + i, plane, v, ep.x3);
  else ld8_h16(p + i, v, ep.f16 ? 2 : 1);
}
// 8 consecutive outputs; `stored` receives the stored values
template <bool X2>
__device__ __forceinline__ void epi_st8(const ConvEpi& ep, uint16_t* p, int64_t i, int64_t plane, const float* v,
                                        float* stored) {
  if constexpr (X2) {
    st8x(p + i, plane, v, stored, ep.x3);
    return;
  }
  const int code = ep.f16 ? 2 : 1;
  uint16_t b[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    b[k] = f32_to_h16c(code, v[k]);
    stored[k] = h16_to_f32c(code, b[k]);
  }
  *reinterpret_cast<uint4*>(p + i) =
      make_uint4((uint32_t)b[0] | ((uint32_t)b[1] << 16), (uint32_t)b[2] | ((uint32_t)b[3] << 16),
                 (uint32_t)b[4] | ((uint32_t)b[5] << 16), (uint32_t)b[6] | ((uint32_t)b[7] << 16));
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

typedef float f32x4 __attribute__((ext_vector_type(4)));

// MFMA 16x16x32 on bf16 or fp16 operands (same rate, same fragment layout)
template <bool F16> struct Mfma16;
template <> struct Mfma16<false> {
  typedef bf16x8 T;
  __device__ static __forceinline__ f32x4 mma(T a, T b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct Mfma16<true> {
  typedef f16x8 T;
  __device__ static __forceinline__ f32x4 mma(T a, T b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};

constexpr int BK = 64;  // bf16 elements per K-step (one 128-B row per tile row)

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// output row of GEMM row m (identity unless the epilogue scatters to a parity class, ConvEpi::omap)
__device__ __forceinline__ int64_t epi_row(const ConvEpi& ep, int m, int Ho, int Wo) {
  if (!ep.omap) return m;
  const int hw = Ho * Wo;
  const int img = m / hw, r = m - img * hw, i = r / Wo, j = r - (r / Wo) * Wo;
  return ((int64_t)img * ep.o_H + i * ep.o_sh + ep.o_ph) * ep.o_W + j * ep.o_sw + ep.o_pw;
}

// dadd element row for output row m of the launch grid (-1: dadd has nothing there)
__device__ __forceinline__ int64_t dadd_row(const ConvEpi& ep, int m, int64_t out_row) {
  if (ep.dadd_s <= 1) return out_row;
  const int s = ep.dadd_s, Ho = ep.dadd_gh, Wo = ep.dadd_gw, hw = Ho * Wo;
  const int img = m / hw, r = m - img * hw, i = r / Wo, j = r - i * Wo;
  if (i % s || j % s) return -1;
  return ((int64_t)img * ((Ho + s - 1) / s) + i / s) * ((Wo + s - 1) / s) + j / s;
}

// per-output-channel epilogue constants
struct EpiCol {
  float bias, s, t, mean, inv;
};

__device__ __forceinline__ EpiCol epi_col(const ConvEpi& ep, int n) {
  EpiCol c;
  c.bias = ep.bias ? ep.bias[n] : (ep.bias_h ? h16_to_f32c(EPC, ep.bias_h[n]) : 0.f);
  c.s = 1.f;
  c.t = 0.f;
  c.mean = 0.f;
  c.inv = 1.f;
  if (ep.y2 || ep.bnb_x) {
    const float g = ep.bn_fix_gamma ? 1.f : ep.bn_gamma[n];
    c.inv = rsqrtf(ep.bn_var[n] + ep.bn_eps);
    c.mean = ep.bn_mean[n];
    c.s = g * c.inv;
    c.t = ep.bn_beta[n] - c.mean * c.s;
  }
  return c;
}

// The workgroup's per-column constants through LDS: column n0 + c is derived ONCE (thread c of the
// workgroup; up to 5 parameter loads and an rsqrt) into a [5][BN] table placed after the staged tile,
// then every thread reads its 8 consecutive columns back as 16-B vectors -- instead of each thread
// issuing 8 x 5 scalar parameter loads before its first store (conv_big.hip: the same change took
// batch-8 test FPS from 749 to 804).  Stage in the same phase as the tile, read after the barrier.
template <int BN, int NT>
__device__ __forceinline__ void epi_cols_stage(float* __restrict__ tab, const ConvEpi& ep, int tid, int n0, int Cout) {
  for (int c = tid; c < BN; c += NT) {
    const EpiCol e = epi_col(ep, n0 + c < Cout ? n0 + c : 0);
    tab[c] = e.bias;
    tab[BN + c] = e.s;
    tab[2 * BN + c] = e.t;
    tab[3 * BN + c] = e.mean;
    tab[4 * BN + c] = e.inv;
  }
}

template <int BN>
__device__ __forceinline__ void epi_cols_load(const float* __restrict__ tab, int cv, EpiCol (&ec)[8]) {
  float v[5][8];
#pragma unroll
  for (int f = 0; f < 5; ++f) {
    const float4 a = *reinterpret_cast<const float4*>(tab + f * BN + cv * 8);
    const float4 b = *reinterpret_cast<const float4*>(tab + f * BN + cv * 8 + 4);
    v[f][0] = a.x; v[f][1] = a.y; v[f][2] = a.z; v[f][3] = a.w;
    v[f][4] = b.x; v[f][5] = b.y; v[f][6] = b.z; v[f][7] = b.w;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) ec[k] = EpiCol{v[0][k], v[1][k], v[2][k], v[3][k], v[4][k]};
}

// fused inverted dropout of output element `idx` (see ConvEpi::drop_p)
__device__ __forceinline__ float epi_dropout(const ConvEpi& ep, int64_t idx, float v) {
  if (ep.drop_p > 0.f) {
    const float u = philox_uniform(ep.drop_seed, (uint64_t)*ep.drop_step, (uint64_t)idx);
    v = u >= ep.drop_p ? v * (1.f / (1.f - ep.drop_p)) : 0.f;
  }
  return v;
}

// ReLU(-and-dropout) backward of the layer whose output is this data gradient's forward input
// (ConvEpi::rmask): keep v where that activation is positive, scaled by rmask_s
__device__ __forceinline__ float epi_rmask(const ConvEpi& ep, int64_t idx, float v) {
  if (ep.rmask) {
    const uint16_t h = ep.rmask[idx];  // bf16 (x2 / x3: the hi plane, which carries the sign)
    v = ((h & 0x8000u) == 0 && (h & 0x7fffu) != 0) ? v * ep.rmask_s : 0.f;
  }
  return v;
}

template <bool X2>
__device__ __forceinline__ void epi_store(const ConvEpi& ep, const EpiCol& c, uint16_t* __restrict__ y, int64_t idx,
                                          float v) {
  v += c.bias;
  if (ep.residual) v += epi_ld1<X2>(ep, ep.residual, idx, ep.x2_py);
  if (ep.relu) v = fmaxf(v, 0.f);
  v = epi_dropout(ep, idx, v);
  v = epi_rmask(ep, idx, v);
  if (X2 && ep.yf) {
    ep.yf[idx] = v;
    return;
  }
  const float ys = epi_st1<X2>(ep, y, idx, ep.x2_py, v);
  if (ep.y2) {
    // the BN reads the STORED (bf16-rounded) conv output, exactly like the unfused pair
    float a = ys * c.s + c.t;
    if (ep.act_relu) a = fmaxf(a, 0.f);
    epi_st1<X2>(ep, ep.y2, idx, ep.x2_py, a);
  }
}

// BN-backward epilogue of one element; returns (g, g * xhat) through sg / sgx
template <bool X2>
__device__ __forceinline__ void epi_bnb(const ConvEpi& ep, const EpiCol& c, uint16_t* __restrict__ y, int64_t idx,
                                        float v, float& sg, float& sgx, int64_t didx) {
  if (ep.dadd && didx >= 0) v += epi_ld1<X2>(ep, ep.dadd, didx, ep.x2_pd);
  const float xv = epi_ld1<X2>(ep, ep.bnb_x, idx, ep.x2_py);
  const float g = (!ep.act_relu || xv * c.s + c.t > 0.f) ? v : 0.f;
  sg += g;
  sgx += g * (xv - c.mean) * c.inv;
  float o = g * c.s;
  if (ep.residual) o += epi_ld1<X2>(ep, ep.residual, idx, ep.x2_py);
  epi_st1<X2>(ep, y, idx, ep.x2_py, o);
}

// Per-column statistics of an LDS-transposed epilogue (thread = 8 consecutive columns cv*8.. of
// some rows): sum over the lanes of each wave sharing the column group (shuffles), then over the
// NW waves through T ([NW][BN][2] floats; the caller has finished reading T), one value per
// column and stat.  With `atomic` the two sums are added to out_a / out_b (fp32 atomics), else
// written to out_a[col] / out_b[col] (a per-row-tile partial row).
template <int BN, int NT>
__device__ __forceinline__ void epi_col_stats(float (&sa)[8], float (&sb)[8], float* __restrict__ T, int tid, int n0,
                                              int Cout, float* out_a, float* out_b, bool atomic, bool skip_b) {
  constexpr int VPR = BN / 8;
  constexpr int NW = NT / 64;
  const int lane = tid & 63, wid = tid >> 6, cv = tid % VPR;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
#pragma unroll
    for (int o = VPR; o < 64; o <<= 1) {
      sa[k] += __shfl_xor(sa[k], o, 64);
      sb[k] += __shfl_xor(sb[k], o, 64);
    }
  }
  __syncthreads();  // T is reused as [NW waves][BN][2] partials
  if (lane < VPR) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      T[(wid * BN + cv * 8 + k) * 2] = sa[k];
      T[(wid * BN + cv * 8 + k) * 2 + 1] = sb[k];
    }
  }
  __syncthreads();
  for (int c = tid; c < BN; c += NT) {
    const int col = n0 + c;
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      a += T[(q * BN + c) * 2];
      b += T[(q * BN + c) * 2 + 1];
    }
    if (col < Cout) {
      if (atomic) {
        if (out_a) atomicAdd(out_a + col, a);
        if (out_b && !skip_b) atomicAdd(out_b + col, b);
      } else {
        out_a[col] = a;
        out_b[col] = b;
      }
    }
  }
}

// BN-backward column sums sum(g) / sum(g * xhat): fp32 atomics into dbeta / dgamma, or (bnb_part,
// deterministic) this row tile's partial row bnb_row0 + m0 / BM of [rows][2][Cout]
template <int BM, int BN, int NT>
__device__ __forceinline__ void epi_bnb_sums(float (&sg)[8], float (&sgx)[8], float* __restrict__ T, int tid, int m0,
                                             int n0, int Cout, const ConvEpi& ep) {
  if (ep.bnb_part) {
    float* row = ep.bnb_part + (int64_t)(ep.bnb_row0 + m0 / BM) * 2 * Cout;
    epi_col_stats<BN, NT>(sg, sgx, T, tid, n0, Cout, row, row + Cout, false, false);
  } else {
    epi_col_stats<BN, NT>(sg, sgx, T, tid, n0, Cout, ep.bnb_dbeta, ep.bnb_dgamma, true, ep.bn_fix_gamma);
  }
}

// training-BN statistics epilogue (ConvEpi::st_part): this row tile's partial row, and the shift row
template <int BM, int BN, int NT>
__device__ __forceinline__ void epi_bn_stats(float (&s1)[8], float (&s2)[8], float* __restrict__ T, int tid, int m0,
                                             int n0, int M, int Cout, const ConvEpi& ep) {
  const int tm = m0 / BM, tiles_m = (M + BM - 1) / BM;
  float* row = ep.st_part + (int64_t)tm * 2 * Cout;
  epi_col_stats<BN, NT>(s1, s2, T, tid, n0, Cout, row, row + Cout, false, false);
  if (tm == 0)
    for (int c = tid; c < BN; c += NT)
      if (n0 + c < Cout) ep.st_part[(int64_t)tiles_m * 2 * Cout + n0 + c] = ep.st_shift[n0 + c];
}

// Shared epilogue of the implicit-GEMM kernels: C/D map col = lane & 15, row = (lane >> 4) * 4 + r.
template <int TM, int TN, int WM, int WN, bool X2 = false>
__device__ __forceinline__ void igemm_epilogue(f32x4 (&acc)[TM][TN], int m0, int n0, int wm, int wn, int lane, int M,
                                               int Cout, const ConvEpi& ep, uint16_t* __restrict__ y, int split,
                                               int splits, float* __restrict__ slab, int Ho = 1, int Wo = 1) {
  if (splits > 1) {  // fp32 partial slab; bias/ReLU/cast happen in the reduce kernel
    float* sp = slab + (int64_t)split * M * Cout;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * WN + j * 16 + (lane & 15);
      if (n >= Cout) continue;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * WM + i * 16 + (lane >> 4) * 4 + r;
          if (m < M) sp[(int64_t)m * Cout + n] = acc[i][j][r];
        }
    }
    return;
  }
  if (ep.bnb_x) {
    // BN-backward epilogue: per-column sums over this wave's rows, reduced across the four
    // 16-lane row groups, then one fp32 atomic per (wave, column, stat)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * WN + j * 16 + (lane & 15);
      float sg = 0.f, sgx = 0.f;
      if (n < Cout) {
        const EpiCol ec = epi_col(ep, n);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = m0 + wm * WM + i * 16 + (lane >> 4) * 4 + r;
            if (m < M) {
              const int64_t orow = epi_row(ep, m, Ho, Wo), drow = dadd_row(ep, m, orow);
              epi_bnb<X2>(ep, ec, y, orow * Cout + n, acc[i][j][r], sg, sgx, drow < 0 ? -1 : drow * Cout + n);
            }
          }
      }
      sg += __shfl_xor(sg, 16, 64);
      sg += __shfl_xor(sg, 32, 64);
      sgx += __shfl_xor(sgx, 16, 64);
      sgx += __shfl_xor(sgx, 32, 64);
      if (lane < 16 && n < Cout) {
        if (ep.bnb_dbeta) atomicAdd(ep.bnb_dbeta + n, sg);
        if (ep.bnb_dgamma && !ep.bn_fix_gamma) atomicAdd(ep.bnb_dgamma + n, sgx);
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * WN + j * 16 + (lane & 15);
    if (n >= Cout) continue;
    const EpiCol ec = epi_col(ep, n);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * WM + i * 16 + (lane >> 4) * 4 + r;
        if (m < M) epi_store<X2>(ep, ec, y, epi_row(ep, m, Ho, Wo) * Cout + n, acc[i][j][r]);
      }
    }
  }
}

// LDS-transposed epilogue (Cout % 8 == 0): the MFMA C/D layout gives each lane 4 rows of ONE
// column, so a direct epilogue issues 2-byte accesses strided by Cout.  Here the fp32 tile is
// scattered into LDS ([BM][BN+4], conflict-free for the 16-lane column runs), and every thread
// then owns 8 consecutive columns of a row: residual / BN-input / dY-add reads, y / y2 stores and
// fp32 split-K slab writes are 16-B vectors, the per-column constants are computed once per
// thread, and the BN-backward column sums reduce across the lanes sharing a column group
// (shuffles), across waves (LDS) and leave the workgroup as one atomic per column and stat.
// KG > 1 (the K-group buffer kernel: KG groups of 4 waves, each accumulating a K slice of the same
// tile): every group stages its partial tile in its own LDS slice and the 256*KG threads read the
// row vectors as the sum of the slices in group order (deterministic), so the cross-group
// reduction costs one extra LDS read per slice and no extra pass.
template <int BM, int BN, int TM, int TN, int WM, int WN, bool X2 = false, int KG = 1>
__device__ __forceinline__ void igemm_epilogue_lds(f32x4 (&acc)[TM][TN], float* __restrict__ T, int m0, int n0, int wm,
                                                   int wn, int lane, int tid, int M, int Cout, const ConvEpi& ep,
                                                   uint16_t* __restrict__ y, int split, int splits,
                                                   float* __restrict__ slab, int Ho = 1, int Wo = 1) {
  constexpr int LDT = BN + 4;      // fp32 row stride of the staged tile
  constexpr int VPR = BN / 8;      // 8-column vectors per row
  constexpr int NT = 256 * KG;     // threads of the workgroup
  constexpr int NV = (BM * VPR + NT - 1) / NT;  // vectors per thread (the last round partial for KG = 4)
  static_assert(BM * VPR % NT == 0 || NT % (BM * VPR) == 0, "vectors per thread");
  __syncthreads();  // every wave is done reading the operand ring
  {
    float* Tq = T + (tid >> 8) * BM * LDT;  // this K group's slice
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Tq[(wm * WM + i * 16 + (lane >> 4) * 4 + r) * LDT + wn * WN + j * 16 + (lane & 15)] = acc[i][j][r];
  }
  // BN epilogues take their column constants from an LDS table; a bias-only epilogue keeps its 8
  // direct loads (cheaper than the table's staging + 10 vector reads: VGG16 fp32 measured -3 %)
  const bool use_tab = ep.y2 || ep.bnb_x;
  float* const tab = T + KG * BM * LDT;  // [5][BN] column constants (callers size the LDS for it)
  if (splits <= 1 && use_tab) epi_cols_stage<BN, NT>(tab, ep, tid, n0, Cout);
  __syncthreads();
  // 8 consecutive accumulators of a staged row: the sum of the K groups' slices
  auto ldrow = [&](int row, int cv8, float* a) {
    const float4* src = reinterpret_cast<const float4*>(T + row * LDT + cv8 * 8);
    float4 a0 = src[0], a1 = src[1];
#pragma unroll
    for (int q = 1; q < KG; ++q) {
      const float4* sq = reinterpret_cast<const float4*>(T + (q * BM + row) * LDT + cv8 * 8);
      const float4 b0 = sq[0], b1 = sq[1];
      a0.x += b0.x; a0.y += b0.y; a0.z += b0.z; a0.w += b0.w;
      a1.x += b1.x; a1.y += b1.y; a1.z += b1.z; a1.w += b1.w;
    }
    a[0] = a0.x; a[1] = a0.y; a[2] = a0.z; a[3] = a0.w; a[4] = a1.x; a[5] = a1.y; a[6] = a1.z; a[7] = a1.w;
  };
  const int cv = tid % VPR;  // this thread's column group (the same for all its vectors)
  const int n = n0 + cv * 8;
  const bool ncol = n < Cout;
  if (splits > 1) {
    float* sp = slab + (int64_t)split * M * Cout;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int row = (tid + v * NT) / VPR, m = m0 + row;
      if (row >= BM || m >= M || !ncol) continue;
      float a[8];
      ldrow(row, cv, a);
      float4* dst = reinterpret_cast<float4*>(sp + (int64_t)m * Cout + n);
      dst[0] = make_float4(a[0], a[1], a[2], a[3]);
      dst[1] = make_float4(a[4], a[5], a[6], a[7]);
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
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int row = (tid + v * NT) / VPR, m = m0 + row;
      if (row >= BM || m >= M || !ncol) continue;
      const int64_t e = epi_row(ep, m, Ho, Wo) * Cout + n;
      float a[8], xv[8], d[8], rs[8];
      ldrow(row, cv, a);
      epi_ld8<X2>(ep, ep.bnb_x, e, ep.x2_py, xv);
      const int64_t drow = ep.dadd ? dadd_row(ep, m, e / Cout) : -1;
      if (drow >= 0) {
        epi_ld8<X2>(ep, ep.dadd, drow * Cout + n, ep.x2_pd, d);
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] += d[k];
      }
      if (ep.residual) epi_ld8<X2>(ep, ep.residual, e, ep.x2_py, rs);
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float g = (!ep.act_relu || xv[k] * ec[k].s + ec[k].t > 0.f) ? a[k] : 0.f;
        sg[k] += g;
        sgx[k] += g * (xv[k] - ec[k].mean) * ec[k].inv;
        o[k] = g * ec[k].s + (ep.residual ? rs[k] : 0.f);
      }
      epi_st8<X2>(ep, y, e, ep.x2_py, o, o);
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
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int row = (tid + v * NT) / VPR, m = m0 + row;
    if (row >= BM || m >= M || !ncol) continue;
    const int64_t e = epi_row(ep, m, Ho, Wo) * Cout + n;
    float a[8];
    ldrow(row, cv, a);
    float rs[8];
    if (ep.residual) epi_ld8<X2>(ep, ep.residual, e, ep.x2_py, rs);
    float t[8], ys[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      t[k] = a[k] + ec[k].bias + (ep.residual ? rs[k] : 0.f);
      if (ep.relu) t[k] = fmaxf(t[k], 0.f);
      t[k] = epi_rmask(ep, e + k, epi_dropout(ep, e + k, t[k]));
    }
    if (X2 && ep.yf) {  // fp32 output (prediction heads of the x2 mode)
      float4* dst = reinterpret_cast<float4*>(ep.yf + e);
      dst[0] = make_float4(t[0], t[1], t[2], t[3]);
      dst[1] = make_float4(t[4], t[5], t[6], t[7]);
      continue;
    }
    epi_st8<X2>(ep, y, e, ep.x2_py, t, ys);  // the BN reads the STORED conv output
    float y2v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float q = ys[k] * ec[k].s + ec[k].t;
      if (ep.act_relu) q = fmaxf(q, 0.f);
      y2v[k] = q;
      const float d = ys[k] - sh[k];
      s1[k] += d;
      s2[k] += d * d;
    }
    if (ep.y2) epi_st8<X2>(ep, ep.y2, e, ep.x2_py, y2v, y2v);
  }
  if (ep.st_part) epi_bn_stats<BM, BN, NT>(s1, s2, T, tid, m0, n0, M, Cout, ep);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until at most `ahead` stages (LPS loads each) are still in flight; ahead <= S - 2 <= 6
template <int LPS>
__device__ __forceinline__ void wait_stages(int ahead) {
  switch (ahead) {
    case 6: wait_vmcnt<6 * LPS>(); break;
    case 5: wait_vmcnt<5 * LPS>(); break;
    case 4: wait_vmcnt<4 * LPS>(); break;
    case 3: wait_vmcnt<3 * LPS>(); break;
    case 2: wait_vmcnt<2 * LPS>(); break;
    case 1: wait_vmcnt<LPS>(); break;
    default: wait_vmcnt<0>(); break;
  }
}

__device__ __forceinline__ void glds16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// ---- buffer-resource LDS-DMA variant: near-zero address arithmetic per K-step ---------------
// PMC on the two kernels above (s3 3x3, 64x64 tile) shows ~100 VALU + ~80 SALU instructions per
// K-step per wave against 8 MFMAs: the im2col address math (integer divisions for the tap,
// 64-bit pixel offsets, four bounds compares per chunk) -- not memory -- paced the loop.  Here
// each thread precomputes, once, a 32-bit byte offset of its A row at tap (0,0) and a bit mask of
// the taps that fall inside the image; the per-K-step part is uniform (SGPR soffset = tap and
// channel-block offset, advanced incrementally) and the per-lane part is one mask test that
// swaps in an out-of-range offset: buffer loads return zeros past num_records, so padding and
// rows >= M / Cout need no zero page and no branch.  Loads go straight to LDS
// (buffer_load_dwordx4 ... lds) S-1 stages ahead, counted vmcnt + raw barrier as above.
constexpr uint32_t kBufOOB = 0x80000000u;

__device__ __forceinline__ void buf_lds16(__amdgpu_buffer_rsrc_t rs, void* lds_wave_base, uint32_t voff,
                                          uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds_wave_base, 16,
                                           (int)voff, (int)soff, 0, 0);
}

// body of the buffer kernel for workgroup `bid` of an `nwg`-workgroup launch; `lds`: S*(BM+BN)*BK
// elements, the block's ONLY LDS (the grouped data + weight gradient launch below shares it with
// the wgrad role)
//
// x2 (fp32-class pairs, X2 = true): a stage holds 32 channels of BOTH planes -- logical 16-B chunks
// 0-3 of a 128-B LDS row are the hi plane's channels c..c+31, chunks 4-7 the lo plane's same
// channels -- so the fragment reads are the bf16 ones (chunk lane>>4 and 4 + lane>>4) and a stage
// runs three MFMAs per fragment pair (A_hi B_hi + A_hi B_lo + A_lo B_hi): 2/3 of the operand
// bytes of three separate K phases for the same MFMA work.  The lo planes sit x2_pa / x2_pb bytes
// further, added to the per-lane offsets of the lo chunks.
//
// BT (data gradient straight from the forward filter, no flipped / transposed copy): B is the
// filter W (Cin_d, taps, Cout_d) itself -- GEMM row k = (tap, channel c) is filter row
// c * taps + (taps - 1 - tap) with its Cout_d outputs contiguous, i.e. B arrives [k][n] instead of
// [n][k].  The stage's B tile is stored k-major (64 rows of 64 outputs, wgrad's chunk swizzle) and
// its fragments are read with ds_read_b64_tr_b16 (rows 8g + 4h + 0..3 of each 32-row half for lane
// group g: the same k order as the A fragments' 16-B chunks).  BN must be 64.
//
// KG > 1 (K groups): 4*KG waves, group q = waves 4q..4q+3 accumulating its contiguous 1/KG of the
// launch's K range for the SAME output tile through its own S-deep LDS sub-ring (the x3 mode with
// KG = 2: one group per phase).  The groups share the workgroup barriers -- one barrier publishes a
// stage of every group -- so each barrier-to-barrier round trip (DMA latency, LDS reads, the serial
// MFMA chain of a small tile: what bounds a batch-1 stage-3 conv at one tile per CU) carries KG
// stages, and 2*KG waves per CU overlap one group's MFMA chain with another's fragment reads.  The
// partial tiles meet in the LDS epilogue (igemm_epilogue_lds, summed in group order).
//
// X3 (the fp32 mode's fused form, X2 = true as well): ONE pass over K with all three planes per
// stage -- the main tiles keep 128-B rows of 32 channels [hi | mid] (chunks 0-3 / 4-7), and a lo
// tile per operand holds the lo plane of the same channels: 64-B rows (swizzle chunk ^ ((row >> 2)
// & 3), conflict-free for 16-row fragment reads) for row-major operands, or for the k-major B of BT
// 32 k-rows laid out like the main tile's first half.  Six MFMAs per fragment set (hh, hm, mh, mm,
// hl, lh): 3/4 of the two-phase form's bytes and half its barriers.
template <int BM, int BN, bool BT, bool X3>
constexpr int igemm_ring_stage() {  // LDS elements of one ring stage
  return (BM + BN) * 64 + (X3 ? BM * 32 + (BT ? 32 * 64 : BN * 32) : 0);
}

template <int BM, int BN, int S, bool F16 = false, bool X2 = false, bool BT = false, int KG = 1, bool X3 = false>
__device__ __forceinline__ void igemm_buf_body(uint16_t* lds, int bid, const uint16_t* __restrict__ x,
                                               const uint16_t* __restrict__ w, uint16_t* __restrict__ y, int NB, int H,
                                               int W, int Cin, int Ho, int Wo, int Cout, int KH, int KW, int stride,
                                               int pad, const ConvEpi& ep, int tiles_n, int nwg, int ntiles, int splits,
                                               float* __restrict__ slab) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int ACH = BM / 32, BCH = BN / 32;
  constexpr int ACL = X3 ? BM / 64 : 0, BCL = X3 ? (BT ? 1 : BN / 64) : 0;  // lo-tile loads per thread
  constexpr int LPS = ACH + BCH + ACL + BCL;
  static_assert(S >= 2 && S <= 8, "pipeline depth");
  static_assert(KG == 1 || (!F16 && BN == 64), "K groups: bf16 / multi-plane 64-column tiles");
  static_assert(!X3 || (X2 && !F16 && BM % 64 == 0 && BN % 64 == 0), "X3: multi-plane 64-multiple tiles");
  constexpr int LBM = X3 ? BM * 32 : 0, LBN = X3 ? (BT ? 32 * 64 : BN * 32) : 0;  // lo tiles per stage
  const int kgi = KG > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 8)) : 0;  // this wave's K group
  uint16_t* As = lds + kgi * S * igemm_ring_stage<BM, BN, BT, X3>();  // the group's sub-ring
  uint16_t* Bs = As + S * BM * BK;
  uint16_t* Al = Bs + S * BN * BK;  // X3 lo tiles
  uint16_t* Bl = Al + S * LBM;

  const int q = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
  const int wgid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + bid / 8;
  const int split = wgid / ntiles, tile = wgid % ntiles;
  const int tm_idx = tile / tiles_n, tn_idx = tile % tiles_n;
  const int m0 = tm_idx * BM, n0 = tn_idx * BN;
  const int M = NB * Ho * Wo;
  const int tid = threadIdx.x, lane = tid & 63, wid = KG > 1 ? __builtin_amdgcn_readfirstlane(tid >> 6) & 3 : tid >> 6;  // wave within the K group
  const int wm = wid >> 1, wn = wid & 1;
  const int K = KH * KW * Cin;

  // the range check covers voffset + soffset: with x2 pairs the records reach through the lo planes
  // (the kBufOOB sentinel of padding taps stays beyond them: operands are < 1 GB per plane)
  // (x3: through the third plane)
  // (readfirstlane: keeps the resources provably uniform -- a VGPR descriptor costs a waterfall
  // loop around every buffer load)
  const int xpl = ep.x2 ? (ep.x3 ? 2 : 1) : 0;
  const int nrec_x = __builtin_amdgcn_readfirstlane((int)((int64_t)NB * H * W * Cin * 2 + (int64_t)xpl * ep.x2_pa));
  const int nrec_w = __builtin_amdgcn_readfirstlane((int)((int64_t)Cout * K * 2 + (int64_t)xpl * ep.x2_pb));
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, nrec_x, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)w, (short)0, nrec_w, 0x00020000);

  const int slot = lane & 7;
  // logical chunk lc of a row: channels lc*8 (16-bit), or (X2) channels (lc&3)*8 of plane lc>>2
  auto chan_bytes = [&](int lc) { return X2 ? (lc & 3) * 16 : lc * 16; };
  // (x2: chunks 4-7 are the lo plane, one plane on; X3: chunks 0-3 the hi plane = memory plane 1,
  // chunks 4-7 the mid plane = memory plane 0)
  auto plane_a = [&](int lc) { return X3 ? (lc < 4 ? ep.x2_pa : 0u) : (X2 && lc >= 4 ? ep.x2_pa : 0u); };
  uint32_t a_off[ACH];
  uint64_t a_mask[ACH];
#pragma unroll
  for (int i = 0; i < ACH; ++i) {
    const int row = 32 * i + 8 * wid + (lane >> 3);
    const int lc = slot ^ ((row >> 1) & 7);
    const int m = m0 + row;
    a_off[i] = 0;
    a_mask[i] = 0;
    if (m < M) {
      const int img = m / (Ho * Wo), rem = m % (Ho * Wo);
      const int hi0 = (rem / Wo) * stride - pad, wi0 = (rem % Wo) * stride - (ep.pad_w >= 0 ? ep.pad_w : pad);
      a_off[i] = (uint32_t)((((int64_t)img * H + hi0) * W + wi0) * Cin * 2 + chan_bytes(lc)) + plane_a(lc);
      for (int fr = 0; fr < KH; ++fr)
        for (int fc = 0; fc < KW; ++fc)
          if ((unsigned)(hi0 + fr) < (unsigned)H && (unsigned)(wi0 + fc) < (unsigned)W)
            a_mask[i] |= 1ull << (fr * KW + fc);
    }
  }
  static_assert(!BT || (BN == 64 && !F16), "BT: 64-column 16-bit bf16 tiles");
  const int taps = KH * KW;
  uint32_t b_off[BCH];
#pragma unroll
  for (int i = 0; i < BCH; ++i) {
    const int row = 32 * i + 8 * wid + (lane >> 3);
    if constexpr (BT) {  // row = k within the stage (x2: rows 32.. are the lo plane of the same channels)
      const int n = n0 + (slot ^ wsw(row)) * 8;
      const int crow = X2 ? (row & 31) : row;
      const uint32_t pl = X3 ? (row < 32 ? ep.x2_pb : 0u) : (X2 && row >= 32 ? ep.x2_pb : 0u);
      b_off[i] = n < Cout ? (uint32_t)(((int64_t)crow * taps * Cout + n) * 2) + pl : kBufOOB;
    } else {
      const int co = n0 + row;
      const int lc = slot ^ ((row >> 1) & 7);
      const uint32_t pl = X3 ? (lc < 4 ? ep.x2_pb : 0u) : (X2 && lc >= 4 ? ep.x2_pb : 0u);
      b_off[i] = co < Cout ? (uint32_t)((int64_t)co * K * 2 + chan_bytes(lc)) + pl : kBufOOB;
    }
  }
  // X3 lo tiles: A (and non-BT B) as 64-B rows of 32 channels, lane -> (row 16 * wave + lane / 4,
  // chunk lane & 3 holding logical chunk (lane & 3) ^ ((row >> 2) & 3)); the BT B lo tile as 32
  // k-rows of 64 outputs like the main B tile's first half
  uint32_t al_off[ACL > 0 ? ACL : 1], bl_off[BCL > 0 ? BCL : 1];
  uint64_t al_mask[ACL > 0 ? ACL : 1];
  if constexpr (X3) {
#pragma unroll
    for (int i = 0; i < ACL; ++i) {
      const int row = 64 * i + 16 * wid + (lane >> 2);
      const int lc = (lane & 3) ^ ((row >> 2) & 3);
      const int m = m0 + row;
      al_off[i] = 0;
      al_mask[i] = 0;
      if (m < M) {
        const int img = m / (Ho * Wo), rem = m % (Ho * Wo);
        const int hi0 = (rem / Wo) * stride - pad, wi0 = (rem % Wo) * stride - (ep.pad_w >= 0 ? ep.pad_w : pad);
        al_off[i] = (uint32_t)((((int64_t)img * H + hi0) * W + wi0) * Cin * 2 + lc * 16) + 2 * ep.x2_pa;
        for (int fr = 0; fr < KH; ++fr)
          for (int fc = 0; fc < KW; ++fc)
            if ((unsigned)(hi0 + fr) < (unsigned)H && (unsigned)(wi0 + fc) < (unsigned)W)
              al_mask[i] |= 1ull << (fr * KW + fc);
      }
    }
#pragma unroll
    for (int i = 0; i < BCL; ++i) {
      if constexpr (BT) {
        const int row = 8 * wid + (lane >> 3);
        const int n = n0 + (slot ^ wsw(row)) * 8;
        bl_off[i] = n < Cout ? (uint32_t)(((int64_t)row * taps * Cout + n) * 2) + 2 * ep.x2_pb : kBufOOB;
      } else {
        const int row = 64 * i + 16 * wid + (lane >> 2);
        const int lc = (lane & 3) ^ ((row >> 2) & 3);
        const int co = n0 + row;
        bl_off[i] = co < Cout ? (uint32_t)((int64_t)co * K * 2 + lc * 16) + 2 * ep.x2_pb : kBufOOB;
      }
    }
  }
  constexpr int KC = X2 ? BK / 2 : BK;  // channels per stage (x2: 32 of each plane)
  const int cin_steps = Cin / KC;
  const int nk1 = KH * KW * cin_steps;              // K steps of one pass
  const int nk_all = X2 && !X3 && ep.x3 ? 2 * nk1 : nk1;  // two-phase x3: (hi, lo), then (mid, hi)
  const int per = (nk_all + splits - 1) / splits;
  const int ks0 = split * per;
  const int nk_sp = max(0, min(nk_all, ks0 + per) - ks0);  // this split's K steps
  // K group kgi: a contiguous 1/KG of them (x3 with KG = 2 and no split: exactly one phase each);
  // every group runs n_iter barrier rounds, idle in the rounds past its own nk
  const int per_g = (nk_sp + KG - 1) / KG;
  const int k_begin = ks0 + kgi * per_g;
  const int nk = max(0, min(nk_sp, (kgi + 1) * per_g) - kgi * per_g);
  const int n_iter = KG > 1 ? per_g : nk;

  // issue cursor (uniform): x3 phase, tap (fr, fc), channel block ci0 of the next stage to load
  int c_ph = k_begin / nk1;
  int c_tap = (k_begin % nk1) / cin_steps, c_ci = ((k_begin % nk1) % cin_steps) * KC;
  int c_fr = c_tap / KW, c_fc = c_tap % KW;
  auto issue = [&](int buf) {
    // the buffer range check sees only the VGPR offset, so the tap shift (which can turn a
    // negative padding-row offset into a valid one) goes there; the channel block is the SGPR part.
    // x3 phase 0 reads every operand one plane further on (common.h: planes 1 / 2 = hi / lo)
    const bool sh = X2 && !X3 && ep.x3 && c_ph == 0;
    const uint32_t tap_a = (uint32_t)((c_fr * W + c_fc) * Cin * 2);
    const uint32_t soff_a = (uint32_t)(c_ci * 2) + (sh ? ep.x2_pa : 0u);
    const uint32_t soff_b = (BT ? (uint32_t)(((int64_t)c_ci * taps + (taps - 1 - c_tap)) * Cout * 2)
                                : (uint32_t)((c_tap * Cin + c_ci) * 2)) + (sh ? ep.x2_pb : 0u);
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const uint32_t vo = ((a_mask[i] >> c_tap) & 1ull) ? a_off[i] + tap_a : kBufOOB;
      buf_lds16(xr, As + (buf * BM + 32 * i + 8 * wid) * BK, vo, soff_a);
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) buf_lds16(wr, Bs + (buf * BN + 32 * i + 8 * wid) * BK, b_off[i], soff_b);
    if constexpr (X3) {
#pragma unroll
      for (int i = 0; i < ACL; ++i) {
        const uint32_t vo = ((al_mask[i] >> c_tap) & 1ull) ? al_off[i] + tap_a : kBufOOB;
        buf_lds16(xr, Al + (buf * BM + 64 * i + 16 * wid) * 32, vo, soff_a);
      }
#pragma unroll
      for (int i = 0; i < BCL; ++i)
        buf_lds16(wr, Bl + buf * LBN + (BT ? 8 * wid * 64 : (64 * i + 16 * wid) * 32), bl_off[i], soff_b);
    }
    c_ci += KC;
    if (c_ci == Cin) {
      c_ci = 0;
      ++c_tap;
      if (++c_fc == KW) {
        c_fc = 0;
        ++c_fr;
      }
      if (c_tap == taps) {  // next x3 phase
        c_tap = 0;
        c_fr = 0;
        ++c_ph;
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
  for (int ks = 0; ks < n_iter; ++ks) {
    wait_stages<LPS>(ks < nk ? min(S - 2, nk - 1 - ks) : 0);
    __builtin_amdgcn_s_barrier();
    if (ks + S - 1 < nk) issue((ks + S - 1) % S);
    if (KG > 1 && ks >= nk) continue;  // this group is done: barriers only
    const int buf = ks % S;
    if constexpr (BT) {
      // A: 16-B chunk reads (chunk 4*kk + g); B: transposed reads of the k-major tile, all in one
      // asm block (through the builtin the compiler drains the in-flight DMA ring first)
      static_assert(TN == 2, "BT: two 16-column fragments per wave");
      bf16x8 af[2][TM], bfr[2][TN];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wm * WM + i * 16 + (lane & 15);
          af[kk][i] = *reinterpret_cast<const bf16x8*>(As + (buf * BM + row) * BK + swz(row, kk * 4 + (lane >> 4)) * 8);
        }
      const int g = lane >> 4, q = (lane & 15) >> 2, pcol = (lane & 3) * 4;
      uint32_t ad[8];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int row = kk * 32 + 8 * g + 4 * h + q, col = wn * WN + j * 16 + pcol;
            ad[kk * 4 + j * 2 + h] = (uint32_t)reinterpret_cast<uintptr_t>(
                Bs + (buf * BN + row) * BK + (((col >> 3) ^ wsw(row)) << 3) + (col & 7));
          }
      s16x4 fr[8];
      asm volatile(
          "ds_read_b64_tr_b16 %0, %8\n\tds_read_b64_tr_b16 %1, %9\n\t"
          "ds_read_b64_tr_b16 %2, %10\n\tds_read_b64_tr_b16 %3, %11\n\t"
          "ds_read_b64_tr_b16 %4, %12\n\tds_read_b64_tr_b16 %5, %13\n\t"
          "ds_read_b64_tr_b16 %6, %14\n\tds_read_b64_tr_b16 %7, %15\n\t"
          "s_waitcnt lgkmcnt(0)"
          : "=&v"(fr[0]), "=&v"(fr[1]), "=&v"(fr[2]), "=&v"(fr[3]), "=&v"(fr[4]), "=&v"(fr[5]), "=&v"(fr[6]),
            "=&v"(fr[7])
          : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3]), "v"(ad[4]), "v"(ad[5]), "v"(ad[6]), "v"(ad[7])
          : "memory");
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bfr[kk][j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(fr[kk * 4 + j * 2], fr[kk * 4 + j * 2 + 1], 0,
                                                                          1, 2, 3, 4, 5, 6, 7));
      if constexpr (X3) {  // lo fragments: A from its 64-B-row tile, B by transposed reads of the k-major lo tile
        bf16x8 afl[TM], bfl[2];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wm * WM + i * 16 + (lane & 15);
          afl[i] = *reinterpret_cast<const bf16x8*>(Al + (buf * BM + row) * 32 + ((g ^ ((row >> 2) & 3)) << 3));
        }
        uint32_t adl[4];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int row = 8 * g + 4 * h + q, col = wn * WN + j * 16 + pcol;
            adl[j * 2 + h] = (uint32_t)reinterpret_cast<uintptr_t>(
                Bl + buf * LBN + row * 64 + (((col >> 3) ^ wsw(row)) << 3) + (col & 7));
          }
        s16x4 frl[4];
        asm volatile(
            "ds_read_b64_tr_b16 %0, %4\n\tds_read_b64_tr_b16 %1, %5\n\t"
            "ds_read_b64_tr_b16 %2, %6\n\tds_read_b64_tr_b16 %3, %7\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(frl[0]), "=&v"(frl[1]), "=&v"(frl[2]), "=&v"(frl[3])
            : "v"(adl[0]), "v"(adl[1]), "v"(adl[2]), "v"(adl[3])
            : "memory");
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bfl[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(frl[j * 2], frl[j * 2 + 1], 0, 1, 2, 3, 4, 5, 6, 7));
        // (hi, mid) halves: af / bfr [0] = hi, [1] = mid
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][i], bfr[0][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][i], bfr[1][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1][i], bfr[0][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1][i], bfr[1][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][i], bfl[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afl[i], bfr[0][j], acc[i][j], 0, 0, 0);
          }
        continue;
      }
      // products per pass: bf16 (k-half 0) (k-half 1); x2 (hi,hi) (hi,lo) (lo,hi)
      constexpr int NPASS = X2 ? 3 : 2;
#pragma unroll
      for (int ps = 0; ps < NPASS; ++ps) {
        const int ka = X2 ? (ps == 2) : ps, kb = X2 ? (ps == 1) : ps;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ka][i], bfr[kb][j], acc[i][j], 0, 0, 0);
      }
      continue;
    }
    if constexpr (X3) {  // hi / mid from the main tiles' chunks 0-3 / 4-7, lo from the 64-B-row tiles
      bf16x8 fh[TM], fm[TM], fl[TM], gh[TN], gm[TN], gl[TN];
      const int g = lane >> 4;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 16 + (lane & 15);
        fh[i] = *reinterpret_cast<const bf16x8*>(As + (buf * BM + row) * BK + swz(row, g) * 8);
        fm[i] = *reinterpret_cast<const bf16x8*>(As + (buf * BM + row) * BK + swz(row, 4 + g) * 8);
        fl[i] = *reinterpret_cast<const bf16x8*>(Al + (buf * BM + row) * 32 + ((g ^ ((row >> 2) & 3)) << 3));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + j * 16 + (lane & 15);
        gh[j] = *reinterpret_cast<const bf16x8*>(Bs + (buf * BN + row) * BK + swz(row, g) * 8);
        gm[j] = *reinterpret_cast<const bf16x8*>(Bs + (buf * BN + row) * BK + swz(row, 4 + g) * 8);
        gl[j] = *reinterpret_cast<const bf16x8*>(Bl + (buf * BN + row) * 32 + ((g ^ ((row >> 2) & 3)) << 3));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh[i], gh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh[i], gm[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fm[i], gh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fm[i], gm[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh[i], gl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fl[i], gh[j], acc[i][j], 0, 0, 0);
        }
      continue;
    }
    if constexpr (X2) {
      bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
      const int ch = lane >> 4, cl = 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 16 + (lane & 15);
        ah[i] = *reinterpret_cast<const bf16x8*>(As + (buf * BM + row) * BK + swz(row, ch) * 8);
        al[i] = *reinterpret_cast<const bf16x8*>(As + (buf * BM + row) * BK + swz(row, cl) * 8);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + j * 16 + (lane & 15);
        bh[j] = *reinterpret_cast<const bf16x8*>(Bs + (buf * BN + row) * BK + swz(row, ch) * 8);
        bl[j] = *reinterpret_cast<const bf16x8*>(Bs + (buf * BN + row) * BK + swz(row, cl) * 8);
      }
      // three passes over the accumulator tile (independent MFMAs back to back)
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
      continue;
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      typename Mfma16<F16>::T af[TM], bfr[TN];
      const int chunk = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const typename Mfma16<F16>::T*>(As + (buf * BM + row) * BK + swz(row, chunk) * 8);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + j * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const typename Mfma16<F16>::T*>(Bs + (buf * BN + row) * BK + swz(row, chunk) * 8);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = Mfma16<F16>::mma(af[i], bfr[j], acc[i][j]);
    }
  }
  static_assert((KG * BM * (BN + 4) + 5 * BN) * 4 <= S * KG * igemm_ring_stage<BM, BN, BT, X3>() * 2,
                "epilogue tile + column table must fit the operand ring");
  if constexpr (KG > 1) {  // (the launcher guarantees Cout % 8 == 0)
    igemm_epilogue_lds<BM, BN, TM, TN, WM, WN, X2, KG>(acc, reinterpret_cast<float*>(lds), m0, n0, wm, wn, lane,
                                                       tid, M, Cout, ep, y, split, splits, slab, Ho, Wo);
    return;
  }
  if (X2 || ep.yf) {  // fp32-class pairs (separate instantiation: the 16-bit loops stay unrolled)
    if (Cout % 8 == 0)
      igemm_epilogue_lds<BM, BN, TM, TN, WM, WN, true>(acc, reinterpret_cast<float*>(lds), m0, n0, wm, wn, lane, tid, M,
                                                       Cout, ep, y, split, splits, slab, Ho, Wo);
    else
      igemm_epilogue<TM, TN, WM, WN, true>(acc, m0, n0, wm, wn, lane, M, Cout, ep, y, split, splits, slab, Ho, Wo);
  } else if (Cout % 8 == 0) {
    igemm_epilogue_lds<BM, BN, TM, TN, WM, WN>(acc, reinterpret_cast<float*>(lds), m0, n0, wm, wn, lane, tid, M, Cout,
                                               ep, y, split, splits, slab, Ho, Wo);
  } else {
    igemm_epilogue<TM, TN, WM, WN>(acc, m0, n0, wm, wn, lane, M, Cout, ep, y, split, splits, slab, Ho, Wo);
  }
}

// split-K reduce of a launch's fp32 slab through the fused epilogue (conv_igemm.hip)
void splitk_reduce_launch(const float* slab, int splits, int M, int Cout, const ConvEpi& ep, uint16_t* y,
                          hipStream_t st);

}  // namespace mxr
