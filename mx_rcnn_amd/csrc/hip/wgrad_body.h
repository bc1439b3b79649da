// MFMA weight-gradient body (LDS-DMA ring) shared by conv_wgrad.hip's kernel and the grouped
// data + weight gradient launch of conv_igemm.hip (the wgrad role of one fused unit-conv backward).
#pragma once
#include "common.h"

namespace mxr {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int WG_BM = 64, WG_BN = 64, WG_BK = 64;  // co x k-cols x pixels per step
constexpr int WG_ROW = 80;                         // padded LDS row, in bf16 elements (160 B)

__device__ __forceinline__ s16x4 tr_read(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(reinterpret_cast<uintptr_t>(p)));
}

template <int N>
__device__ __forceinline__ void wait_vmcnt_wg() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS row holding MFMA k-index (kk*32) + 8g + j, for the first (j<4) / second (j>=4) read
__device__ __forceinline__ int krow(int kk, int g, int second) { return kk * 32 + (second ? 16 : 0) + 4 * g; }

// ---- LDS-DMA variant ------------------------------------------------------------------------
// Same GEMM and transposed fragment reads, restructured like conv_igemm_buf_kernel: both
// operands arrive by buffer_load_dwordx4 ... lds (S-deep ring, counted vmcnt, raw barrier), so
// the per-step VALU is the pixel -> (img, ho, wo) split of two rows (multiply-high divisions by
// precomputed magic numbers instead of integer division) and the per-lane validity selects.
// DMA writes LDS lane-linearly, so the 160-B row padding of the kernel above becomes an XOR
// swizzle of the 16-B chunk, chunk ^ ((row >> 1) & 3) * 2: the 8 rows x 32 B read by each
// half-wave of ds_read_b64_tr_b16 then fall on 16 distinct 16-B bank slots (conflict-free).
// The epilogue goes through LDS as well: with one split the tile is written straight to the
// bf16 gradient (accumulating into it when asked), otherwise as float4 slab rows.
struct FastDiv {
  uint32_t mul, shift;
};

inline FastDiv make_fastdiv(uint32_t d) {  // n / d == (mulhi(n, mul) + n) >> shift for n < 2^31
  uint32_t l = 0;
  while ((1u << l) < d) ++l;
  FastDiv f;
  f.shift = l;
  f.mul = (uint32_t)(((((uint64_t)1 << l) - d) << 32) / d + 1);
  return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, FastDiv f) { return (__umulhi(n, f.mul) + n) >> f.shift; }

__device__ __forceinline__ int wsw(int row) { return ((row >> 1) & 3) << 1; }

constexpr uint32_t kWgOOB = 0x80000000u;

// all arguments of one weight-gradient launch (the kernel below, or the wgrad role of the grouped
// data + weight gradient launch in conv_igemm.hip)
struct WgradParams {
  const uint16_t* dy;
  const uint16_t* x;
  float* slab;
  uint16_t* dw;
  int accumulate, NB, H, W, Cin, Ho, Wo, Cout, KW, stride, pad, tiles_n, ntiles, splits, per, nwg;
  FastDiv fd_hw, fd_w;
  // fp32-class operands (common.h x2): dY and X are hi / lo plane pairs.  A stage then holds 32
  // pixels of both planes (LDS rows 0-31 hi, 32-63 lo, the same pixels), read by the same
  // fragment loads as a 64-pixel bf16 stage, and runs three MFMAs per fragment pair (dY_hi X_hi +
  // dY_hi X_lo + dY_lo X_hi); the gradient is fp32 (dwf instead of dw)
  // x3 (the fp32 mode, common.h): dY and X are (mid, hi, lo) triples, x2_pdy / x2_px the plane
  // spacings; the pixel loop runs twice, first one plane further on ((hi, lo): hh + hl + lh), then at
  // the base ((mid, hi): mm + mh + hm)
  int x2 = 0;
  int x3 = 0;
  uint32_t x2_pdy = 0, x2_px = 0;  // lo-plane offsets, bytes
  float* dwf = nullptr;
  // fused SGD-momentum (sgd_w set, splits == 1): the tile's gradient updates the parameter in place
  // -- fp32 master, momentum and the shadow the next forward reads -- instead of being stored;
  // the gradient is rounded as the unfused path would have stored it (bf16 when sgd_gbf16)
  float* sgd_w = nullptr;
  float* sgd_mom = nullptr;
  uint16_t* sgd_wb = nullptr;  // bf16 shadow, or the x2 / x3 planes sgd_plane elements apart
  int64_t sgd_plane = 0;
  int sgd_x3 = 0, sgd_gbf16 = 0;
  const float* sgd_lr = nullptr;
  float sgd_mu = 0.f, sgd_wd = 0.f, sgd_rescale = 1.f, sgd_clip = -1.f;
};

constexpr int kWgradLdsElems = 3 * 2 * WG_BK * 64;  // the S = 3 ring: [S][dY|X][64 px][64 ch] (48 KB)

// workgroup `wgid` of the launch; `lds`: KG * S * 2 * 64 * 64 bf16 (16-B aligned); X2 must equal p.x2.
// KG > 1: 4*KG waves, group q over a contiguous 1/KG of the pixel loop through its own sub-ring
// (the grouped dgrad + wgrad launch's K-group form, conv_igemm.hip); the partial tiles are summed
// in group order in the LDS epilogue.
// X3 (the fp32 mode's fused form, X2 = true as well): rows 0-31 of a stage are the hi plane of 32
// pixels, rows 32-63 the mid plane, and a lo tile per operand (32 rows laid out like rows 0-31)
// after the S main stages holds the lo plane: one pass, six MFMAs per fragment set (hh, hm, mh,
// mm, hl, lh).
template <bool X3>
constexpr int wgrad_ring_stage() { return 2 * WG_BK * 64 + (X3 ? 2 * 32 * 64 : 0); }

template <int S, bool X2 = false, int KG = 1, bool X3 = false, bool SGD = false>
__device__ __forceinline__ void wgrad_buf_body(uint16_t* lds, int wgid, const WgradParams& p) {
  constexpr int LPS = X3 ? 6 : 4;  // DMA instructions per thread per stage (2 dY rows + 2 X rows [+ 2 lo])
  constexpr int NT = 256 * KG;
  constexpr int GSTRIDE = S * wgrad_ring_stage<X3>();  // one group's ring, elements
  static_assert(S >= 2 && S <= 4, "pipeline depth");
  static_assert(!X3 || X2, "X3 is a multi-plane mode");
  const int kgi = KG > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 8)) : 0;
  lds += kgi * GSTRIDE;  // this group's sub-ring
  uint16_t* lo_ring = lds + S * 2 * WG_BK * 64;  // X3: [S][dY lo | X lo][32 px][64 ch]
  const uint16_t* __restrict__ dy = p.dy;
  const uint16_t* __restrict__ x = p.x;
  float* __restrict__ slab = p.slab;
  uint16_t* __restrict__ dw = p.dw;
  const int accumulate = p.accumulate, NB = p.NB, H = p.H, W = p.W, Cin = p.Cin, Ho = p.Ho, Wo = p.Wo;
  const int Cout = p.Cout, KW = p.KW, stride = p.stride, pad = p.pad, tiles_n = p.tiles_n, ntiles = p.ntiles;
  const int splits = p.splits, per = p.per;
  const FastDiv fd_hw = p.fd_hw, fd_w = p.fd_w;
  const int split = wgid / ntiles, tile = wgid % ntiles;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int co0 = tm * WG_BM, k0 = tn * WG_BN;
  const int tap = k0 / Cin, ci0 = k0 % Cin;
  const int fr = tap / KW, fc = tap % KW;
  const int P = NB * Ho * Wo, HWo = Ho * Wo;
  const int tid = threadIdx.x, lane = tid & 63, wid = KG > 1 ? __builtin_amdgcn_readfirstlane(tid >> 6) & 3 : tid >> 6;  // wave within the group
  const int wm = wid >> 1, wn = wid & 1;
  const int steps_all = (P + WG_BK - 1) / WG_BK;
  const int s_begin = split * per, s_end = min(steps_all, s_begin + per);
  const int nsteps = max(0, s_end - s_begin);
  constexpr int PX = X2 ? WG_BK / 2 : WG_BK;  // pixels per stage
  const int nloop1 = X2 ? 2 * nsteps : nsteps;           // one pass
  const int nloop = X2 && !X3 && p.x3 ? 2 * nloop1 : nloop1;  // two-phase x3: (hi, lo), then (mid, hi)

  // records through the lo planes for x2 pairs, the third plane for x3 (the range check covers
  // voffset + soffset)
  // (readfirstlane: keeps the resources provably uniform -- a VGPR descriptor costs a waterfall
  // loop around every buffer load)
  const int npl = X2 ? (p.x3 ? 2 : 1) : 0;
  const int nrec_dy = __builtin_amdgcn_readfirstlane((int)((int64_t)P * Cout * 2 + (int64_t)npl * p.x2_pdy));
  const int nrec_x = __builtin_amdgcn_readfirstlane((int)((int64_t)NB * H * W * Cin * 2 + (int64_t)npl * p.x2_px));
  const __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc((void*)dy, (short)0, nrec_dy, 0x00020000);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, nrec_x, 0x00020000);
  int rowi[2], chk[2], prow[2];
  uint32_t a_off[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    rowi[i] = 32 * i + 8 * wid + (lane >> 3);  // LDS row
    prow[i] = X2 ? rowi[i] - 32 * i : rowi[i];  // pixel within the stage (x2: row 32 + r is pixel r's lo)
    chk[i] = (lane & 7) ^ wsw(rowi[i]);
    a_off[i] = co0 + chk[i] * 8 < Cout ? (uint32_t)((prow[i] * Cout + co0 + chk[i] * 8) * 2) : kWgOOB;
  }
  const uint32_t lo_dy = 2 * p.x2_pdy, lo_x = 2 * p.x2_px;  // X3: byte offsets of the lo planes
  auto issue = [&](int it, int buf) {
    const bool ph0 = X2 && !X3 && p.x3 && it < nloop1;  // two-phase x3 (hi, lo): one plane further on
    if (X2 && !X3 && p.x3 && !ph0) it -= nloop1;
    const int p0 = s_begin * WG_BK + it * PX;
    uint16_t* Ab = lds + buf * 2 * WG_BK * 64;
    uint16_t* Bb = Ab + WG_BK * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      // planes of rows 0-31 / 32-63: x2 (hi, lo) = memory planes (0, 1); X3 (hi, mid) = (1, 0)
      const uint32_t pdy = X3 ? (i ? 0u : p.x2_pdy) : (X2 && i ? p.x2_pdy : 0u) + (ph0 ? p.x2_pdy : 0u);
      const uint32_t px = X3 ? (i ? 0u : p.x2_px) : (X2 && i ? p.x2_px : 0u) + (ph0 ? p.x2_px : 0u);
      const int p = p0 + prow[i];
      const uint32_t va = p < P ? a_off[i] : kWgOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(dyr, (__attribute__((address_space(3))) void*)(Ab + (32 * i + 8 * wid) * 64),
                                               16, (int)va, (int)((uint32_t)p0 * Cout * 2 + pdy), 0, 0);
      uint32_t vb = kWgOOB;
      if (p < P) {
        const int img = (int)fdiv((uint32_t)p, fd_hw), rem = p - img * HWo;
        const int ho = (int)fdiv((uint32_t)rem, fd_w), wo = rem - ho * Wo;
        const int hi = ho * stride - pad + fr, wi = wo * stride - pad + fc;
        if ((unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W)
          vb = (uint32_t)(((((int64_t)img * H + hi) * W + wi) * Cin + ci0 + chk[i] * 8) * 2);
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void*)(Bb + (32 * i + 8 * wid) * 64),
                                               16, (int)vb, (int)px, 0, 0);
      if (X3 && i == 0) {  // the lo plane of the same 32 pixels (memory plane 2)
        uint16_t* La = lo_ring + buf * 2 * 32 * 64;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(dyr, (__attribute__((address_space(3))) void*)(La + 8 * wid * 64), 16,
                                                 (int)va, (int)((uint32_t)p0 * Cout * 2 + lo_dy), 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void*)(La + (32 + 8 * wid) * 64),
                                                 16, (int)vb, (int)lo_x, 0, 0);
      }
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fused SGD (KG = 1): the master / momentum rows this thread updates in the epilogue are loaded
  // now, under the pixel loop, instead of after it
  constexpr int SGD_V = (512 + 255) / 256;
  float4 sgd_wp[SGD_V][2], sgd_mp[SGD_V][2];
  if constexpr (SGD && KG == 1) {
#pragma unroll
    for (int v = 0; v < SGD_V; ++v) {
      const int e = tid + v * 256, co = co0 + (e >> 3);
      if (e < 512 && co < Cout) {
        const int64_t o = (int64_t)co * (tiles_n * WG_BN) + k0 + (e & 7) * 8;
        sgd_wp[v][0] = reinterpret_cast<const float4*>(p.sgd_w + o)[0];
        sgd_wp[v][1] = reinterpret_cast<const float4*>(p.sgd_w + o)[1];
        sgd_mp[v][0] = reinterpret_cast<const float4*>(p.sgd_mom + o)[0];
        sgd_mp[v][1] = reinterpret_cast<const float4*>(p.sgd_mom + o)[1];
      }
    }
  }
  const int g = lane >> 4, q = (lane & 15) >> 2, pcol = (lane & 3) * 4;
  // swizzled element offset of (row, col), col a multiple of 4 inside one 16-B chunk
  auto lidx = [](int row, int col) { return row * 64 + (((col >> 3) ^ wsw(row)) << 3) + (col & 7); };

  // this group's contiguous slice of the loop (all of it for KG = 1; x3 with KG = 2: one phase)
  const int per_it = (nloop + KG - 1) / KG;
  const int it0 = kgi * per_it;
  const int nl = max(0, min(nloop, it0 + per_it) - it0);
  const int n_iter = KG > 1 ? per_it : nl;
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nl) issue(it0 + s, s);
  for (int st = 0; st < n_iter; ++st) {
    const int ahead = st < nl ? min(S - 2, nl - 1 - st) : 0;
    if (ahead >= 2) wait_vmcnt_wg<2 * LPS>();
    else if (ahead == 1) wait_vmcnt_wg<LPS>();
    else wait_vmcnt_wg<0>();
    __builtin_amdgcn_s_barrier();
    if (st + S - 1 < nl) issue(it0 + st + S - 1, (st + S - 1) % S);
    if (KG > 1 && st >= nl) continue;  // this group is done: barriers only
    const uint16_t* Ab = lds + (st % S) * 2 * WG_BK * 64;
    const uint16_t* Bb = Ab + WG_BK * 64;
    // all 16 transposed fragment reads of the step in ONE asm block: through the builtin, the
    // compiler cannot tell the ring slot being read from the slots the in-flight LDS-DMA loads
    // fill, and drained EVERY load (s_waitcnt vmcnt(0)) before the reads -- no pipelining at
    // all; the counted vmcnt wait above is the real dependency
    uint32_t ad[16];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
          ad[kk * 8 + i * 2 + h] = (uint32_t)reinterpret_cast<uintptr_t>(
              Ab + lidx(krow(kk, g, h) + q, wm * 32 + i * 16 + pcol));
#pragma unroll
        for (int j = 0; j < 2; ++j)
          ad[kk * 8 + 4 + j * 2 + h] = (uint32_t)reinterpret_cast<uintptr_t>(
              Bb + lidx(krow(kk, g, h) + q, wn * 32 + j * 16 + pcol));
      }
    s16x4 fr[16];
    asm volatile(
        "ds_read_b64_tr_b16 %0, %16\n\tds_read_b64_tr_b16 %1, %17\n\t"
        "ds_read_b64_tr_b16 %2, %18\n\tds_read_b64_tr_b16 %3, %19\n\t"
        "ds_read_b64_tr_b16 %4, %20\n\tds_read_b64_tr_b16 %5, %21\n\t"
        "ds_read_b64_tr_b16 %6, %22\n\tds_read_b64_tr_b16 %7, %23\n\t"
        "ds_read_b64_tr_b16 %8, %24\n\tds_read_b64_tr_b16 %9, %25\n\t"
        "ds_read_b64_tr_b16 %10, %26\n\tds_read_b64_tr_b16 %11, %27\n\t"
        "ds_read_b64_tr_b16 %12, %28\n\tds_read_b64_tr_b16 %13, %29\n\t"
        "ds_read_b64_tr_b16 %14, %30\n\tds_read_b64_tr_b16 %15, %31\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(fr[0]), "=&v"(fr[1]), "=&v"(fr[2]), "=&v"(fr[3]), "=&v"(fr[4]), "=&v"(fr[5]), "=&v"(fr[6]),
          "=&v"(fr[7]), "=&v"(fr[8]), "=&v"(fr[9]), "=&v"(fr[10]), "=&v"(fr[11]), "=&v"(fr[12]), "=&v"(fr[13]),
          "=&v"(fr[14]), "=&v"(fr[15])
        : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3]), "v"(ad[4]), "v"(ad[5]), "v"(ad[6]), "v"(ad[7]),
          "v"(ad[8]), "v"(ad[9]), "v"(ad[10]), "v"(ad[11]), "v"(ad[12]), "v"(ad[13]), "v"(ad[14]), "v"(ad[15])
        : "memory");
    bf16x8 af[2][2], bfr[2][2];  // [kk][i]: x2 kk = plane (hi / lo of the same 32 pixels)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[kk][i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(fr[kk * 8 + i * 2], fr[kk * 8 + i * 2 + 1], 0,
                                                                       1, 2, 3, 4, 5, 6, 7));
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bfr[kk][j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(fr[kk * 8 + 4 + j * 2],
                                                                        fr[kk * 8 + 4 + j * 2 + 1], 0, 1, 2, 3, 4, 5,
                                                                        6, 7));
    }
    if constexpr (X3) {  // lo fragments by transposed reads of the lo tiles; six products
      const uint16_t* La = lo_ring + (st % S) * 2 * 32 * 64;
      uint32_t adl[8];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
          adl[i * 2 + h] = (uint32_t)reinterpret_cast<uintptr_t>(La + lidx(krow(0, g, h) + q, wm * 32 + i * 16 + pcol));
#pragma unroll
        for (int j = 0; j < 2; ++j)
          adl[4 + j * 2 + h] = (uint32_t)reinterpret_cast<uintptr_t>(
              La + 32 * 64 + lidx(krow(0, g, h) + q, wn * 32 + j * 16 + pcol));
      }
      s16x4 frl[8];
      asm volatile(
          "ds_read_b64_tr_b16 %0, %8\n\tds_read_b64_tr_b16 %1, %9\n\t"
          "ds_read_b64_tr_b16 %2, %10\n\tds_read_b64_tr_b16 %3, %11\n\t"
          "ds_read_b64_tr_b16 %4, %12\n\tds_read_b64_tr_b16 %5, %13\n\t"
          "ds_read_b64_tr_b16 %6, %14\n\tds_read_b64_tr_b16 %7, %15\n\t"
          "s_waitcnt lgkmcnt(0)"
          : "=&v"(frl[0]), "=&v"(frl[1]), "=&v"(frl[2]), "=&v"(frl[3]), "=&v"(frl[4]), "=&v"(frl[5]),
            "=&v"(frl[6]), "=&v"(frl[7])
          : "v"(adl[0]), "v"(adl[1]), "v"(adl[2]), "v"(adl[3]), "v"(adl[4]), "v"(adl[5]), "v"(adl[6]),
            "v"(adl[7])
          : "memory");
      bf16x8 afl[2], bfl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        afl[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(frl[i * 2], frl[i * 2 + 1], 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bfl[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(frl[4 + j * 2], frl[4 + j * 2 + 1], 0, 1, 2, 3, 4,
                                                                    5, 6, 7));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {  // [0] = hi, [1] = mid
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][i], bfr[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][i], bfr[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1][i], bfr[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1][i], bfr[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][i], bfl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afl[i], bfr[0][j], acc[i][j], 0, 0, 0);
        }
      continue;
    }
    // products (a, b) per pass: bf16 (0,0) (1,1); x2 (hi,hi) (hi,lo) (lo,hi)
    constexpr int NPASS = X2 ? 3 : 2;
#pragma unroll
    for (int ps = 0; ps < NPASS; ++ps) {
      const int ka = X2 ? (ps == 2) : ps, kb = X2 ? (ps == 1) : ps;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ka][i], bfr[kb][j], acc[i][j], 0, 0, 0);
    }
  }

  // epilogue through LDS: T[co][k] fp32 (row stride 68; one slice per K group, summed in group
  // order), then 8-column vectors per thread
  __syncthreads();
  float* T = reinterpret_cast<float*>(lds - kgi * GSTRIDE);  // the workgroup's LDS
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        T[(kgi * 64 + wm * 32 + i * 16 + (lane >> 4) * 4 + r) * 68 + wn * 32 + j * 16 + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  const int ldk = tiles_n * WG_BN;
#pragma unroll
  for (int v = 0; v < (512 + NT - 1) / NT; ++v) {
    const int e = tid + v * NT, row = e >> 3, cv = e & 7;
    const int co = co0 + row;
    if (e >= 512 || co >= Cout) continue;
    const float4* src = reinterpret_cast<const float4*>(T + row * 68 + cv * 8);
    float4 a0 = src[0], a1 = src[1];
#pragma unroll
    for (int q = 1; q < KG; ++q) {
      const float4* sq = reinterpret_cast<const float4*>(T + (q * 64 + row) * 68 + cv * 8);
      const float4 b0 = sq[0], b1 = sq[1];
      a0.x += b0.x; a0.y += b0.y; a0.z += b0.z; a0.w += b0.w;
      a1.x += b1.x; a1.y += b1.y; a1.z += b1.z; a1.w += b1.w;
    }
    const int64_t o = (int64_t)co * ldk + k0 + cv * 8;
    if (SGD) {  // fused update (the host guarantees sgd_w, splits == 1 and 16-B aligned rows)
      float g[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      if (p.sgd_gbf16) {
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] = bf16_to_f32(f32_to_bf16(g[k]));
      }
      const float lr = *p.sgd_lr;
      float4* wp = reinterpret_cast<float4*>(p.sgd_w + o);
      float4* mp = reinterpret_cast<float4*>(p.sgd_mom + o);
      float4 w0, w1, m0, m1;
      if constexpr (KG == 1 && NT == 256) {  // prefetched before the pixel loop
        w0 = sgd_wp[v][0]; w1 = sgd_wp[v][1]; m0 = sgd_mp[v][0]; m1 = sgd_mp[v][1];
      } else {
        w0 = wp[0]; w1 = wp[1]; m0 = mp[0]; m1 = mp[1];
      }
      float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      float mv[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) wv[k] = sgd_one(wv[k], mv[k], g[k], lr, p.sgd_mu, p.sgd_wd, p.sgd_rescale, p.sgd_clip);
      wp[0] = make_float4(wv[0], wv[1], wv[2], wv[3]);
      wp[1] = make_float4(wv[4], wv[5], wv[6], wv[7]);
      mp[0] = make_float4(mv[0], mv[1], mv[2], mv[3]);
      mp[1] = make_float4(mv[4], mv[5], mv[6], mv[7]);
      if (p.sgd_wb && p.sgd_plane) {
        const int code = p.sgd_x3 ? kCodeX3 : kCodeX2;
        st4c(p.sgd_wb, o, code, p.sgd_plane, wv);
        st4c(p.sgd_wb, o + 4, code, p.sgd_plane, wv + 4);
      } else if (p.sgd_wb) {
        st8_bf16(p.sgd_wb + o, wv);
      }
      continue;
    }
    if (splits > 1) {
      float4* d = reinterpret_cast<float4*>(slab + (int64_t)split * Cout * ldk + o);
      d[0] = a0;
      d[1] = a1;
    } else if (p.dwf) {  // fp32 gradient (x2 mode)
      float4* d = reinterpret_cast<float4*>(p.dwf + o);
      if (accumulate) {
        const float4 q0 = d[0], q1 = d[1];
        d[0] = make_float4(a0.x + q0.x, a0.y + q0.y, a0.z + q0.z, a0.w + q0.w);
        d[1] = make_float4(a1.x + q1.x, a1.y + q1.y, a1.z + q1.z, a1.w + q1.w);
      } else {
        d[0] = a0;
        d[1] = a1;
      }
    } else {
      float a[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      if (accumulate) {
        float prev[8];
        ld8_bf16(dw + o, prev);
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] += prev[k];
      }
      st8_bf16(dw + o, a);
    }
  }
}

// sum of the split-K slabs (+ the existing gradient when accumulating) -> bf16; 4 * nt elements per
// nt-thread workgroup `gid` (the wgrad_reduce kernel, or a role of the grouped launch)
__device__ __forceinline__ void wgrad_reduce_body(int gid, const float* __restrict__ slab, int splits, int64_t n,
                                                  uint16_t* __restrict__ out, int accumulate, float* outf = nullptr,
                                                  int nt = 256) {
  const int64_t e = ((int64_t)gid * nt + threadIdx.x) * 4;
  if (e >= n) return;
  float4 a = *reinterpret_cast<const float4*>(slab + e);
#pragma unroll 4
  for (int s = 1; s < splits; ++s) {
    const float4 b = *reinterpret_cast<const float4*>(slab + (int64_t)s * n + e);
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  }
  if (outf) {  // fp32 gradient (x2 mode)
    float4* d = reinterpret_cast<float4*>(outf + e);
    if (accumulate) {
      const float4 q = *d;
      a.x += q.x; a.y += q.y; a.z += q.z; a.w += q.w;
    }
    *d = a;
    return;
  }
  if (accumulate) {  // add into the existing gradient (flat-buffer view), no separate add kernel
    const ushort4 o = *reinterpret_cast<const ushort4*>(out + e);
    a.x += bf16_to_f32(o.x); a.y += bf16_to_f32(o.y); a.z += bf16_to_f32(o.z); a.w += bf16_to_f32(o.w);
  }
  *reinterpret_cast<ushort4*>(out + e) = make_ushort4(f32_to_bf16(a.x), f32_to_bf16(a.y), f32_to_bf16(a.z),
                                                      f32_to_bf16(a.w));
}

// a deferred split-K reduce carried into the next grouped launch (role 0 there)
struct WgradReduceParams {
  const float* slab = nullptr;
  uint16_t* dw = nullptr;
  float* dwf = nullptr;  // fp32 gradient instead of dw (x2 mode)
  int64_t n = 0;
  int splits = 0, accumulate = 1, nwg = 0;
};

// host helpers (conv_wgrad.hip)
WgradParams wgrad_params(const uint16_t* dy, const uint16_t* x, uint16_t* dw, float* slab, int NB, int H, int W,
                         int Cin, int Ho, int Wo, int Cout, int KH, int KW, int stride, int pad, int splits,
                         int accumulate);
void wgrad_reduce(const float* slab, int splits, int64_t n, uint16_t* dw, int accumulate, hipStream_t st,
                  float* dwf = nullptr);

}  // namespace mxr
