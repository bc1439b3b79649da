// Large-tile implicit-GEMM convolution for the large-M GEMMs (batch-8 inference, the VGG16 trunk at
// 600x1000, the RPN 3x3 over a batch): BM = 256 output pixels x BN = 256 / 128 output channels per
// 512-thread workgroup (8 waves), v_mfma_f32_16x16x32_{bf16,f16}, every wave owning a 128x64 /
// 64x64 accumulator block (128 / 64 AGPRs).
//
// Why a second kernel: the 64x64 buffer kernel (conv_igemm.hip) runs one K stage per barrier with
// the next two stages in flight; on a large grid each CU then streams 2 x 64 operand rows per
// 64x64x64 MFMA block, and the per-stage DMA round trip (tools/microbench/dma_stream.hip: ~0.3 us
// for a 16 KB stage at every CU loading) bounds it at 480-800 TF/s on these shapes
// (tools/microbench/conv_tiles.py).  Here a K tile is BK = 32 channels of one filter tap for 256
// rows of A and BN rows of B (32 / 24 KB), the LDS holds FOUR K tiles (a ring three tiles deep in
// flight: 96 KB of DMA outstanding per CU, never drained to zero inside the loop), and one barrier
// per K tile separates 32 (16) MFMAs per wave -- 1024 (512) MFMA cycles per SIMD against 32 (24)
// KB of operand bytes per CU.
//
// LDS image: [buf][row][32] bf16, 64-B rows, 16-B chunk c of row r stored at chunk c ^ ((r >> 2) & 3):
// the 16 rows a ds_read_b128 fragment read touches (same logical chunk) land on 16 distinct 16-B
// slots of the 256-B bank row -- conflict-free.  The DMA image is lane-linear (4 lanes per row), so
// the swizzle is applied to each lane's SOURCE chunk.
//
// Operands and padding follow the buffer kernel: NHWC activations, filter (Cout, KH, KW, Cin),
// per-lane 32-bit row offsets + a 64-bit tap mask, padding taps read as zeros through the buffer
// range check.  Epilogue per wave through a private 16-row LDS slab: bias, residual, ReLU, frozen
// BN(+ReLU) second output (ConvEpi::y2), bf16 or fp16 storage, 16-B vector loads / stores.
#include "common.h"
#include "../kernels.h"

namespace mxr {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr uint32_t kOOB = 0x80000000u;
constexpr int BK = 32;       // channels per K tile
constexpr int NBUF = 4;      // K tiles resident in LDS (3 in flight); short-K tiles 205-207: 2 or 3

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, void* lds_wave_base, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds_wave_base, 16, (int)voff,
                                           (int)soff, 0, 0);
}

template <bool F16>
__device__ __forceinline__ f32x4_t mma(const uint4& a, const uint4& b, f32x4_t c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c, 0,
                                                  0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                   c, 0, 0, 0);
}

template <int BM_, int BN>
struct BigCfg {
  static constexpr int BM = BM_;
  static constexpr int WGN = BN / 64;        // waves along N (64 columns each)
  static constexpr int WGM = 8 / WGN;        // waves along M
  static constexpr int WM = BM / WGM;        // rows per wave (128, 64 or 32)
  static constexpr int TM = WM / 16, TN = 4; // 16x16 accumulator tiles per wave
  static constexpr int ROWS = BM + BN;       // LDS rows per K tile
  // DMA instruction i of wave w loads LDS rows i*128 + 16w .. +15 (A rows first, then B rows): a wave
  // issues LPT_HI instructions per K tile if its last block exists (w < NHI), else LPT_LO
  static constexpr int LPT_HI = (ROWS + 127) / 128, LPT_LO = ROWS / 128;
  static constexpr int NHI = (ROWS % 128) / 16;  // waves with the extra (partial-round) instruction
  static_assert(BM % 16 == 0 && BN % 64 == 0 && ROWS % 16 == 0, "16-row DMA blocks never straddle A / B");
  static constexpr int EPI_LD = 64 + 4;      // fp32 row stride of the per-wave epilogue slab
};

// The LDS ring arrives as a plain pointer parameter (no __restrict__, not the __shared__ object
// itself): referenced directly, hipcc's wait-count pass drained every in-flight LDS-DMA
// (s_waitcnt vmcnt(0)) before the fragment reads of each K tile -- the same effect the buffer
// kernel documents for a __restrict__ ring (conv_igemm.hip).
template <int BM_, int BN, bool F16, int NR = NBUF>
__device__ __forceinline__ void conv_big_body(uint16_t* lds, const uint16_t* __restrict__ x,
                                              const uint16_t* __restrict__ w, uint16_t* __restrict__ y, int NB, int H,
                                              int W, int Cin, int Ho, int Wo, int Cout, int KH, int KW, int stride,
                                              int pad, const ConvEpi& ep, int tiles_n, int nwg) {
  using C = BigCfg<BM_, BN>;
  constexpr int BM = C::BM, TM = C::TM, TN = C::TN, WM = C::WM;

  const int bid = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tm_idx = wgid / tiles_n, tn_idx = wgid % tiles_n;
  const int m0 = tm_idx * BM, n0 = tn_idx * BN;
  const int M = NB * Ho * Wo;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / C::WGN, wn = wid % C::WGN;
  const int K = KH * KW * Cin;

  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, (int)((int64_t)NB * H * W * Cin * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)w, (short)0, (int)((int64_t)Cout * K * 2), 0x00020000);

  // DMA roles: instruction i of a thread loads LDS row i*128 + tid/4 (A rows first, then B rows),
  // logical 16-B chunk (tid & 3) ^ ((row >> 2) & 3) of that row's 32 channels
  const int lpt = wid < C::NHI ? C::LPT_HI : C::LPT_LO;  // wave-uniform
  uint32_t off[C::LPT_HI];
  uint64_t amask[C::LPT_HI];
#pragma unroll
  for (int i = 0; i < C::LPT_HI; ++i) {
    const int row = i * 128 + (tid >> 2);
    const int lc = (tid & 3) ^ ((row >> 2) & 3);
    off[i] = kOOB;
    amask[i] = 0;
    if (row >= C::ROWS) continue;
    if (row < BM) {
      const int m = m0 + row;
      if (m < M) {
        const int img = m / (Ho * Wo), rem = m % (Ho * Wo);
        const int hi0 = (rem / Wo) * stride - pad, wi0 = (rem % Wo) * stride - pad;
        off[i] = (uint32_t)(((((int64_t)img * H + hi0) * W + wi0) * Cin + lc * 8) * 2);
        for (int fr = 0; fr < KH; ++fr)
          for (int fc = 0; fc < KW; ++fc)
            if ((unsigned)(hi0 + fr) < (unsigned)H && (unsigned)(wi0 + fc) < (unsigned)W)
              amask[i] |= 1ull << (fr * KW + fc);
      }
    } else {
      const int co = n0 + row - BM;
      if (co < Cout) off[i] = (uint32_t)(((int64_t)co * K + lc * 8) * 2);
    }
  }
  const int cin_steps = Cin / BK;
  const int nk = KH * KW * cin_steps;
  int c_tap = 0, c_ci = 0, c_fr = 0, c_fc = 0;
  auto issue = [&](int buf) {
    const uint32_t tap_a = (uint32_t)((c_fr * W + c_fc) * Cin * 2);
    const uint32_t soff_a = (uint32_t)(c_ci * 2);
    const uint32_t soff_b = (uint32_t)((c_tap * Cin + c_ci) * 2);
    uint16_t* base = lds + (buf * C::ROWS + wid * 16) * BK;  // this wave's 16 rows of instruction 0
#pragma unroll
    for (int i = 0; i < C::LPT_HI; ++i) {
      const int row0 = i * 128 + wid * 16;  // wave-uniform role of this instruction
      if (row0 >= C::ROWS) continue;
      if (row0 < BM) {
        const uint32_t vo = ((amask[i] >> c_tap) & 1ull) ? off[i] + tap_a : kOOB;
        dma16(xr, base + i * 128 * BK, vo, soff_a);
      } else {
        dma16(wr, base + i * 128 * BK, off[i], soff_b);
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

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NR - 1; ++s)
    if (s < nk) issue(s);
  // fragment read offsets (elements) within a K tile: A row wm*WM + i*16 + (lane & 15), B row
  // BM + wn*64 + j*16 + (lane & 15), logical chunk lane >> 4
  const int fr_row = lane & 15, fr_ch = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    // K tile kt landed: at most min(NR - 2, nk-1-kt) younger tiles of this thread still in flight
    const int ahead = min(NR - 2, nk - 1 - kt);
    if (ahead >= 2) {
      if (C::NHI == 0 || lpt == C::LPT_LO) vm_wait<2 * C::LPT_LO>();
      else vm_wait<2 * C::LPT_HI>();
    } else if (ahead == 1) {
      if (C::NHI == 0 || lpt == C::LPT_LO) vm_wait<C::LPT_LO>();
      else vm_wait<C::LPT_HI>();
    } else {
      vm_wait<0>();
    }
    __builtin_amdgcn_s_barrier();  // every wave's DMA of tile kt landed; tile kt-1's buffer is free
    if (kt + NR - 1 < nk) issue((kt + NR - 1) % NR);
    const uint16_t* T = lds + (kt % NR) * C::ROWS * BK;
    uint4 af[TM], bf[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = BM + wn * 64 + j * 16 + fr_row;
      bf[j] = *reinterpret_cast<const uint4*>(T + row * BK + ((fr_ch ^ ((row >> 2) & 3)) << 3));
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * WM + i * 16 + fr_row;
      af[i] = *reinterpret_cast<const uint4*>(T + row * BK + ((fr_ch ^ ((row >> 2) & 3)) << 3));
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mma<F16>(af[i], bf[j], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
  }

  // ---- epilogue: per wave, 16 output rows at a time through a private fp32 slab ----------------
  __syncthreads();  // every wave is done with the operand ring (and every DMA retired: vmcnt(0) above)
  float* slab = reinterpret_cast<float*>(lds) + wid * 16 * C::EPI_LD;
  const int code = F16 ? 2 : 1;
  const int er = lane >> 2;             // slab row of this lane
  const int ec = (lane & 3) * 16;       // first of its 16 columns
  const int n = n0 + wn * 64 + ec;
  // per-column epilogue coefficients: each lane derives ONE of the wave's 64 columns (bias, BN
  // scale, BN shift: 5 loads + 1 rsqrt) into a per-wave LDS table, then reads its 16 columns back as
  // 16-B vectors -- instead of 16 columns x 5 scalar loads per lane
  float* coef = reinterpret_cast<float*>(lds) + 8 * 16 * C::EPI_LD + wid * 3 * 64;
  {
    const int col = min(n0 + wn * 64 + lane, Cout - 1);
    float cb = ep.bias ? ep.bias[col] : (ep.bias_h ? h16_to_f32(ep.bias_h[col], code) : 0.f), cs = 1.f, ct = 0.f;
    if (ep.y2) {
      const float g = ep.bn_fix_gamma ? 1.f : ep.bn_gamma[col];
      const float inv = rsqrtf(ep.bn_var[col] + ep.bn_eps);
      cs = g * inv;
      ct = ep.bn_beta[col] - ep.bn_mean[col] * cs;
    }
    coef[lane] = cb;
    coef[64 + lane] = cs;
    coef[128 + lane] = ct;
  }
  float bias[16], bs[16], bt[16];  // (same-wave LDS write -> read: in order)
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 b4 = *reinterpret_cast<const float4*>(coef + ec + 4 * q);
    bias[4 * q] = b4.x; bias[4 * q + 1] = b4.y; bias[4 * q + 2] = b4.z; bias[4 * q + 3] = b4.w;
    if (ep.y2) {  // (no second output: the BN columns are never read)
      const float4 s4 = *reinterpret_cast<const float4*>(coef + 64 + ec + 4 * q);
      const float4 t4 = *reinterpret_cast<const float4*>(coef + 128 + ec + 4 * q);
      bs[4 * q] = s4.x; bs[4 * q + 1] = s4.y; bs[4 * q + 2] = s4.z; bs[4 * q + 3] = s4.w;
      bt[4 * q] = t4.x; bt[4 * q + 1] = t4.y; bt[4 * q + 2] = t4.z; bt[4 * q + 3] = t4.w;
    } else {
      bs[4 * q] = bs[4 * q + 1] = bs[4 * q + 2] = bs[4 * q + 3] = 1.f;
      bt[4 * q] = bt[4 * q + 1] = bt[4 * q + 2] = bt[4 * q + 3] = 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) slab[((lane >> 4) * 4 + r) * C::EPI_LD + j * 16 + (lane & 15)] = acc[i][j][r];
    // same-wave LDS write -> read: in order, no barrier needed
    const int m = m0 + wm * WM + i * 16 + er;
    if (m < M && n < Cout) {
      const int64_t e = (int64_t)m * Cout + n;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (n + h * 8 >= Cout) break;
        float v[8], rs[8];
        const float4* src = reinterpret_cast<const float4*>(slab + er * C::EPI_LD + ec + h * 8);
        const float4 a0 = src[0], a1 = src[1];
        v[0] = a0.x; v[1] = a0.y; v[2] = a0.z; v[3] = a0.w; v[4] = a1.x; v[5] = a1.y; v[6] = a1.z; v[7] = a1.w;
        if (ep.residual) ld8_h16(ep.residual + e + h * 8, rs, code);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float t = v[k] + bias[h * 8 + k] + (ep.residual ? rs[k] : 0.f);
          if (ep.relu) t = fmaxf(t, 0.f);
          v[k] = t;
        }
        uint16_t yb[8];
        float y2v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          yb[k] = f32_to_h16(v[k], code);
          float qv = h16_to_f32(yb[k], code) * bs[h * 8 + k] + bt[h * 8 + k];  // BN reads the STORED output
          if (ep.act_relu) qv = fmaxf(qv, 0.f);
          y2v[k] = qv;
        }
        *reinterpret_cast<uint4*>(y + e + h * 8) =
            make_uint4((uint32_t)yb[0] | ((uint32_t)yb[1] << 16), (uint32_t)yb[2] | ((uint32_t)yb[3] << 16),
                       (uint32_t)yb[4] | ((uint32_t)yb[5] << 16), (uint32_t)yb[6] | ((uint32_t)yb[7] << 16));
        if (ep.y2) st8_h16(ep.y2 + e + h * 8, y2v, code);
      }
    }
  }
}

// LDS: the ring, and at least what the epilogue reuses it for: 8 per-wave slabs (16 rows x EPI_LD
// fp32) and 8 per-wave coefficient tables (3 x 64 fp32)
template <int BM, int BN, int NR>
constexpr int big_lds_elems() {
  constexpr int ring = NR * BigCfg<BM, BN>::ROWS * BK, slabs = (8 * 16 * BigCfg<BM, BN>::EPI_LD + 8 * 3 * 64) * 2;
  return ring > slabs ? ring : slabs;
}

template <int BM, int BN, bool F16, int NBR = NBUF>
__global__ void __launch_bounds__(512)
conv_big_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, uint16_t* __restrict__ y, int NB,
                int H, int W, int Cin, int Ho, int Wo, int Cout, int KH, int KW, int stride, int pad, const ConvEpi ep,
                int tiles_n, int nwg) {
  // one LDS array (a second __shared__ object can make hipcc drain the DMA ring before each read)
  __shared__ __attribute__((aligned(16))) uint16_t lds[big_lds_elems<BM, BN, NBR>()];
  conv_big_body<BM, BN, F16, NBR>(lds, x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, tiles_n, nwg);
}

}  // namespace

// tile codes 200 (256x256) / 201 (256x128) / 202 (128x128) / 203 (128x256) / 204 (160x256: the batch-8
// stage-3 1x1 reduce, M = 33 600 = 210 x 160 rows, one tile per CU on 210 CUs with no partial
// second round; 8 waves as 2 x 4 of 80 x 64 accumulators); -1 when the shape or
// epilogue is not supported.  The 128-row tiles serve N = 256 GEMMs of a few tens of thousands of
// rows (the batch-8 stage-3 reduce / 3x3 convs: 75 workgroups of 256x256 leave 181 of 256 CUs
// idle; 128x128 gives 300, two resident per CU with the 64 KB ring)
int conv_big_fwd(const uint16_t* x, const uint16_t* w, uint16_t* y, int NB, int H, int W, int Cin, int Ho, int Wo,
                 int Cout, int KH, int KW, int stride, int pad, const ConvEpi& ep, int tile, hipStream_t st) {
  if (tile < 200 || tile > 207) return -1;
  if (Cin % BK != 0 || Cout % 16 != 0 || KH * KW > 64) return -1;
  if (ep.x2 || ep.yf || ep.bt || ep.omap || ep.pad_w >= 0 || ep.bnb_x || ep.st_part || ep.bnb_part || ep.rmask ||
      ep.drop_p > 0.f)
    return -1;
  if ((ep.y2) && (!ep.bn_beta || !ep.bn_mean || !ep.bn_var || (!ep.bn_fix_gamma && !ep.bn_gamma))) return -1;
  if ((int64_t)NB * H * W * Cin * 2 >= (int64_t)kOOB || (int64_t)Cout * KH * KW * Cin * 2 >= (int64_t)kOOB) return -1;
  const int M = NB * Ho * Wo;
  const int bm = tile == 204 ? 160 : (tile == 200 || tile == 201 || tile == 207) ? 256 : 128;
  const int bn = (tile == 200 || tile == 203 || tile == 204 || tile == 207) ? 256 : 128;
  const int tiles_n = (Cout + bn - 1) / bn;
  const int nwg = ((M + bm - 1) / bm) * tiles_n;
#define MXR_BIG(BM_, BN_, F_, R_)                                                                          \
  conv_big_kernel<BM_, BN_, F_, R_><<<nwg, 512, 0, st>>>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, \
                                                        pad, ep, tiles_n, nwg)
#define MXR_BIG2(BM_, BN_, R_)      \
  do {                              \
    if (ep.f16)                     \
      MXR_BIG(BM_, BN_, true, R_);  \
    else                            \
      MXR_BIG(BM_, BN_, false, R_); \
  } while (0)
  // 205-207: shallow rings for short-K GEMMs (the 1x1 expands, K = 256 / 512): less LDS per
  // workgroup, so more workgroups per CU and one's epilogue stores overlap another's K loop
  switch (tile) {
    case 200: MXR_BIG2(256, 256, NBUF); break;
    case 201: MXR_BIG2(256, 128, NBUF); break;
    case 202: MXR_BIG2(128, 128, NBUF); break;
    case 203: MXR_BIG2(128, 256, NBUF); break;
    case 205: MXR_BIG2(128, 128, 2); break;
    case 206: MXR_BIG2(128, 128, 3); break;
    case 207: MXR_BIG2(256, 256, 2); break;
    default: MXR_BIG2(160, 256, NBUF); break;
  }
#undef MXR_BIG2
#undef MXR_BIG
  return tile;
}

}  // namespace mxr
