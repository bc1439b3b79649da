// MFMA weight gradient for NHWC bf16 convolutions (SURVEY kernel K2, the `igemm_wrw` MIOpen
// kernel it replaces took 2.2 ms/step in the first ResNet-101 profile).
//
//   dW[co][k] = sum_p dY[p][co] * X[p shifted by tap(k)][ci(k)],   k = (fr, fc, ci)
//
// GEMM view: M = Cout, N = KH*KW*Cin, K = output pixels.  Both operands arrive from HBM
// with the CHANNEL dimension contiguous (NHWC rows), but MFMA wants 8 consecutive K
// (pixels) per lane.  Tiles are therefore staged as [pixel][channel] rows in LDS and the
// fragments are read with gfx950's transposing `ds_read_b64_tr_b16` (4 pixel-rows x 16
// channels per 16-lane group, delivered column-major), two reads per 8-deep fragment.
//
// LDS rows are padded to 160 B (BM/BN = 64 channels = 128 B + 32 B) and the MFMA k-index
// is permuted onto LDS rows (k = 8g + j -> row 4g + j for j < 4, 16 + 4g + j - 4 otherwise)
// so each 32-lane half of a transposed read touches 8 consecutive rows whose 32-B column
// windows land on 8 disjoint bank slots: conflict-free.  The permutation is applied to both
// operands, so the sum over K is unchanged.
//
// Split-K over pixels with fp32 slab partials (the output is small, the reduction long);
// the shared split-K reduce kernel of conv_igemm.hip casts to bf16.
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "../kernels.h"

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

__global__ void __launch_bounds__(256)
conv_wgrad_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x, float* __restrict__ slab, int NB,
                  int H, int W, int Cin, int Ho, int Wo, int Cout, int KW, int stride, int pad, int tiles_n,
                  int ntiles, int splits, int per) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * WG_BK * WG_ROW];
  uint16_t* As = lds;                        // [2][BK][ROW]  dY tile: pixels x co
  uint16_t* Bs = lds + 2 * WG_BK * WG_ROW;   // [2][BK][ROW]  X tile:  pixels x ci
  const int wgid = blockIdx.x;
  const int split = wgid / ntiles, tile = wgid % ntiles;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int co0 = tm * WG_BM, k0 = tn * WG_BN;          // k0: column in (fr, fc, ci) space
  const int tap = k0 / Cin, ci0 = k0 % Cin;              // Cin % 64 == 0: a tile never straddles taps
  const int fr = tap / KW, fc = tap % KW;
  const int P = NB * Ho * Wo;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int steps_all = (P + WG_BK - 1) / WG_BK;
  const int s_begin = split * per, s_end = min(steps_all, s_begin + per);
  const int nsteps = max(0, s_end - s_begin);

  // per thread: 2 chunks of 16 B for each operand per step (64 rows x 8 chunks / 256)
  uint4 ra[2], rb[2];
  auto load = [&](int sl) {
    const int p0 = (s_begin + sl) * WG_BK;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int qq = tid + i * 256, row = qq >> 3, ch = qq & 7;
      const int p = p0 + row;
      ra[i] = make_uint4(0, 0, 0, 0);
      rb[i] = make_uint4(0, 0, 0, 0);
      if (p < P) {
        if (co0 + ch * 8 < Cout)
          ra[i] = *reinterpret_cast<const uint4*>(dy + (int64_t)p * Cout + co0 + ch * 8);
        const int img = p / (Ho * Wo), rem = p % (Ho * Wo);
        const int hi = (rem / Wo) * stride - pad + fr, wi = (rem % Wo) * stride - pad + fc;
        if (hi >= 0 && hi < H && wi >= 0 && wi < W)
          rb[i] = *reinterpret_cast<const uint4*>(x + (((int64_t)img * H + hi) * W + wi) * Cin + ci0 + ch * 8);
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int qq = tid + i * 256, row = qq >> 3, ch = qq & 7;
      *reinterpret_cast<uint4*>(As + (buf * WG_BK + row) * WG_ROW + ch * 8) = ra[i];
      *reinterpret_cast<uint4*>(Bs + (buf * WG_BK + row) * WG_ROW + ch * 8) = rb[i];
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed-read lane addressing: lane 4q+p of a 16-lane group -> row q, columns 4p..4p+3
  const int g = lane >> 4, q = (lane & 15) >> 2, pcol = (lane & 3) * 4;
  if (nsteps > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  for (int st = 0; st < nsteps; ++st) {
    const int buf = st & 1;
    if (st + 1 < nsteps) load(st + 1);
    const uint16_t* Ab = As + buf * WG_BK * WG_ROW;
    const uint16_t* Bb = Bs + buf * WG_BK * WG_ROW;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int col = wm * 32 + i * 16 + pcol;
        const s16x4 lo = tr_read(Ab + (krow(kk, g, 0) + q) * WG_ROW + col);
        const s16x4 hi = tr_read(Ab + (krow(kk, g, 1) + q) * WG_ROW + col);
        af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = wn * 32 + j * 16 + pcol;
        const s16x4 lo = tr_read(Bb + (krow(kk, g, 0) + q) * WG_ROW + col);
        const s16x4 hi = tr_read(Bb + (krow(kk, g, 1) + q) * WG_ROW + col);
        bfr[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (st + 1 < nsteps) store(buf ^ 1);
    __syncthreads();
  }

  // partial tile -> slab[split][co][k]  (C/D map: col = lane & 15, row = (lane >> 4) * 4 + r)
  float* sp = slab + (int64_t)split * Cout * (int64_t)tiles_n * WG_BN;
  const int ldk = tiles_n * WG_BN;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        const int k = k0 + wn * 32 + j * 16 + (lane & 15);
        if (co < Cout) sp[(int64_t)co * ldk + k] = acc[i][j][r];
      }
}

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

static FastDiv make_fastdiv(uint32_t d) {  // n / d == (mulhi(n, mul) + n) >> shift for n < 2^31
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

template <int S>
__global__ void __launch_bounds__(256)
conv_wgrad_buf_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x, float* __restrict__ slab,
                      uint16_t* __restrict__ dw, int accumulate, int NB, int H, int W, int Cin, int Ho, int Wo,
                      int Cout, int KW, int stride, int pad, int tiles_n, int ntiles, int splits, int per,
                      FastDiv fd_hw, FastDiv fd_w) {
  constexpr int LPS = 4;  // DMA instructions per thread per stage (2 dY rows + 2 X rows)
  static_assert(S >= 2 && S <= 4, "pipeline depth");
  __shared__ __attribute__((aligned(16))) uint16_t lds[S * 2 * WG_BK * 64];  // [S][dY|X][64 px][64 ch]
  const int wgid = blockIdx.x;
  const int split = wgid / ntiles, tile = wgid % ntiles;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int co0 = tm * WG_BM, k0 = tn * WG_BN;
  const int tap = k0 / Cin, ci0 = k0 % Cin;
  const int fr = tap / KW, fc = tap % KW;
  const int P = NB * Ho * Wo, HWo = Ho * Wo;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int steps_all = (P + WG_BK - 1) / WG_BK;
  const int s_begin = split * per, s_end = min(steps_all, s_begin + per);
  const int nsteps = max(0, s_end - s_begin);

  const __amdgpu_buffer_rsrc_t dyr =
      __builtin_amdgcn_make_buffer_rsrc((void*)dy, (short)0, (int)((int64_t)P * Cout * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, (int)((int64_t)NB * H * W * Cin * 2), 0x00020000);
  int rowi[2], chk[2];
  uint32_t a_off[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    rowi[i] = 32 * i + 8 * wid + (lane >> 3);
    chk[i] = (lane & 7) ^ wsw(rowi[i]);
    a_off[i] = co0 + chk[i] * 8 < Cout ? (uint32_t)((rowi[i] * Cout + co0 + chk[i] * 8) * 2) : kWgOOB;
  }
  auto issue = [&](int sl, int buf) {
    const int p0 = (s_begin + sl) * WG_BK;
    uint16_t* Ab = lds + buf * 2 * WG_BK * 64;
    uint16_t* Bb = Ab + WG_BK * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int p = p0 + rowi[i];
      const uint32_t va = p < P ? a_off[i] : kWgOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(dyr, (__attribute__((address_space(3))) void*)(Ab + (32 * i + 8 * wid) * 64),
                                               16, (int)va, (int)((uint32_t)p0 * Cout * 2), 0, 0);
      uint32_t vb = kWgOOB;
      if (p < P) {
        const int img = (int)fdiv((uint32_t)p, fd_hw), rem = p - img * HWo;
        const int ho = (int)fdiv((uint32_t)rem, fd_w), wo = rem - ho * Wo;
        const int hi = ho * stride - pad + fr, wi = wo * stride - pad + fc;
        if ((unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W)
          vb = (uint32_t)(((((int64_t)img * H + hi) * W + wi) * Cin + ci0 + chk[i] * 8) * 2);
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void*)(Bb + (32 * i + 8 * wid) * 64),
                                               16, (int)vb, 0, 0, 0);
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, q = (lane & 15) >> 2, pcol = (lane & 3) * 4;
  // swizzled element offset of (row, col), col a multiple of 4 inside one 16-B chunk
  auto lidx = [](int row, int col) { return row * 64 + (((col >> 3) ^ wsw(row)) << 3) + (col & 7); };

#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nsteps) issue(s, s);
  for (int st = 0; st < nsteps; ++st) {
    const int ahead = min(S - 2, nsteps - 1 - st);
    if (ahead >= 2) wait_vmcnt_wg<2 * LPS>();
    else if (ahead == 1) wait_vmcnt_wg<LPS>();
    else wait_vmcnt_wg<0>();
    __builtin_amdgcn_s_barrier();
    if (st + S - 1 < nsteps) issue(st + S - 1, (st + S - 1) % S);
    const uint16_t* Ab = lds + (st % S) * 2 * WG_BK * 64;
    const uint16_t* Bb = Ab + WG_BK * 64;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int col = wm * 32 + i * 16 + pcol;
        const s16x4 lo = tr_read(Ab + lidx(krow(kk, g, 0) + q, col));
        const s16x4 hi = tr_read(Ab + lidx(krow(kk, g, 1) + q, col));
        af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = wn * 32 + j * 16 + pcol;
        const s16x4 lo = tr_read(Bb + lidx(krow(kk, g, 0) + q, col));
        const s16x4 hi = tr_read(Bb + lidx(krow(kk, g, 1) + q, col));
        bfr[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }

  // epilogue through LDS: T[co][k] fp32 (row stride 68), then 8-column vectors per thread
  float* T = reinterpret_cast<float*>(lds);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        T[(wm * 32 + i * 16 + (lane >> 4) * 4 + r) * 68 + wn * 32 + j * 16 + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  const int ldk = tiles_n * WG_BN;
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    const int e = tid + v * 256, row = e >> 3, cv = e & 7;
    const int co = co0 + row;
    if (co >= Cout) continue;
    const float4* src = reinterpret_cast<const float4*>(T + row * 68 + cv * 8);
    const float4 a0 = src[0], a1 = src[1];
    const int64_t o = (int64_t)co * ldk + k0 + cv * 8;
    if (splits > 1) {
      float4* d = reinterpret_cast<float4*>(slab + (int64_t)split * Cout * ldk + o);
      d[0] = a0;
      d[1] = a1;
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

__global__ void __launch_bounds__(256)
wgrad_reduce_kernel(const float* __restrict__ slab, int splits, int64_t n, uint16_t* __restrict__ out,
                    int accumulate) {
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (e >= n) return;
  float4 a = *reinterpret_cast<const float4*>(slab + e);
  for (int s = 1; s < splits; ++s) {
    const float4 b = *reinterpret_cast<const float4*>(slab + (int64_t)s * n + e);
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  }
  if (accumulate) {  // add into the existing gradient (flat-buffer view), no separate add kernel
    const ushort4 o = *reinterpret_cast<const ushort4*>(out + e);
    a.x += bf16_to_f32(o.x); a.y += bf16_to_f32(o.y); a.z += bf16_to_f32(o.z); a.w += bf16_to_f32(o.w);
  }
  *reinterpret_cast<ushort4*>(out + e) = make_ushort4(f32_to_bf16(a.x), f32_to_bf16(a.y), f32_to_bf16(a.z),
                                                      f32_to_bf16(a.w));
}

int conv_wgrad_plan(int NB, int Ho, int Wo, int Cin, int Cout, int KH, int KW, int* splits_out) {
  // LDS-DMA kernel (tools/microbench/conv_tiles.py --wgrad on the ResNet-101 C4 shapes): split
  // the pixel reduction up to ~9 workgroups per CU while every split keeps >= 16 64-pixel steps
  const int P = NB * Ho * Wo;
  const int tiles = ((Cout + WG_BM - 1) / WG_BM) * (KH * KW * Cin / WG_BN);
  const int steps = (P + WG_BK - 1) / WG_BK;
  static const int min_steps = [] {  // A/B knob MXR_WGRAD_MIN_STEPS: 64-pixel steps kept per split
    const char* e = std::getenv("MXR_WGRAD_MIN_STEPS");
    return e ? std::max(1, std::atoi(e)) : 16;
  }();
  int splits = 1;
  while (splits < 64 && tiles * splits * 2 <= 2304 && steps / (splits * 2) >= min_steps) splits *= 2;
  *splits_out = splits;
  return splits;
}

int conv_wgrad(const uint16_t* dy, const uint16_t* x, uint16_t* dw, float* slab, int NB, int H, int W, int Cin,
               int Ho, int Wo, int Cout, int KH, int KW, int stride, int pad, int splits, int accumulate,
               hipStream_t st, int variant) {
  if (Cin % WG_BN != 0 || Cout % 8 != 0) return -1;
  const int P = NB * Ho * Wo;
  const int tiles_m = (Cout + WG_BM - 1) / WG_BM, tiles_n = KH * KW * Cin / WG_BN;
  const int ntiles = tiles_m * tiles_n;
  const int steps = (P + WG_BK - 1) / WG_BK;
  const int per = (steps + splits - 1) / splits;
  const int64_t n = (int64_t)Cout * KH * KW * Cin;
  const bool buf_ok = (int64_t)P * Cout * 2 < (int64_t)kWgOOB && (int64_t)NB * H * W * Cin * 2 < (int64_t)kWgOOB;
  if (variant == 0 && buf_ok) {
    conv_wgrad_buf_kernel<3><<<ntiles * splits, 256, 0, st>>>(dy, x, slab, dw, accumulate, NB, H, W, Cin, Ho, Wo, Cout,
                                                              KW, stride, pad, tiles_n, ntiles, splits, per,
                                                              make_fastdiv(Ho * Wo), make_fastdiv(Wo));
    if (splits > 1) wgrad_reduce_kernel<<<div_up((n + 3) / 4, 256), 256, 0, st>>>(slab, splits, n, dw, accumulate);
    return splits;
  }
  conv_wgrad_kernel<<<ntiles * splits, 256, 0, st>>>(dy, x, slab, NB, H, W, Cin, Ho, Wo, Cout, KW, stride, pad,
                                                     tiles_n, ntiles, splits, per);
  wgrad_reduce_kernel<<<div_up((n + 3) / 4, 256), 256, 0, st>>>(slab, splits, n, dw, accumulate);
  return splits;
}

}  // namespace mxr
