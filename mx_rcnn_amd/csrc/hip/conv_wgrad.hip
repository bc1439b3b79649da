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
#include "wgrad_body.h"

namespace mxr {

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

template <int S, bool X2 = false, bool X3 = false, bool SGD = false>
__global__ void __launch_bounds__(256) conv_wgrad_buf_kernel(WgradParams p) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[S * wgrad_ring_stage<X3>()];  // [S][dY|X][64 px][64 ch] (+ lo)
  wgrad_buf_body<S, X2, 1, X3, SGD>(lds, blockIdx.x, p);
}

__global__ void __launch_bounds__(256)
wgrad_reduce_kernel(const float* __restrict__ slab, int splits, int64_t n, uint16_t* __restrict__ out,
                    int accumulate, float* __restrict__ outf) {
  wgrad_reduce_body((int)blockIdx.x, slab, splits, n, out, accumulate, outf);
}

WgradParams wgrad_params(const uint16_t* dy, const uint16_t* x, uint16_t* dw, float* slab, int NB, int H, int W,
                         int Cin, int Ho, int Wo, int Cout, int KH, int KW, int stride, int pad, int splits,
                         int accumulate) {
  WgradParams p;
  p.dy = dy; p.x = x; p.slab = slab; p.dw = dw; p.accumulate = accumulate;
  p.NB = NB; p.H = H; p.W = W; p.Cin = Cin; p.Ho = Ho; p.Wo = Wo; p.Cout = Cout; p.KW = KW;
  p.stride = stride; p.pad = pad;
  p.tiles_n = KH * KW * Cin / WG_BN;
  p.ntiles = ((Cout + WG_BM - 1) / WG_BM) * p.tiles_n;
  p.splits = splits;
  const int steps = (NB * Ho * Wo + WG_BK - 1) / WG_BK;
  p.per = (steps + splits - 1) / splits;
  p.nwg = p.ntiles * splits;
  p.fd_hw = make_fastdiv(Ho * Wo);
  p.fd_w = make_fastdiv(Wo);
  return p;
}

void wgrad_reduce(const float* slab, int splits, int64_t n, uint16_t* dw, int accumulate, hipStream_t st,
                  float* dwf) {
  wgrad_reduce_kernel<<<div_up((n + 3) / 4, 256), 256, 0, st>>>(slab, splits, n, dw, accumulate, dwf);
}

void wgrad_reduce_run(const float* slab, int splits, int64_t n, uint16_t* dw, hipStream_t st, float* dwf) {
  wgrad_reduce(slab, splits, n, dw, 1, st, dwf);
}

int conv_wgrad_plan(int NB, int Ho, int Wo, int Cin, int Cout, int KH, int KW, int* splits_out, int planes) {
  // LDS-DMA kernel (tools/microbench/conv_tiles.py --wgrad on the ResNet-101 C4 shapes): split
  // the pixel reduction up to ~9 workgroups per CU while every split keeps >= 16 64-pixel steps
  const int P = NB * Ho * Wo;
  const int tiles = ((Cout + WG_BM - 1) / WG_BM) * (KH * KW * Cin / WG_BN);
  const int steps = (P + WG_BK - 1) / WG_BK;
  // 64-pixel steps kept per split (A/B knob MXR_WGRAD_MIN_STEPS): 8 with multi-plane operands, whose
  // steps are 2-3x longer (fp32 headline 75.6 vs 75.0 img/s, bf16x3 101.7 vs 100.9), 16 for bf16
  // (152.1 vs 150.3)
  static const int env_steps = [] {
    const char* e = std::getenv("MXR_WGRAD_MIN_STEPS");
    return e ? std::max(1, std::atoi(e)) : 0;
  }();
  const int min_steps = env_steps > 0 ? env_steps : (planes > 0 ? 8 : 16);
  int splits = 1;
  while (splits < 64 && tiles * splits * 2 <= 2304 && steps / (splits * 2) >= min_steps) splits *= 2;
  *splits_out = splits;
  return splits;
}

int conv_wgrad(const uint16_t* dy, const uint16_t* x, uint16_t* dw, float* slab, int NB, int H, int W, int Cin,
               int Ho, int Wo, int Cout, int KH, int KW, int stride, int pad, int splits, int accumulate,
               hipStream_t st, int variant, const WgradX2& x2) {
  if (Cin % WG_BN != 0 || Cout % 8 != 0) return -1;
  const int P = NB * Ho * Wo;
  const int tiles_m = (Cout + WG_BM - 1) / WG_BM, tiles_n = KH * KW * Cin / WG_BN;
  const int ntiles = tiles_m * tiles_n;
  const int steps = (P + WG_BK - 1) / WG_BK;
  const int per = (steps + splits - 1) / splits;
  const int64_t n = (int64_t)Cout * KH * KW * Cin;
  const bool buf_ok = (int64_t)P * Cout * 2 < (int64_t)kWgOOB && (int64_t)NB * H * W * Cin * 2 < (int64_t)kWgOOB;
  if (x2.x2 && !(variant == 0 && buf_ok)) return -1;  // pairs: the LDS-DMA kernel only
  if (x2.x2 && ((int64_t)P * Cout * 2 + (x2.x3 ? 2 : 1) * (int64_t)x2.pdy >= (int64_t)kWgOOB ||
                (int64_t)NB * H * W * Cin * 2 + (x2.x3 ? 2 : 1) * (int64_t)x2.px >= (int64_t)kWgOOB))
    return -1;  // every plane inside the 32-bit buffer offsets
  if (variant == 0 && buf_ok) {
    WgradParams p = wgrad_params(dy, x, dw, slab, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, splits, accumulate);
    p.x2 = x2.x2;
    p.x3 = x2.x3;
    p.x2_pdy = x2.pdy;
    p.x2_px = x2.px;
    p.dwf = x2.dwf;
    if (p.x3)
      conv_wgrad_buf_kernel<3, true, true><<<ntiles * splits, 256, 0, st>>>(p);  // fp32 triples: fused one pass
    else if (p.x2)
      conv_wgrad_buf_kernel<3, true><<<ntiles * splits, 256, 0, st>>>(p);
    else
      conv_wgrad_buf_kernel<3><<<ntiles * splits, 256, 0, st>>>(p);
    if (splits > 1)
      wgrad_reduce_kernel<<<div_up((n + 3) / 4, 256), 256, 0, st>>>(slab, splits, n, dw, accumulate, x2.dwf);
    return splits;
  }
  conv_wgrad_kernel<<<ntiles * splits, 256, 0, st>>>(dy, x, slab, NB, H, W, Cin, Ho, Wo, Cout, KW, stride, pad,
                                                     tiles_n, ntiles, splits, per);
  wgrad_reduce_kernel<<<div_up((n + 3) / 4, 256), 256, 0, st>>>(slab, splits, n, dw, accumulate, nullptr);
  return splits;
}

int conv_wgrad_sgd(const uint16_t* dy, const uint16_t* x, int NB, int H, int W, int Cin, int Ho, int Wo, int Cout, int KH,
                   int KW, int stride, int pad, hipStream_t st, const WgradX2& x2, const WgradSgd& sgd) {
  if (Cin % WG_BN != 0 || Cout % 8 != 0 || !sgd.w || !sgd.mom || !sgd.lr) return -1;
  const int P = NB * Ho * Wo;
  const bool buf_ok = (int64_t)P * Cout * 2 < (int64_t)kWgOOB && (int64_t)NB * H * W * Cin * 2 < (int64_t)kWgOOB;
  if (!buf_ok) return -1;
  if (x2.x2 && ((int64_t)P * Cout * 2 + (x2.x3 ? 2 : 1) * (int64_t)x2.pdy >= (int64_t)kWgOOB ||
                (int64_t)NB * H * W * Cin * 2 + (x2.x3 ? 2 : 1) * (int64_t)x2.px >= (int64_t)kWgOOB))
    return -1;
  WgradParams p = wgrad_params(dy, x, nullptr, nullptr, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, 1, 0);
  p.x2 = x2.x2;
  p.x3 = x2.x3;
  p.x2_pdy = x2.pdy;
  p.x2_px = x2.px;
  p.sgd_w = sgd.w;
  p.sgd_mom = sgd.mom;
  p.sgd_wb = sgd.wb;
  p.sgd_plane = sgd.plane;
  p.sgd_x3 = sgd.x3;
  p.sgd_gbf16 = sgd.gbf16;
  p.sgd_lr = sgd.lr;
  p.sgd_mu = sgd.mu;
  p.sgd_wd = sgd.wd;
  p.sgd_rescale = sgd.rescale;
  p.sgd_clip = sgd.clip;
  if (p.x3)
    conv_wgrad_buf_kernel<3, true, true, true><<<p.ntiles, 256, 0, st>>>(p);
  else if (p.x2)
    conv_wgrad_buf_kernel<3, true, false, true><<<p.ntiles, 256, 0, st>>>(p);
  else
    conv_wgrad_buf_kernel<3, false, false, true><<<p.ntiles, 256, 0, st>>>(p);
  return 1;
}

}  // namespace mxr
