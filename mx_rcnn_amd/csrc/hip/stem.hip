// Stem convolution: the trunk's first layer, 3 input channels (ResNet bn_data -> conv0 7x7/2 ->
// bn0 -> relu, `rcnn/resnet.py:146-150`; VGG conv1_1 3x3/1 + bias + relu, `rcnn/symbol.py:11-13`).
//
// The MFMA implicit-GEMM conv kernels stream K in 64-channel blocks, which a 3-channel input does
// not have: K = KH*KW*3 (147 for conv0) is tiny, while M (one output pixel per row: 267K for an
// 800x1333 image) is the largest of the whole network.  So the stem gets its own kernel:
//   * one workgroup per (image, output row, 64-pixel strip), 4 waves, all 64 output channels;
//   * the strip's input patch (KH rows x (63*S+KW) columns x 3 channels) is read once into LDS
//     with the frozen input affine applied (bn_data; identity for VGG) and zero padding AFTER
//     the affine (the unfused path pads the normalised tensor), rounded to the storage type;
//   * the im2col A fragments are gathered from the LDS patch through a per-k offset table
//     (k = (fr*KW + fc)*3 + c, padded to a multiple of 32 with zeros); the B fragments are 16-B
//     reads of the packed [64][KP] filter (20 KB, L1/L2 resident: staging it per workgroup cost
//     2x the kernel time), and the frozen BN affines are folded from gamma / beta / moving
//     statistics in the kernel (no folded copies to keep in sync with the BN buffers);
//   * 16x16x32 MFMA, fp32 accumulation; epilogue y = relu?(acc*scale[n] + shift[n]) (the
//     frozen bn0, or the bias), staged through LDS and written as 16-B row vectors.
// It replaces three launches of the unfused path (input BN, vendor conv, BN+ReLU) with one.
#include "common.h"
#include "../kernels.h"

namespace mxr {

namespace {
typedef __bf16 sbf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 sf16x8 __attribute__((ext_vector_type(8)));
typedef float sf32x4 __attribute__((ext_vector_type(4)));

template <bool F16>
__device__ __forceinline__ sf32x4 stem_mfma(const uint4& a, const uint4& b, sf32x4 c) {
  if constexpr (F16) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(sf16x8, a), __builtin_bit_cast(sf16x8, b), c, 0,
                                                  0, 0);
  } else {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(sbf16x8, a), __builtin_bit_cast(sbf16x8, b), c,
                                                   0, 0, 0);
  }
}
}  // namespace

constexpr int STEM_BM = 64;   // output pixels per workgroup (one row strip)
constexpr int STEM_CO = 64;   // output channels (all of them)
constexpr int STEM_LDT = STEM_CO + 8;  // 16-bit row stride of the staged output tile

// NP = 2 (bf16x3 mode): x is the fp32 image, the patch is kept as hi / lo bf16 planes, the packed
// filter is an x2 pair (lo plane 64 * KP on), three MFMAs per fragment pair, y an x2 pair.
// NP = 3 (fp32 mode): patch and packed filter as (hi, mid, lo) planes in that logical order, six
// MFMAs per fragment pair, y an x3 triple (memory planes mid, hi, lo; common.h)
template <int KH, int KW, int S, bool F16, int NP = 1>
__global__ void __launch_bounds__(256)
stem_conv_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, const StemArgs a,
                 uint16_t* __restrict__ y, int N, int H, int W, int Ho, int Wo, int pad, int relu, int strips, int nwg) {
  constexpr int K = KH * KW * 3;
  constexpr int KP = (K + 31) / 32 * 32;
  constexpr int PW = (STEM_BM - 1) * S + KW;  // patch columns
  constexpr int code = F16 ? 2 : 1;
  constexpr bool X2 = NP >= 2, X3 = NP == 3;
  __shared__ __attribute__((aligned(16))) uint16_t patch[NP][KH * PW * 4];
  __shared__ int koff[KP];
  __shared__ float in_aff[6], out_aff[2 * STEM_CO];
  __shared__ __attribute__((aligned(16))) uint16_t T[NP][STEM_BM * STEM_LDT];

  // XCD-aware order: consecutive tiles (neighbouring output rows share KH-S input rows) on one XCD
  const int bid = blockIdx.x;
  const int q = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
  const int tile = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + bid / 8;
  const int strip = tile % strips, row = tile / strips;
  const int ho = row % Ho, n = row / Ho;
  const int wo0 = strip * STEM_BM;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // phase 1: folded affines, im2col offset table
  if (tid < 3) {
    float sc = 1.f, sh = 0.f;
    if (a.in_m) {
      sc = (a.in_fixg ? 1.f : a.in_g[tid]) * rsqrtf(a.in_v[tid] + a.in_eps);
      sh = a.in_b[tid] - a.in_m[tid] * sc;
    }
    in_aff[tid] = sc;
    in_aff[3 + tid] = sh;
  }
  if (tid < STEM_CO) {
    float sc = 1.f, sh = 0.f;
    if (a.out_m) {
      sc = (a.out_fixg ? 1.f : a.out_g[tid]) * rsqrtf(a.out_v[tid] + a.out_eps);
      sh = a.out_b[tid] - a.out_m[tid] * sc;
    } else if (a.bias) {
      sh = ld(a.bias, tid, a.bias_code);
    }
    out_aff[tid] = sc;
    out_aff[STEM_CO + tid] = sh;
  }
  for (int k = tid; k < KP; k += 256) {
    if (k < K) {
      const int tap = k / 3, c = k - 3 * tap, fr = tap / KW, fc = tap - fr * KW;
      koff[k] = (fr * PW + fc) * 4 + c;
    } else {
      koff[k] = -1;
    }
  }
  __syncthreads();

  // phase 2: the strip's input patch, input affine applied, zero padding after it
  const int hi0 = ho * S - pad, wi0 = wo0 * S - pad;
  const float s0 = in_aff[0], s1 = in_aff[1], s2 = in_aff[2];
  const float b0 = in_aff[3], b1 = in_aff[4], b2 = in_aff[5];
  for (int e = tid; e < KH * PW; e += 256) {
    const int r = e / PW, c = e - r * PW;
    const int hi = hi0 + r, wi = wi0 + c;
    uint2 v = make_uint2(0u, 0u), vl = make_uint2(0u, 0u), vm = make_uint2(0u, 0u);
    if ((unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W) {
      if constexpr (X3) {
        const float* px = reinterpret_cast<const float*>(x) + (((int64_t)n * H + hi) * W + wi) * 3;
        uint16_t h0, m0, l0, h1, m1, l1, h2, m2, l2;
        split3_bf16(px[0] * s0 + b0, h0, m0, l0);
        split3_bf16(px[1] * s1 + b1, h1, m1, l1);
        split3_bf16(px[2] * s2 + b2, h2, m2, l2);
        v = make_uint2((uint32_t)h0 | ((uint32_t)h1 << 16), h2);
        vm = make_uint2((uint32_t)m0 | ((uint32_t)m1 << 16), m2);
        vl = make_uint2((uint32_t)l0 | ((uint32_t)l1 << 16), l2);
      } else if constexpr (X2) {
        const float* px = reinterpret_cast<const float*>(x) + (((int64_t)n * H + hi) * W + wi) * 3;
        uint16_t h0, l0, h1, l1, h2, l2;
        split_bf16(px[0] * s0 + b0, h0, l0);
        split_bf16(px[1] * s1 + b1, h1, l1);
        split_bf16(px[2] * s2 + b2, h2, l2);
        v = make_uint2((uint32_t)h0 | ((uint32_t)h1 << 16), h2);
        vl = make_uint2((uint32_t)l0 | ((uint32_t)l1 << 16), l2);
      } else {
        const uint16_t* px = x + (((int64_t)n * H + hi) * W + wi) * 3;
        const uint32_t c0 = f32_to_h16(h16_to_f32(px[0], code) * s0 + b0, code);
        const uint32_t c1 = f32_to_h16(h16_to_f32(px[1], code) * s1 + b1, code);
        const uint32_t c2 = f32_to_h16(h16_to_f32(px[2], code) * s2 + b2, code);
        v = make_uint2(c0 | (c1 << 16), c2);
      }
    }
    *reinterpret_cast<uint2*>(patch[0] + e * 4) = v;
    if constexpr (X2) *reinterpret_cast<uint2*>(patch[NP - 1] + e * 4) = vl;
    if constexpr (X3) *reinterpret_cast<uint2*>(patch[1] + e * 4) = vm;
  }
  __syncthreads();

  // A row = this wave's pixel (lane & 15) of 16; k chunk = lane >> 4 (8 consecutive k)
  const int p = wave * 16 + (lane & 15);
  const int pbase = p * S * 4;
  const int chunk = lane >> 4;
  sf32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = sf32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KP / 32; ++ks) {
    const int k0 = ks * 32 + chunk * 8;
    uint4 af[NP];
#pragma unroll
    for (int pl = 0; pl < NP; ++pl) {
      uint32_t aw[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int o0 = koff[k0 + 2 * e], o1 = koff[k0 + 2 * e + 1];
        const uint32_t lo = o0 >= 0 ? patch[pl][o0 + pbase] : 0u;
        const uint32_t hi = o1 >= 0 ? patch[pl][o1 + pbase] : 0u;
        aw[e] = lo | (hi << 16);
      }
      af[pl] = make_uint4(aw[0], aw[1], aw[2], aw[3]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint4 bf = *reinterpret_cast<const uint4*>(w + (j * 16 + (lane & 15)) * KP + k0);
      acc[j] = stem_mfma<F16>(af[0], bf, acc[j]);
      if constexpr (X3) {  // logical planes (hi, mid, lo): hm + mh + hl + lh + mm
        const uint4 bm = *reinterpret_cast<const uint4*>(w + STEM_CO * KP + (j * 16 + (lane & 15)) * KP + k0);
        const uint4 bl = *reinterpret_cast<const uint4*>(w + 2 * STEM_CO * KP + (j * 16 + (lane & 15)) * KP + k0);
        acc[j] = stem_mfma<F16>(af[0], bm, acc[j]);
        acc[j] = stem_mfma<F16>(af[1], bf, acc[j]);
        acc[j] = stem_mfma<F16>(af[0], bl, acc[j]);
        acc[j] = stem_mfma<F16>(af[2], bf, acc[j]);
        acc[j] = stem_mfma<F16>(af[1], bm, acc[j]);
      } else if constexpr (X2) {  // A_hi B_lo + A_lo B_hi
        const uint4 bl = *reinterpret_cast<const uint4*>(w + STEM_CO * KP + (j * 16 + (lane & 15)) * KP + k0);
        acc[j] = stem_mfma<F16>(af[0], bl, acc[j]);
        acc[j] = stem_mfma<F16>(af[1], bf, acc[j]);
      }
    }
  }

  // epilogue: acc[j][r] is (pixel wave*16 + (lane>>4)*4 + r, channel j*16 + (lane&15))
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int co = j * 16 + (lane & 15);
    const float sc = out_aff[co], sh = out_aff[STEM_CO + co];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = acc[j][r] * sc + sh;
      if (relu) v = fmaxf(v, 0.f);
      if constexpr (X3) {  // T planes in memory order (mid, hi, lo)
        uint16_t h, m, l;
        split3_bf16(v, h, m, l);
        T[0][(wave * 16 + chunk * 4 + r) * STEM_LDT + co] = m;
        T[1][(wave * 16 + chunk * 4 + r) * STEM_LDT + co] = h;
        T[2][(wave * 16 + chunk * 4 + r) * STEM_LDT + co] = l;
      } else if constexpr (X2) {
        uint16_t h, l;
        split_bf16(v, h, l);
        T[0][(wave * 16 + chunk * 4 + r) * STEM_LDT + co] = h;
        T[NP - 1][(wave * 16 + chunk * 4 + r) * STEM_LDT + co] = l;
      } else {
        T[0][(wave * 16 + chunk * 4 + r) * STEM_LDT + co] = f32_to_h16(v, code);
      }
    }
  }
  __syncthreads();
  // 64 pixels x 64 channels = 512 vectors of 8 channels: two per thread
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    const int idx = tid + v * 256;
    const int px = idx >> 3, cv = idx & 7;
    const int wo = wo0 + px;
    if (wo < Wo) {
      const int64_t o = (((int64_t)n * Ho + ho) * Wo + wo) * STEM_CO + cv * 8;
      *reinterpret_cast<uint4*>(y + o) = *reinterpret_cast<const uint4*>(T[0] + px * STEM_LDT + cv * 8);
#pragma unroll
      for (int pl = 1; pl < NP; ++pl)  // further planes: one (N, Ho, Wo, 64) block apart
        *reinterpret_cast<uint4*>(y + pl * (int64_t)N * Ho * Wo * STEM_CO + o) =
            *reinterpret_cast<const uint4*>(T[pl] + px * STEM_LDT + cv * 8);
    }
  }
}

int stem_conv(const uint16_t* x, const uint16_t* w, const StemArgs& a, uint16_t* y, int N, int H, int W, int Ho,
              int Wo, int KH, int KW, int stride, int pad, int relu, int code, hipStream_t st) {
  const int strips = div_up(Wo, STEM_BM);
  const int64_t nwg64 = (int64_t)N * Ho * strips;
  if (nwg64 <= 0) return 0;
  if (nwg64 > (1 << 30)) return 2;
  const int nwg = (int)nwg64;
#define MXR_STEM(KH_, KW_, S_)                                                                                   \
  if (KH == KH_ && KW == KW_ && stride == S_) {                                                                \
    if (code == 4)                                                                                             \
      stem_conv_kernel<KH_, KW_, S_, false, 3><<<nwg, 256, 0, st>>>(x, w, a, y, N, H, W, Ho, Wo, pad, relu,        \
                                                                    strips, nwg);                               \
    else if (code == 3)                                                                                        \
      stem_conv_kernel<KH_, KW_, S_, false, 2><<<nwg, 256, 0, st>>>(x, w, a, y, N, H, W, Ho, Wo, pad, relu,        \
                                                                    strips, nwg);                               \
    else if (code == 2)                                                                                        \
      stem_conv_kernel<KH_, KW_, S_, true><<<nwg, 256, 0, st>>>(x, w, a, y, N, H, W, Ho, Wo, pad, relu, strips, nwg); \
    else                                                                                                       \
      stem_conv_kernel<KH_, KW_, S_, false><<<nwg, 256, 0, st>>>(x, w, a, y, N, H, W, Ho, Wo, pad, relu, strips, nwg); \
    return 0;                                                                                                  \
  }
  MXR_STEM(7, 7, 2)
  MXR_STEM(3, 3, 1)
#undef MXR_STEM
  return 1;  // unsupported geometry
}

}  // namespace mxr
