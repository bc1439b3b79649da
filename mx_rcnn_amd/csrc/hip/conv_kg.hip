// K-group implicit-GEMM convolution (tile codes 27-29): the buffer-resource LDS-DMA kernel of
// conv_igemm.hip with KG groups of four waves per 64x64 output tile, each group accumulating a
// contiguous 1/KG of the K range through its own LDS sub-ring, the partial tiles summed in the LDS
// epilogue (igemm_body.h: igemm_buf_body / igemm_epilogue_lds with KG > 1).
//
// Why: a batch-1 stage-3 conv (M = 4200 rows) gives one 64x64 tile per CU, and one tile's main
// loop is bound by the barrier-to-barrier round trip -- DMA issue, LDS fragment reads, the serial
// MFMA chain of four waves -- not by bytes or MFMA rate (profiles/r3_conv_study.md).  K groups put
// KG stages behind every barrier and 4*KG waves on the CU, so one group's fragment reads and waits
// overlap another group's MFMAs.  The fp32 triples (x3) run the fused one-pass body per group:
//   27: S = 3, KG = 2 (96 KB of LDS; x3 144 KB)   28: S = 2, KG = 2 (64 KB; x3 96 KB)
//   29: S = 2, KG = 4 (128 KB; not x3)
// The summation order differs from tile 23's (K split into group slices), so a tile choice moves
// results at the rounding level; the per-shape autotune (bindings.cpp) caches its choice.
#include "igemm_body.h"

namespace mxr {

template <int S, bool X2, bool BT, int KG, bool X3 = false>
__global__ void __launch_bounds__(256 * KG)
conv_igemm_kg_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, uint16_t* __restrict__ y, int NB,
                     int H, int W, int Cin, int Ho, int Wo, int Cout, int KH, int KW, int stride, int pad,
                     const ConvEpi ep, int tiles_n, int nwg, int ntiles, int splits, float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[S * KG * igemm_ring_stage<64, 64, BT, X3>()];
  igemm_buf_body<64, 64, S, false, X2, BT, KG, X3>(lds, blockIdx.x, x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW,
                                                   stride, pad, ep, tiles_n, nwg, ntiles, splits, slab);
}

template <int S, int KG>
static void launch_kg(const uint16_t* x, const uint16_t* w, uint16_t* y, int NB, int H, int W, int Cin, int Ho, int Wo,
                      int Cout, int KH, int KW, int stride, int pad, const ConvEpi& ep, int splits, float* slab,
                      hipStream_t st) {
  const int M = NB * Ho * Wo;
  const int tiles_n = (Cout + 63) / 64, ntiles = ((M + 63) / 64) * tiles_n, nwg = ntiles * splits;
#define MXR_KG(X_, B_, ...)                                                                                     \
  conv_igemm_kg_kernel<S, X_, B_, KG, ##__VA_ARGS__><<<nwg, 256 * KG, 0, st>>>(                                   \
      x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, tiles_n, nwg, ntiles, splits, slab)
  if constexpr (S * KG * igemm_ring_stage<64, 64, false, true>() * 2 <= 160 * 1024) {
    // fp32 triples: the fused one-pass form per group (all three planes per stage)
    if (ep.x3 && ep.bt) {
      MXR_KG(true, true, true);
      if (splits > 1) splitk_reduce_launch(slab, splits, M, Cout, ep, y, st);
      return;
    }
    if (ep.x3) {
      MXR_KG(true, false, true);
      if (splits > 1) splitk_reduce_launch(slab, splits, M, Cout, ep, y, st);
      return;
    }
  }
  if (ep.x2 && ep.bt) MXR_KG(true, true);
  else if (ep.x2) MXR_KG(true, false);
  else if (ep.bt) MXR_KG(false, true);
  else MXR_KG(false, false);
#undef MXR_KG
  if (splits > 1) splitk_reduce_launch(slab, splits, M, Cout, ep, y, st);
}

int conv_igemm_kg(int tile, const uint16_t* x, const uint16_t* w, uint16_t* y, int NB, int H, int W, int Cin, int Ho,
                  int Wo, int Cout, int KH, int KW, int stride, int pad, const ConvEpi& ep, int splits, float* slab,
                  hipStream_t st) {
  if (ep.f16 || Cout % 8 != 0 || Cin % BK != 0 || KH * KW > 64) return -1;
  if (ep.x3 && tile == 29) return -1;  // x3: four 24 KB-per-stage sub-rings do not fit the LDS
  switch (tile) {
    case 27: launch_kg<3, 2>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
    case 28: launch_kg<2, 2>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
    case 29: launch_kg<2, 4>(x, w, y, NB, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ep, splits, slab, st); break;
    default: return -1;
  }
  return tile;
}

}  // namespace mxr
