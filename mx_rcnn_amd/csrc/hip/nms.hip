// Bitmask greedy NMS for the proposal layer (kernel K6/K7;
// reference semantics `helper/processing/nms.py:4-38`: suppress j when IoU(i,j) > thresh,
// +1-pixel areas, boxes visited in descending score order).
//
// Stage 1 (nms_mask): one 64-thread workgroup (one wave64) per (row block, column block,
// image) of the upper triangle; lane i owns row i of the 64x64 tile and emits one 64-bit
// word of "j suppressed by i" bits -- the word width IS the wave width.
// Stage 2 (nms_reduce): one workgroup per image.  Wave 0 resolves a 64-box block
// serially in scalar registers (iterating only over KEPT boxes via find-first-set), then
// every thread ORs the kept rows into the LDS `removed` bitmap column-parallel.  The kept
// list lives in LDS and the kernel writes the final (post, 5) RoI block directly,
// including the reference's random pad (slot >= n_keep takes keep[floor(u*n_keep)]).
// Early exit once `post` boxes are kept.  No host synchronisation anywhere.
#include "common.h"
#include "../kernels.h"

namespace mxr {

__global__ void __launch_bounds__(64)
nms_mask_kernel(const float* __restrict__ boxes, const int32_t* __restrict__ n_valid, int P, int nb,
                float thresh, uint64_t* __restrict__ mask) {
  const int rb = blockIdx.y, cb = blockIdx.x, b = blockIdx.z;
  if (cb < rb) return;
  const int nv = n_valid[b];
  const int row0 = rb * 64, col0 = cb * 64;
  if (row0 >= nv || col0 >= nv) return;
  __shared__ float4 cbox[64];
  const float4* bx = reinterpret_cast<const float4*>(boxes) + (int64_t)b * P;
  const int tid = threadIdx.x;
  if (col0 + tid < nv) cbox[tid] = bx[col0 + tid];
  __syncthreads();
  const int i = row0 + tid;
  if (i >= nv) return;
  const float4 r = bx[i];
  const float rarea = (r.z - r.x + 1.f) * (r.w - r.y + 1.f);
  const int ncol = min(64, nv - col0);
  uint64_t bits = 0;
  const int jstart = (rb == cb) ? tid + 1 : 0;
  for (int j = jstart; j < ncol; ++j) {
    const float4 c = cbox[j];
    const float carea = (c.z - c.x + 1.f) * (c.w - c.y + 1.f);
    if (iou_plus1(r.x, r.y, r.z, r.w, rarea, c.x, c.y, c.z, c.w, carea) > thresh) bits |= (1ull << j);
  }
  mask[((int64_t)b * P + i) * nb + cb] = bits;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, lane);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_or64(uint64_t v) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo |= __shfl_xor(lo, o, 64);
    hi |= __shfl_xor(hi, o, 64);
  }
  return ((uint64_t)hi << 32) | lo;
}

// One workgroup (16 waves) per image.  Per 64-box block rb:
//  1. wave 0 resolves the block: lane i holds row i's diagonal word (boxes j > i it suppresses);
//     iterate kept <- cand & ~OR_{i in kept} diag_i to its fixpoint (a wave OR-reduction per
//     iteration; greedy NMS is the unique fixpoint, reached in "longest suppression chain"
//     iterations -- typically 1-3);
//  2. all threads OR the kept rows of block rb into the LDS `removed` bitmap of the later
//     column blocks.  Thread (jq, c) owns column block c (< 256) and rows jq*16..+15 of the
//     block; the 16 mask words for block rb+1 are PREFETCHED into registers while block rb is
//     being resolved, so each iteration's global-load latency overlaps the previous iteration.
__global__ void __launch_bounds__(1024)
nms_reduce_kernel(const float* __restrict__ boxes, const float* __restrict__ scores,
                  const int32_t* __restrict__ n_valid, const uint64_t* __restrict__ mask, int P, int nb, int post,
                  const float* __restrict__ rand_u, float* __restrict__ rois, float* __restrict__ out_scores,
                  int64_t* __restrict__ keep_idx, int32_t* __restrict__ n_keep_out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // single dynamic LDS region (Guideline 17): [kept_bits u64 | nkeep i32 | pad][removed nb*u64][keep_list]
  uint64_t& s_kept_bits = *reinterpret_cast<uint64_t*>(smem);
  int& s_nkeep = *reinterpret_cast<int*>(smem + 8);
  uint64_t* removed = reinterpret_cast<uint64_t*>(smem + 16);                            // nb words
  int32_t* keep_list = reinterpret_cast<int32_t*>(smem + 16 + ((nb * 8 + 15) / 16) * 16);  // post ints
  const int b = blockIdx.x, tid = threadIdx.x;
  const int nv = n_valid[b];
  const uint64_t* mb = mask + (int64_t)b * P * nb;
  for (int c = tid; c < nb; c += blockDim.x) removed[c] = 0;
  if (tid == 0) s_nkeep = 0;
  const int nbv = (nv + 63) / 64;
  const int jq = tid >> 8, cidx = tid & 255;
  // prefetch registers: this thread's 16 words of (row block rb, column cidx)
  uint64_t pf[16];
  auto fetch = [&](int rb) {
    const int nrow = min(64, P - rb * 64);
    const bool colok = (cidx > rb) && (cidx < nbv);
    // unconditional loads from clamped (always in-bounds) addresses, masked afterwards, so the
    // 16 loads issue back to back instead of branching around each one
    const int col = min(cidx, nb - 1);
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
      const int j = jq * 16 + jj;
      const uint64_t v = mb[(int64_t)min(rb * 64 + j, P - 1) * nb + col];
      pf[jj] = (colok && j < nrow) ? v : 0ull;
    }
  };
  uint64_t diag_next = 0;
  if (nbv > 0) {
    fetch(0);
    if (tid < 64) diag_next = (tid < nv) ? mb[(int64_t)tid * nb] : 0ull;
  }
  __syncthreads();
  for (int rb = 0; rb < nbv; ++rb) {
    if (s_nkeep >= post) break;  // uniform: read after a barrier
    if (tid < 64) {
      const int i = rb * 64 + tid;
      const uint64_t diag = diag_next;
      if (rb + 1 < nbv) {
        const int i2 = i + 64;
        diag_next = (i2 < nv) ? mb[(int64_t)i2 * nb + rb + 1] : 0ull;
      }
      const int nrow = min(64, nv - rb * 64);
      const uint64_t valid = (nrow == 64) ? ~0ull : ((1ull << nrow) - 1ull);
      const uint64_t cand = valid & ~removed[rb];
      uint64_t kept = cand;
      for (int it = 0; it < 65; ++it) {
        const uint64_t sup = wave_or64(((kept >> tid) & 1ull) ? diag : 0ull);
        const uint64_t next = cand & ~sup;
        if (next == kept) break;
        kept = next;
      }
      const int nk = s_nkeep;
      if (nk + __popcll(kept) > post) {  // keep only the lowest (post - nk) boxes of this block
        int need = post - nk;
        uint64_t trunc = 0, k = kept;
        while (need-- > 0 && k) { trunc |= k & (~k + 1); k &= k - 1; }
        kept = trunc;
      }
      if ((kept >> tid) & 1ull) keep_list[nk + __popcll(kept & ((1ull << tid) - 1ull))] = i;
      __builtin_amdgcn_wave_barrier();
      if (tid == 0) {
        s_kept_bits = kept;
        s_nkeep = nk + __popcll(kept);
      }
    }
    __syncthreads();
    const uint64_t kept = s_kept_bits;
    uint64_t acc = 0;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) acc |= ((kept >> (jq * 16 + jj)) & 1ull) ? pf[jj] : 0ull;
    if (acc) atomicOr(reinterpret_cast<unsigned long long*>(&removed[cidx]), (unsigned long long)acc);
    if (rb + 1 < nbv) fetch(rb + 1);
    __syncthreads();
  }
  const int nk = s_nkeep;
  if (tid == 0) n_keep_out[b] = nk;
  const float4* bx = reinterpret_cast<const float4*>(boxes) + (int64_t)b * P;
  for (int s = tid; s < post; s += blockDim.x) {
    int idx;
    if (s < nk) {
      idx = keep_list[s];
    } else if (nk > 0) {
      int r = (int)(rand_u[(int64_t)b * post + s] * nk);
      idx = keep_list[min(max(r, 0), nk - 1)];
    } else {
      idx = 0;
    }
    const float4 bb = bx[idx];
    float* ro = rois + ((int64_t)b * post + s) * 5;
    ro[0] = (float)b; ro[1] = bb.x; ro[2] = bb.y; ro[3] = bb.z; ro[4] = bb.w;
    out_scores[(int64_t)b * post + s] = scores[(int64_t)b * P + idx];
    keep_idx[(int64_t)b * post + s] = idx;
  }
}

void nms_mask(const float* boxes, const int32_t* n_valid, int B, int P, float thresh, uint64_t* mask,
              hipStream_t st) {
  if (B == 0 || P == 0) return;
  const int nb = div_up(P, 64);
  dim3 grid(nb, nb, B);
  nms_mask_kernel<<<grid, 64, 0, st>>>(boxes, n_valid, P, nb, thresh, mask);
}

void nms_reduce(const float* boxes, const float* scores, const int32_t* n_valid, const uint64_t* mask, int B,
                int P, int post, const float* rand_u, float* rois, float* out_scores, int64_t* keep_idx,
                int32_t* n_keep, hipStream_t st) {
  if (B == 0) return;
  const int nb = div_up(P, 64);
  const size_t lds = 16 + ((nb * 8 + 15) / 16) * 16 + (size_t)post * 4;
  nms_reduce_kernel<<<B, 1024, lds, st>>>(boxes, scores, n_valid, mask, P, nb, post, rand_u, rois, out_scores,
                                         keep_idx, n_keep);
}

}  // namespace mxr
