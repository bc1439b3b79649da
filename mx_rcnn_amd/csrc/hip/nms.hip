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

__global__ void __launch_bounds__(1024)
nms_reduce_kernel(const float* __restrict__ boxes, const float* __restrict__ scores,
                  const int32_t* __restrict__ n_valid, const uint64_t* __restrict__ mask, int P, int nb, int post,
                  const float* __restrict__ rand_u, float* __restrict__ rois, float* __restrict__ out_scores,
                  int64_t* __restrict__ keep_idx, int32_t* __restrict__ n_keep_out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // single dynamic LDS region (Guideline 17): [kept_bits u64 | nkeep i32 | pad][removed nb*u64][keep_list]
  uint64_t& s_kept_bits = *reinterpret_cast<uint64_t*>(smem);
  int& s_nkeep = *reinterpret_cast<int*>(smem + 8);
  uint64_t* removed = reinterpret_cast<uint64_t*>(smem + 16);                          // nb words
  int32_t* keep_list = reinterpret_cast<int32_t*>(smem + 16 + ((nb * 8 + 15) / 16) * 16);  // post ints
  const int b = blockIdx.x, tid = threadIdx.x;
  const int nv = n_valid[b];
  const uint64_t* mb = mask + (int64_t)b * P * nb;
  for (int c = tid; c < nb; c += blockDim.x) removed[c] = 0;
  if (tid == 0) s_nkeep = 0;
  __syncthreads();
  const int nbv = (nv + 63) / 64;
  for (int rb = 0; rb < nbv; ++rb) {
    if (s_nkeep >= post) break;  // uniform: read after a barrier
    if (tid < 64) {
      // Resolve the 64-box block without a serial scalar chain: lane j holds COLUMN j of the
      // block's diagonal 64x64 suppression tile (bit i set when box i suppresses box j), and
      // the wave iterates kept <- {j candidate : no kept i < j suppresses j} to its fixpoint.
      // Greedy NMS is the unique fixpoint (membership of j depends only on i < j), and the
      // iteration count is the longest suppression chain in the block (usually a few), not
      // the number of kept boxes.
      const int i = rb * 64 + tid;
      const uint64_t diag = (i < nv) ? mb[(int64_t)i * nb + rb] : 0ull;
      const int nrow = min(64, nv - rb * 64);
      const uint64_t valid = (nrow == 64) ? ~0ull : ((1ull << nrow) - 1ull);
      const uint64_t cand = valid & ~removed[rb];
      uint64_t col = 0;
      for (int r = 0; r < 64; ++r) {
        const uint64_t row = readlane64(diag, r);
        col |= ((row >> tid) & 1ull) << r;
      }
      uint64_t kept = cand;
      for (int it = 0; it < 65; ++it) {
        const bool keep_me = ((cand >> tid) & 1ull) && !(col & kept);
        const uint64_t next = __ballot(keep_me);
        if (next == kept) break;
        kept = next;
      }
      int nk = s_nkeep;
      const int cnt = __popcll(kept);
      if (nk + cnt > post) {  // keep only the lowest (post - nk) boxes of this block
        int need = post - nk;
        uint64_t trunc = 0, k = kept;
        while (need-- > 0 && k) { trunc |= k & (~k + 1); k &= k - 1; }
        kept = trunc;
      }
      if ((kept >> tid) & 1ull) {
        const int pos = nk + __popcll(kept & ((1ull << tid) - 1ull));
        keep_list[pos] = i;
      }
      __builtin_amdgcn_wave_barrier();
      if (tid == 0) {
        s_kept_bits = kept;
        s_nkeep = nk + __popcll(kept);
      }
    }
    __syncthreads();
    const uint64_t kept = s_kept_bits;
    if (kept && s_nkeep < post) {
      // column-parallel OR of the kept rows: 4 thread groups each own 16 of the block's 64
      // rows; loads are unconditional (masked after) so hipcc keeps 16 independent loads in
      // flight instead of branching around each one
      const int jq = tid >> 8, cidx = tid & 255;
      const int nrow = min(64, P - rb * 64);
      for (int c = rb + 1 + cidx; c < nbv; c += 256) {
        uint64_t acc = 0;
        const uint64_t* col = mb + (int64_t)(rb * 64) * nb + c;
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
          const int j = jq * 16 + jj;
          if (j < nrow) {
            const uint64_t v = col[(int64_t)j * nb];
            acc |= ((kept >> j) & 1ull) ? v : 0ull;
          }
        }
        if (acc) atomicOr(reinterpret_cast<unsigned long long*>(&removed[c]), (unsigned long long)acc);
      }
    }
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
