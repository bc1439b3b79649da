// Bitmask greedy NMS for the proposal layer (kernel K6/K7;
// reference semantics `helper/processing/nms.py:4-38`: suppress j when IoU(i,j) > thresh,
// +1-pixel areas, boxes visited in descending score order).
//
// The suppression matrix is stored TRANSPOSED, one 64-bit word per (row block, box):
//   maskT[rb][j] bit i  <=>  box rb*64+i (higher score, rb*64+i < j) suppresses box j,
// with the columns of each row block PAIRED: the words of boxes cb*64+l and (cb^1)*64+l sit
// side by side (word index (cb>>1)*128 + 2l + (cb&1)), so one 16-B load per lane fetches lane l's
// words of two column blocks.  The reducer streams the whole upper triangle through ONE CU,
// whose address path costs about the same per wave-load at 8 and 16 B per lane: 16-B loads
// halve the wave-loads (and the per-iteration time, which that path sets).
// With lane = box j, "is j suppressed by any kept box of block rb" is a single
// `ballot((maskT[rb][j] & kept[rb]) != 0)` -- the 64-bit word width IS the wave width, so the
// serial part of greedy NMS runs on wave-wide bit operations instead of shuffles or atomics.
//
// Stage 1 (nms_mask): 256-thread workgroup per (4 column blocks, row block, image); lane = box
// j, the 64 row boxes sit in LDS.  Rows of maskT are contiguous in j (coalesced stores).
// Stage 2 (nms_reduce): one 1024-thread workgroup per image, ONE barrier per 64-box block t:
//   wave 0    resolves block t: cand = valid & ~(removed[t] | ballot(maskT[t-1][j] & kept[t-1]))
//             then the in-block fixpoint kept = cand & ~ballot(maskT[t][j] & kept) (the unique
//             greedy fixpoint; chain-length iterations of ~5 instructions each);
//   waves 1-15 fold block t-1's kept rows into removed[c] for every column block c >= t+1
//             (one ballot per column block, each c owned by one wave -> plain LDS RMW);
//   the words for the next block are prefetched into registers one iteration ahead, so the
//   per-block critical path is LDS + ballots + one barrier, never a global-memory round trip.
// The kept list lives in LDS; the kernel writes the final (post, 5) RoI block directly,
// including the reference's random pad (slot >= n_keep takes keep[floor(u*n_keep)]).  Early
// exit once `post` boxes are kept.  No host synchronisation anywhere.
//   That reducer streams the whole 9 MB triangle (P = 12000) through one CU at that CU's share of
//   the memory bandwidth (~270 us); it stays as the MXR_NMS_SERIAL=1 path.
// Stage 2, default (nms_reduce_mc): a chain of workgroups, one per PER = 8 column blocks, so the
// triangle is read by ceil(nb / 8) CUs and only the 64-box resolve stays serial:
//   phase A  every wave owns one column block c of its workgroup and folds the kept rows r < lo
//            (published by earlier workgroups) into its removed word, polling the per-block
//            records 16 rows at a time; the mask words of a chunk are loaded before its poll;
//   phase B  wave 0 resolves the workgroup's own blocks in order from LDS only (the PER x PER own
//            triangle of mask words is staged there during phase A), publishing each block's
//            kept word and running count as it goes -- no barrier, no global round trip inside;
//   every workgroup then writes the output rows of its own kept boxes, and the one that resolves
//   the last needed block (count reaches `post`, or the last valid block) adds the random pad.
//   Measured (MXR_NMS_PROBE timeline, 12000 boxes): ~0.35 us per block in phase B, ~2 us per
//   hand-off between workgroups; 8 blocks per workgroup beat 16 (fewer folds per block).
// A published record is two 64-bit words {kept lo/hi 32 bits | (count + 1) << 32}: each word is
// stored and loaded whole (relaxed, agent scope), a nonzero upper half means "written", so a
// reader never needs an ordering fence between the two.  The records are zeroed by nms_mask and
// again by the last workgroup to finish (a per-image exit counter), so a mask buffer may be
// reduced more than once.  A workgroup only ever waits for lower-numbered workgroups of its image,
// which are dispatched before it, and every poll gives up after NMSC_SPIN empty rounds (the
// output then reports n_keep = -1) -- the kernel always drains.
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "../kernels.h"

namespace mxr {

constexpr int NMS_HELPERS = 15;  // helper waves in the 1024-thread reducer
constexpr int NMS_PF = 7;        // prefetched column-block PAIRS per helper lane (15 * 7 = 105 pairs
                                 // >= 188 blocks of the 12000-box training NMS; farther pairs take
                                 // plain loads)

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

// words per row block (column blocks padded to an even count)
__host__ __device__ __forceinline__ int64_t nms_row_words(int nb) { return (int64_t)((nb + 1) >> 1) * 128; }
// index of lane l's word of column block cb within a row block
__device__ __forceinline__ int64_t nms_col(int cb, int l) { return (int64_t)(cb >> 1) * 128 + l * 2 + (cb & 1); }

__global__ void __launch_bounds__(256)
nms_mask_kernel(const float* __restrict__ boxes, const int32_t* __restrict__ n_valid, int P, int nb,
                float thresh, uint64_t* __restrict__ maskT, uint64_t* __restrict__ rec) {
  const int rb = blockIdx.y, b = blockIdx.z;
  if (blockIdx.x == 0) {  // clear the multi-workgroup reducer's block records and exit counter
    if (threadIdx.x < 2) rec[((int64_t)b * nb + rb) * 2 + threadIdx.x] = 0ull;
    if (rb == 0 && threadIdx.x == 2) rec[(int64_t)gridDim.z * nb * 2 + b] = 0ull;
  }
  if (blockIdx.x * 4 + 3 < rb) return;  // whole group below the diagonal
  const int cb = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int nv = min(n_valid[b], P);  // a count above P must not walk past the image's boxes
  const int row0 = rb * 64;
  const int64_t Pp = nms_row_words(nb);
  __shared__ float4 rbox[64];
  __shared__ float rarea[64];
  const float4* bx = reinterpret_cast<const float4*>(boxes) + (int64_t)b * P;
  if (threadIdx.x < 64) {
    const int i = row0 + threadIdx.x;
    const float4 r = i < nv ? bx[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    rbox[threadIdx.x] = r;
    rarea[threadIdx.x] = (r.z - r.x + 1.f) * (r.w - r.y + 1.f);
  }
  __syncthreads();
  if (cb < rb || cb >= nb) return;
  const int j = cb * 64 + lane;
  uint64_t bits = 0;
  if (j < nv) {
    const float4 c = bx[j];
    const float carea = (c.z - c.x + 1.f) * (c.w - c.y + 1.f);
    const int iend = min(64, j - row0);  // rows i with row0 + i < j (all < nv since j < nv)
    for (int i = 0; i < iend; ++i) {
      const float4 r = rbox[i];
      if (iou_plus1(r.x, r.y, r.z, r.w, rarea[i], c.x, c.y, c.z, c.w, carea) > thresh) bits |= (1ull << i);
    }
  }
  maskT[((int64_t)b * nb + rb) * Pp + nms_col(cb, lane)] = bits;
}

// Output row s of image b: RoI [b, box], its score and index.
__device__ __forceinline__ void nms_write_row(const float* __restrict__ boxes, const float* __restrict__ scores, int b,
                                              int P, int post, int s, int idx, float* __restrict__ rois,
                                              float* __restrict__ out_scores, int64_t* __restrict__ keep_idx) {
  idx = min(max(idx, 0), P - 1);  // never read outside the image's box block
  const float4 bb = reinterpret_cast<const float4*>(boxes)[(int64_t)b * P + idx];
  float* ro = rois + ((int64_t)b * post + s) * 5;
  ro[0] = (float)b; ro[1] = bb.x; ro[2] = bb.y; ro[3] = bb.z; ro[4] = bb.w;
  out_scores[(int64_t)b * post + s] = scores[(int64_t)b * P + idx];
  keep_idx[(int64_t)b * post + s] = idx;
}

// Output slots [s0, post) (the whole workgroup; keep_list holds nk entries and is visible to every
// thread): slot s < nk takes keep[s], later slots the reference's random pad keep[floor(u * nk)].
__device__ __forceinline__ void nms_write_out(const float* __restrict__ boxes, const float* __restrict__ scores, int b,
                                              int P, int post, int nk, int s0, const int32_t* keep_list,
                                              const float* __restrict__ rand_u, float* __restrict__ rois,
                                              float* __restrict__ out_scores, int64_t* __restrict__ keep_idx,
                                              int32_t* __restrict__ n_keep_out) {
  if (threadIdx.x == 0) n_keep_out[b] = nk;
  for (int s = s0 + threadIdx.x; s < post; s += blockDim.x) {
    int idx;
    if (s < nk) {
      idx = keep_list[s];
    } else if (nk > 0) {
      int r = (int)(rand_u[(int64_t)b * post + s] * nk);
      idx = keep_list[min(max(r, 0), nk - 1)];
    } else {
      idx = 0;
    }
    nms_write_row(boxes, scores, b, P, post, s, idx, rois, out_scores, keep_idx);
  }
}

__global__ void __launch_bounds__(1024)
nms_reduce_kernel(const float* __restrict__ boxes, const float* __restrict__ scores,
                  const int32_t* __restrict__ n_valid, const uint64_t* __restrict__ maskT, int P, int nb, int post,
                  const float* __restrict__ rand_u, float* __restrict__ rois, float* __restrict__ out_scores,
                  int64_t* __restrict__ keep_idx, int32_t* __restrict__ n_keep_out, int32_t* keep_ws,
                  int fallback = 0, int32_t* gave_up = nullptr) {
  // fallback: launched behind the multi-workgroup reducer, which wrote n_keep = -1 for an image
  // whose chain gave up; only those images are redone here (the rest exit at once), and each one
  // redone adds 1 to *gave_up (the caller's give-up counter, if any)
  if (fallback) {
    if (n_keep_out[blockIdx.x] != -1) return;  // uniform per workgroup
    if (threadIdx.x == 0 && gave_up) __hip_atomic_fetch_add(gave_up, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // single dynamic LDS region (Guideline 17): [nkeep 2 x i32 | pad][removed nb u64][keptw nb u64][keep_list post i32];
  // the keep list moves to global memory (keep_ws, (B, post) int32) when it does not fit in LDS
  // (post = all boxes of a > 32K-box image)
  // The kept count is double-buffered: iteration t reads s_nk[t & 1] (written in t-1) and wave 0
  // writes s_nk[(t + 1) & 1].  A single slot let a late helper wave read wave 0's iteration-t
  // update at the top of iteration t, break out of the loop alone and skip the barrier the
  // rest of the workgroup waits on (reached whenever `post` boxes are kept, i.e. every
  // test-time call with post = 300).
  int* s_nk = reinterpret_cast<int*>(smem);
  uint64_t* removed = reinterpret_cast<uint64_t*>(smem + 16);
  uint64_t* keptw = removed + nb;
  const int b = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  int32_t* keep_list = keep_ws ? keep_ws + (int64_t)b * post : reinterpret_cast<int32_t*>(keptw + nb);
  const int nv = min(n_valid[b], P);
  const int64_t Pp = nms_row_words(nb);
  const uint64_t* mb = maskT + (int64_t)b * nb * Pp;
  for (int c = tid; c < nb; c += blockDim.x) {
    removed[c] = 0;
    keptw[c] = 0;
  }
  if (tid < 2) s_nk[tid] = 0;
  const int nbv = (nv + 63) / 64;
  // wave 0: words of block t (diag = maskT[t][j], wprev = maskT[t-1][j]); helpers: the column
  // block pairs of the next iteration.  Every prefetch is loaded into the variable it is
  // consumed from, AFTER the consumption: a loop-carried copy (x = x_next) would make the
  // compiler wait for the prefetch at the end of every iteration.
  uint64_t diag = 0, wprev = 0;
  u64x2 pf[NMS_PF];
#pragma unroll
  for (int k = 0; k < NMS_PF; ++k) pf[k] = u64x2{0ull, 0ull};
  if (wave == 0 && nbv > 0) diag = mb[nms_col(0, lane)];
  __syncthreads();
  int t = 0;
  for (; t < nbv; ++t) {
    if (s_nk[t & 1] >= post) break;  // uniform: written before the last barrier, not rewritten until the next
    if (wave == 0) {
      const int j = t * 64 + lane;
      const uint64_t kp = t > 0 ? keptw[t - 1] : 0ull;
      const uint64_t sp = __ballot((wprev & kp) != 0ull);
      const int nrow = min(64, nv - t * 64);
      const uint64_t valid = nrow >= 64 ? ~0ull : ((1ull << nrow) - 1ull);
      const uint64_t cand = valid & ~(removed[t] | sp);
      uint64_t kept = cand;
      for (int it = 0; it < 65; ++it) {
        const uint64_t sup = __ballot((diag & kept) != 0ull);
        const uint64_t next = cand & ~sup;
        if (next == kept) break;
        kept = next;
      }
      // prefetch block t+1 (clamped to an in-range word on the last block)
      const int tn = min(t + 1, nb - 1);
      diag = mb[(int64_t)tn * Pp + nms_col(tn, lane)];
      wprev = mb[(int64_t)t * Pp + nms_col(tn, lane)];
      const int nk = s_nk[t & 1];
      if (nk + __popcll(kept) > post) {  // keep only the lowest (post - nk) boxes of this block
        int need = post - nk;
        uint64_t trunc = 0, k = kept;
        while (need-- > 0 && k) {
          trunc |= k & (~k + 1);
          k &= k - 1;
        }
        kept = trunc;
      }
      if ((kept >> lane) & 1ull) keep_list[nk + __popcll(kept & ((1ull << lane) - 1ull))] = j;
      if (lane == 0) {
        keptw[t] = kept;
        s_nk[(t + 1) & 1] = nk + __popcll(kept);
      }
    } else {
      const int h = wave - 1;
      // vmcnt(0) through the builtin, which the compiler's wait-count pass sees: it then knows the
      // previous iteration's prefetch has landed, and issues this iteration's guarded prefetch
      // loads back to back instead of draining before each (the skipped-slot path could otherwise
      // still have a load in flight into the same registers).
      __builtin_amdgcn_s_waitcnt(0x0F70);  // gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15 (no wait)
      if (t >= 1) {
        const uint64_t kp = keptw[t - 1];
        if (kp) {
          // fold kept rows of block t-1 into columns c >= t+1 (c = t is wave 0's, via wprev);
          // pair q holds columns 2q, 2q+1; the first pair may start at column t
          const int q0 = (t + 1) >> 1;
#pragma unroll
          for (int k = 0; k < NMS_PF; ++k) {
            const int c0 = 2 * (q0 + h + NMS_HELPERS * k);
            if (c0 >= t + 1 && c0 < nbv) {
              const uint64_t bits = __ballot((pf[k].x & kp) != 0ull);
              // ds_or_b64 without return: no LDS round trip on the helper's path
              if (lane == 0 && bits) atomicOr(reinterpret_cast<unsigned long long*>(&removed[c0]), bits);
            }
            if (c0 + 1 < nbv) {
              const uint64_t bits = __ballot((pf[k].y & kp) != 0ull);
              if (lane == 0 && bits) atomicOr(reinterpret_cast<unsigned long long*>(&removed[c0 + 1]), bits);
            }
          }
          // pairs beyond the prefetch window (only when P > ~13K, e.g. the alternate-training
          // proposal dump with pre-NMS = all anchors): plain loads of row block t-1, same fold
          for (int q = q0 + h + NMS_HELPERS * NMS_PF; 2 * q < nbv; q += NMS_HELPERS) {
            const u64x2 wv = *reinterpret_cast<const u64x2*>(mb + (int64_t)(t - 1) * Pp + (int64_t)q * 128 + lane * 2);
            const int c0 = 2 * q;
            if (c0 >= t + 1) {
              const uint64_t bits = __ballot((wv.x & kp) != 0ull);
              if (lane == 0 && bits) atomicOr(reinterpret_cast<unsigned long long*>(&removed[c0]), bits);
            }
            if (c0 + 1 < nbv) {
              const uint64_t bits = __ballot((wv.y & kp) != 0ull);
              if (lane == 0 && bits) atomicOr(reinterpret_cast<unsigned long long*>(&removed[c0 + 1]), bits);
            }
          }
        }
      }
      // prefetch row block t for iteration t+1: the pairs q0' + h + 15k (q0' = (t+2)/2) whose
      // first column is < nbv.  One CU streams the whole triangle and every wave-load costs the
      // CU's address path about the same at 8 and 16 B per lane, so a slot fetches two column
      // blocks and unneeded slots do not issue at all.  These are ordinary loads: the compiler
      // tracks them, so a wave leaving the loop with a prefetch in flight waits before any
      // register of it is reused.  (Round 2 issued them as inline asm, invisible to the compiler's
      // wait-count pass: after an early exit at `post` kept boxes, a late prefetch could land in
      // registers the epilogue had reused for the kept count, corrupting the keep list.)
      const int q0n = (t + 2) >> 1;
      const uint64_t* rowp = mb + (int64_t)t * Pp + (int64_t)(q0n + h) * 128 + lane * 2;
#pragma unroll
      for (int k = 0; k < NMS_PF; ++k) {
        if (2 * (q0n + h + NMS_HELPERS * k) < nbv) pf[k] = *reinterpret_cast<const u64x2*>(rowp + NMS_HELPERS * 128 * k);
      }
    }
    __syncthreads();
  }
  // the loop ends right after a barrier (break) or after the last one (t == nbv): s_nk[t & 1]
  // is the final count either way
  nms_write_out(boxes, scores, b, P, post, min(s_nk[t & 1], post), 0, keep_list, rand_u, rois, out_scores, keep_idx,
                n_keep_out);
}

// ---- multi-workgroup reducer -------------------------------------------------------------------
constexpr int NMSC_PER = 8;  // column blocks per workgroup, one wave each (MXR_NMS_PER=16 for the A/B)
constexpr int NMSC_SPIN = 1 << 20;  // empty poll rounds before a workgroup gives up (MXR_NMS_SPIN overrides)

__device__ __forceinline__ uint64_t nmsc_load(const uint64_t* p) {
  return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void nmsc_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// own-triangle slot of (row k, column c), k <= c < PER, in units of 64 words
__host__ __device__ constexpr int nmsc_tri(int k, int c) { return c * (c + 1) / 2 + k; }

template <int PER>
__global__ void __launch_bounds__(PER * 64)
nms_reduce_mc_kernel(const float* __restrict__ boxes, const float* __restrict__ scores,
                     const int32_t* __restrict__ n_valid, const uint64_t* __restrict__ maskT, uint64_t* rec, int P,
                     int nb, int post, const float* __restrict__ rand_u, float* __restrict__ rois,
                     float* __restrict__ out_scores, int64_t* __restrict__ keep_idx,
                     int32_t* __restrict__ n_keep_out, int32_t* keep_ws, uint64_t* probe, int spin_max) {
  // dynamic LDS: [own triangle (PER * (PER + 1) / 2) x 64 u64][kept nb u64][rem PER u64][count nb i32][keep list post i32]
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint64_t* tri = reinterpret_cast<uint64_t*>(smem);
  uint64_t* s_kept = tri + (PER * (PER + 1) / 2) * 64;
  uint64_t* s_rem = s_kept + nb;
  int* s_nk = reinterpret_cast<int*>(s_rem + PER);
  __shared__ int s_flag[4];  // 0: final record seen, 1: final block resolved here (-1: none), 2: gave up, 3: last out
  const int b = blockIdx.y, w = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  int32_t* keep_list = keep_ws ? keep_ws + (int64_t)b * post : s_nk + nb;
  const int nv = min(n_valid[b], P), nbv = (nv + 63) / 64;
  const int64_t Pp = nms_row_words(nb);
  const uint64_t* mb = maskT + (int64_t)b * nb * Pp;
  uint64_t* rb = rec + (int64_t)b * nb * 2;
  uint64_t* cnt = rec + (int64_t)gridDim.y * nb * 2 + b;
  const int lo = w * PER, hi = min(lo + PER, nbv);
  if (tid == 0) {
    s_flag[0] = 0;
    s_flag[1] = -1;
    s_flag[2] = 0;
  }
  // MXR_NMS_PROBE timeline (wall clock): per block {resolve start, publish, fixpoint rounds, kept},
  // per workgroup {start, phase A done, phase B done, end}
  uint64_t* pb = probe ? probe + (int64_t)b * nb * 8 : nullptr;
  uint64_t* pw = pb ? pb + (int64_t)nb * 4 + (int64_t)w * 4 : nullptr;
  if (pw && tid == 0) pw[0] = wall_clock64();
  __syncthreads();
  bool assemble = nbv == 0 && w == 0;  // no valid box: workgroup 0 writes the padded output
  int tf = -1;
  if (lo < nbv) {
    const int c = lo + wave;
    const bool active = c < hi;
    if (active) {  // stage this wave's column of the own triangle (rows lo..c)
      uint64_t own[PER];
#pragma unroll
      for (int k = 0; k < PER; ++k) own[k] = k <= wave ? mb[(int64_t)(lo + k) * Pp + nms_col(c, lane)] : 0ull;
#pragma unroll
      for (int k = 0; k < PER; ++k)
        if (k <= wave) tri[nmsc_tri(k, wave) * 64 + lane] = own[k];
    }
    // phase A: fold the kept rows of earlier workgroups into column c
    uint64_t rem = 0;
    bool stop = false, gave_up = false;
    if (active) {
      for (int r0 = 0; r0 < lo && !stop; r0 += 16) {
        const int nr = min(16, lo - r0);
        uint64_t wd[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) wd[i] = i < nr ? mb[(int64_t)(r0 + i) * Pp + nms_col(c, lane)] : 0ull;
        int got = 0, spins = 0;
        while (got < nr && !stop) {
          uint64_t w0 = 0, w1 = 0;
          if (lane >= got && lane < nr) {
            w0 = nmsc_load(rb + 2 * (r0 + lane));
            w1 = nmsc_load(rb + 2 * (r0 + lane) + 1);
          }
          const bool ok = lane < got || (lane < nr && (w0 >> 32) != 0ull && (w1 >> 32) != 0ull);
          const int n = min(nr, (int)__builtin_ctzll(~__ballot(ok)));  // ready prefix of the chunk
          if (n == got) {
            if (++spins > spin_max) {
              stop = gave_up = true;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
          }
          spins = 0;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            if (i >= got && i < n && !stop) {
              const uint32_t k0 = __builtin_amdgcn_readlane((int)(uint32_t)w0, i);
              const uint32_t k1 = __builtin_amdgcn_readlane((int)(uint32_t)w1, i);
              const int nk = __builtin_amdgcn_readlane((int)(uint32_t)(w0 >> 32), i) - 1;
              const uint64_t kp = (uint64_t)k0 | ((uint64_t)k1 << 32);
              rem |= __ballot((wd[i] & kp) != 0ull);
              if (wave == 0 && lane == 0) {
                s_kept[r0 + i] = kp;
                s_nk[r0 + i] = nk;
              }
              if (nk >= post) stop = true;  // the chain ended before this workgroup's blocks
            }
          }
          got = n;
        }
      }
      if (lane == 0) {
        s_rem[wave] = rem;
        if (stop) s_flag[gave_up ? 2 : 0] = 1;
      }
    }
    __syncthreads();
    if (pw && tid == 0) pw[1] = wall_clock64();
    if (s_flag[0] == 0 && s_flag[2] == 0) {
      // phase B: wave 0 resolves blocks lo..hi-1 from LDS
      if (wave == 0) {
        uint64_t rm[PER];
#pragma unroll
        for (int k = 0; k < PER; ++k) rm[k] = s_rem[k];
        int nk = lo > 0 ? s_nk[lo - 1] : 0;
#pragma unroll
        for (int k = 0; k < PER; ++k) {
          const int t = lo + k;
          if (t >= hi) break;
          uint64_t row[PER];
#pragma unroll
          for (int c2 = k; c2 < PER; ++c2) row[c2] = lo + c2 < hi ? tri[nmsc_tri(k, c2) * 64 + lane] : 0ull;
          const int nrow = min(64, nv - t * 64);
          const uint64_t valid = nrow >= 64 ? ~0ull : ((1ull << nrow) - 1ull);
          const uint64_t cand = valid & ~rm[k];
          const uint64_t t_res = pb ? wall_clock64() : 0ull;
          uint64_t kept = cand;
          int rounds = 0;
          for (int it = 0; it < 65; ++it) {
            const uint64_t sup = __ballot((row[k] & kept) != 0ull);
            const uint64_t next = cand & ~sup;
            ++rounds;
            if (next == kept) break;
            kept = next;
          }
          if (nk + __popcll(kept) > post) {  // keep only the lowest (post - nk) boxes of this block
            int need = post - nk;
            uint64_t trunc = 0, kk = kept;
            while (need-- > 0 && kk) {
              trunc |= kk & (~kk + 1);
              kk &= kk - 1;
            }
            kept = trunc;
          }
          nk += __popcll(kept);
          if (lane == 0) {
            const uint64_t tag = (uint64_t)(nk + 1) << 32;
            nmsc_store(rb + 2 * t, (kept & 0xffffffffull) | tag);
            nmsc_store(rb + 2 * t + 1, (kept >> 32) | tag);
            s_kept[t] = kept;
            s_nk[t] = nk;
            if (pb) {
              pb[t * 4] = t_res;
              pb[t * 4 + 1] = wall_clock64();
              pb[t * 4 + 2] = rounds;
              pb[t * 4 + 3] = __popcll(kept);
            }
          }
          if (nk >= post || t == nbv - 1) {
            tf = t;
            break;
          }
#pragma unroll
          for (int c2 = k + 1; c2 < PER; ++c2) rm[c2] |= __ballot((row[c2] & kept) != 0ull);
        }
        if (lane == 0) s_flag[1] = tf;
      }
      __syncthreads();
      if (pw && tid == 0) pw[2] = wall_clock64();
      tf = s_flag[1];
      assemble = tf >= 0;
      // every workgroup writes the output rows of its own kept boxes (their slots are final: all
      // below the kept count); the final workgroup adds only the random pad
      const int tend = tf >= 0 ? tf + 1 : hi;
      for (int t = lo + wave; t < tend; t += PER) {
        const uint64_t kept = s_kept[t];
        if ((kept >> lane) & 1ull)
          nms_write_row(boxes, scores, b, P, post, (t > 0 ? s_nk[t - 1] : 0) + __popcll(kept & ((1ull << lane) - 1ull)),
                        t * 64 + lane, rois, out_scores, keep_idx);
      }
    } else if (s_flag[2] && tid == 0) {
      // a poll gave up: this image's output is not assembled; the serial reducer launched behind
      // this kernel (nms_reduce) sees the -1 and redoes the image from the same mask
      n_keep_out[b] = -1;
    }
  }
  if (assemble) {
    // keep list from the kept words: block t's boxes follow the s_nk[t - 1] boxes kept before it
    for (int t = wave; t <= tf; t += PER) {
      const uint64_t kept = s_kept[t];
      const int base = t > 0 ? s_nk[t - 1] : 0;
      if ((kept >> lane) & 1ull) keep_list[base + __popcll(kept & ((1ull << lane) - 1ull))] = t * 64 + lane;
    }
    __syncthreads();
    const int nk = tf >= 0 ? min(s_nk[tf], post) : 0;
    nms_write_out(boxes, scores, b, P, post, nk, nk, keep_list, rand_u, rois, out_scores, keep_idx, n_keep_out);
  }
  // the last workgroup of the image to finish clears the records for the next reduce
  __syncthreads();
  if (pw && tid == 0) pw[3] = wall_clock64();
  if (tid == 0)
    s_flag[3] = __hip_atomic_fetch_add(cnt, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1u;
  __syncthreads();
  if (s_flag[3]) {
    for (int i = tid; i < 2 * nb; i += blockDim.x) nmsc_store(rb + i, 0ull);
    if (tid == 0) nmsc_store(cnt, 0ull);
  }
}

// MXR_NMS_CHECK=1 oracle: the plain greedy flag loop on the device (one 1024-thread workgroup per
// image, a suppression bit per box in LDS, one barrier per visited box), with the same IoU
// arithmetic as nms_mask_kernel, so it checks the reducer's logic rather than float rounding.
// result[b] = {first keep position where the reducer differs (-1 if none), greedy kept count}.
__global__ void __launch_bounds__(1024)
nms_check_kernel(const float* __restrict__ boxes, const int32_t* __restrict__ n_valid, int P, float thresh, int post,
                 const int64_t* __restrict__ keep_idx, const int32_t* __restrict__ n_keep, int32_t* __restrict__ result) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* removed = reinterpret_cast<uint32_t*>(smem);  // ceil(P / 32) words
  __shared__ int s_bad;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int nv = min(n_valid[b], P);
  const int nw = (P + 31) / 32;
  for (int w = tid; w < nw; w += blockDim.x) removed[w] = 0u;
  if (tid == 0) s_bad = -1;
  __syncthreads();
  const float4* bx = reinterpret_cast<const float4*>(boxes) + (int64_t)b * P;
  const int64_t* kp = keep_idx + (int64_t)b * post;
  const int nk_dev = n_keep[b];
  int cnt = 0;
  for (int i = 0; i < nv && cnt < post; ++i) {
    if ((removed[i >> 5] >> (i & 31)) & 1u) continue;  // uniform: read after the last barrier
    if (tid == 0 && s_bad < 0 && (cnt >= nk_dev || kp[cnt] != i)) s_bad = cnt;
    ++cnt;
    const float4 r = bx[i];
    const float ra = (r.z - r.x + 1.f) * (r.w - r.y + 1.f);
    for (int j = i + 1 + tid; j < nv; j += blockDim.x) {
      const float4 c = bx[j];
      const float ca = (c.z - c.x + 1.f) * (c.w - c.y + 1.f);
      if (iou_plus1(r.x, r.y, r.z, r.w, ra, c.x, c.y, c.z, c.w, ca) > thresh) atomicOr(&removed[j >> 5], 1u << (j & 31));
    }
    __syncthreads();
  }
  __syncthreads();
  if (tid == 0) {
    int bad = s_bad;
    if (bad < 0 && nk_dev != cnt) bad = min(cnt, nk_dev);
    result[2 * b] = bad;
    result[2 * b + 1] = cnt;
  }
}

void nms_check(const float* boxes, const int32_t* n_valid, int B, int P, float thresh, int post,
               const int64_t* keep_idx, const int32_t* n_keep, int32_t* result, hipStream_t st) {
  if (B == 0 || P == 0) return;
  nms_check_kernel<<<B, 1024, (size_t)((P + 31) / 32) * 4, st>>>(boxes, n_valid, P, thresh, post, keep_idx, n_keep,
                                                                 result);
}

static bool nms_probe() {
  static const bool on = [] {
    const char* e = getenv("MXR_NMS_PROBE");
    return e && e[0] == '1';
  }();
  return on;
}

int64_t nms_mask_words(int B, int P) {
  const int nb = div_up(P, 64);
  // transposed mask, then the reducer's block records (2 words per block) and exit counters,
  // then (MXR_NMS_PROBE=1) the reducer's timeline, 8 words per block
  return (int64_t)B * nb * nms_row_words(nb) + (int64_t)B * nb * 2 + B + (nms_probe() ? (int64_t)B * nb * 8 : 0);
}

void nms_mask(const float* boxes, const int32_t* n_valid, int B, int P, float thresh, uint64_t* mask,
              hipStream_t st) {
  if (B == 0 || P == 0) return;
  const int nb = div_up(P, 64);
  dim3 grid(div_up(nb, 4), nb, B);
  nms_mask_kernel<<<grid, 256, 0, st>>>(boxes, n_valid, P, nb, thresh, mask, mask + (int64_t)B * nb * nms_row_words(nb));
}

static size_t nms_serial_lds(int nb, int post) { return 16 + (size_t)nb * 16 + (size_t)post * 4; }
static size_t nms_mc_lds(int nb, int post, int per = NMSC_PER) {
  return (size_t)(per * (per + 1) / 2) * 64 * 8 + (size_t)nb * 8 + per * 8 + (size_t)nb * 4 + (size_t)post * 4;
}

size_t nms_reduce_lds(int P, int post) {
  const int nb = div_up(P, 64);
  return std::max(nms_serial_lds(nb, post), nms_mc_lds(nb, post, 16));
}

bool nms_keep_in_lds(int P, int post) { return nms_reduce_lds(P, post) <= 160 * 1024; }

void nms_reduce(const float* boxes, const float* scores, const int32_t* n_valid, const uint64_t* mask, int B,
                int P, int post, const float* rand_u, float* rois, float* out_scores, int64_t* keep_idx,
                int32_t* n_keep, int32_t* keep_ws, hipStream_t st, int32_t* gave_up) {
  if (B == 0) return;
  const int nb = div_up(P, 64);
  const int lpost = keep_ws ? 0 : post;
  static const bool serial = [] {
    const char* e = getenv("MXR_NMS_SERIAL");
    return e && e[0] == '1';
  }();
  if (serial) {
    nms_reduce_kernel<<<B, 1024, nms_serial_lds(nb, lpost), st>>>(boxes, scores, n_valid, mask, P, nb, post, rand_u,
                                                                  rois, out_scores, keep_idx, n_keep, keep_ws);
    return;
  }
  // the records follow the mask (nms_mask_words); written here, cleared by nms_mask and by the kernel
  uint64_t* rec = const_cast<uint64_t*>(mask) + (int64_t)B * nb * nms_row_words(nb);
  static const int per = [] {
    const char* e = getenv("MXR_NMS_PER");
    return e && atoi(e) == 16 ? 16 : NMSC_PER;
  }();
  dim3 grid(div_up(nb, per), B);
  uint64_t* probe = nms_probe() ? rec + (int64_t)B * nb * 2 + B : nullptr;
  // poll budget (read per call: tests/test_nms_multi.py drives the give-up path with 0)
  const char* sp = getenv("MXR_NMS_SPIN");
  const int spin_max = sp ? std::max(0, atoi(sp)) : NMSC_SPIN;
  if (per == 16)
    nms_reduce_mc_kernel<16><<<grid, 16 * 64, nms_mc_lds(nb, lpost, 16), st>>>(boxes, scores, n_valid, mask, rec, P, nb,
                                                                          post, rand_u, rois, out_scores, keep_idx,
                                                                          n_keep, keep_ws, probe, spin_max);
  else
    nms_reduce_mc_kernel<NMSC_PER><<<grid, NMSC_PER * 64, nms_mc_lds(nb, lpost), st>>>(
        boxes, scores, n_valid, mask, rec, P, nb, post, rand_u, rois, out_scores, keep_idx, n_keep, keep_ws, probe,
        spin_max);
  // the always-launched fallback: exits at once unless a chain gave up on an image (n_keep = -1),
  // then finishes that image serially, so a scheduling stall never leaves RoIs unassembled
  nms_reduce_kernel<<<B, 1024, nms_serial_lds(nb, lpost), st>>>(boxes, scores, n_valid, mask, P, nb, post, rand_u,
                                                                rois, out_scores, keep_idx, n_keep, keep_ws, 1, gave_up);
}

}  // namespace mxr
