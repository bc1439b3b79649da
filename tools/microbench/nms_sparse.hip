// Standalone copy of the sparse-list NMS (commit ef4c548, reverted from the extension after an
// intermittent fault under bench_test.py) for a controlled re-test: tools/microbench/nms_sparse_bench.hip
// runs it against the dense kernel, including the per-class path (post == P, n_valid < P).

// Bitmask greedy NMS for the proposal layer (kernel K6/K7;
// reference semantics `helper/processing/nms.py:4-38`: suppress j when IoU(i,j) > thresh,
// +1-pixel areas, boxes visited in descending score order).
//
// Suppression words, one 64-bit word per (row block r, box j):
//   word[r][j] bit i  <=>  box r*64+i (higher score, r*64+i < j) suppresses box j.
// With lane = box j, "is j suppressed by any kept box of block r" is a single
// `ballot((word[r][j] & kept[r]) != 0)` -- the 64-bit word width IS the wave width, so the
// serial part of greedy NMS runs on wave-wide bit operations instead of shuffles or atomics.
//
// Storage (one workspace, nms_mask_words): the two near-diagonal column blocks of every row
// block are dense (near[r][0][j] = words vs block r, near[r][1][j] = vs block r+1: what the
// resolving wave reads); every farther column is SPARSE: only nonzero words, as (word, j)
// entries appended to a per-row-block list.  Proposals are score-sorted, i.e. spatially random,
// so almost every 64x64 block pair contains some overlapping pair (dense at block level) but
// only a few percent of the per-box words are nonzero: the dense triangle was 9 MB for
// 12000 boxes and streaming it through the one CU that runs the serial scan took ~250 of its
// ~300 us (the CU's outstanding-miss limit caps it near 30 GB/s); the lists are ~20x smaller.
//
// Stage 1 (nms_mask): 256-thread workgroup per (4 column blocks, row block, image); lane = box
// j, the 64 row boxes sit in LDS; nonzero far words are appended with one atomic per wave.
// Stage 2 (nms_reduce): one 1024-thread workgroup per image, ONE barrier per 64-box block t:
//   wave 0    resolves block t: cand = valid & ~(removed[t] | ballot(near[t-1][1][j] & kept[t-1]))
//             then the in-block fixpoint kept = cand & ~ballot(near[t][0][j] & kept) (the unique
//             greedy fixpoint; chain-length iterations of ~5 instructions each);
//   waves 1-15 fold block t-1's kept rows into removed[] through row t-1's sparse list (one
//             entry per lane, LDS atomic OR of the suppressed box's bit);
//   every global read is prefetched two iterations ahead into registers (double-buffered), so
//   the per-block critical path is LDS + ballots + one barrier.
// The kept list lives in LDS; the kernel writes the final (post, 5) RoI block directly,
// including the reference's random pad (slot >= n_keep takes keep[floor(u*n_keep)]).  Early
// exit once `post` boxes are kept.  No host synchronisation anywhere.
#include "common.h"
#include "../kernels.h"

namespace mxr_sparse {
using mxr::div_up;
using mxr::iou_plus1;

#ifdef NMS_DEBUG
__device__ int g_nms_dbg[4];  // [mask ent OOB, reduce ent OOB, near OOB, removed OOB]
#define NMS_CHECK(cond, slot) if (!(cond)) { atomicAdd(&g_nms_dbg[slot], 1); } else
#else
#define NMS_CHECK(cond, slot)
#endif

constexpr int NMS_HELPERS = 15;  // helper waves in the 1024-thread reducer

struct NmsEntry {  // one nonzero far word
  uint64_t word;
  uint32_t j;      // box index (column)
  uint32_t pad;
};

struct NmsLayout {  // carve the workspace
  uint64_t* near;   // [B][nb][2][64]
  int32_t* cnt;     // [B][nb] entries per row-block list
  NmsEntry* ent;    // [B][nb][cap]
  int64_t cap;
};

__host__ __device__ __forceinline__ int64_t nms_cnt_words(int B, int nb) {
  return (((int64_t)B * nb + 3) / 4) * 2;  // int32 counts, padded to 16 B
}

__host__ __device__ __forceinline__ NmsLayout nms_layout(uint64_t* ws, int B, int nb) {
  NmsLayout L;
  L.near = ws;
  L.cnt = reinterpret_cast<int32_t*>(ws + (int64_t)B * nb * 128);
  L.ent = reinterpret_cast<NmsEntry*>(ws + (int64_t)B * nb * 128 + nms_cnt_words(B, nb));
  L.cap = (int64_t)nb * 64;
  return L;
}

__global__ void __launch_bounds__(256)
nms_mask_kernel(const float* __restrict__ boxes, const int32_t* __restrict__ n_valid, int P, int nb, int B,
                float thresh, uint64_t* __restrict__ ws) {
  const int rb = blockIdx.y, b = blockIdx.z;
  if (blockIdx.x * 4 + 3 < rb) return;  // whole group below the diagonal
  const int cb = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int nv = min(n_valid[b], P);
  const int row0 = rb * 64;
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
  const bool active = cb >= rb && cb < nb;  // wave-uniform
  const int j = cb * 64 + lane;
  uint64_t bits = 0;
  if (active && j < nv && row0 < nv) {
    const float4 c = bx[j];
    const float carea = (c.z - c.x + 1.f) * (c.w - c.y + 1.f);
    const int iend = min(64, j - row0);  // rows i with row0 + i < j (all < nv since j < nv)
    for (int i = 0; i < iend; ++i) {
      const float4 r = rbox[i];
      if (iou_plus1(r.x, r.y, r.z, r.w, rarea[i], c.x, c.y, c.z, c.w, carea) > thresh) bits |= (1ull << i);
    }
  }
  const NmsLayout L = nms_layout(ws, B, nb);
  const int64_t row = (int64_t)b * nb + rb;
  if (active && cb <= rb + 1) L.near[row * 128 + (cb - rb) * 64 + lane] = bits;
  // far words: one list append per WORKGROUP (the 4 waves share the row block)
  const bool far = active && cb >= rb + 2;
  const uint64_t nz = far ? __ballot(bits != 0ull) : 0ull;
  __shared__ int s_wc[4], s_base;
  const int wv = threadIdx.x >> 6;
  if (lane == 0) s_wc[wv] = __popcll(nz);
  __syncthreads();
  if (threadIdx.x == 0) {
    const int tot = s_wc[0] + s_wc[1] + s_wc[2] + s_wc[3];
    s_base = tot ? atomicAdd(L.cnt + row, tot) : 0;
  }
  __syncthreads();
  if (bits && far) {
    int off = s_base;
    for (int w = 0; w < wv; ++w) off += s_wc[w];
    NmsEntry e;
    e.word = bits;
    e.j = (uint32_t)j;
    e.pad = 0u;
    const int64_t slot_i = off + __popcll(nz & ((1ull << lane) - 1ull));
    NMS_CHECK(slot_i < L.cap, 0)
    L.ent[row * L.cap + slot_i] = e;
  }
}

template <int N>
__device__ __forceinline__ void nms_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

typedef unsigned int nms_u4 __attribute__((ext_vector_type(4)));

// 16 B per lane global -> LDS DMA (lane-linear destination at the wave-uniform base)
__device__ __forceinline__ void nms_dma16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

constexpr int NMS_KPF = 2;  // 64-entry chunks per helper and row block held in the ring (1920 entries)
constexpr int NMS_RING_H = 2 * NMS_KPF * NMS_HELPERS * 64 * 16;  // [parity][chunk][helper][lane] x 16 B
constexpr int NMS_RING_W = 4 * 128 * 8;                // wave-0 near ring: [row & 3][128 words]

__global__ void __launch_bounds__(1024)
nms_reduce_kernel(const float* __restrict__ boxes, const float* __restrict__ scores,
                  const int32_t* __restrict__ n_valid, const uint64_t* __restrict__ ws, int P, int nb, int B,
                  int post, const float* __restrict__ rand_u, float* __restrict__ rois,
                  float* __restrict__ out_scores, int64_t* __restrict__ keep_idx, int32_t* __restrict__ n_keep_out) {
  // The DMA rings are their own LDS objects: the compiler then sees that the scan state (the
  // dynamic region) cannot alias an in-flight DMA and does not drain vmcnt before touching it.
  __shared__ __attribute__((aligned(16))) unsigned char ring_h[NMS_RING_H];
  __shared__ __attribute__((aligned(16))) uint64_t ring_w[NMS_RING_W / 8];
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // dynamic LDS: [nkeep i32 | pad][removed nb u64][keptw nb u64][cnt nb i32 (even)][keep_list post i32]
  unsigned char* rest = smem;
  int* s_nk = reinterpret_cast<int*>(rest);  // double-buffered kept count (see csrc/hip/nms.hip)
  uint64_t* removed = reinterpret_cast<uint64_t*>(rest + 16);
  uint64_t* keptw = removed + nb;
  int32_t* s_cnt = reinterpret_cast<int32_t*>(keptw + nb);
  int32_t* keep_list = s_cnt + ((nb + 1) & ~1);
  const int b = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int nv = min(n_valid[b], P);
  const NmsLayout L = nms_layout(const_cast<uint64_t*>(ws), B, nb);
  const uint64_t* near = L.near + (int64_t)b * nb * 128;
  const NmsEntry* ent = L.ent + (int64_t)b * nb * L.cap;
  for (int c = tid; c < nb; c += blockDim.x) {
    removed[c] = 0;
    keptw[c] = 0;
    s_cnt[c] = L.cnt[(int64_t)b * nb + c];
  }
  if (tid < 2) s_nk[tid] = 0;
  const int nbv = (nv + 63) / 64;
  const int h = wave - 1;
  // Prefetch distance 2 through LDS-DMA rings (the asynchronous writes land in LDS, never in
  // registers the compiler may have reassigned): wave 0 streams row block r's dense near words
  // (1 KB) into ring_w[r & 3]; helper h streams its 64-entry share of row r's sparse list into
  // ring_h[r & 1][h].  Counted vmcnt waits: wave 0 issues exactly one DMA per iteration (rows
  // clamped in range), a helper at most one.
  auto w0_issue = [&](int r) {
    const int rc = min(r, nb - 1);
    nms_dma16(near + (int64_t)rc * 128 + 2 * lane, ring_w + (r & 3) * 128);
  };
  auto h_issue = [&](int r) -> int {  // row r's first NMS_KPF * 960 entries, this wave's chunks
    const int n = s_cnt[r];
    int issued = 0;
#pragma unroll
    for (int k = 0; k < NMS_KPF; ++k) {
      const int e = (h + NMS_HELPERS * k) * 64;
      if (e < n) {
        nms_dma16(ent + (int64_t)r * L.cap + e + lane,
                  ring_h + (((r & 1) * NMS_KPF + k) * NMS_HELPERS + h) * 64 * 16);
        ++issued;
      }
    }
    return issued;
  };
  __syncthreads();  // s_cnt visible
  int issued_prev = 0;
  if (wave == 0) {
    w0_issue(0);
    w0_issue(1);
  } else if (nbv > 0) {
    issued_prev = h_issue(0);
  }
  int t = 0;
  for (; t < nbv; ++t) {
    if (s_nk[t & 1] >= post) break;  // uniform: not rewritten before the next barrier
    if (wave == 0) {
      nms_wait_vm<1>();  // row t's near words (issued two iterations ago) are in ring_w[t & 3]
      uint64_t diag, wprev;  // (asm reads, as for the helpers' ring; wprev is ANDed with kp = 0 at t = 0)
      const uint32_t ld_ = (uint32_t)reinterpret_cast<uintptr_t>(ring_w + (t & 3) * 128 + lane);
      const uint32_t lw_ = (uint32_t)reinterpret_cast<uintptr_t>(ring_w + ((t - 1) & 3) * 128 + 64 + lane);
      asm volatile("ds_read_b64 %0, %2\n\tds_read_b64 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                   : "=v"(diag), "=v"(wprev) : "v"(ld_), "v"(lw_) : "memory");
      const int j = t * 64 + lane;
      const uint64_t kp = t > 0 ? keptw[t - 1] : 0ull;
      const uint64_t sp = __ballot((wprev & kp) != 0ull);
      const int nrow = min(64, nv - t * 64);
      const uint64_t valid = nrow >= 64 ? ~0ull : ((1ull << nrow) - 1ull);
      const uint64_t cand = valid & ~(removed[t] | sp);
      uint64_t kept = cand;
#ifndef NMS_ABL_NOFIX  // ablation switch for tools/microbench/nms_bench.hip
      for (int it = 0; it < 65; ++it) {
        const uint64_t sup = __ballot((diag & kept) != 0ull);
        const uint64_t next = cand & ~sup;
        if (next == kept) break;
        kept = next;
      }
#endif
      w0_issue(t + 2);  // into the slot of row t-2, read for the last time in iteration t-1
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
#ifndef NMS_ABL_NOHELP  // ablation switch for tools/microbench/nms_bench.hip
      // row t-1's entries (issued two iterations ago) have landed; row t's may be in flight
      if (issued_prev >= 2) nms_wait_vm<2>();
      else if (issued_prev == 1) nms_wait_vm<1>();
      else nms_wait_vm<0>();
      if (t >= 1) {
        const int r = t - 1;
        const uint64_t kp = keptw[r];
        const int n = s_cnt[r];
        if (kp) {
#pragma unroll
          for (int k = 0; k < NMS_KPF; ++k) {
            const int e = (h + NMS_HELPERS * k) * 64 + lane;
            if (e < n) {
              // read through asm: hipcc cannot tell this slot from the one still being filled and
              // would drain every DMA first (the counted wait above is the real dependency)
              nms_u4 w;
              const uint32_t la = (uint32_t)reinterpret_cast<uintptr_t>(
                  ring_h + ((((r & 1) * NMS_KPF + k) * NMS_HELPERS + h) * 64 + lane) * 16);
              asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(w) : "v"(la) : "memory");
              const uint64_t word = ((uint64_t)w.y << 32) | w.x;
              NMS_CHECK((int)(w.z >> 6) < nb, 3)
              if (word & kp) {  // asm LDS OR (as an atomicOr, hipcc would drain the DMAs first)
                const uint32_t ra = (uint32_t)reinterpret_cast<uintptr_t>(&removed[w.z >> 6]);
                const uint64_t bit = 1ull << (w.z & 63);
                asm volatile("ds_or_b64 %0, %1" ::"v"(ra), "v"(bit) : "memory");
              }
            }
          }
          // entries past the ring (> 1920 nonzero far words in this row block): plain loads
          for (int e2 = (NMS_HELPERS * NMS_KPF + h) * 64 + lane; e2 < n; e2 += NMS_HELPERS * 64) {
            const NmsEntry x = ent[(int64_t)r * L.cap + e2];
            if (x.word & kp) atomicOr(reinterpret_cast<unsigned long long*>(&removed[x.j >> 6]), 1ull << (x.j & 63));
          }
        }
      }
      // row t+1 into the parity slot just consumed (its ds_reads completed above)
      issued_prev = t + 1 < nbv ? h_issue(t + 1) : 0;
#endif
    }
    // barrier without the vmcnt(0) drain __syncthreads() implies: the scan state is LDS only
    // (lgkmcnt), the prefetch DMAs must stay in flight across it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  // drain the DMAs still in flight before the block can retire
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int nk = min(s_nk[t & 1], post);
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

int64_t nms_mask_words(int B, int P) {
  const int nb = (int)div_up(P, 64);
  return (int64_t)B * nb * 128 + nms_cnt_words(B, nb) + (int64_t)B * nb * nb * 64 * 2;
}

void nms_mask(const float* boxes, const int32_t* n_valid, int B, int P, float thresh, uint64_t* ws,
              hipStream_t st) {
  if (B == 0 || P == 0) return;
  const int nb = div_up(P, 64);
  const NmsLayout L = nms_layout(ws, B, nb);
  (void)hipMemsetAsync(L.cnt, 0, nms_cnt_words(B, nb) * 8, st);
  dim3 grid(div_up(nb, 4), nb, B);
  nms_mask_kernel<<<grid, 256, 0, st>>>(boxes, n_valid, P, nb, B, thresh, ws);
}

size_t nms_reduce_lds(int P, int post) {  // dynamic part (the static rings add NMS_RING_H + NMS_RING_W)
  const int nb = div_up(P, 64);
  return 16 + (size_t)nb * 16 + (size_t)((nb + 1) & ~1) * 4 + (size_t)post * 4;
}

void nms_reduce(const float* boxes, const float* scores, const int32_t* n_valid, const uint64_t* ws, int B,
                int P, int post, const float* rand_u, float* rois, float* out_scores, int64_t* keep_idx,
                int32_t* n_keep, hipStream_t st) {
  if (B == 0) return;
  const int nb = div_up(P, 64);
  nms_reduce_kernel<<<B, 1024, nms_reduce_lds(P, post), st>>>(boxes, scores, n_valid, ws, P, nb, B, post, rand_u,
                                                             rois, out_scores, keep_idx, n_keep);
}

}  // namespace mxr_sparse
