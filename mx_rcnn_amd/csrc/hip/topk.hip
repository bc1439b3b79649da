// Proposal pre-NMS top-k (SURVEY kernel K5; reference `rcnn/rpn/proposal.py:123-127`:
// order = scores.ravel().argsort()[::-1][:pre_nms_topN]) -> the P best decoded boxes of each image
// in descending score order, ties by lower anchor index (a stable descending sort), plus the
// count of valid (finite-score) entries among them.  Two launches, deterministic, graph-safe;
// replaces a full device radix sort of all anchors + gather + count.
//
//   topk_select_kernel  grid B, 1024 threads, the image's keys held in registers (<= 64 per thread):
//       radix-select the P-th largest key (4 passes of 8-bit LDS histograms over an order-preserving
//       uint32 image of the float keys, wave-aggregated atomics), then collect the candidates:
//       every key above it (one slot atomic per wave) and, in ANCHOR ORDER, just enough keys equal
//       to it (row by row, ballot prefixes) -- exactly the stable top-P set.
//   topk_rank_kernel    grid (ceil(P/64), B): four lanes rank one candidate against all P of its
//       image by counting (64-bit compares of (key, ~index) packed words streamed through LDS, the
//       reads are broadcasts) and the first scatters key + box to its rank.
#include "common.h"
#include "../kernels.h"

namespace mxr {

__device__ __forceinline__ uint32_t ord_key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ float unord_key(uint32_t o) {
  const uint32_t u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
  return __uint_as_float(u);
}

constexpr int kTopkThreads = 1024;
constexpr int kTopkPer = 64;  // keys held in registers per thread: N <= 65536

// thread t holds keys t, t + 1024, ... (coalesced loads, anchor order = (row j, thread t))
__global__ void __launch_bounds__(kTopkThreads)
topk_select_kernel(const float* __restrict__ keys, int N, int P, uint32_t* __restrict__ cand_key,
                   int* __restrict__ cand_idx, int* __restrict__ n_valid) {
  __shared__ unsigned int hist[256];
  __shared__ unsigned int prefix_s, remain_s, slot_s, valid_s;
  __shared__ unsigned int wcnt[kTopkThreads / 64];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const float* k = keys + (int64_t)b * N;
  uint32_t* ck = cand_key + (int64_t)b * P;
  int* ci = cand_idx + (int64_t)b * P;
  const int rows = (N + kTopkThreads - 1) / kTopkThreads;
  uint32_t u[kTopkPer];
  unsigned int nv = 0;
#pragma unroll
  for (int j = 0; j < kTopkPer; ++j) {
    const int i = j * kTopkThreads + tid;
    const float f = (j < rows && i < N) ? k[i] : -INFINITY;
    nv += f > -INFINITY;
    u[j] = (j < rows && i < N) ? ord_key(f) : 0u;  // 0: below every real key (-inf maps to 0x007fffff)
  }
  if (tid == 0) {
    prefix_s = 0;
    remain_s = (unsigned int)P;
    slot_s = 0;
    valid_s = 0;
  }
  __syncthreads();
  if (nv) atomicAdd(&valid_s, nv);
  // 4 radix passes (most significant byte first) for the P-th largest ordered key
  for (int pass = 3; pass >= 0; --pass) {
    for (int i = tid; i < 256; i += kTopkThreads) hist[i] = 0;
    __syncthreads();
    const unsigned int pre = prefix_s;
    const unsigned int hi_mask = pass == 3 ? 0u : (0xffffffffu << (8 * (pass + 1)));
#pragma unroll
    for (int j = 0; j < kTopkPer; ++j) {
      if (j >= rows) break;
      const bool in = u[j] != 0u && (u[j] & hi_mask) == (pre & hi_mask);
      const unsigned int bin = (u[j] >> (8 * pass)) & 255u;
      // one LDS atomic per DISTINCT bin of the wave (the scores cluster in a few bins; 64 lanes
      // adding to one address would serialise on the CU's single LDS across all 16 waves)
      uint64_t active = __ballot(in);
      while (active) {
        const int leader = __ffsll((long long)active) - 1;
        const unsigned int b0 = __shfl(bin, leader, 64);
        const uint64_t m = __ballot(bin == b0) & active;
        if (lane == leader) atomicAdd(&hist[b0], (unsigned int)__popcll(m));
        active &= ~m;
      }
    }
    __syncthreads();
    if (tid == 0) {
      const unsigned int rem = remain_s;
      unsigned int acc = 0;
      int bin = 255;
      for (; bin > 0; --bin) {
        if (acc + hist[bin] >= rem) break;
        acc += hist[bin];
      }
      remain_s = rem - acc;
      prefix_s = pre | ((unsigned int)bin << (8 * pass));
    }
    __syncthreads();
  }
  const uint32_t T = prefix_s;
  const unsigned int need_eq = remain_s;  // keys equal to T to take, lowest anchor index first
  const unsigned int base = (unsigned int)P - need_eq;
  unsigned int eq_done = 0;  // equal keys taken in earlier rows (uniform)
#pragma unroll
  for (int j = 0; j < kTopkPer; ++j) {
    if (j >= rows) break;
    const int i = j * kTopkThreads + tid;
    // strictly greater: any order, one LDS atomic per wave
    const bool gt = u[j] > T;
    const uint64_t mg = __ballot(gt);
    if (mg) {
      unsigned int s0 = 0;
      if (lane == __ffsll((long long)mg) - 1) s0 = atomicAdd(&slot_s, (unsigned int)__popcll(mg));
      s0 = __shfl(s0, __ffsll((long long)mg) - 1, 64);
      if (gt) {
        const unsigned int s = s0 + (unsigned int)__popcll(mg & ((1ull << lane) - 1ull));
        ck[s] = u[j];
        ci[s] = i;
      }
    }
    // equal to T: in anchor order within the row (wave prefix + per-wave counts through LDS)
    if (eq_done < need_eq) {
      const bool eq = u[j] == T && i < N;
      const uint64_t me = __ballot(eq);
      if (lane == 0) wcnt[wid] = (unsigned int)__popcll(me);
      __syncthreads();
      unsigned int before = eq_done, row_total = 0;
      for (int w = 0; w < kTopkThreads / 64; ++w) {
        const unsigned int c = wcnt[w];
        if (w < wid) before += c;
        row_total += c;
      }
      before += (unsigned int)__popcll(me & ((1ull << lane) - 1ull));
      if (eq && before < need_eq) {
        ck[base + before] = T;
        ci[base + before] = i;
      }
      eq_done += row_total;
      __syncthreads();  // wcnt is rewritten by the next row
    }
  }
  if (tid == 0) n_valid[b] = (int)min((unsigned int)P, valid_s);
}

// 64 candidates per workgroup, 4 lanes per candidate (each counts a quarter of every tile), so a
// 12000-candidate image spreads over ~190 workgroups; tile reads are 16-B broadcasts, 8 compares
// per LDS round trip.
__global__ void __launch_bounds__(256)
topk_rank_kernel(const uint32_t* __restrict__ cand_key, const int* __restrict__ cand_idx,
                 const float* __restrict__ boxes, int N, int P, float* __restrict__ skeys, float* __restrict__ sboxes) {
  __shared__ __attribute__((aligned(16))) uint64_t tile[2048];
  const int b = blockIdx.y, tid = threadIdx.x;
  const int q = tid & 3;                    // quarter of each tile this lane counts
  const int i = blockIdx.x * 64 + (tid >> 2);
  const uint32_t* ck = cand_key + (int64_t)b * P;
  const int* ci = cand_idx + (int64_t)b * P;
  uint64_t mine = 0;
  int idx = 0;
  if (i < P) {
    idx = ci[i];
    mine = ((uint64_t)ck[i] << 32) | (uint32_t)~(uint32_t)idx;  // larger = earlier in the order
  }
  int rank = 0;
  for (int t0 = 0; t0 < P; t0 += 2048) {
    const int m = min(2048, P - t0);
    for (int j = tid; j < 2048; j += 256)
      tile[j] = j < m ? ((uint64_t)ck[t0 + j] << 32) | (uint32_t)~(uint32_t)ci[t0 + j] : 0ull;  // pad never ranks above
    __syncthreads();
    // the 4 lanes of a candidate read 4 ADJACENT 16-B pairs (one 64-B run: conflict-free), every
    // candidate of the wave the same run (broadcast)
    const ulonglong2* tv = reinterpret_cast<const ulonglong2*>(tile) + q;
#pragma unroll 16
    for (int j = 0; j < 256; ++j) {
      const ulonglong2 v = tv[4 * j];
      rank += (v.x > mine) + (v.y > mine);
    }
    __syncthreads();
  }
  rank += __shfl_xor(rank, 1, 64);
  rank += __shfl_xor(rank, 2, 64);
  if (i < P && q == 0) {
    skeys[(int64_t)b * P + rank] = unord_key((uint32_t)(mine >> 32));
    const float4 bx = *reinterpret_cast<const float4*>(boxes + ((int64_t)b * N + idx) * 4);
    *reinterpret_cast<float4*>(sboxes + ((int64_t)b * P + rank) * 4) = bx;
  }
}

int proposal_topk(const float* keys, const float* boxes, int B, int N, int P, uint32_t* ws_key, int* ws_idx,
                  float* skeys, float* sboxes, int* n_valid, hipStream_t st) {
  if (B <= 0 || N <= 0 || P <= 0 || P > N || N > kTopkThreads * kTopkPer) return -1;
  topk_select_kernel<<<B, kTopkThreads, 0, st>>>(keys, N, P, ws_key, ws_idx, n_valid);
  topk_rank_kernel<<<dim3(div_up(P, 64), B), 256, 0, st>>>(ws_key, ws_idx, boxes, N, P, skeys, sboxes);
  return 0;
}

}  // namespace mxr
