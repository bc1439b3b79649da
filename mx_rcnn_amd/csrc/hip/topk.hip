// Proposal pre-NMS top-k (SURVEY kernel K5; reference `rcnn/rpn/proposal.py:123-127`:
// order = scores.ravel().argsort()[::-1][:pre_nms_topN]) -> the P best decoded boxes of each image
// in descending score order, ties by lower anchor index (a stable descending sort), plus the
// count of valid (finite-score) entries among them.  Six launches, deterministic, graph-safe;
// replaces a full device sort of all anchors + gather + count.
//
//   topk_hist_kernel<0..2>, topk_count_kernel, topk_write_kernel  grid (ceil(N / 2048), B): grid
//       radix select of the P-th largest key and the stable top-P candidate set (below)
//   topk_chunk_sort_kernel + topk_merge_rank_kernel (P <= 20480, below), else
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

// ---- grid radix select ------------------------------------------------------------------------
// The P-th largest ordered key of each image, found digit by digit (bits 31..21, 20..10, 9..0)
// by a GRID of workgroups per image: a single workgroup per image (the first version) walked the
// 50 400 keys four times from one CU -- 160-340 us, latency bound, and 1 CU of 256 busy.  Here each
// workgroup owns kTkChunk consecutive keys (8 per thread, anchor order = thread order), builds
// its chunk's digit histogram in LDS (wave-aggregated atomics: one per distinct bin of a wave)
// and adds it to the image's global histogram (integer atomics: order-independent, so
// deterministic).  The next launch's workgroups each scan the finished histogram themselves (a
// 256-thread block scan of 8 KB, identical in every workgroup: no extra launch, no global
// hand-off but a state row that chunk 0 records for the later launches).  Then a count launch
// (> T, == T, finite per chunk) and a write launch (chunk prefix + block scan: every key above T
// and the first need_eq keys equal to T in anchor order -- exactly the stable top-P set) feed
// the rank kernel below.
constexpr int kTkThreads = 256;
constexpr int kTkPer = 8;
constexpr int kTkChunk = kTkThreads * kTkPer;
constexpr int kTkBins = 2048;

struct TkWs {  // int32 workspace of one call (zeroed by the caller)
  uint32_t* hist;   // [B][3][kTkBins]
  uint32_t* state;  // [B][3][2]: (prefix, remain) after digit pass p
  uint32_t* cnt;    // [B][G][3]: (> T, == T, finite) per chunk
};

__host__ __device__ inline int64_t topk_ws_words(int B, int G) {
  return (int64_t)B * 3 * kTkBins + (int64_t)B * 6 + (int64_t)B * G * 3;
}

__device__ __forceinline__ TkWs tk_ws(uint32_t* ws, int B, int G) {
  TkWs w;
  w.hist = ws;
  w.state = ws + (int64_t)B * 3 * kTkBins;
  w.cnt = w.state + (int64_t)B * 6;
  return w;
}

// exclusive block scan of one value per thread (256 threads); returns the exclusive prefix, total in *tot
__device__ __forceinline__ uint32_t tk_block_scan(uint32_t v, uint32_t* wsum, uint32_t* tot) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) wsum[wid] = inc;
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kTkThreads / 64; ++w) {
    const uint32_t c = wsum[w];
    if (w < wid) before += c;
    all += c;
  }
  __syncthreads();  // wsum reusable
  *tot = all;
  return before + inc - v;
}

// largest bin with (keys in higher bins) < remain <= (keys in it and higher bins): the digit of
// the remain-th largest key, and remain minus the keys above that bin
__device__ __forceinline__ void tk_pick(const uint32_t* __restrict__ hist, int nbins, uint32_t remain,
                                        uint32_t* wsum, uint32_t* s_bin, uint32_t* s_rem) {
  const int per = nbins / kTkThreads;  // 8 or 4 bins per thread, thread 0 the highest
  const int top = nbins - 1 - threadIdx.x * per;
  uint32_t h[8];
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    h[k] = k < per ? hist[top - k] : 0u;
    s += h[k];
  }
  uint32_t tot;
  uint32_t acc = tk_block_scan(s, wsum, &tot);
  if (threadIdx.x == 0) {  // (unreachable with consistent counts: remain <= keys under the prefix)
    *s_bin = 0u;
    *s_rem = remain;
  }
  __syncthreads();
  if (acc < remain && remain <= acc + s) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k < per && acc + h[k] >= remain) {
        *s_bin = (uint32_t)(top - k);
        *s_rem = remain - acc;
        break;
      }
      acc += h[k];
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void tk_load(const float* __restrict__ k, int N, int i0, uint32_t (&u)[kTkPer],
                                        uint32_t& valid_mask) {
  valid_mask = 0;
#pragma unroll
  for (int j = 0; j < kTkPer; ++j) {
    const int i = i0 + j;
    u[j] = 0u;  // below every real key (-inf maps to 0x007fffff)
    if (i < N) {
      const float f = k[i];
      u[j] = ord_key(f);
      valid_mask |= (f > -INFINITY ? 1u : 0u) << j;
    }
  }
}

// the prefix / remain this launch starts from: digit passes 0..PASS-1 finished
template <int PASS>
__device__ __forceinline__ void tk_resolve(const TkWs& w, int b, int P, uint32_t* wsum, uint32_t& pre,
                                           uint32_t& rem) {
  __shared__ uint32_t s_bin, s_rem;
  if (PASS == 0) {
    pre = 0;
    rem = (uint32_t)P;
    return;
  }
  uint32_t* st = w.state + (int64_t)b * 6;
  const uint32_t pre0 = PASS >= 2 ? st[2 * (PASS - 2)] : 0u;
  const uint32_t rem0 = PASS >= 2 ? st[2 * (PASS - 2) + 1] : (uint32_t)P;
  const int nbins = PASS - 1 == 2 ? 1024 : kTkBins;
  const int shift = PASS - 1 == 0 ? 21 : (PASS - 1 == 1 ? 10 : 0);
  tk_pick(w.hist + ((int64_t)b * 3 + PASS - 1) * kTkBins, nbins, rem0, wsum, &s_bin, &s_rem);
  pre = pre0 | (s_bin << shift);
  rem = s_rem;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st[2 * (PASS - 1)] = pre;
    st[2 * (PASS - 1) + 1] = rem;
  }
}

template <int PASS>
__global__ void __launch_bounds__(kTkThreads)
topk_hist_kernel(const float* __restrict__ keys, int N, int P, uint32_t* __restrict__ ws) {
  __shared__ uint32_t h[kTkBins];
  __shared__ uint32_t wsum[kTkThreads / 64];
  const int b = blockIdx.y, G = gridDim.x, lane = threadIdx.x & 63;
  const TkWs w = tk_ws(ws, gridDim.y, G);
  for (int i = threadIdx.x; i < kTkBins; i += kTkThreads) h[i] = 0u;
  uint32_t pre, rem;
  tk_resolve<PASS>(w, b, P, wsum, pre, rem);
  uint32_t u[kTkPer], vm;
  tk_load(keys + (int64_t)b * N, N, blockIdx.x * kTkChunk + threadIdx.x * kTkPer, u, vm);
  const int shift = PASS == 0 ? 21 : (PASS == 1 ? 10 : 0);
  const uint32_t dmask = PASS == 2 ? 1023u : 2047u;
  const int i0 = blockIdx.x * kTkChunk + threadIdx.x * kTkPer;
  __syncthreads();  // h zeroed
#pragma unroll
  for (int j = 0; j < kTkPer; ++j) {
    const bool in = i0 + j < N && (PASS == 0 || (u[j] >> (shift + (PASS == 1 ? 11 : 10))) ==
                                                    (pre >> (shift + (PASS == 1 ? 11 : 10))));
    const uint32_t bin = (u[j] >> shift) & dmask;
    uint64_t active = __ballot(in);
    // the wave's most frequent bins with one LDS atomic each (clustered scores put most of a wave in
    // a few top-digit bins), then the scattered rest directly (the low digits are spread: a
    // per-distinct-bin loop would run up to 64 rounds)
    for (int it = 0; it < 4 && active; ++it) {
      const int leader = __ffsll((long long)active) - 1;
      const uint32_t b0 = __shfl(bin, leader, 64);
      const uint64_t m = __ballot(bin == b0) & active;
      if (lane == leader) atomicAdd(&h[b0], (uint32_t)__popcll(m));
      active &= ~m;
    }
    if ((active >> lane) & 1ull) atomicAdd(&h[bin], 1u);
  }
  __syncthreads();
  uint32_t* gh = w.hist + ((int64_t)b * 3 + PASS) * kTkBins;
  for (int i = threadIdx.x; i < (PASS == 2 ? 1024 : kTkBins); i += kTkThreads)
    if (h[i]) atomicAdd(gh + i, h[i]);
}

// T and need_eq (the last digit pass), then this chunk's (> T, == T, finite) counts
__global__ void __launch_bounds__(kTkThreads)
topk_count_kernel(const float* __restrict__ keys, int N, int P, uint32_t* __restrict__ ws) {
  __shared__ uint32_t wsum[kTkThreads / 64];
  const int b = blockIdx.y, G = gridDim.x;
  const TkWs w = tk_ws(ws, gridDim.y, G);
  uint32_t T, need;
  tk_resolve<3>(w, b, P, wsum, T, need);
  uint32_t u[kTkPer], vm;
  tk_load(keys + (int64_t)b * N, N, blockIdx.x * kTkChunk + threadIdx.x * kTkPer, u, vm);
  const int i0 = blockIdx.x * kTkChunk + threadIdx.x * kTkPer;
  uint32_t gt = 0, eq = 0;
#pragma unroll
  for (int j = 0; j < kTkPer; ++j) {
    gt += u[j] > T;
    eq += u[j] == T && i0 + j < N;
  }
  uint32_t tg, te, tv;
  tk_block_scan(gt, wsum, &tg);
  tk_block_scan(eq, wsum, &te);
  tk_block_scan((uint32_t)__popc(vm), wsum, &tv);
  if (threadIdx.x == 0) {
    uint32_t* c = w.cnt + ((int64_t)b * G + blockIdx.x) * 3;
    c[0] = tg;
    c[1] = te;
    c[2] = tv;
  }
}

// candidates: keys > T at (chunks before + block prefix), the first need_eq keys == T (anchor
// order) after them; chunk 0 also writes the image's valid count
__global__ void __launch_bounds__(kTkThreads)
topk_write_kernel(const float* __restrict__ keys, int N, int P, uint32_t* __restrict__ ws,
                  uint32_t* __restrict__ cand_key, int* __restrict__ cand_idx, int* __restrict__ n_valid) {
  __shared__ uint32_t wsum[kTkThreads / 64];
  const int b = blockIdx.y, G = gridDim.x;
  const TkWs w = tk_ws(ws, gridDim.y, G);
  {  // every histogram reader (the digit passes, the count kernel) is done: leave them zeroed for the
     // next call (the workspace is persistent and self-cleaning, bindings.cpp clean_ws)
    uint32_t* hb = w.hist + (int64_t)b * 3 * kTkBins;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < 3 * kTkBins; i += G * blockDim.x) hb[i] = 0u;
  }
  const uint32_t* st = w.state + (int64_t)b * 6;
  const uint32_t T = st[4], need = st[5];
  const uint32_t* c = w.cnt + (int64_t)b * G * 3;
  uint32_t gbase = 0, ebase = 0;
  for (int q = 0; q < (int)blockIdx.x; ++q) {
    gbase += c[3 * q];
    ebase += c[3 * q + 1];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    uint32_t nv = 0;
    for (int q = 0; q < G; ++q) nv += c[3 * q + 2];
    n_valid[b] = (int)min((uint32_t)P, nv);
  }
  if (ebase >= need && c[3 * blockIdx.x] == 0) return;  // nothing of this chunk is taken (uniform)
  uint32_t u[kTkPer], vm;
  const int i0 = blockIdx.x * kTkChunk + threadIdx.x * kTkPer;
  tk_load(keys + (int64_t)b * N, N, i0, u, vm);
  uint32_t gt = 0, eq = 0;
#pragma unroll
  for (int j = 0; j < kTkPer; ++j) {
    gt += u[j] > T;
    eq += u[j] == T && i0 + j < N;
  }
  uint32_t tot;
  uint32_t gs = gbase + tk_block_scan(gt, wsum, &tot);
  uint32_t es = ebase + tk_block_scan(eq, wsum, &tot);
  const uint32_t base = (uint32_t)P - need;
  uint32_t* ck = cand_key + (int64_t)b * P;
  int* ci = cand_idx + (int64_t)b * P;
  // (bounds are guaranteed by the counts -- #(> T) = P - need -- and checked anyway: a wrong slot
  // must not become a wild store)
#pragma unroll
  for (int j = 0; j < kTkPer; ++j) {
    if (u[j] > T) {
      if (gs < base) {
        ck[gs] = u[j];
        ci[gs] = i0 + j;
      }
      ++gs;
    } else if (u[j] == T && i0 + j < N) {
      if (es < need) {
        ck[base + es] = T;
        ci[base + es] = i0 + j;
      }
      ++es;
    }
  }
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
  if (i < P && q == 0 && rank < P && (unsigned)idx < (unsigned)N) {  // ranks: a permutation of 0..P-1 (distinct (key, index) words)
    skeys[(int64_t)b * P + rank] = unord_key((uint32_t)(mine >> 32));
    const float4 bx = *reinterpret_cast<const float4*>(boxes + ((int64_t)b * N + idx) * 4);
    *reinterpret_cast<float4*>(sboxes + ((int64_t)b * P + rank) * 4) = bx;
  }
}

// ---- ranking the P candidates: chunk sort + merge ranks (O(P log P)) -------------------------------
// topk_rank_kernel counts, for every candidate, the candidates above it: O(P^2) compares (79 us at
// P = 12000).  Here each 1024-candidate chunk is bitonic-sorted in LDS and written back in place
// (candidate slots of the chunk, key and index words), then every candidate's rank is its position
// in its chunk plus, for each other chunk, the number of its words above (a binary search over the
// whole sorted candidate set held in LDS: P * 8 B, P <= 20480).  Words (key, ~index) are distinct,
// so the ranks are a permutation and the order is the stable descending one.
constexpr int kTkSortChunk = 1024;
constexpr int kTkMergeMaxP = 20480;  // 160 KB of 8-B words

__global__ void __launch_bounds__(512)
topk_chunk_sort_kernel(uint32_t* __restrict__ cand_key, int* __restrict__ cand_idx, int P) {
  __shared__ uint64_t w[kTkSortChunk];
  const int b = blockIdx.y, c0 = blockIdx.x * kTkSortChunk, tid = threadIdx.x;
  const int len = min(kTkSortChunk, P - c0);
  uint32_t* ck = cand_key + (int64_t)b * P + c0;
  int* ci = cand_idx + (int64_t)b * P + c0;
  for (int i = tid; i < kTkSortChunk; i += 512)
    w[i] = i < len ? ((uint64_t)ck[i] << 32) | (uint32_t)~(uint32_t)ci[i] : 0ull;  // pads sort last
  __syncthreads();
  for (int k = 2; k <= kTkSortChunk; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int i = tid + q * 512, ixj = i ^ j;
        if (ixj > i) {
          const uint64_t a = w[i], c = w[ixj];
          const bool desc = (i & k) == 0;
          if ((a < c) == desc) {
            w[i] = c;
            w[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < len; i += 512) {
    ck[i] = (uint32_t)(w[i] >> 32);
    ci[i] = (int)~(uint32_t)w[i];
  }
}

__global__ void __launch_bounds__(1024)
topk_merge_rank_kernel(const uint32_t* __restrict__ cand_key, const int* __restrict__ cand_idx,
                       const float* __restrict__ boxes, int N, int P, float* __restrict__ skeys,
                       float* __restrict__ sboxes) {
  extern __shared__ uint64_t all[];  // the whole sorted candidate set of this image
  const int b = blockIdx.y, tid = threadIdx.x;
  const uint32_t* ck = cand_key + (int64_t)b * P;
  const int* ci = cand_idx + (int64_t)b * P;
  for (int i = tid; i < P; i += 1024) all[i] = ((uint64_t)ck[i] << 32) | (uint32_t)~(uint32_t)ci[i];
  __syncthreads();
  const int mine = blockIdx.x, p = mine * kTkSortChunk + tid;
  if (p >= P) return;
  const uint64_t v = all[p];
  int rank = tid;  // position in its own (sorted) chunk
  const int nch = (P + kTkSortChunk - 1) / kTkSortChunk;
  for (int c = 0; c < nch; ++c) {
    if (c == mine) continue;
    const uint64_t* s = all + c * kTkSortChunk;
    int lo = 0, hi = min(kTkSortChunk, P - c * kTkSortChunk);  // count of s[] > v: a prefix (descending)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (s[mid] > v) lo = mid + 1;
      else hi = mid;
    }
    rank += lo;
  }
  const int idx = (int)~(uint32_t)v;
  if (rank < P && (unsigned)idx < (unsigned)N) {
    skeys[(int64_t)b * P + rank] = unord_key((uint32_t)(v >> 32));
    const float4 bx = *reinterpret_cast<const float4*>(boxes + ((int64_t)b * N + idx) * 4);
    *reinterpret_cast<float4*>(sboxes + ((int64_t)b * P + rank) * 4) = bx;
  }
}

int64_t proposal_topk_ws_words(int B, int N) { return topk_ws_words(B, (N + kTkChunk - 1) / kTkChunk); }

int proposal_topk(const float* keys, const float* boxes, int B, int N, int P, uint32_t* ws, uint32_t* ws_key,
                  int* ws_idx, float* skeys, float* sboxes, int* n_valid, hipStream_t st) {
  if (B <= 0 || N <= 0 || P <= 0 || P > N || B > 65535) return -1;
  const dim3 grid((N + kTkChunk - 1) / kTkChunk, B);
  // ws: histograms zeroed on entry (atomics); the write kernel zeroes them again after use
  topk_hist_kernel<0><<<grid, kTkThreads, 0, st>>>(keys, N, P, ws);
  topk_hist_kernel<1><<<grid, kTkThreads, 0, st>>>(keys, N, P, ws);
  topk_hist_kernel<2><<<grid, kTkThreads, 0, st>>>(keys, N, P, ws);
  topk_count_kernel<<<grid, kTkThreads, 0, st>>>(keys, N, P, ws);
  topk_write_kernel<<<grid, kTkThreads, 0, st>>>(keys, N, P, ws, ws_key, ws_idx, n_valid);
  if (P <= kTkMergeMaxP) {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)topk_merge_rank_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                kTkMergeMaxP * 8);
      attr = true;
    }
    const dim3 g2(div_up(P, kTkSortChunk), B);
    topk_chunk_sort_kernel<<<g2, 512, 0, st>>>(ws_key, ws_idx, P);
    topk_merge_rank_kernel<<<g2, 1024, (size_t)P * 8, st>>>(ws_key, ws_idx, boxes, N, P, skeys, sboxes);
  } else {
    topk_rank_kernel<<<dim3(div_up(P, 64), B), 256, 0, st>>>(ws_key, ws_idx, boxes, N, P, skeys, sboxes);
  }
  return 0;
}

}  // namespace mxr
