// Fused RPN anchor-target subsampling and R-CNN proposal-target sampling (SURVEY §2.11-B/C;
// reference `rcnn/minibatch.py:319-395` and `rcnn/rpn/proposal_target.py:135-195`).
//
// The torch formulation of these two steps (random-rank argsort per pool, where/gather/one-hot
// chains) was ~120 tiny launches per training step, each a graph node costing a few
// microseconds regardless of its work.  Here:
//
//   anchor_sample  (1 workgroup / image): fg/bg counts, uniform random subsets without
//                  replacement (fg to RPN_FG_FRACTION * RPN_BATCH_SIZE, bg to the rest), written
//                  as a kept-anchor bitmap + number of examples
//   anchor_output  (grid over anchors): final labels in the reference (a, h, w) order and the
//                  bbox target / inside / outside weights in (4A, H, W) planes
//   proposal_sample (2 workgroups / image: the fg and the bg half of the sample): gt rows appended to
//                  the proposals, fg / bg pools with
//                  the reference fallbacks, fixed-size fg (with-replacement pad prepended) and bg
//                  samples, labels zeroed past fg_this, class-specific normalised targets and
//                  weights (R x 4C)
//
// Random subsets: "the k smallest random keys among the pool" (ties by index) is a uniform
// k-subset.  It is found without sorting the pool: collect the pool members whose key is below
// a threshold t set for ~k + 4 sqrt(k) + 32 expected hits, then rank the (few hundred) hits by
// counting in LDS; t is widened / narrowed in the rare rounds that catch too few / too many.
// The keys are a torch.rand draw (graph-safe Philox offsets), so results are reproducible for a
// fixed generator state; the RNG stream is not numpy's (documented deviation).
#include "common.h"
#include "../kernels.h"

namespace mxr {

constexpr int SEL_CAP = 1024;  // LDS candidate list (one element per thread when ranking)

struct SelScratch {
  float key[SEL_CAP];
  int idx[SEL_CAP];
  int cnt;
};

// Selects take = min(k, count) pool members with the smallest (key, index); writes them in
// ascending key order to out[0..take).  count = |pool|.  take == count needs count <= SEL_CAP.
// Block-uniform arguments; all threads must call.
template <class Pool, class Key>
__device__ int select_smallest(int n, int count, int k, Pool pool, Key key, SelScratch& s, int* out) {
  const int take = min(k, count);
  if (take <= 0) return 0;
  float t = take >= count ? 2.f : fminf(1.f, ((float)take + 4.f * sqrtf((float)take) + 32.f) / (float)count);
  for (int round = 0; round < 48; ++round) {
    if (threadIdx.x == 0) s.cnt = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      if (!pool(i)) continue;
      const float kv = key(i);
      if (kv < t) {
        const int p = atomicAdd(&s.cnt, 1);
        if (p < SEL_CAP) {
          s.key[p] = kv;
          s.idx[p] = i;
        }
      }
    }
    __syncthreads();
    const int c = s.cnt;
    if (c >= take && c <= SEL_CAP) {
      for (int e = threadIdx.x; e < c; e += blockDim.x) {
        const float ke = s.key[e];
        const int ie = s.idx[e];
        int r = 0, j = 0;
        // 8 candidates per step: their (broadcast) LDS reads are issued together, so the loop pays
        // one LDS latency per 8 comparisons instead of one per comparison
        for (; j + 8 <= c; j += 8) {
          float kj[8];
          int ij[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            kj[u] = s.key[j + u];
            ij[u] = s.idx[j + u];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) r += (kj[u] < ke) || (kj[u] == ke && ij[u] < ie);
        }
        for (; j < c; ++j) {
          const float kj = s.key[j];
          r += (kj < ke) || (kj == ke && s.idx[j] < ie);
        }
        if (r < take) out[r] = ie;
      }
      __syncthreads();
      return take;
    }
    __syncthreads();  // every thread has read s.cnt before the next round resets it
    if (c < take) t = t >= 1.f ? 2.f : fminf(1.f, t * 2.f);
    else t *= fmaxf(0.05f, ((float)take + 4.f * sqrtf((float)take) + 32.f) / (float)c);
  }
  return 0;  // not reached for key distributions in [0, 1)
}

// ------------------------------------------------------------------------------- anchors
// label_pre (B, N) int32 in {-1, 0, 1}; keys (B, N) uniform [0,1).  Writes kept (B, NW) uint32
// bitmap (bit = anchor selected), meta (B, 4) int32 = [all_fg, all_bg, n_fg, n_bg].
__global__ void __launch_bounds__(1024)
anchor_sample_kernel(const int32_t* __restrict__ label_pre, const float* __restrict__ keys, int N, int num_fg,
                     int batch, uint32_t* __restrict__ kept, int32_t* __restrict__ meta) {
  __shared__ SelScratch s;
  __shared__ int s_acc;
  __shared__ int sel[SEL_CAP];
  const int b = blockIdx.x;
  const int32_t* lab = label_pre + (int64_t)b * N;
  const float* key = keys + (int64_t)b * N;
  const int NW = (N + 31) / 32;
  uint32_t* kb = kept + (int64_t)b * NW;
  for (int w = threadIdx.x; w < NW; w += blockDim.x) kb[w] = 0u;
  int nfg = 0, nbg = 0;
  {
    int cf = 0, cb = 0;
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
      const int l = lab[i];
      cf += l == 1;
      cb += l == 0;
    }
    if (threadIdx.x == 0) s_acc = 0;
    __syncthreads();
    atomicAdd(&s_acc, cf);
    __syncthreads();
    nfg = s_acc;
    __syncthreads();
    if (threadIdx.x == 0) s_acc = 0;
    __syncthreads();
    atomicAdd(&s_acc, cb);
    __syncthreads();
    nbg = s_acc;
    __syncthreads();
  }
  const bool all_fg = nfg <= num_fg;
  int n_fg = nfg;
  if (!all_fg) {
    n_fg = select_smallest(N, nfg, num_fg, [&](int i) { return lab[i] == 1; }, [&](int i) { return key[i]; }, s, sel);
    for (int e = threadIdx.x; e < n_fg; e += blockDim.x) atomicOr(kb + (sel[e] >> 5), 1u << (sel[e] & 31));
    __syncthreads();
  }
  const int k_bg = max(batch - n_fg, 0);
  const bool all_bg = nbg <= k_bg;
  int n_bg = nbg;
  if (!all_bg) {
    n_bg = select_smallest(N, nbg, k_bg, [&](int i) { return lab[i] == 0; }, [&](int i) { return key[i]; }, s, sel);
    for (int e = threadIdx.x; e < n_bg; e += blockDim.x) atomicOr(kb + (sel[e] >> 5), 1u << (sel[e] & 31));
  }
  if (threadIdx.x == 0) {
    meta[b * 4 + 0] = all_fg;
    meta[b * 4 + 1] = all_bg;
    meta[b * 4 + 2] = n_fg;
    meta[b * 4 + 3] = n_bg;
  }
}

// One thread per (image, anchor a, position hw): reads the (h, w, a)-ordered assignment, writes
// label (B, A*H*W) and the (B, 4A, H, W) target / inside / outside planes.
__global__ void __launch_bounds__(256)
anchor_output_kernel(const int32_t* __restrict__ label_pre, const float* __restrict__ targets,
                     const uint32_t* __restrict__ kept, const int32_t* __restrict__ meta, int B, int A, int HW,
                     float iw0, float iw1, float iw2, float iw3, float pos_weight, int32_t* __restrict__ label,
                     float* __restrict__ bbox_target, float* __restrict__ inside, float* __restrict__ outside,
                     int64_t kept_stride, int32_t* __restrict__ clean_ws = nullptr, int64_t clean_n = 0) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t i = t; i < clean_n; i += (int64_t)gridDim.x * blockDim.x) clean_ws[i] = 0;
  const int64_t per = (int64_t)A * HW;
  if (t >= (int64_t)B * per) return;
  const int b = (int)(t / per);
  const int r = (int)(t % per);
  const int a = r / HW, hw = r % HW;
  const int N = HW * A;
  const int i = hw * A + a;
  const int NW = (N + 31) / 32;
  const int l = label_pre[(int64_t)b * N + i];
  const int32_t* m = meta + b * 4;
  const bool bit = (kept[(int64_t)b * (kept_stride > 0 ? kept_stride : NW) + (i >> 5)] >> (i & 31)) & 1u;
  int lo = -1;
  if (l == 1 && (m[0] || bit)) lo = 1;
  else if (l == 0 && (m[1] || bit)) lo = 0;
  label[(int64_t)b * per + r] = lo;
  const float4 tg = *reinterpret_cast<const float4*>(targets + ((int64_t)b * N + i) * 4);
  float pw, nw;
  if (pos_weight < 0.f) {
    const int ne = max(m[2] + m[3], 1);
    pw = nw = 1.f / (float)ne;
  } else {
    pw = pos_weight / (float)max(m[2], 1);
    nw = (1.f - pos_weight) / (float)max(m[3], 1);
  }
  const float ow = lo == 1 ? pw : (lo == 0 ? nw : 0.f);
  const float fgw = lo == 1 ? 1.f : 0.f;
  const float tv[4] = {tg.x, tg.y, tg.z, tg.w};
  const float iw[4] = {iw0, iw1, iw2, iw3};
  const int64_t base = ((int64_t)b * 4 * A + 4 * a) * HW + hw;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    bbox_target[base + (int64_t)c * HW] = tv[c];
    inside[base + (int64_t)c * HW] = fgw * iw[c];
    outside[base + (int64_t)c * HW] = ow;
  }
}

void anchor_sample(const int32_t* label_pre, const float* targets, const float* keys, int B, int A, int H, int W,
                   int num_fg, int batch, const float* inside_w, float pos_weight, uint32_t* kept_ws,
                   int32_t* meta_ws, int32_t* label, float* bbox_target, float* inside, float* outside,
                   hipStream_t st) {
  if (B == 0) return;
  const int N = H * W * A;
  anchor_sample_kernel<<<B, 1024, 0, st>>>(label_pre, keys, N, num_fg, batch, kept_ws, meta_ws);
  const int64_t total = (int64_t)B * N;
  anchor_output_kernel<<<div_up(total, 256), 256, 0, st>>>(label_pre, targets, kept_ws, meta_ws, B, A, H * W,
                                                           inside_w[0], inside_w[1], inside_w[2], inside_w[3],
                                                           pos_weight, label, bbox_target, inside, outside, 0);
}

// ---- multi-workgroup subsampling -------------------------------------------------------------
// anchor_sample above runs the whole image on one workgroup (~115 us on ResNet-101's 50 400
// anchors, ~400 us on VGG16): every pass over the anchors is one CU's bandwidth.  Here the key
// histograms of the fg / bg pools come from the assignment pass (grid-wide atomics), and one
// grid-wide mark pass selects: with the pool's k-th smallest key in bin T, every member in a bin
// below T is taken, members of bin T are collected into a short list, and the grid's last
// workgroup per image (device-scope counter, release / acquire fences) takes the `rem` smallest
// (key, index) of that list -- exactly the set select_smallest picks, at ~N / 4096 boundary
// candidates instead of N.  An overfull boundary list (pathological key repeats) falls back to
// select_smallest restricted to bin T.
constexpr int kBoundCap = 2048;

struct AnchorThr {
  int tbin[2], rem[2];
  int all_fg, all_bg, n_fg, n_bg;
};

// Block-wide (256 threads): in histogram h (kSampleBins bins), the bin holding the k-th smallest
// key (k >= 1) and how many of that bin's members are taken; total = sum of h.  part: 512 ints LDS.
__device__ void hist_kth(const int32_t* __restrict__ h, int k, int* part, int* res, int& total) {
  const int tid = threadIdx.x;
  constexpr int PER = kSampleBins / 256;
  int v[PER], sum = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    v[j] = h[tid * PER + j];
    sum += v[j];
  }
  part[tid] = sum;
  __syncthreads();
  int* a = part;
  int* bb = part + 256;
  for (int off = 1; off < 256; off <<= 1) {  // inclusive scan (Hillis-Steele, double-buffered)
    bb[tid] = a[tid] + (tid >= off ? a[tid - off] : 0);
    __syncthreads();
    int* t = a;
    a = bb;
    bb = t;
  }
  const int incl = a[tid], excl = incl - sum;
  total = a[255];
  if (k >= 1 && excl < k && k <= incl) {
    int c = excl;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (c + v[j] >= k) {
        res[0] = tid * PER + j;
        res[1] = k - c;
        break;
      }
      c += v[j];
    }
  }
  __syncthreads();
}

// thresholds of both pools (block-uniform result in s)
__device__ void anchor_thresholds(const int32_t* __restrict__ hist, int num_fg, int batch, int* part, AnchorThr& s) {
  int nfg = 0, nbg = 0;
  if (threadIdx.x == 0) {
    s.tbin[0] = s.tbin[1] = kSampleBins;  // "take every member"
    s.rem[0] = s.rem[1] = 0;
  }
  __syncthreads();
  __shared__ int sres[2];
  hist_kth(hist, num_fg, part, sres, nfg);  // writes sres only when num_fg < nfg somewhere
  const bool all_fg = nfg <= num_fg;
  const int n_fg = all_fg ? nfg : num_fg;
  if (threadIdx.x == 0 && !all_fg) {
    s.tbin[0] = num_fg > 0 ? sres[0] : 0;
    s.rem[0] = num_fg > 0 ? sres[1] : 0;
  }
  __syncthreads();
  const int k_bg = max(batch - n_fg, 0);
  hist_kth(hist + kSampleBins, k_bg, part, sres, nbg);
  const bool all_bg = nbg <= k_bg;
  if (threadIdx.x == 0) {
    if (!all_bg) {
      s.tbin[1] = k_bg > 0 ? sres[0] : 0;
      s.rem[1] = k_bg > 0 ? sres[1] : 0;
    }
    s.all_fg = all_fg;
    s.all_bg = all_bg;
    s.n_fg = n_fg;
    s.n_bg = all_bg ? nbg : k_bg;
  }
  __syncthreads();
}

// grid (ceil(N / 256), B) x 256.  ws per image: [kept NW words | bcnt fg, bcnt bg, done, pad | list fg | list bg]
__global__ void __launch_bounds__(256)
anchor_mark_kernel(const int32_t* __restrict__ label_pre, const float* __restrict__ keys,
                   const int32_t* __restrict__ hist, int N, int num_fg, int batch, int32_t* __restrict__ ws,
                   int64_t per, int NW, int32_t* __restrict__ meta) {
  __shared__ int part[512];
  __shared__ AnchorThr thr;
  __shared__ int s_last;
  __shared__ SelScratch sc;
  __shared__ int sel[SEL_CAP];
  const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  const int32_t* h = hist + (int64_t)b * 2 * kSampleBins;
  anchor_thresholds(h, num_fg, batch, part, thr);
  int32_t* base = ws + (int64_t)b * per;
  uint32_t* kept = reinterpret_cast<uint32_t*>(base);
  int32_t* cnt = base + NW;  // [0] fg boundary count, [1] bg, [2] done blocks
  int32_t* list = cnt + 4;   // [2][kBoundCap]
  const int32_t* lab = label_pre + (int64_t)b * N;
  const float* key = keys + (int64_t)b * N;
  const int t = blockIdx.x * 256 + tid;
  bool take = false;
  if (t < N) {
    const int l = lab[t];
    if (l == 0 || l == 1) {
      const int p = l == 1 ? 0 : 1;
      const int bin = sample_bin(key[t]);
      if (bin < thr.tbin[p]) {
        take = true;
      } else if (bin == thr.tbin[p] && thr.rem[p] > 0) {
        const int pos = atomicAdd(cnt + p, 1);
        if (pos < kBoundCap) list[p * kBoundCap + pos] = t;
      }
    }
  }
  const unsigned long long m = __ballot(take);
  if ((lane & 31) == 0 && t < N) {
    const uint32_t wbits = (uint32_t)(m >> (lane & 32));
    if (wbits) atomicOr(kept + (t >> 5), wbits);
  }
  // the last workgroup of this image resolves the boundary bins
  __threadfence();
  __syncthreads();
  if (tid == 0) s_last = atomicAdd(cnt + 2, 1) == (int)gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  for (int p = 0; p < 2; ++p) {
    const int rem = thr.rem[p];
    if (rem <= 0) continue;
    const int c = atomicAdd(cnt + p, 0);
    const int32_t* lp = list + p * kBoundCap;
    if (c <= kBoundCap) {
      for (int e = tid; e < c; e += 256) {
        const int ie = lp[e];
        const float ke = key[ie];
        int r = 0;
        for (int j = 0; j < c; ++j) {
          const int ij = lp[j];
          const float kj = key[ij];
          r += (kj < ke) || (kj == ke && ij < ie);
        }
        if (r < rem) atomicOr(kept + (ie >> 5), 1u << (ie & 31));
      }
    } else {
      const int lv = p == 0 ? 1 : 0, tb = thr.tbin[p];
      const int got = select_smallest(N, c, rem, [&](int i) { return lab[i] == lv && sample_bin(key[i]) == tb; },
                                      [&](int i) { return key[i]; }, sc, sel);
      for (int e = tid; e < got; e += 256) atomicOr(kept + (sel[e] >> 5), 1u << (sel[e] & 31));
    }
    __syncthreads();
  }
  if (tid == 0) {
    meta[b * 4 + 0] = thr.all_fg;
    meta[b * 4 + 1] = thr.all_bg;
    meta[b * 4 + 2] = thr.n_fg;
    meta[b * 4 + 3] = thr.n_bg;
  }
}

int64_t anchor_mark_ws_ints(int B, int64_t N) { return (int64_t)B * (div_up(N, 32) + 4 + 2 * kBoundCap); }

void anchor_sample_hist(const int32_t* label_pre, const float* targets, const float* keys, const int32_t* hist,
                        int B, int A, int H, int W, int num_fg, int batch, const float* inside_w, float pos_weight,
                        int32_t* ws, int32_t* meta, int32_t* label, float* bbox_target, float* inside, float* outside,
                        hipStream_t st, int32_t* clean_ws, int64_t clean_n) {
  if (B == 0) return;
  const int N = H * W * A;
  const int NW = (int)div_up(N, 32);
  const int64_t per = NW + 4 + 2 * kBoundCap;
  anchor_mark_kernel<<<dim3((unsigned)div_up(N, 256), B), 256, 0, st>>>(label_pre, keys, hist, N, num_fg, batch, ws,
                                                                        per, NW, meta);
  const int64_t total = (int64_t)B * N;
  anchor_output_kernel<<<div_up(total, 256), 256, 0, st>>>(label_pre, targets, reinterpret_cast<const uint32_t*>(ws),
                                                           meta, B, A, H * W, inside_w[0], inside_w[1], inside_w[2],
                                                           inside_w[3], pos_weight, label, bbox_target, inside,
                                                           outside, per, clean_ws, clean_n);
}

// ------------------------------------------------------------------------------- proposals
// rois (B, P, 5), gt (B, G, 5) (rows >= n_gt[b] padding), max_ov / argmax (B, P) of the proposal
// rows vs the image's gt (HIP iou_max), rnd (B, 2M + 2R') uniform [0,1) with M = P + G.
// Outputs: out_rois (B*R, 5), label (B*R) int32, bbox_target / inside / outside (B*R, 4C).
constexpr int PT_MAX_ROWS = 16384;  // LDS row arrays: 16384 x 8 B = 128 KB

struct PtParams {
  int P, G, R, F, C;
  float fg_thresh, bg_hi, bg_lo;
  int is_train, normalize;
  float means[4], stds[4], iw[4];
};

__global__ void __launch_bounds__(1024)
proposal_sample_kernel(const float* __restrict__ rois, const float* __restrict__ gt, const int32_t* __restrict__ n_gt,
                       const float* __restrict__ max_ov_p, const int32_t* __restrict__ argmax_p,
                       const float* __restrict__ rnd, const PtParams prm, float* __restrict__ out_rois,
                       int32_t* __restrict__ out_label, float* __restrict__ bbox_target, float* __restrict__ inside,
                       float* __restrict__ outside) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int P = prm.P, G = prm.G, R = prm.R, F = prm.F, C = prm.C;
  const int M = P + G;
  float* s_ov = reinterpret_cast<float*>(smem);                    // [M]
  int* s_am = reinterpret_cast<int*>(s_ov + M);                    // [M]
  SelScratch& s = *reinterpret_cast<SelScratch*>(s_am + M);
  int* sel_fg = reinterpret_cast<int*>(&s + 1);                    // [F]
  int* sel_bg = sel_fg + F;                                        // [R - F]
  int* keep = sel_bg + (R - F);                                    // [R]
  float* s_t = reinterpret_cast<float*>(keep + R);                 // [R][4]
  int* s_lab = reinterpret_cast<int*>(s_t + 4 * R);                // [R]
  int* s_acc = s_lab + R;
  float* gb = reinterpret_cast<float*>(s_acc + 4);                 // [G][5]: the image's gt rows
  const int b = blockIdx.x;
  const int ng = n_gt[b];
  const float* rb = rois + (int64_t)b * P * 5;
  for (int i = threadIdx.x; i < P; i += blockDim.x) {
    s_ov[i] = max_ov_p[(int64_t)b * P + i];
    s_am[i] = argmax_p[(int64_t)b * P + i];
  }
  for (int i = threadIdx.x; i < G * 5; i += blockDim.x) gb[i] = gt[(int64_t)b * G * 5 + i];
  __syncthreads();
  for (int g = threadIdx.x; g < G; g += blockDim.x) {  // gt rows vs gt (first max, like numpy)
    float best = 0.f;
    int bi = 0;
    if (g < ng) {
      const float* q = gb + g * 5;
      const float qa = (q[2] - q[0] + 1.f) * (q[3] - q[1] + 1.f);
      best = -1.f;
      for (int j = 0; j < ng; ++j) {
        const float* o = gb + j * 5;
        const float oa = (o[2] - o[0] + 1.f) * (o[3] - o[1] + 1.f);
        const float v = iou_plus1(q[0], q[1], q[2], q[3], qa, o[0], o[1], o[2], o[3], oa);
        if (v > best) {
          best = v;
          bi = j;
        }
      }
    }
    s_ov[P + g] = best;
    s_am[P + g] = bi;
  }
  __syncthreads();
  auto valid = [&](int i) { return i < P || (i - P) < ng; };
  auto is_fg = [&](int i) { return valid(i) && s_ov[i] >= prm.fg_thresh; };
  auto is_bg0 = [&](int i) { return valid(i) && s_ov[i] < prm.bg_hi && s_ov[i] >= prm.bg_lo; };
  auto is_bgfb = [&](int i) { return valid(i) && s_ov[i] < prm.bg_hi + 0.2f && s_ov[i] >= 0.f; };
  int nfg = 0, nbg0 = 0, nbgfb = 0, nval = 0;
  {
    int a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    for (int i = threadIdx.x; i < M; i += blockDim.x) {
      a0 += is_fg(i);
      a1 += is_bg0(i);
      a2 += is_bgfb(i);
      a3 += valid(i);
    }
    int* acc4 = s_acc;  // 4 counters
    if (threadIdx.x < 4) acc4[threadIdx.x] = 0;
    __syncthreads();
    if (a0) atomicAdd(acc4 + 0, a0);
    if (a1) atomicAdd(acc4 + 1, a1);
    if (a2) atomicAdd(acc4 + 2, a2);
    if (a3) atomicAdd(acc4 + 3, a3);
    __syncthreads();
    nfg = acc4[0];
    nbg0 = acc4[1];
    nbgfb = acc4[2];
    nval = acc4[3];
    __syncthreads();
  }
  const bool bg_use_fb = prm.is_train && nbg0 == 0;
  const int nbg = bg_use_fb ? nbgfb : nbg0;
  const bool fg_any = nfg > 0, bg_any = nbg > 0;
  auto fg_pool = [&](int i) { return fg_any ? is_fg(i) : valid(i); };
  auto bg_pool = [&](int i) { return bg_any ? (bg_use_fb ? is_bgfb(i) : is_bg0(i)) : valid(i); };
  const float* kf = rnd + (int64_t)b * (2 * M + R);
  const float* kg = kf + M;
  const float* ur = kg + M;  // R pad draws: [0, F) fg, [F, R) bg
  const int cf = fg_any ? nfg : nval, cb = bg_any ? nbg : nval;
  // the two halves of the sample are independent: workgroup (b, 0) selects and writes the fg slots
  // [0, F), workgroup (b, 1) the bg slots [F, R) -- the two selections run side by side
  const bool bg_half = blockIdx.y == 1;
  const int j0 = bg_half ? F : 0, j1 = bg_half ? R : F;
  int tf = 0, tb = 0;
  if (!bg_half) tf = select_smallest(M, cf, F, fg_pool, [&](int i) { return kf[i]; }, s, sel_fg);
  else tb = select_smallest(M, cb, R - F, bg_pool, [&](int i) { return kg[i]; }, s, sel_bg);
  // sample_slots: [0, pad) with-replacement picks from the sample, [pad, n) the sample in key order
  for (int j = j0 + threadIdx.x; j < j1; j += blockDim.x) {
    const bool f = j < F;
    const int n = f ? F : R - F, take = f ? tf : tb, jj = f ? j : j - F;
    const int* sl = f ? sel_fg : sel_bg;
    const int pad = n - take;
    int idx = 0;
    if (take > 0) {
      if (jj < pad) idx = sl[min((int)(ur[j] * (float)take), take - 1)];
      else idx = sl[jj - pad];
    }
    keep[j] = idx;
  }
  __syncthreads();
  const int fg_this = min(nfg, F);
  for (int j = j0 + threadIdx.x; j < j1; j += blockDim.x) {
    const int idx = keep[j];
    float bx[5];
    if (idx < P) {
      for (int q = 0; q < 5; ++q) bx[q] = rb[idx * 5 + q];
    } else {
      bx[0] = (float)b;
      for (int q = 0; q < 4; ++q) bx[q + 1] = gb[(idx - P) * 5 + q];
    }
    const int am = s_am[idx];
    const float* gs = gb + min(am, max(G - 1, 0)) * 5;
    int lab = (G > 0 && j < fg_this) ? (int)gs[4] : 0;
    float* ro = out_rois + ((int64_t)b * R + j) * 5;
    for (int q = 0; q < 5; ++q) ro[q] = bx[q];
    out_label[(int64_t)b * R + j] = lab;
    // bbox_transform(ex = roi, gt = assigned gt), optionally (t - mean) / std; zero unless fg
    float t4[4] = {0.f, 0.f, 0.f, 0.f};
    if (lab > 0 && G > 0) {
      const float ew = bx[3] - bx[1] + 1.f, eh = bx[4] - bx[2] + 1.f;
      const float ex = bx[1] + 0.5f * (ew - 1.f), ey = bx[2] + 0.5f * (eh - 1.f);
      const float gw = gs[2] - gs[0] + 1.f, gh = gs[3] - gs[1] + 1.f;
      const float gx = gs[0] + 0.5f * (gw - 1.f), gy = gs[1] + 0.5f * (gh - 1.f);
      t4[0] = (gx - ex) / (ew + 1e-14f);
      t4[1] = (gy - ey) / (eh + 1e-14f);
      t4[2] = logf(gw / ew);
      t4[3] = logf(gh / eh);
      if (prm.normalize)
        for (int q = 0; q < 4; ++q) t4[q] = (t4[q] - prm.means[q]) / prm.stds[q];
    }
    for (int q = 0; q < 4; ++q) s_t[j * 4 + q] = t4[q];
    s_lab[j] = lab;
  }
  __syncthreads();
  // class-specific (R, 4C) rows: one wave per sample row, one float4 (a class's 4 values) per lane
  const int C4 = 4 * C;
  const float4 iw4 = make_float4(prm.iw[0], prm.iw[1], prm.iw[2], prm.iw[3]);
  const float4 ow4 = make_float4(prm.iw[0] > 0.f ? 1.f : 0.f, prm.iw[1] > 0.f ? 1.f : 0.f,
                                 prm.iw[2] > 0.f ? 1.f : 0.f, prm.iw[3] > 0.f ? 1.f : 0.f);
  const int nwaves = blockDim.x >> 6, lane = threadIdx.x & 63;
  for (int j = j0 + (threadIdx.x >> 6); j < j1; j += nwaves) {
    const int lab = s_lab[j];
    const float4 t4 = make_float4(s_t[j * 4], s_t[j * 4 + 1], s_t[j * 4 + 2], s_t[j * 4 + 3]);
    const int64_t row = ((int64_t)b * R + j) * C4;
    float4* bt = reinterpret_cast<float4*>(bbox_target + row);
    float4* in = reinterpret_cast<float4*>(inside + row);
    float4* ou = reinterpret_cast<float4*>(outside + row);
    for (int cls = lane; cls < C; cls += 64) {
      const bool hit = lab > 0 && cls == lab;  // component selects (a float4 select went through scratch)
      bt[cls] = make_float4(hit ? t4.x : 0.f, hit ? t4.y : 0.f, hit ? t4.z : 0.f, hit ? t4.w : 0.f);
      in[cls] = make_float4(hit ? iw4.x : 0.f, hit ? iw4.y : 0.f, hit ? iw4.z : 0.f, hit ? iw4.w : 0.f);
      ou[cls] = make_float4(hit ? ow4.x : 0.f, hit ? ow4.y : 0.f, hit ? ow4.z : 0.f, hit ? ow4.w : 0.f);
    }
  }
}

size_t proposal_sample_lds(int P, int G, int R, int F) {
  const int M = P + G;
  return (size_t)M * 8 + sizeof(SelScratch) + (size_t)(F + (R - F) + R) * 4 + (size_t)R * 16 + (size_t)R * 4 + 16 +
         (size_t)G * 20;
}

int proposal_sample(const float* rois, const float* gt, const int32_t* n_gt, const float* max_ov, const int32_t* argmax,
                    const float* rnd, int B, int P, int G, int R, int F, int C, float fg_thresh, float bg_hi,
                    float bg_lo, int is_train, int normalize, const float* means, const float* stds,
                    const float* inside_w, float* out_rois, int32_t* out_label, float* bbox_target, float* inside,
                    float* outside, hipStream_t st) {
  if (P + G > PT_MAX_ROWS || F > SEL_CAP || R - F > SEL_CAP || F < 0 || F > R) return -1;
  const size_t lds = proposal_sample_lds(P, G, R, F);
  if (lds > 160 * 1024) return -1;
  if (B == 0) return 0;
  PtParams prm;
  prm.P = P; prm.G = G; prm.R = R; prm.F = F; prm.C = C;
  prm.fg_thresh = fg_thresh; prm.bg_hi = bg_hi; prm.bg_lo = bg_lo;
  prm.is_train = is_train; prm.normalize = normalize;
  for (int q = 0; q < 4; ++q) {
    prm.means[q] = means[q];
    prm.stds[q] = stds[q];
    prm.iw[q] = inside_w[q];
  }
  proposal_sample_kernel<<<dim3(B, 2), 1024, lds, st>>>(rois, gt, n_gt, max_ov, argmax, rnd, prm, out_rois, out_label,
                                               bbox_target, inside, outside);
  return 0;
}

}  // namespace mxr
