// Test-time detection post-processing on the device (SURVEY kernels K18 / K19).
//
// Reference (`rcnn/tester.py:50-65`, `rcnn/detector.py:74`): per image and per class j >= 1,
// keep RoIs with score > thresh, decode the class's box deltas against the RoI, clip to the
// image, greedy NMS (IoU > 0.3 suppresses), then keep at most max_per_image detections over all
// classes: the score of the max_per_image-th best is the image threshold and every detection
// scoring >= it stays (ties can exceed the cap).  Here that is two launches, no host sync:
//
//   det_class_nms_kernel  grid (B, C-1): one workgroup per (image, class).  Threshold-collect
//       the class scores into LDS (LDS atomic slot counter), bitonic-sort them (score desc, RoI
//       index asc on ties: a fixed, deterministic tie rule -- the reference's `argsort()[::-1]`
//       (helper/processing/nms.py:19) orders tied scores by DESCENDING index after numpy's
//       unstable quicksort, so tied-score parity is unpinned), decode + clip the survivors, greedy
//       NMS over the sorted list (a suppression bitmask resolved by one wave; above 512
//       candidates suppression flags with one barrier per kept box), write the kept (score, box)
//       list of the class.
//   det_topk_kernel       grid B: one workgroup per image.  Radix-select the max_per_image-th
//       largest kept score (4 passes of 8-bit LDS histograms over the float bits; scores are
//       positive so their bits order like the values), then compact the detections scoring >= it
//       in class order into a fixed (cap, 6) output [x1 y1 x2 y2 score class] in ORIGINAL image
//       pixels (boxes / im_scale), plus the count.
//
// nest_kernel (K19, `helper/processing/nms.py:40-70`, predict.py): box i is dropped when
// inter(i, j) / area(i) > thresh for any other box j; one thread per box, the other boxes
// streamed through LDS in 256-box tiles.
#include "common.h"
#include "../kernels.h"

namespace mxr {

constexpr int kDetMaxR = 1024;  // RoIs per image handled by one (image, class) workgroup
constexpr int kDetBits = 512;   // classes with up to this many candidates take the bitmask NMS

__device__ __forceinline__ bool det_before(float sa, int ia, float sb, int ib) {
  return sa > sb || (sa == sb && ia < ib);
}

__global__ void __launch_bounds__(256)
det_class_nms_kernel(const float* __restrict__ rois, const float* __restrict__ scores,
                     const float* __restrict__ deltas, const float* __restrict__ im_info, int R, int C, float thresh,
                     float nms_thresh, float* __restrict__ ks, float* __restrict__ kb, int* __restrict__ kn) {
  __shared__ float key[kDetMaxR];
  __shared__ int idx[kDetMaxR];
  __shared__ float box[kDetMaxR][4];
  __shared__ unsigned char sup[kDetMaxR];
  __shared__ uint64_t smask[kDetBits * (kDetBits / 64)];
  __shared__ int n_s, kept_s;
  const int b = blockIdx.x, c = blockIdx.y + 1, tid = threadIdx.x;
  if (tid == 0) n_s = 0;
  __syncthreads();
  const int64_t base = (int64_t)b * R;
  for (int r = tid; r < R; r += 256) {
    const float s = scores[(base + r) * C + c];
    if (s > thresh) {
      const int slot = atomicAdd(&n_s, 1);
      key[slot] = s;
      idx[slot] = r;
    }
  }
  __syncthreads();
  const int n = n_s;
  int P = 1;
  while (P < n) P <<= 1;
  for (int i = n + tid; i < P; i += 256) {
    key[i] = -INFINITY;
    idx[i] = 0x7fffffff;
  }
  __syncthreads();
  // bitonic sort, descending by (score, -index)
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < P; i += 256) {
        const int l = i ^ j;
        if (l > i) {
          const bool desc = (i & k) == 0;
          const bool swap = desc ? det_before(key[l], idx[l], key[i], idx[i]) : det_before(key[i], idx[i], key[l], idx[l]);
          if (swap) {
            const float tk = key[i];
            key[i] = key[l];
            key[l] = tk;
            const int ti = idx[i];
            idx[i] = idx[l];
            idx[l] = ti;
          }
        }
      }
      __syncthreads();
    }
  }
  // decode + clip (bbox_pred / clip_boxes, +1 pixel convention)
  const float H = im_info[b * 3 + 0], W = im_info[b * 3 + 1];
  for (int i = tid; i < n; i += 256) {
    const int64_t row = base + idx[i];
    const float* ro = rois + row * 5;
    const float w = ro[3] - ro[1] + 1.f, h = ro[4] - ro[2] + 1.f;
    const float cx = ro[1] + 0.5f * (w - 1.f), cy = ro[2] + 0.5f * (h - 1.f);
    const float* d = deltas + row * 4 * C + 4 * c;
    const float pcx = d[0] * w + cx, pcy = d[1] * h + cy;
    const float pw = expf(d[2]) * w, ph = expf(d[3]) * h;
    box[i][0] = fminf(fmaxf(pcx - 0.5f * (pw - 1.f), 0.f), W - 1.f);
    box[i][1] = fminf(fmaxf(pcy - 0.5f * (ph - 1.f), 0.f), H - 1.f);
    box[i][2] = fminf(fmaxf(pcx + 0.5f * (pw - 1.f), 0.f), W - 1.f);
    box[i][3] = fminf(fmaxf(pcy + 0.5f * (ph - 1.f), 0.f), H - 1.f);
    sup[i] = 0;
  }
  __syncthreads();
  if (n <= kDetBits) {
    // greedy NMS in score order as a suppression bitmask: every thread fills words of
    // mask[i][w] (bit t: box i suppresses box 64w + t > i), then ONE wave resolves the boxes in
    // order with the removed set held one 64-bit word per lane -- no barrier per kept box (the
    // loop below pays one per kept box: ~100 us for a class with a few hundred survivors)
    const int nw = (n + 63) >> 6;
    for (int e = tid; e < n * nw; e += 256) {
      const int i = e / nw, w = e - i * nw;
      const float ax1 = box[i][0], ay1 = box[i][1], ax2 = box[i][2], ay2 = box[i][3];
      const float aa = (ax2 - ax1 + 1.f) * (ay2 - ay1 + 1.f);
      uint64_t bits = 0;
      const int j1 = min(n, 64 * w + 64);
      for (int j = max(64 * w, i + 1); j < j1; ++j) {
        const float bb = (box[j][2] - box[j][0] + 1.f) * (box[j][3] - box[j][1] + 1.f);
        if (iou_plus1(ax1, ay1, ax2, ay2, aa, box[j][0], box[j][1], box[j][2], box[j][3], bb) > nms_thresh)
          bits |= 1ull << (j - 64 * w);
      }
      smask[e] = bits;
    }
    __syncthreads();
    if (tid < 64) {
      uint64_t rem = 0;  // lane l: removed bits of boxes 64l .. 64l + 63
      for (int i = 0; i < n; ++i) {
        const uint64_t wi = __shfl(rem, i >> 6, 64);
        if (!((wi >> (i & 63)) & 1ull) && tid < nw) rem |= smask[i * nw + tid];
      }
      for (int j = tid; j < n; j += 64) sup[j] = (unsigned char)((__shfl(rem, j >> 6, 64) >> (j & 63)) & 1ull);
    }
    __syncthreads();
  } else {
  // greedy NMS in score order
  for (int i = 0; i < n; ++i) {
    if (sup[i]) continue;  // uniform: every thread reads the same LDS flag after the barrier
    const float ax1 = box[i][0], ay1 = box[i][1], ax2 = box[i][2], ay2 = box[i][3];
    const float aa = (ax2 - ax1 + 1.f) * (ay2 - ay1 + 1.f);
    for (int j = i + 1 + tid; j < n; j += 256) {
      if (sup[j]) continue;
      const float bb = (box[j][2] - box[j][0] + 1.f) * (box[j][3] - box[j][1] + 1.f);
      if (iou_plus1(ax1, ay1, ax2, ay2, aa, box[j][0], box[j][1], box[j][2], box[j][3], bb) > nms_thresh) sup[j] = 1;
    }
    __syncthreads();
  }
  }
  // compact the kept list (order preserved): one wave ballots 64 flags at a time
  if (tid < 64) {
    int kept = 0;
    const int64_t o = ((int64_t)b * (C - 1) + (c - 1)) * R;
    for (int i0 = 0; i0 < n; i0 += 64) {
      const int i = i0 + tid;
      const bool k = i < n && !sup[i];
      const uint64_t m = __ballot(k);
      if (k) {
        const int pos = kept + __popcll(m & ((1ull << tid) - 1ull));
        ks[o + pos] = key[i];
        float4 bx = make_float4(box[i][0], box[i][1], box[i][2], box[i][3]);
        *reinterpret_cast<float4*>(kb + (o + pos) * 4) = bx;
      }
      kept += __popcll(m);
    }
    if (tid == 0) kn[b * (C - 1) + (c - 1)] = kept;
  }
}

__global__ void __launch_bounds__(256)
det_topk_kernel(const float* __restrict__ ks, const float* __restrict__ kb, const int* __restrict__ kn, int R, int C,
                const float* __restrict__ im_info, int max_per, int cap, float* __restrict__ dets,
                int* __restrict__ counts) {
  __shared__ unsigned int hist[256];
  __shared__ unsigned int prefix_s, remain_s;
  __shared__ int off[1024 + 1];
  __shared__ int kn_s[1024];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nc = C - 1;
  const int64_t cbase = (int64_t)b * nc;
  // per-class kept counts staged in LDS once: the passes below walk the classes wave-parallel
  // (one class per wave at a time, its scores lane-parallel) instead of every thread stepping
  // through all classes in order behind a dependent count load each (4 x 80 serial round trips)
  for (int c = tid; c < nc; c += 256) kn_s[c] = kn[cbase + c];
  __syncthreads();
  // image threshold: the max_per-th largest kept score (0 when fewer are kept)
  int total = 0;
  for (int c = 0; c < nc; ++c) total += kn_s[c];
  unsigned int th_bits = 0;
  if (max_per > 0 && total > max_per) {
    if (tid == 0) {
      prefix_s = 0;
      remain_s = (unsigned int)max_per;  // rank (1-based) of the wanted key among keys matching the prefix
    }
    for (int pass = 3; pass >= 0; --pass) {
      for (int i = tid; i < 256; i += 256) hist[i] = 0;
      __syncthreads();
      const unsigned int pre = prefix_s;
      const unsigned int hi_mask = pass == 3 ? 0u : (0xffffffffu << (8 * (pass + 1)));
      for (int c = wid; c < nc; c += 4) {
        const int cnt = kn_s[c];
        const float* s = ks + (cbase + c) * R;
        for (int i = lane; i < cnt; i += 64) {
          const unsigned int u = __float_as_uint(s[i]);
          if ((u & hi_mask) == (pre & hi_mask)) atomicAdd(&hist[(u >> (8 * pass)) & 255u], 1u);
        }
      }
      __syncthreads();
      if (tid == 0) {
        unsigned int rem = remain_s, acc = 0;
        int bin = 255;
        for (; bin > 0; --bin) {  // from the largest keys down
          if (acc + hist[bin] >= rem) break;
          acc += hist[bin];
        }
        remain_s = rem - acc;
        prefix_s = pre | ((unsigned int)bin << (8 * pass));
      }
      __syncthreads();
    }
    th_bits = prefix_s;
  }
  // per-class selected counts (the kept lists are score-sorted: the selection is a prefix)
  for (int c = tid; c < nc; c += 256) {
    const int cnt = kn_s[c];
    const float* s = ks + (cbase + c) * R;
    int lo = 0, hi = cnt;  // first index with bits < th_bits
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (__float_as_uint(s[mid]) >= th_bits) lo = mid + 1; else hi = mid;
    }
    off[c + 1] = lo;
  }
  __syncthreads();
  if (tid == 0) {
    off[0] = 0;
    for (int c = 0; c < nc; ++c) off[c + 1] += off[c];
    counts[b] = min(off[nc], cap);
  }
  __syncthreads();
  const float inv = 1.f / im_info[b * 3 + 2];
  for (int c = wid; c < nc; c += 4) {
    const int o0 = off[c], cnt = off[c + 1] - off[c];
    for (int i = lane; i < cnt; i += 64) {
      const int dst = o0 + i;
      if (dst >= cap) break;
      const int64_t src = (cbase + c) * R + i;
      float* d = dets + ((int64_t)b * cap + dst) * 6;
      const float4 bx = *reinterpret_cast<const float4*>(kb + src * 4);
      d[0] = bx.x * inv;
      d[1] = bx.y * inv;
      d[2] = bx.z * inv;
      d[3] = bx.w * inv;
      d[4] = ks[src];
      d[5] = (float)(c + 1);
    }
  }
}

int det_postprocess(const float* rois, const float* scores, const float* deltas, const float* im_info, int B, int R,
                    int C, float thresh, float nms_thresh, int max_per, int cap, float* ws_scores, float* ws_boxes,
                    int* ws_counts, float* dets, int* counts, hipStream_t st) {
  if (R > kDetMaxR || C < 2 || C - 1 > 1024 || B <= 0 || cap <= 0) return -1;
  det_class_nms_kernel<<<dim3(B, C - 1), 256, 0, st>>>(rois, scores, deltas, im_info, R, C, thresh, nms_thresh,
                                                        ws_scores, ws_boxes, ws_counts);
  det_topk_kernel<<<B, 256, 0, st>>>(ws_scores, ws_boxes, ws_counts, R, C, im_info, max_per, cap, dets, counts);
  return 0;
}

__global__ void __launch_bounds__(256)
nest_kernel(const float* __restrict__ dets, int n, int stride, float thresh, uint8_t* __restrict__ keep) {
  __shared__ float tile[256][4];
  const int i = blockIdx.x * 256 + threadIdx.x;
  float x1 = 0.f, y1 = 0.f, x2 = 0.f, y2 = 0.f, area = 1.f;
  if (i < n) {
    x1 = dets[(int64_t)i * stride + 0];
    y1 = dets[(int64_t)i * stride + 1];
    x2 = dets[(int64_t)i * stride + 2];
    y2 = dets[(int64_t)i * stride + 3];
    area = (x2 - x1 + 1.f) * (y2 - y1 + 1.f);
  }
  bool k = true;
  for (int t0 = 0; t0 < n; t0 += 256) {
    const int j = t0 + threadIdx.x;
    if (j < n) {
#pragma unroll
      for (int q = 0; q < 4; ++q) tile[threadIdx.x][q] = dets[(int64_t)j * stride + q];
    }
    __syncthreads();
    const int m = min(256, n - t0);
    for (int q = 0; q < m; ++q) {
      if (t0 + q == i) continue;
      const float w = fmaxf(0.f, fminf(x2, tile[q][2]) - fmaxf(x1, tile[q][0]) + 1.f);
      const float h = fmaxf(0.f, fminf(y2, tile[q][3]) - fmaxf(y1, tile[q][1]) + 1.f);
      if (w * h / area > thresh) k = false;
    }
    __syncthreads();
  }
  if (i < n) keep[i] = k ? 1 : 0;
}

int nest_filter(const float* dets, int n, int stride, float thresh, uint8_t* keep, hipStream_t st) {
  if (n <= 0) return 0;
  nest_kernel<<<div_up(n, 256), 256, 0, st>>>(dets, n, stride, thresh, keep);
  return 0;
}

}  // namespace mxr
