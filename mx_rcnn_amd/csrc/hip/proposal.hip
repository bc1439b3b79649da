// Fused RPN proposal front end (reference
// `rcnn/rpn/proposal.py:57-119`): fg softmax of the 2-way RPN logits, anchor
// enumeration (base + shift), delta decode, clip to the image and the min-size
// filter, in ONE pass over the RPN head outputs.  One thread per
// (image, h, w, a); consecutive threads walk the anchor index a fastest so the
// NHWC head outputs (channels innermost) are read contiguously.
//
// Deliberate deviation: in TRAIN the reference crops the
// deltas to (int(im_h/16), int(im_w/16)) but not the scores; here both are
// cropped identically (crop_to_im=1), so score/box pairs always line up.
#include "common.h"
#include "../kernels.h"

namespace mxr {

__global__ void __launch_bounds__(256)
proposal_decode_kernel(const void* __restrict__ cls, int cls_bf16, int64_t cs0, int64_t cs1, int64_t cs2, int64_t cs3,
                       const void* __restrict__ dlt, int dlt_bf16, int64_t ds0, int64_t ds1, int64_t ds2, int64_t ds3,
                       int is_prob, const float* __restrict__ im_info, const float* __restrict__ base_anchors, int A,
                       int H, int W, float feat_stride, float min_size, int crop_to_im,
                       float* __restrict__ boxes, float* __restrict__ keys) {
  const int b = blockIdx.y;
  const int64_t N = (int64_t)H * W * A;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N) return;
  const float im_h = im_info[b * 3 + 0], im_w = im_info[b * 3 + 1], im_scale = im_info[b * 3 + 2];
  int Hc = H, Wc = W;
  if (crop_to_im) {
    Hc = min(H, (int)(im_h / feat_stride));
    Wc = min(W, (int)(im_w / feat_stride));
  }
  float4* bo = reinterpret_cast<float4*>(boxes) + (int64_t)b * N + t;
  float* ko = keys + (int64_t)b * N + t;
  if (t >= (int64_t)Hc * Wc * A) {
    *bo = make_float4(0.f, 0.f, 0.f, 0.f);
    *ko = -INFINITY;
    return;
  }
  const int a = (int)(t % A);
  const int64_t hw = t / A;
  const int w = (int)(hw % Wc);
  const int h = (int)(hw / Wc);

  // fg probability: softmax over (bg = channel a, fg = channel A + a)
  const int64_t cb = (int64_t)b * cs0 + (int64_t)h * cs2 + (int64_t)w * cs3;
  float score;
  if (is_prob) {
    score = ld(cls, cb + (int64_t)(A + a) * cs1, cls_bf16);
  } else {
    const float s_bg = ld(cls, cb + (int64_t)a * cs1, cls_bf16);
    const float s_fg = ld(cls, cb + (int64_t)(A + a) * cs1, cls_bf16);
    const float m = fmaxf(s_bg, s_fg);
    const float e_bg = __expf(s_bg - m), e_fg = __expf(s_fg - m);
    score = e_fg / (e_bg + e_fg);
  }
  // anchor (h, w, a)
  const float sx = w * feat_stride, sy = h * feat_stride;
  const float ax1 = base_anchors[a * 4 + 0] + sx, ay1 = base_anchors[a * 4 + 1] + sy;
  const float ax2 = base_anchors[a * 4 + 2] + sx, ay2 = base_anchors[a * 4 + 3] + sy;
  const float aw = ax2 - ax1 + 1.f, ah = ay2 - ay1 + 1.f;
  const float acx = ax1 + 0.5f * (aw - 1.f), acy = ay1 + 0.5f * (ah - 1.f);
  const int64_t db = (int64_t)b * ds0 + (int64_t)h * ds2 + (int64_t)w * ds3 + (int64_t)(4 * a) * ds1;
  const float dx = ld(dlt, db, dlt_bf16), dy = ld(dlt, db + ds1, dlt_bf16);
  const float dw = ld(dlt, db + 2 * ds1, dlt_bf16), dh = ld(dlt, db + 3 * ds1, dlt_bf16);
  const float pcx = dx * aw + acx, pcy = dy * ah + acy;
  const float pw = expf(dw) * aw, ph = expf(dh) * ah;
  float x1 = pcx - 0.5f * (pw - 1.f), y1 = pcy - 0.5f * (ph - 1.f);
  float x2 = pcx + 0.5f * (pw - 1.f), y2 = pcy + 0.5f * (ph - 1.f);
  // clip (clip_boxes): x in [0, im_w-1], y in [0, im_h-1]
  x1 = fmaxf(fminf(x1, im_w - 1.f), 0.f);
  y1 = fmaxf(fminf(y1, im_h - 1.f), 0.f);
  x2 = fmaxf(fminf(x2, im_w - 1.f), 0.f);
  y2 = fmaxf(fminf(y2, im_h - 1.f), 0.f);
  *bo = make_float4(x1, y1, x2, y2);
  const float ms = min_size * im_scale;
  const bool keep = (x2 - x1 + 1.f >= ms) && (y2 - y1 + 1.f >= ms) && !isnan(score);
  *ko = keep ? score : -INFINITY;
}

void proposal_decode(const void* cls, int cls_bf16, int64_t cs0, int64_t cs1, int64_t cs2, int64_t cs3,
                     const void* dlt, int dlt_bf16, int64_t ds0, int64_t ds1, int64_t ds2, int64_t ds3,
                     int is_prob, const float* im_info, const float* base_anchors, int A,
                     int B, int H, int W, float feat_stride, float min_size,
                     int crop_to_im, float* boxes, float* keys, hipStream_t st) {
  const int64_t N = (int64_t)H * W * A;
  if (N == 0 || B == 0) return;
  dim3 grid(div_up(N, 256), B);
  proposal_decode_kernel<<<grid, 256, 0, st>>>(cls, cls_bf16, cs0, cs1, cs2, cs3, dlt, dlt_bf16, ds0, ds1, ds2, ds3,
                                               is_prob, im_info, base_anchors, A, H, W, feat_stride, min_size,
                                               crop_to_im, boxes, keys);
}

}  // namespace mxr

namespace mxr {

// Post-sort assembly of the top-P proposals (one workgroup per image): the first P sorted keys,
// the boxes gathered by the sort order, and the count of valid (finite-key) proposals.  Sorted
// descending, the valid keys form a prefix, so n_valid is the count over the first P.  Replaces
// the slice copy, the gather and the compare / sum / cast chain (five launches) on the proposal
// chain's serial path.
__global__ void __launch_bounds__(1024)
proposal_gather_kernel(const float* __restrict__ skeys, const int64_t* __restrict__ order,
                       const float* __restrict__ boxes, int64_t N, int P, float* __restrict__ out_keys,
                       float* __restrict__ out_boxes, int32_t* __restrict__ n_valid) {
  __shared__ int s_cnt;
  const int b = blockIdx.x;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  const float* kb = skeys + (int64_t)b * N;
  const int64_t* ob = order + (int64_t)b * N;
  const float4* bb = reinterpret_cast<const float4*>(boxes) + (int64_t)b * N;
  int cnt = 0;
  for (int i = threadIdx.x; i < P; i += blockDim.x) {
    const float k = kb[i];
    int64_t o = ob[i];
    o = o < 0 ? 0 : (o >= N ? N - 1 : o);
    out_keys[(int64_t)b * P + i] = k;
    reinterpret_cast<float4*>(out_boxes)[(int64_t)b * P + i] = bb[o];
    cnt += k > -INFINITY;
  }
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
  if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(&s_cnt, cnt);
  __syncthreads();
  if (threadIdx.x == 0) n_valid[b] = s_cnt;
}

void proposal_gather(const float* skeys, const int64_t* order, const float* boxes, int B, int64_t N, int P,
                     float* out_keys, float* out_boxes, int32_t* n_valid, hipStream_t st) {
  if (B == 0) return;
  proposal_gather_kernel<<<B, 1024, 0, st>>>(skeys, order, boxes, N, P, out_keys, out_boxes, n_valid);
}

}  // namespace mxr
