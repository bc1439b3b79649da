// IoU matrix reductions and RPN anchor-target assignment (kernels K8/K9;
// reference `rcnn/minibatch.py:204-395`, `rcnn/rpn/proposal_target.py:135-145`,
// `helper/processing/bbox_regression.py:11-31`).
//
// The (N x G) IoU matrix is never materialised: every thread owns one box row and streams
// the image's gt boxes from LDS, keeping the running row max / first argmax in registers.
// The per-gt column max (needed by the "best anchor for each gt is positive" rule) is reduced
// per workgroup in LDS with integer atomicMax on the float bits (IoU >= 0, so the int order
// is the float order), then ONE global atomic per (workgroup, gt).
#include "common.h"
#include "../kernels.h"

namespace mxr {

constexpr int kGtTile = 512;  // gt boxes staged per LDS pass

__global__ void __launch_bounds__(256)
iou_max_kernel(const float* __restrict__ boxes, int bs, int off, int N, const float* __restrict__ gt,
               const int32_t* __restrict__ n_gt, int G, const uint8_t* __restrict__ row_mask,
               float* __restrict__ max_ov, int32_t* __restrict__ argmax, float* __restrict__ gt_max) {
  __shared__ float4 sg[kGtTile];
  __shared__ float sa[kGtTile];
  __shared__ int smax[kGtTile];
  const int b = blockIdx.y;
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int ng = min(n_gt[b], G);
  const bool active = n < N;
  float x1 = 0, y1 = 0, x2 = 0, y2 = 0, area = 0;
  bool use_row = false;
  if (active) {
    const float* p = boxes + ((int64_t)b * N + n) * bs + off;
    x1 = p[0]; y1 = p[1]; x2 = p[2]; y2 = p[3];
    area = (x2 - x1 + 1.f) * (y2 - y1 + 1.f);
    use_row = row_mask ? row_mask[(int64_t)b * N + n] != 0 : true;
  }
  float best = -1.f;
  int arg = 0;
  const float* gb = gt + (int64_t)b * G * 5;
  for (int g0 = 0; g0 < ng; g0 += kGtTile) {
    const int cnt = min(kGtTile, ng - g0);
    __syncthreads();
    for (int k = threadIdx.x; k < cnt; k += blockDim.x) {
      const float* q = gb + (int64_t)(g0 + k) * 5;
      sg[k] = make_float4(q[0], q[1], q[2], q[3]);
      sa[k] = (q[2] - q[0] + 1.f) * (q[3] - q[1] + 1.f);
      smax[k] = 0;
    }
    __syncthreads();
    if (active) {
      for (int k = 0; k < cnt; ++k) {
        const float4 q = sg[k];
        const float ov = iou_plus1(x1, y1, x2, y2, area, q.x, q.y, q.z, q.w, sa[k]);
        if (ov > best) { best = ov; arg = g0 + k; }
        if (gt_max && use_row && ov > 0.f) atomicMax(&smax[k], __float_as_int(ov));
      }
    }
    if (gt_max) {
      __syncthreads();
      for (int k = threadIdx.x; k < cnt; k += blockDim.x)
        if (smax[k] > 0) atomicMax(reinterpret_cast<int*>(gt_max) + (int64_t)b * G + g0 + k, smax[k]);
    }
  }
  if (active) {
    max_ov[(int64_t)b * N + n] = ng > 0 ? best : 0.f;
    argmax[(int64_t)b * N + n] = arg;
  }
}

void iou_max(const float* boxes, int bs, int off, int B, int N, const float* gt, const int32_t* n_gt, int G,
             const uint8_t* row_mask, float* max_ov, int32_t* argmax, float* gt_max, hipStream_t st) {
  if (B == 0 || N == 0) return;
  dim3 grid(div_up(N, 256), B);
  iou_max_kernel<<<grid, 256, 0, st>>>(boxes, bs, off, N, gt, n_gt, G, row_mask, max_ov, argmax, gt_max);
}

// ---------------------------------------------------------------------------------------
// Anchor target.  Pass 1: inside test + IoU row max/argmax + per-gt max over inside anchors.
__device__ __forceinline__ void anchor_box(const float* base, int A, int W, float stride, int64_t t,
                                           float& x1, float& y1, float& x2, float& y2) {
  const int a = (int)(t % A);
  const int64_t hw = t / A;
  const int w = (int)(hw % W), h = (int)(hw / W);
  x1 = base[a * 4 + 0] + w * stride; y1 = base[a * 4 + 1] + h * stride;
  x2 = base[a * 4 + 2] + w * stride; y2 = base[a * 4 + 3] + h * stride;
}

__global__ void __launch_bounds__(256)
anchor_pass1_kernel(const float* __restrict__ base, int A, int H, int W, float stride,
                    const float* __restrict__ im_info, int border, const float* __restrict__ gt,
                    const int32_t* __restrict__ n_gt, int G, float* __restrict__ max_ov,
                    int32_t* __restrict__ argmax, float* __restrict__ gt_max, int32_t* __restrict__ zero_ws,
                    int64_t zero_n) {
  __shared__ float4 sg[kGtTile];
  __shared__ float sa[kGtTile];
  __shared__ int smax[kGtTile];
  const int b = blockIdx.y;
  const int64_t N = (int64_t)H * W * A;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (zero_ws) {  // the sampling chain's mark workspace, consumed by the previous call's output kernel
    const int64_t nt = (int64_t)gridDim.x * gridDim.y * blockDim.x;
    for (int64_t i = ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x; i < zero_n; i += nt)
      zero_ws[i] = 0;
  }
  const int ng = min(n_gt[b], G);
  const float im_h = im_info[b * 3], im_w = im_info[b * 3 + 1];
  float x1 = 0, y1 = 0, x2 = 0, y2 = 0;
  bool inside = false;
  if (t < N) {
    anchor_box(base, A, W, stride, t, x1, y1, x2, y2);
    inside = x1 >= -border && y1 >= -border && x2 < im_w + border && y2 < im_h + border;
  }
  const float area = (x2 - x1 + 1.f) * (y2 - y1 + 1.f);
  float best = -1.f;
  int arg = 0;
  const float* gb = gt + (int64_t)b * G * 5;
  for (int g0 = 0; g0 < ng; g0 += kGtTile) {
    const int cnt = min(kGtTile, ng - g0);
    __syncthreads();
    for (int k = threadIdx.x; k < cnt; k += blockDim.x) {
      const float* q = gb + (int64_t)(g0 + k) * 5;
      sg[k] = make_float4(q[0], q[1], q[2], q[3]);
      sa[k] = (q[2] - q[0] + 1.f) * (q[3] - q[1] + 1.f);
      smax[k] = 0;
    }
    __syncthreads();
    if (inside) {
      for (int k = 0; k < cnt; ++k) {
        const float4 q = sg[k];
        const float ov = iou_plus1(x1, y1, x2, y2, area, q.x, q.y, q.z, q.w, sa[k]);
        if (ov > best) { best = ov; arg = g0 + k; }
        if (ov > 0.f) atomicMax(&smax[k], __float_as_int(ov));
      }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < cnt; k += blockDim.x)
      if (smax[k] > 0) atomicMax(reinterpret_cast<int*>(gt_max) + (int64_t)b * G + g0 + k, smax[k]);
  }
  if (t < N) {
    max_ov[(int64_t)b * N + t] = inside ? (ng > 0 ? best : 0.f) : -1.f;  // -1 marks "outside"
    argmax[(int64_t)b * N + t] = arg;
  }
}

// Pass 2: labels (pre-sampling) and regression targets.
__global__ void __launch_bounds__(256)
anchor_pass2_kernel(const float* __restrict__ base, int A, int H, int W, float stride,
                    const float* __restrict__ gt, const int32_t* __restrict__ n_gt, int G,
                    float neg_thresh, float pos_thresh, int clobber, const float* __restrict__ max_ov,
                    const int32_t* __restrict__ argmax, const float* __restrict__ gt_max,
                    int32_t* __restrict__ label, float* __restrict__ targets, const float* __restrict__ keys,
                    int32_t* __restrict__ hist) {
  __shared__ float4 sg[kGtTile];
  __shared__ float sa[kGtTile];
  __shared__ float sm[kGtTile];
  const int b = blockIdx.y;
  const int64_t N = (int64_t)H * W * A;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int ng = min(n_gt[b], G);
  float x1 = 0, y1 = 0, x2 = 0, y2 = 0, mo = -1.f;
  if (t < N) {
    anchor_box(base, A, W, stride, t, x1, y1, x2, y2);
    mo = max_ov[(int64_t)b * N + t];
  }
  const bool inside = mo >= 0.f;
  const float area = (x2 - x1 + 1.f) * (y2 - y1 + 1.f);
  bool is_gt_best = false;
  const float* gb = gt + (int64_t)b * G * 5;
  for (int g0 = 0; g0 < ng; g0 += kGtTile) {
    const int cnt = min(kGtTile, ng - g0);
    __syncthreads();
    for (int k = threadIdx.x; k < cnt; k += blockDim.x) {
      const float* q = gb + (int64_t)(g0 + k) * 5;
      sg[k] = make_float4(q[0], q[1], q[2], q[3]);
      sa[k] = (q[2] - q[0] + 1.f) * (q[3] - q[1] + 1.f);
      sm[k] = gt_max[(int64_t)b * G + g0 + k];
    }
    __syncthreads();
    if (inside && !is_gt_best) {
      for (int k = 0; k < cnt; ++k) {
        const float4 q = sg[k];
        // exact equality with the column max (reference: where(overlaps == gt_max_overlaps));
        // like the reference this also matches a gt whose best overlap is 0
        if (iou_plus1(x1, y1, x2, y2, area, q.x, q.y, q.z, q.w, sa[k]) == sm[k]) { is_gt_best = true; break; }
      }
    }
  }
  if (t >= N) return;
  int lab = -1;
  float4 tg = make_float4(0.f, 0.f, 0.f, 0.f);
  if (inside) {
    if (ng == 0) {
      lab = 0;
    } else {
      if (!clobber && mo < neg_thresh) lab = 0;
      if (is_gt_best) lab = 1;
      if (mo >= pos_thresh) lab = 1;
      if (clobber && mo < neg_thresh) lab = 0;
      const float* q = gb + (int64_t)argmax[(int64_t)b * N + t] * 5;
      const float ew = x2 - x1 + 1.f, eh = y2 - y1 + 1.f;
      const float ecx = x1 + 0.5f * (ew - 1.f), ecy = y1 + 0.5f * (eh - 1.f);
      const float gw = q[2] - q[0] + 1.f, gh = q[3] - q[1] + 1.f;
      const float gcx = q[0] + 0.5f * (gw - 1.f), gcy = q[1] + 0.5f * (gh - 1.f);
      tg = make_float4((gcx - ecx) / (ew + 1e-14f), (gcy - ecy) / (eh + 1e-14f), logf(gw / ew), logf(gh / eh));
    }
  }
  label[(int64_t)b * N + t] = lab;
  reinterpret_cast<float4*>(targets)[(int64_t)b * N + t] = tg;
  // subsampling histograms (sample.hip anchor_mark): per image and pool (fg, bg), the count of
  // labelled anchors per key bin
  if (hist != nullptr && lab >= 0)
    atomicAdd(hist + ((int64_t)b * 2 + (lab == 1 ? 0 : 1)) * kSampleBins + sample_bin(keys[(int64_t)b * N + t]), 1);
}

void anchor_target_assign(const float* base_anchors, int A, int H, int W, float feat_stride,
                          const float* im_info, int allowed_border, const float* gt, const int32_t* n_gt, int G,
                          int B, float neg_thresh, float pos_thresh, int clobber_positives, float* max_ov,
                          int32_t* argmax, float* gt_max, int32_t* label, float* targets, hipStream_t st,
                          const float* keys, int32_t* hist, int32_t* zero_ws, int64_t zero_n) {
  const int64_t N = (int64_t)H * W * A;
  if (B == 0 || N == 0) return;
  dim3 grid(div_up(N, 256), B);
  anchor_pass1_kernel<<<grid, 256, 0, st>>>(base_anchors, A, H, W, feat_stride, im_info, allowed_border, gt, n_gt,
                                            G, max_ov, argmax, gt_max, zero_ws, zero_n);
  anchor_pass2_kernel<<<grid, 256, 0, st>>>(base_anchors, A, H, W, feat_stride, gt, n_gt, G, neg_thresh,
                                            pos_thresh, clobber_positives, max_ov, argmax, gt_max, label, targets,
                                            keys, hist);
}

}  // namespace mxr
