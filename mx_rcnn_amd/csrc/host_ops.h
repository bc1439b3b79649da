// Host (CPU) twins of the frozen BN+ReLU forward, the SGD-momentum update, the RPN / R-CNN softmax-CE and smooth-L1
// losses, the RPN anchor-target assignment, the proposal-target IoU pass, the
// proposal decode, the proposal NMS and the RoI max-pool forward /
// backward, written against raw pointers so the same code is linked into the extension
// (bindings.cpp wraps it in ATen tensors and at::parallel_for) and into the sanitizer driver
// tests/native/host_ops_test.cpp (built with -fsanitize=address,undefined and
// -fsanitize=thread, no torch).
//
// Semantics follow the GPU kernels, which follow the reference:
//   * NMS: greedy over score-sorted boxes, +1-pixel areas, suppress j when IoU(i, j) > thresh
//     (helper/processing/nms.py:4 nms).
//   * RoI pool: MXNet ROIPooling -- roundf corners, float bin edges with floor/ceil, first
//     maximum in row-major order (strict '>'), empty bins -> 0 with argmax -1
//     (rcnn/symbol.py:92 mx.symbol.ROIPooling call site).
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

namespace mxr {
namespace host {

// boxes: n x 4 (x1, y1, x2, y2) in descending-score order.  Kept positions are appended to
// `keep`; max_keep <= 0 means no cap.
// T = double: the reference's float64 proposal arithmetic; T = float: bit-identical to the GPU
// mask kernel's fp32 IoU (iou_plus1), i.e. the oracle of the device reducer's logic
template <typename T>
inline void nms_greedy(const T* b, int64_t n, double thresh, int64_t max_keep, std::vector<int64_t>& keep) {
  if (n <= 0) return;
  const T th = (T)thresh;
  std::vector<T> area(n);
  for (int64_t i = 0; i < n; ++i) area[i] = (b[4 * i + 2] - b[4 * i] + (T)1) * (b[4 * i + 3] - b[4 * i + 1] + (T)1);
  std::vector<uint8_t> removed(n, 0);
  for (int64_t i = 0; i < n; ++i) {
    if (removed[i]) continue;
    keep.push_back(i);
    if (max_keep > 0 && (int64_t)keep.size() >= max_keep) break;
    const T x1 = b[4 * i], y1 = b[4 * i + 1], x2 = b[4 * i + 2], y2 = b[4 * i + 3];
    for (int64_t j = i + 1; j < n; ++j) {
      if (removed[j]) continue;
      const T w = std::min(x2, b[4 * j + 2]) - std::max(x1, b[4 * j]) + (T)1;
      const T h = std::min(y2, b[4 * j + 3]) - std::max(y1, b[4 * j + 1]) + (T)1;
      if (w <= (T)0 || h <= (T)0) continue;
      const T inter = w * h;
      if (inter / (area[i] + area[j] - inter) > th) removed[j] = 1;
    }
  }
}

// RoIs [r0, r1) of a (B, C, H, W) fp32 feature map; out / arg are (R, C, PH, PW) and must be
// pre-filled with 0 / -1 (untouched for empty bins and RoIs with an out-of-range batch index).
// Disjoint RoI ranges write disjoint output rows, so callers may run ranges concurrently.
inline void roi_pool_range(const float* f, int64_t B, int64_t C, int64_t H, int64_t W, const float* ro, int64_t r0,
                           int64_t r1, int64_t PH, int64_t PW, float sc, float* o, int32_t* a) {
  for (int64_t r = r0; r < r1; ++r) {
    const float* roi = ro + r * 5;
    const float bf = roi[0];
    if (!(bf > -1.f) || bf >= (float)B) continue;  // truncation as (int64_t); NaN rejected before the cast
    const int64_t b = (int64_t)bf;
    const int x1 = (int)std::round(roi[1] * sc), y1 = (int)std::round(roi[2] * sc);
    const int x2 = (int)std::round(roi[3] * sc), y2 = (int)std::round(roi[4] * sc);
    const int rw = std::max(x2 - x1 + 1, 1), rh = std::max(y2 - y1 + 1, 1);
    const float bh = (float)rh / (float)PH, bw = (float)rw / (float)PW;
    for (int64_t ph = 0; ph < PH; ++ph) {
      const int hs = (int)std::min<int64_t>(std::max<int64_t>((int64_t)std::floor((float)ph * bh) + y1, 0), H);
      const int he = (int)std::min<int64_t>(std::max<int64_t>((int64_t)std::ceil((float)(ph + 1) * bh) + y1, 0), H);
      for (int64_t pw = 0; pw < PW; ++pw) {
        const int ws = (int)std::min<int64_t>(std::max<int64_t>((int64_t)std::floor((float)pw * bw) + x1, 0), W);
        const int we = (int)std::min<int64_t>(std::max<int64_t>((int64_t)std::ceil((float)(pw + 1) * bw) + x1, 0), W);
        if (he <= hs || we <= ws) continue;
        for (int64_t c = 0; c < C; ++c) {
          const float* fc = f + ((b * C + c) * H) * W;
          float best = fc[hs * W + ws];
          int bi = hs * (int)W + ws;
          for (int h = hs; h < he; ++h)
            for (int w = ws; w < we; ++w) {
              const float v = fc[h * W + w];
              if (v > best) {
                best = v;
                bi = h * (int)W + w;
              }
            }
          const int64_t oi = ((r * C + c) * PH + ph) * PW + pw;
          o[oi] = best;
          a[oi] = bi;
        }
      }
    }
  }
}

// RoI max-pool backward for channels [c0, c1): gin (B, C, H, W) fp32, pre-zeroed; gout / arg
// (R, C, PH*PW).  Each channel's gradients are summed in ascending RoI order, so the result is
// bitwise reproducible and channel ranges can run concurrently without atomics.
inline void roi_pool_bwd_channels(const float* gout, const int32_t* arg, const float* ro, int64_t R, int64_t B,
                                  int64_t C, int64_t H, int64_t W, int64_t PHW, int64_t c0, int64_t c1, float* gin) {
  for (int64_t r = 0; r < R; ++r) {
    const float bf = ro[r * 5];
    if (!(bf > -1.f) || bf >= (float)B) continue;
    const int64_t b = (int64_t)bf;
    for (int64_t c = c0; c < c1; ++c) {
      const float* g = gout + (r * C + c) * PHW;
      const int32_t* a = arg + (r * C + c) * PHW;
      float* dst = gin + (b * C + c) * H * W;
      for (int64_t k = 0; k < PHW; ++k)
        if (a[k] >= 0 && a[k] < H * W) dst[a[k]] += g[k];
    }
  }
}

// One image of the proposal decode (rcnn/rpn/proposal.py:39-149 steps 1-4):
// fg score (softmax over the (bg, fg) logit pair, or the given probability), anchor at
// (x * stride, y * stride) + base[a], +1-convention delta decode, clip to the image, min-size
// filter (filtered / NaN -> key -inf).  cls (2A, H, W), dlt (4A, H, W) NCHW fp32; rows are
// (h, w, a) over the Hc x Wc grid (crop: int(im / stride) as the TRAIN deltas), the rest of
// the H*W*A outputs keep key -inf and box 0.
inline void proposal_decode_image(const float* cls, const float* dlt, int64_t A, int64_t H, int64_t W, float im_h,
                                  float im_w, float im_scale, const float* base, float stride, float min_size,
                                  bool crop, bool is_prob, float* boxes, float* keys) {
  const int64_t N = H * W * A, HW = H * W;
  for (int64_t i = 0; i < N; ++i) {
    keys[i] = -INFINITY;
    boxes[4 * i] = boxes[4 * i + 1] = boxes[4 * i + 2] = boxes[4 * i + 3] = 0.f;
  }
  int64_t Hc = H, Wc = W;
  if (crop) {
    Hc = std::min<int64_t>(H, (int64_t)(im_h / stride));
    Wc = std::min<int64_t>(W, (int64_t)(im_w / stride));
  }
  const float wmax = im_w - 1.f, hmax = im_h - 1.f, ms = min_size * im_scale;
  for (int64_t y = 0; y < Hc; ++y)
    for (int64_t x = 0; x < Wc; ++x)
      for (int64_t a = 0; a < A; ++a) {
        const int64_t pix = y * W + x, row = (y * Wc + x) * A + a;
        float fg;
        if (is_prob) {
          fg = cls[(A + a) * HW + pix];
        } else {
          const float l0 = cls[a * HW + pix], l1 = cls[(A + a) * HW + pix];
          const float m = std::max(l0, l1), e0 = std::exp(l0 - m), e1 = std::exp(l1 - m);
          fg = e1 / (e0 + e1);
        }
        const float ax1 = (float)x * stride + base[4 * a], ay1 = (float)y * stride + base[4 * a + 1];
        const float ax2 = (float)x * stride + base[4 * a + 2], ay2 = (float)y * stride + base[4 * a + 3];
        const float w = ax2 - ax1 + 1.f, h = ay2 - ay1 + 1.f;
        const float cx = ax1 + 0.5f * (w - 1.f), cy = ay1 + 0.5f * (h - 1.f);
        const float* d = dlt + (4 * a) * HW + pix;
        const float pcx = d[0] * w + cx, pcy = d[HW] * h + cy;
        const float pw = std::exp(d[2 * HW]) * w, ph = std::exp(d[3 * HW]) * h;
        float* o = boxes + 4 * row;
        o[0] = std::max(std::min(pcx - 0.5f * (pw - 1.f), wmax), 0.f);
        o[1] = std::max(std::min(pcy - 0.5f * (ph - 1.f), hmax), 0.f);
        o[2] = std::max(std::min(pcx + 0.5f * (pw - 1.f), wmax), 0.f);
        o[3] = std::max(std::min(pcy + 0.5f * (ph - 1.f), hmax), 0.f);
        const bool ok = (o[2] - o[0] + 1.f >= ms) && (o[3] - o[1] + 1.f >= ms) && !std::isnan(fg);
        keys[row] = ok ? fg : -INFINITY;
      }
}

// RPN anchor-target assignment (rcnn/minibatch.py assign_anchor, before the
// fg/bg subsampling), one image.  Anchors are (h, w, a) rows at (x * stride, y * stride) +
// base[a]; an anchor is inside when it lies within the image grown by `border`.  IoU uses
// +1-pixel areas.  Pass 1 (anchor_gt_max) takes each gt's best IoU over the inside anchors;
// pass 2 (anchor_assign_range, anchor rows [n0, n1), runnable concurrently) labels each
// inside anchor: bg if its best IoU < neg, fg if it ties a gt's best or reaches pos (bg rule
// last when clobber), and encodes its best gt.  Outside anchors: label -1, target 0.
inline bool anchor_at(const float* base, int64_t A, int64_t W, float stride, int64_t n, float im_h, float im_w,
                      int border, float* an) {
  const int64_t a = n % A, x = (n / A) % W, y = n / (A * W);
  an[0] = (float)x * stride + base[4 * a];
  an[1] = (float)y * stride + base[4 * a + 1];
  an[2] = (float)x * stride + base[4 * a + 2];
  an[3] = (float)y * stride + base[4 * a + 3];
  return an[0] >= (float)-border && an[1] >= (float)-border && an[2] < im_w + (float)border &&
         an[3] < im_h + (float)border;
}

inline float iou1(const float* a, const float* g) {
  const float iw = std::min(a[2], g[2]) - std::max(a[0], g[0]) + 1.f;
  const float ih = std::min(a[3], g[3]) - std::max(a[1], g[1]) + 1.f;
  if (!(iw > 0.f && ih > 0.f)) return 0.f;
  const float inter = iw * ih;
  const float aa = (a[2] - a[0] + 1.f) * (a[3] - a[1] + 1.f), ga = (g[2] - g[0] + 1.f) * (g[3] - g[1] + 1.f);
  return inter / (aa + ga - inter);
}

// gt: ng rows of stride gt_stride (x1, y1, x2, y2, ...); gmax: ng floats, the best IoU of each gt over
// the inside anchors (-INFINITY when no anchor is inside: then no anchor ever reads it).  A gt whose best
// IoU is 0 marks every inside zero-IoU anchor as its foreground, as in the reference.
inline void anchor_gt_max(const float* base, int64_t A, int64_t H, int64_t W, float stride, float im_h, float im_w,
                          int border, const float* gt, int64_t gt_stride, int64_t ng, float* gmax) {
  for (int64_t g = 0; g < ng; ++g) gmax[g] = -INFINITY;
  float an[4];
  for (int64_t n = 0; n < H * W * A; ++n) {
    if (!anchor_at(base, A, W, stride, n, im_h, im_w, border, an)) continue;
    for (int64_t g = 0; g < ng; ++g) gmax[g] = std::max(gmax[g], iou1(an, gt + g * gt_stride));
  }
}

inline void anchor_assign_range(const float* base, int64_t A, int64_t W, float stride, float im_h, float im_w,
                                int border, const float* gt, int64_t gt_stride, int64_t ng, const float* gmax,
                                float neg, float pos, bool clobber, int64_t n0, int64_t n1, int32_t* labels,
                                float* targets) {
  float an[4];
  for (int64_t n = n0; n < n1; ++n) {
    float* t = targets + 4 * n;
    t[0] = t[1] = t[2] = t[3] = 0.f;
    labels[n] = -1;
    if (!anchor_at(base, A, W, stride, n, im_h, im_w, border, an)) continue;
    if (ng == 0) {
      labels[n] = 0;
      continue;
    }
    float mo = -INFINITY;
    int64_t am = 0;
    bool best = false;
    for (int64_t g = 0; g < ng; ++g) {
      const float v = iou1(an, gt + g * gt_stride);
      if (v > mo) {
        mo = v;
        am = g;
      }
      best = best || v == gmax[g];
    }
    int32_t lab = -1;
    if (!clobber && mo < neg) lab = 0;
    if (best) lab = 1;
    if (mo >= pos) lab = 1;
    if (clobber && mo < neg) lab = 0;
    labels[n] = lab;
    const float* q = gt + am * gt_stride;
    const float ew = an[2] - an[0] + 1.f, eh = an[3] - an[1] + 1.f;
    const float ecx = an[0] + 0.5f * (ew - 1.f), ecy = an[1] + 0.5f * (eh - 1.f);
    const float gw = q[2] - q[0] + 1.f, gh = q[3] - q[1] + 1.f;
    const float gcx = q[0] + 0.5f * (gw - 1.f), gcy = q[1] + 0.5f * (gh - 1.f);
    t[0] = (gcx - ecx) / (ew + 1e-14f);
    t[1] = (gcy - ecy) / (eh + 1e-14f);
    t[2] = std::log(gw / ew);
    t[3] = std::log(gh / eh);
  }
}

// Row max / first argmax of IoU(boxes[n, off:off+4], gt[:ng]) for rows [n0, n1) (the
// proposal-target overlap pass, rcnn/rpn/proposal_target.py _sample_rois bbox_overlaps +
// argmax).  An image without gt gives 0 / 0 (numpy argmax of an all-zero row).
inline void iou_max_rows(const float* boxes, int64_t bstride, int64_t off, int64_t n0, int64_t n1, const float* gt,
                         int64_t gt_stride, int64_t ng, float* mx, int32_t* am) {
  for (int64_t n = n0; n < n1; ++n) {
    const float* a = boxes + n * bstride + off;
    float best = ng > 0 ? -INFINITY : 0.f;
    int32_t bi = 0;
    for (int64_t g = 0; g < ng; ++g) {
      const float v = iou1(a, gt + g * gt_stride);
      if (v > best) {
        best = v;
        bi = (int32_t)g;
      }
    }
    mx[n] = best;
    am[n] = bi;
  }
}

// RPN SoftmaxOutput(multi_output, use_ignore=-1, normalization='valid') in one pass per
// element (rcnn/symbol.py:194 rpn_cls_prob): logits (B, 2A, H, W) viewed as (B, 2, A*H*W)
// (bg = first A channels), label (B, A*H*W) in {-1, 0, 1}.  grad = (p - onehot) * valid *
// grad_scale / max(#valid, 1); returns the mean -log p over the valid labels.  The loss is
// accumulated in double in element order (reproducible).
inline float rpn_softmax_ce(const float* logits, const int32_t* label, int64_t B, int64_t AHW, float grad_scale,
                            float* grad) {
  int64_t nvalid = 0;
  for (int64_t i = 0; i < B * AHW; ++i) nvalid += label[i] >= 0;
  const float norm = (float)std::max<int64_t>(nvalid, 1), gs = grad_scale / norm;
  double loss = 0.0;
  for (int64_t b = 0; b < B; ++b)
    for (int64_t i = 0; i < AHW; ++i) {
      const int64_t i0 = b * 2 * AHW + i, i1 = i0 + AHW;
      const int32_t l = label[b * AHW + i];
      const float m = std::max(logits[i0], logits[i1]);
      const float e0 = std::exp(logits[i0] - m), e1 = std::exp(logits[i1] - m), s = e0 + e1;
      const float p0 = e0 / s, p1 = e1 / s;
      if (l < 0) {
        grad[i0] = grad[i1] = 0.f;
        continue;
      }
      grad[i0] = (p0 - (l == 0 ? 1.f : 0.f)) * gs;
      grad[i1] = (p1 - (l == 1 ? 1.f : 0.f)) * gs;
      loss -= std::log((double)std::max(l == 1 ? p1 : p0, 1e-14f));
    }
  return (float)(loss / norm);
}

// MakeLoss(outside * smooth_l1(inside * (pred - target), sigma), grad_scale) value and
// gradient in one pass (rcnn/symbol.py:378 bbox_loss): f(x) = 0.5 (sigma x)^2 if |x| < 1 /
// sigma^2 else |x| - 0.5 / sigma^2.  Returns sum(outside * f), double-accumulated.
inline float smooth_l1(const float* pred, const float* tgt, const float* iw, const float* ow, int64_t n, float sigma,
                       float grad_scale, float* grad) {
  const float s2 = sigma * sigma;
  double loss = 0.0;
  for (int64_t i = 0; i < n; ++i) {
    const float x = iw[i] * (pred[i] - tgt[i]), ax = std::fabs(x);
    const bool small = ax < 1.f / s2;
    const float f = small ? 0.5f * s2 * x * x : ax - 0.5f / s2;
    const float d = small ? s2 * x : (float)((x > 0.f) - (x < 0.f));
    grad[i] = grad_scale * ow[i] * d * iw[i];
    loss += (double)(ow[i] * f);
  }
  return (float)loss;
}

// SGD with momentum, MXNet semantics (SURVEY 2.9 SGD row): g = clip(rescale * grad, +-clip)
// (clip <= 0: none), mom = momentum * mom - lr * (g + wd * w), w += mom; elements [n0, n1).
inline void sgd_momentum_range(float* w, float* mom, const float* grad, int64_t n0, int64_t n1, float lr,
                               float momentum, float wd, float rescale, float clip) {
  for (int64_t i = n0; i < n1; ++i) {
    float g = grad[i] * rescale;
    if (clip > 0.f) g = std::min(std::max(g, -clip), clip);
    const float m = mom[i] * momentum - lr * (g + wd * w[i]);
    mom[i] = m;
    w[i] += m;
  }
}

// R-CNN head SoftmaxOutput (normalization 'batch' / 'null', rcnn/symbol.py cls_prob) for rows
// [r0, r1) of (R, C) logits: prob = softmax(row), grad = (prob - onehot) * valid * grad_scale /
// norm (label < 0 = ignored row).  Returns the rows' summed -log p (divide by norm outside);
// rows are independent, so ranges may run concurrently.
inline double row_softmax_ce_range(const float* logits, const int32_t* label, int64_t C, int64_t r0, int64_t r1,
                                   float norm, float grad_scale, float* prob, float* grad) {
  double loss = 0.0;
  const float gs = grad_scale / norm;
  for (int64_t r = r0; r < r1; ++r) {
    const float* x = logits + r * C;
    float* p = prob + r * C;
    float m = x[0];
    for (int64_t c = 1; c < C; ++c) m = std::max(m, x[c]);
    float s = 0.f;
    for (int64_t c = 0; c < C; ++c) {
      p[c] = std::exp(x[c] - m);
      s += p[c];
    }
    for (int64_t c = 0; c < C; ++c) p[c] /= s;
    const int32_t l = label[r];
    const bool valid = l >= 0 && l < C;
    for (int64_t c = 0; c < C; ++c) grad[r * C + c] = valid ? (p[c] - (c == l ? 1.f : 0.f)) * gs : 0.f;
    if (valid) loss -= std::log((double)std::max(p[l], 1e-14f));
  }
  return loss;
}

// Frozen BatchNorm (+ReLU) forward, use_global_stats semantics (SURVEY 2.9 BatchNorm row:
// gamma * (x - mean) / sqrt(var + eps) + beta, gamma := 1 with fix_gamma) folded to a
// per-channel scale / shift, elements [n0, n1) of a tensor whose channel of element i is
// (i / inner) % C (inner = H*W for NCHW, 1 for channels_last).
inline void bn_frozen_range(const float* x, float* y, int64_t n0, int64_t n1, int64_t C, int64_t inner,
                            const float* scale, const float* shift, bool relu) {
  for (int64_t i = n0; i < n1; ++i) {
    const int64_t c = (i / inner) % C;
    const float v = x[i] * scale[c] + shift[c];
    y[i] = relu ? std::max(v, 0.f) : v;
  }
}

}  // namespace host
}  // namespace mxr
