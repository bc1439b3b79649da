// Host (CPU) twins of the proposal NMS and the RoI max-pool forward, written against raw
// pointers so the same code is linked into the extension (bindings.cpp wraps it in ATen
// tensors and at::parallel_for) and into the sanitizer driver tests/native/host_ops_test.cpp
// (built with -fsanitize=address,undefined and -fsanitize=thread, no torch).
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
inline void nms_greedy(const double* b, int64_t n, double thresh, int64_t max_keep, std::vector<int64_t>& keep) {
  if (n <= 0) return;
  std::vector<double> area(n);
  for (int64_t i = 0; i < n; ++i) area[i] = (b[4 * i + 2] - b[4 * i] + 1.0) * (b[4 * i + 3] - b[4 * i + 1] + 1.0);
  std::vector<uint8_t> removed(n, 0);
  for (int64_t i = 0; i < n; ++i) {
    if (removed[i]) continue;
    keep.push_back(i);
    if (max_keep > 0 && (int64_t)keep.size() >= max_keep) break;
    const double x1 = b[4 * i], y1 = b[4 * i + 1], x2 = b[4 * i + 2], y2 = b[4 * i + 3];
    for (int64_t j = i + 1; j < n; ++j) {
      if (removed[j]) continue;
      const double w = std::min(x2, b[4 * j + 2]) - std::max(x1, b[4 * j]) + 1.0;
      const double h = std::min(y2, b[4 * j + 3]) - std::max(y1, b[4 * j + 1]) + 1.0;
      if (w <= 0.0 || h <= 0.0) continue;
      const double inter = w * h;
      if (inter / (area[i] + area[j] - inter) > thresh) removed[j] = 1;
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

}  // namespace host
}  // namespace mxr
