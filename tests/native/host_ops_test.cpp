// Sanitizer driver for the host C++ twins in mx_rcnn_amd/csrc/host_ops.h (host
// code under -fsanitize=address,undefined and -fsanitize=thread; device sanitizers are not
// available on this pool).  No torch: built and run by tests/test_native_sanitizers.py.
//
// Checks, each on deterministic pseudo-random inputs:
//   * NMS against an independent IoU-matrix greedy oracle, the max_keep cap, n = 0 / 1,
//     degenerate boxes, bitwise repeatability;
//   * RoI pool against a per-bin brute-force oracle, including RoIs outside the map, bad
//     batch indices (negative, >= B, NaN) and 1-pixel RoIs;
//   * RoI pool backward against a float64 scatter (invalid batch indices, out-of-range
//     argmax), channel ranges on threads bitwise equal to one pass;
//   * proposal decode invariants (scores in [0, 1], boxes clipped, min size, crop rows -inf,
//     NaN score and exp overflow inputs);
//   * anchor assignment: anchor-row ranges on threads bitwise equal to one pass, label
//     invariants with 0 / some / all gt (fg present without clobber, none without gt);
//   * IoU row max: ranges on threads equal one pass, IoU 1 for boxes equal to a gt, no-gt rows;
//   * losses: softmax-CE gradient pairs cancel, ignored labels carry no gradient, large logits
//     stay finite; smooth-L1 gradient bounded by the outside weight and masked by inside;
//   * head softmax-CE: row ranges on threads equal one pass, rows sum to 1, gradients to 0;
//   * frozen BN+ReLU: NCHW and channels_last channel indexing, threaded ranges;
//   * SGD-momentum: element ranges on threads equal one pass and the hand-written update;
//   * RoI pool ranges run concurrently on std::threads equal the serial result (the
//     at::parallel_for contract; -fsanitize=thread checks the disjoint-write claim).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <thread>
#include <vector>

#include "host_ops.h"

namespace {

int g_fail = 0;
#define CHECK(cond, ...)                         \
  do {                                           \
    if (!(cond)) {                               \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);         \
      std::fprintf(stderr, "\n");                \
      ++g_fail;                                  \
    }                                            \
  } while (0)

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed * 6364136223846793005ull + 1442695040888963407ull) {}
  uint32_t next() {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(s >> 33);
  }
  double uni() { return next() / 2147483648.0; }  // [0, 1)
};

std::vector<double> rand_boxes(Rng& g, int64_t n, double extent) {
  std::vector<double> b(4 * n);
  for (int64_t i = 0; i < n; ++i) {
    const double x = g.uni() * extent, y = g.uni() * extent;
    const double w = g.uni() * extent * 0.3, h = g.uni() * extent * 0.3;
    b[4 * i] = x;
    b[4 * i + 1] = y;
    b[4 * i + 2] = x + w;
    b[4 * i + 3] = y + h;
  }
  return b;
}

// oracle: full IoU matrix first, then the greedy pass
std::vector<int64_t> nms_oracle(const std::vector<double>& b, int64_t n, double thr, int64_t max_keep) {
  std::vector<double> iou(n * n, 0.0);
  for (int64_t i = 0; i < n; ++i)
    for (int64_t j = 0; j < n; ++j) {
      const double ai = (b[4 * i + 2] - b[4 * i] + 1) * (b[4 * i + 3] - b[4 * i + 1] + 1);
      const double aj = (b[4 * j + 2] - b[4 * j] + 1) * (b[4 * j + 3] - b[4 * j + 1] + 1);
      const double w = std::fmin(b[4 * i + 2], b[4 * j + 2]) - std::fmax(b[4 * i], b[4 * j]) + 1;
      const double h = std::fmin(b[4 * i + 3], b[4 * j + 3]) - std::fmax(b[4 * i + 1], b[4 * j + 1]) + 1;
      if (w > 0 && h > 0) iou[i * n + j] = w * h / (ai + aj - w * h);
    }
  std::vector<int64_t> keep;
  std::vector<char> dead(n, 0);
  for (int64_t i = 0; i < n; ++i) {
    if (dead[i]) continue;
    if (max_keep > 0 && (int64_t)keep.size() >= max_keep) break;
    keep.push_back(i);
    for (int64_t j = i + 1; j < n; ++j)
      if (iou[i * n + j] > thr) dead[j] = 1;
  }
  return keep;
}

void test_nms() {
  Rng g(7);
  for (int trial = 0; trial < 40; ++trial) {
    const int64_t n = 1 + (int64_t)(g.uni() * 600);
    const double thr = trial % 3 == 0 ? 0.3 : 0.7;
    const int64_t cap = trial % 4 == 0 ? 1 + (int64_t)(g.uni() * 50) : -1;
    std::vector<double> b = rand_boxes(g, n, 500.0);
    if (trial % 5 == 0) {  // degenerate boxes: zero / negative extents
      b[0] = b[2] = 10.0;
      if (n > 1) b[4 + 2] = b[4] - 3.0;
    }
    std::vector<int64_t> k1, k2;
    mxr::host::nms_greedy(b.data(), n, thr, cap, k1);
    mxr::host::nms_greedy(b.data(), n, thr, cap, k2);
    const std::vector<int64_t> ref = nms_oracle(b, n, thr, cap);
    CHECK(k1 == ref, "nms trial %d: %zu kept vs oracle %zu", trial, k1.size(), ref.size());
    CHECK(k1 == k2, "nms trial %d not repeatable", trial);
    if (cap > 0) CHECK((int64_t)k1.size() <= cap, "nms cap exceeded");
  }
  std::vector<int64_t> k;
  mxr::host::nms_greedy<float>(nullptr, 0, 0.7, -1, k);
  CHECK(k.empty(), "nms n=0");
  const double one[4] = {1, 2, 3, 4};
  mxr::host::nms_greedy(one, 1, 0.7, -1, k);
  CHECK(k.size() == 1 && k[0] == 0, "nms n=1");
}

void roi_oracle(const std::vector<float>& f, int64_t B, int64_t C, int64_t H, int64_t W, const float* roi, int64_t PH,
                int64_t PW, float sc, float* o, int32_t* a) {
  // same bin definition, independently written: per bin, scan all pixels and keep those inside
  const float bf = roi[0];
  if (!(bf > -1.f) || bf >= (float)B) return;
  const int64_t b = (int64_t)bf;
  const int x1 = (int)std::round(roi[1] * sc), y1 = (int)std::round(roi[2] * sc);
  const int x2 = (int)std::round(roi[3] * sc), y2 = (int)std::round(roi[4] * sc);
  const float bh = (float)std::max(y2 - y1 + 1, 1) / (float)PH, bw = (float)std::max(x2 - x1 + 1, 1) / (float)PW;
  for (int64_t c = 0; c < C; ++c)
    for (int64_t ph = 0; ph < PH; ++ph)
      for (int64_t pw = 0; pw < PW; ++pw) {
        const long hs = (long)std::floor((float)ph * bh) + y1, he = (long)std::ceil((float)(ph + 1) * bh) + y1;
        const long ws = (long)std::floor((float)pw * bw) + x1, we = (long)std::ceil((float)(pw + 1) * bw) + x1;
        float best = -std::numeric_limits<float>::infinity();
        int bi = -1;
        for (long h = 0; h < H; ++h)
          for (long w = 0; w < W; ++w) {
            if (h < hs || h >= he || w < ws || w >= we) continue;
            const float v = f[((b * C + c) * H + h) * W + w];
            if (bi < 0 || v > best) {
              best = v;
              bi = (int)(h * W + w);
            }
          }
        const int64_t oi = (c * PH + ph) * PW + pw;
        o[oi] = bi < 0 ? 0.f : best;
        a[oi] = bi;
      }
}

void test_roi_pool() {
  Rng g(11);
  const int64_t B = 2, C = 5, H = 23, W = 31, PH = 7, PW = 7, R = 64;
  const float sc = 1.f / 16.f;
  std::vector<float> f(B * C * H * W);
  for (auto& v : f) v = (float)(g.uni() * 2 - 1);
  std::vector<float> rois(R * 5);
  for (int64_t r = 0; r < R; ++r) {
    float* q = &rois[r * 5];
    q[0] = (float)(r % B);
    const float x = (float)(g.uni() * W * 16 * 1.2 - 40), y = (float)(g.uni() * H * 16 * 1.2 - 40);
    q[1] = x;
    q[2] = y;
    q[3] = x + (float)(g.uni() * 300);
    q[4] = y + (float)(g.uni() * 300);
  }
  rois[5 * 3] = -1.f;                                     // negative batch index: skipped
  rois[5 * 4] = (float)B;                                 // batch index past the end: skipped
  rois[5 * 5] = std::numeric_limits<float>::quiet_NaN();  // NaN batch index: skipped
  rois[5 * 6 + 3] = rois[5 * 6 + 1];                      // 1-pixel wide RoI
  rois[5 * 6 + 4] = rois[5 * 6 + 2];
  rois[5 * 7 + 1] = rois[5 * 7 + 3] = 5000.f;             // entirely right of the map
  const int64_t per = C * PH * PW;
  std::vector<float> o(R * per, 0.f);
  std::vector<int32_t> a(R * per, -1);
  mxr::host::roi_pool_range(f.data(), B, C, H, W, rois.data(), 0, R, PH, PW, sc, o.data(), a.data());
  std::vector<float> ro(per);
  std::vector<int32_t> ra(per);
  for (int64_t r = 0; r < R; ++r) {
    std::fill(ro.begin(), ro.end(), 0.f);
    std::fill(ra.begin(), ra.end(), -1);
    roi_oracle(f, B, C, H, W, &rois[r * 5], PH, PW, sc, ro.data(), ra.data());
    CHECK(std::memcmp(ro.data(), &o[r * per], per * sizeof(float)) == 0, "roi %ld values differ", (long)r);
    CHECK(std::memcmp(ra.data(), &a[r * per], per * sizeof(int32_t)) == 0, "roi %ld argmax differs", (long)r);
  }
  for (int r : {3, 4, 5, 7})
    for (int64_t i = 0; i < per; ++i) CHECK(a[r * per + i] == -1 && o[r * per + i] == 0.f, "roi %d must be empty", r);

  // concurrent disjoint ranges (the at::parallel_for split) == serial, bitwise
  std::vector<float> o2(R * per, 0.f);
  std::vector<int32_t> a2(R * per, -1);
  const int T = 4;
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    const int64_t r0 = R * t / T, r1 = R * (t + 1) / T;
    th.emplace_back([&, r0, r1] {
      mxr::host::roi_pool_range(f.data(), B, C, H, W, rois.data(), r0, r1, PH, PW, sc, o2.data(), a2.data());
    });
  }
  for (auto& x : th) x.join();
  CHECK(std::memcmp(o.data(), o2.data(), o.size() * sizeof(float)) == 0, "threaded roi pool values differ");
  CHECK(std::memcmp(a.data(), a2.data(), a.size() * sizeof(int32_t)) == 0, "threaded roi pool argmax differs");
}

void test_roi_pool_bwd() {
  Rng g(13);
  const int64_t B = 2, C = 6, H = 17, W = 21, PHW = 49, R = 40;
  std::vector<float> gout(R * C * PHW), rois(R * 5, 0.f);
  std::vector<int32_t> arg(R * C * PHW);
  for (auto& v : gout) v = (float)(g.uni() - 0.5);
  for (auto& v : arg) v = (int32_t)(g.uni() * (H * W + 8)) - 4;  // includes -1..-4 and > H*W: skipped
  for (int64_t r = 0; r < R; ++r) rois[r * 5] = (float)(r % (B + 1)) - (r % 7 == 0 ? 3.f : 0.f);  // some invalid
  std::vector<double> ref(B * C * H * W, 0.0);
  for (int64_t r = 0; r < R; ++r) {
    const float bf = rois[r * 5];
    if (!(bf > -1.f) || bf >= (float)B) continue;
    const int64_t b = (int64_t)bf;
    for (int64_t c = 0; c < C; ++c)
      for (int64_t k = 0; k < PHW; ++k) {
        const int32_t a = arg[(r * C + c) * PHW + k];
        if (a >= 0 && a < H * W) ref[(b * C + c) * H * W + a] += gout[(r * C + c) * PHW + k];
      }
  }
  std::vector<float> gin(B * C * H * W, 0.f), gin2(B * C * H * W, 0.f);
  mxr::host::roi_pool_bwd_channels(gout.data(), arg.data(), rois.data(), R, B, C, H, W, PHW, 0, C, gin.data());
  for (size_t i = 0; i < gin.size(); ++i) CHECK(std::fabs(gin[i] - ref[i]) < 1e-4, "bwd %zu: %f vs %f", i, gin[i], ref[i]);
  std::vector<std::thread> th;
  for (int t = 0; t < 3; ++t)
    th.emplace_back([&, t] {
      mxr::host::roi_pool_bwd_channels(gout.data(), arg.data(), rois.data(), R, B, C, H, W, PHW, C * t / 3,
                                       C * (t + 1) / 3, gin2.data());
    });
  for (auto& x : th) x.join();
  CHECK(std::memcmp(gin.data(), gin2.data(), gin.size() * sizeof(float)) == 0, "threaded bwd differs");
}

void test_proposal_decode() {
  Rng g(17);
  const int64_t A = 9, H = 19, W = 25, N = H * W * A;
  std::vector<float> cls(2 * A * H * W), dlt(4 * A * H * W), base(4 * A);
  for (auto& v : cls) v = (float)(g.uni() * 6 - 3);
  for (auto& v : dlt) v = (float)(g.uni() - 0.5);
  dlt[7] = std::numeric_limits<float>::infinity();  // exp overflow path
  cls[5] = std::numeric_limits<float>::quiet_NaN();  // NaN score -> filtered
  for (int64_t a = 0; a < A; ++a) {
    const float s = 8.f * (float)(1 + a % 3) * 4.f;
    base[4 * a] = -s;
    base[4 * a + 1] = -s / (1 + a / 3);
    base[4 * a + 2] = s + 15.f;
    base[4 * a + 3] = s / (1 + a / 3) + 15.f;
  }
  const float im_h = 250.f, im_w = 330.f;  // crop grid 15 x 20 < 19 x 25
  for (int crop = 0; crop < 2; ++crop) {
    std::vector<float> boxes(4 * N), keys(N);
    mxr::host::proposal_decode_image(cls.data(), dlt.data(), A, H, W, im_h, im_w, 1.f, base.data(), 16.f, 16.f,
                                     crop != 0, false, boxes.data(), keys.data());
    const int64_t Hc = crop ? 15 : H, Wc = crop ? 20 : W;
    int64_t n_fin = 0;
    for (int64_t i = 0; i < N; ++i) {
      if (i >= Hc * Wc * A) CHECK(std::isinf(keys[i]) && keys[i] < 0, "row %ld beyond the grid must be -inf", (long)i);
      if (!std::isfinite(keys[i])) continue;
      ++n_fin;
      CHECK(keys[i] >= 0.f && keys[i] <= 1.f, "score %f out of [0, 1]", keys[i]);
      const float* b = &boxes[4 * i];
      CHECK(b[0] >= 0 && b[2] <= im_w - 1 && b[1] >= 0 && b[3] <= im_h - 1, "box %ld outside the image", (long)i);
      CHECK(b[2] - b[0] + 1 >= 16.f && b[3] - b[1] + 1 >= 16.f, "box %ld below min size", (long)i);
    }
    CHECK(n_fin > N / 10, "too few boxes survive (%ld)", (long)n_fin);
  }
}

void test_anchor_assign() {
  Rng g(19);
  const int64_t A = 9, H = 21, W = 27, N = H * W * A, G = 5, gs = 5;
  std::vector<float> base(4 * A), gt(G * gs, 0.f);
  for (int64_t a = 0; a < A; ++a) {
    const float s = 16.f * (float)(1 + a % 3), r = 1.f + (float)(a / 3) * 0.5f;
    base[4 * a] = -s * r;
    base[4 * a + 1] = -s / r;
    base[4 * a + 2] = s * r + 15.f;
    base[4 * a + 3] = s / r + 15.f;
  }
  for (int64_t i = 0; i < G; ++i) {
    const float x = (float)(g.uni() * 350), y = (float)(g.uni() * 260), w = (float)(g.uni() * 120 + 8);
    gt[i * gs] = x;
    gt[i * gs + 1] = y;
    gt[i * gs + 2] = x + w;
    gt[i * gs + 3] = y + w * 0.7f;
  }
  const float im_h = 330.f, im_w = 430.f;
  for (int clobber = 0; clobber < 2; ++clobber)
    for (int64_t ng : {(int64_t)0, (int64_t)2, G}) {
      std::vector<float> gmax(G), t1(4 * N), t2(4 * N);
      std::vector<int32_t> l1(N), l2(N);
      mxr::host::anchor_gt_max(base.data(), A, H, W, 16.f, im_h, im_w, 0, gt.data(), gs, ng, gmax.data());
      mxr::host::anchor_assign_range(base.data(), A, W, 16.f, im_h, im_w, 0, gt.data(), gs, ng, gmax.data(), 0.3f,
                                     0.7f, clobber != 0, 0, N, l1.data(), t1.data());
      std::vector<std::thread> th;
      for (int t = 0; t < 4; ++t)
        th.emplace_back([&, t] {
          mxr::host::anchor_assign_range(base.data(), A, W, 16.f, im_h, im_w, 0, gt.data(), gs, ng, gmax.data(),
                                         0.3f, 0.7f, clobber != 0, N * t / 4, N * (t + 1) / 4, l2.data(), t2.data());
        });
      for (auto& x : th) x.join();
      CHECK(l1 == l2 && std::memcmp(t1.data(), t2.data(), t1.size() * sizeof(float)) == 0,
            "threaded anchor assignment differs (ng %ld)", (long)ng);
      int64_t nfg = 0, nbg = 0;
      for (int64_t n = 0; n < N; ++n) {
        CHECK(l1[n] >= -1 && l1[n] <= 1, "label %d", l1[n]);
        nfg += l1[n] == 1;
        nbg += l1[n] == 0;
        if (l1[n] != 1) CHECK(t1[4 * n] == 0.f || ng > 0, "target without gt");
      }
      // without clobber every gt's best anchor is fg; with clobber the bg rule may override it
      CHECK(ng == 0 ? nfg == 0 && nbg > 0 : (clobber || nfg >= 1), "fg %ld bg %ld with %ld gt", (long)nfg, (long)nbg,
            (long)ng);
    }
}

void test_iou_max() {
  Rng g(23);
  const int64_t N = 300, bs = 5, G = 6;
  std::vector<float> boxes(N * bs), gt(G * 5);
  for (int64_t n = 0; n < N; ++n) {
    const float x = (float)(g.uni() * 400), y = (float)(g.uni() * 300);
    boxes[n * bs] = 0.f;
    boxes[n * bs + 1] = x;
    boxes[n * bs + 2] = y;
    boxes[n * bs + 3] = x + (float)(g.uni() * 120);
    boxes[n * bs + 4] = y + (float)(g.uni() * 120);
  }
  for (int64_t j = 0; j < G; ++j)
    for (int k = 0; k < 4; ++k) gt[j * 5 + k] = boxes[(j * 37) * bs + 1 + k];  // gt j == box 37 j
  for (int64_t ng : {(int64_t)0, G}) {
    std::vector<float> m1(N), m2(N);
    std::vector<int32_t> a1(N), a2(N);
    mxr::host::iou_max_rows(boxes.data(), bs, 1, 0, N, gt.data(), 5, ng, m1.data(), a1.data());
    std::vector<std::thread> th;
    for (int t = 0; t < 3; ++t)
      th.emplace_back([&, t] {
        mxr::host::iou_max_rows(boxes.data(), bs, 1, N * t / 3, N * (t + 1) / 3, gt.data(), 5, ng, m2.data(),
                                a2.data());
      });
    for (auto& x : th) x.join();
    CHECK(m1 == m2 && a1 == a2, "threaded iou_max differs");
    for (int64_t n = 0; n < N; ++n) {
      CHECK(m1[n] >= 0.f && m1[n] <= 1.f && a1[n] >= 0 && a1[n] < std::max<int64_t>(ng, 1), "row %ld", (long)n);
      if (ng == 0) CHECK(m1[n] == 0.f && a1[n] == 0, "no-gt row %ld", (long)n);
    }
    if (ng > 0)
      for (int64_t j = 0; j < G; ++j) CHECK(m1[j * 37] == 1.f, "box equal to gt %ld must have IoU 1", (long)j);
  }
}

void test_losses() {
  Rng g(29);
  const int64_t B = 2, AHW = 9 * 5 * 7;
  std::vector<float> logits(B * 2 * AHW), grad(B * 2 * AHW);
  std::vector<int32_t> label(B * AHW);
  for (auto& v : logits) v = (float)(g.uni() * 40 - 20);  // large logits: exp stability
  for (auto& l : label) l = (int32_t)(g.uni() * 3) - 1;
  const float loss = mxr::host::rpn_softmax_ce(logits.data(), label.data(), B, AHW, 1.f, grad.data());
  CHECK(std::isfinite(loss) && loss >= 0.f, "rpn ce loss %f", loss);
  for (int64_t b = 0; b < B; ++b)
    for (int64_t i = 0; i < AHW; ++i) {
      const float g0 = grad[b * 2 * AHW + i], g1 = grad[b * 2 * AHW + AHW + i];
      CHECK(std::fabs(g0 + g1) < 1e-6f, "softmax grads of one anchor must cancel");
      if (label[b * AHW + i] < 0) CHECK(g0 == 0.f && g1 == 0.f, "ignored label with gradient");
    }
  std::vector<int32_t> none(B * AHW, -1);
  CHECK(mxr::host::rpn_softmax_ce(logits.data(), none.data(), B, AHW, 1.f, grad.data()) == 0.f, "all ignored");
  const int64_t n = 4 * 21 * 16;
  std::vector<float> p(n), t(n), iw(n), ow(n), gr(n);
  for (int64_t i = 0; i < n; ++i) {
    p[i] = (float)(g.uni() * 4 - 2);
    t[i] = (float)(g.uni() * 4 - 2);
    iw[i] = g.uni() < 0.5 ? 1.f : 0.f;
    ow[i] = iw[i] / 16.f;
  }
  const float sl = mxr::host::smooth_l1(p.data(), t.data(), iw.data(), ow.data(), n, 3.f, 1.f, gr.data());
  CHECK(std::isfinite(sl) && sl >= 0.f, "smooth l1 %f", sl);
  for (int64_t i = 0; i < n; ++i) {
    if (iw[i] == 0.f) CHECK(gr[i] == 0.f, "masked element with gradient");
    CHECK(std::fabs(gr[i]) <= 1.f / 16.f + 1e-7f, "smooth-L1 gradient not bounded by the outside weight");
  }
}

void test_sgd() {
  Rng g(37);
  const int64_t n = 10007;
  std::vector<float> w(n), m(n), gr(n);
  for (int64_t i = 0; i < n; ++i) {
    w[i] = (float)(g.uni() - 0.5);
    m[i] = (float)(g.uni() - 0.5) * 0.1f;
    gr[i] = (float)(g.uni() * 4 - 2);
  }
  std::vector<float> w1 = w, m1 = m, w2 = w, m2 = m;
  mxr::host::sgd_momentum_range(w1.data(), m1.data(), gr.data(), 0, n, 0.01f, 0.9f, 5e-4f, 0.5f, 0.3f);
  std::vector<std::thread> th;
  for (int t = 0; t < 4; ++t)
    th.emplace_back([&, t] {
      mxr::host::sgd_momentum_range(w2.data(), m2.data(), gr.data(), n * t / 4, n * (t + 1) / 4, 0.01f, 0.9f, 5e-4f,
                                    0.5f, 0.3f);
    });
  for (auto& x : th) x.join();
  CHECK(w1 == w2 && m1 == m2, "threaded SGD differs");
  for (int64_t i = 0; i < n; i += 997) {
    const float gc = std::min(std::max(gr[i] * 0.5f, -0.3f), 0.3f);
    const float me = m[i] * 0.9f - 0.01f * (gc + 5e-4f * w[i]);
    CHECK(m1[i] == me && w1[i] == w[i] + me, "SGD element %ld", (long)i);
  }
}

void test_row_softmax_ce() {
  Rng g(41);
  const int64_t R = 257, C = 21;
  std::vector<float> x(R * C), p1(R * C), g1(R * C), p2(R * C), g2(R * C);
  std::vector<int32_t> lab(R);
  for (auto& v : x) v = (float)(g.uni() * 60 - 30);
  for (auto& l : lab) l = (int32_t)(g.uni() * (C + 1)) - 1;
  const double l1 = mxr::host::row_softmax_ce_range(x.data(), lab.data(), C, 0, R, (float)R, 1.f, p1.data(), g1.data());
  double parts[4];
  std::vector<std::thread> th;
  for (int t = 0; t < 4; ++t)
    th.emplace_back([&, t] {
      parts[t] = mxr::host::row_softmax_ce_range(x.data(), lab.data(), C, R * t / 4, R * (t + 1) / 4, (float)R, 1.f,
                                                 p2.data(), g2.data());
    });
  for (auto& x_ : th) x_.join();
  CHECK(p1 == p2 && g1 == g2, "threaded row CE differs");
  CHECK(std::fabs(l1 - (parts[0] + parts[1] + parts[2] + parts[3])) < 1e-9 * std::max(1.0, l1), "row CE partials");
  for (int64_t r = 0; r < R; ++r) {
    double ps = 0.0, gsum = 0.0;
    for (int64_t c = 0; c < C; ++c) {
      ps += p1[r * C + c];
      gsum += g1[r * C + c];
    }
    CHECK(std::fabs(ps - 1.0) < 1e-5, "row %ld probabilities sum to %f", (long)r, ps);
    CHECK(std::fabs(gsum) < 1e-6, "row %ld gradient sums to %g", (long)r, gsum);
  }
}

void test_bn_frozen() {
  Rng g(47);
  const int64_t N = 2, C = 13, HW = 37, n = N * C * HW;
  std::vector<float> x(n), y1(n), y2(n), sc(C), sh(C);
  for (auto& v : x) v = (float)(g.uni() * 8 - 4);
  for (int64_t c = 0; c < C; ++c) {
    sc[c] = (float)(g.uni() * 2 - 1);
    sh[c] = (float)(g.uni() - 0.5);
  }
  for (int64_t inner : {HW, (int64_t)1}) {  // NCHW, channels_last
    mxr::host::bn_frozen_range(x.data(), y1.data(), 0, n, C, inner, sc.data(), sh.data(), true);
    std::vector<std::thread> th;
    for (int t = 0; t < 3; ++t)
      th.emplace_back([&, t] {
        mxr::host::bn_frozen_range(x.data(), y2.data(), n * t / 3, n * (t + 1) / 3, C, inner, sc.data(), sh.data(),
                                   true);
      });
    for (auto& x_ : th) x_.join();
    CHECK(y1 == y2, "threaded BN differs");
    for (int64_t i = 0; i < n; ++i) {
      const int64_t c = (i / inner) % C;
      CHECK(y1[i] == std::max(x[i] * sc[c] + sh[c], 0.f), "BN element %ld", (long)i);
    }
  }
}

}  // namespace

int main() {
  test_nms();
  test_roi_pool();
  test_roi_pool_bwd();
  test_proposal_decode();
  test_anchor_assign();
  test_iou_max();
  test_losses();
  test_sgd();
  test_row_softmax_ce();
  test_bn_frozen();
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("host_ops_test OK\n");
  return 0;
}
