// Sanitizer driver for the host C++ twins in mx_rcnn_amd/csrc/host_ops.h (host
// code under -fsanitize=address,undefined and -fsanitize=thread; device sanitizers are not
// available on this pool).  No torch: built and run by tests/test_native_sanitizers.py.
//
// Checks, each on deterministic pseudo-random inputs:
//   * NMS against an independent IoU-matrix greedy oracle, the max_keep cap, n = 0 / 1,
//     degenerate boxes, bitwise repeatability;
//   * RoI pool against a per-bin brute-force oracle, including RoIs outside the map, bad
//     batch indices (negative, >= B, NaN) and 1-pixel RoIs;
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
  mxr::host::nms_greedy(nullptr, 0, 0.7, -1, k);
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

}  // namespace

int main() {
  test_nms();
  test_roi_pool();
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("host_ops_test OK\n");
  return 0;
}
