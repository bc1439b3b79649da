// Stand-alone timing of the proposal NMS kernels on RPN-shaped data (random-init RPN: boxes =
// ResNet C4 anchors (scales 4,8,16,32, ratios .5,1,2, stride 16) on a 50x84 grid with small
// jitter, random scores, top 12000 -> keep 6000).  Build variants with -D flags to ablate:
//   hipcc -O3 --offload-arch=gfx950 -I mx_rcnn_amd/csrc -I mx_rcnn_amd/csrc/hip \
//         tools/microbench/nms_bench.hip -o /tmp/nms_bench && /tmp/nms_bench
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "nms.hip"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
  const int P = argc > 1 ? atoi(argv[1]) : 12000, post = argc > 2 ? atoi(argv[2]) : 6000;
  const float thresh = 0.7f;
  std::mt19937 rng(123);
  std::uniform_real_distribution<float> U(0.f, 1.f);
  // anchors
  std::vector<float> base;
  const float ratios[3] = {0.5f, 1.f, 2.f}, scales[4] = {4, 8, 16, 32};
  for (float r : ratios)
    for (float s : scales) {
      const float w = 16.f, h = 16.f, area = w * h;
      const float ws = std::round(std::sqrt(area / r)), hs = std::round(ws * r);
      const float cx = 7.5f, cy = 7.5f, W = ws * s, H = hs * s;
      base.insert(base.end(), {cx - 0.5f * (W - 1), cy - 0.5f * (H - 1), cx + 0.5f * (W - 1), cy + 0.5f * (H - 1)});
    }
  const int FH = 50, FW = 84, A = 12;
  std::vector<std::pair<float, int>> sc;
  std::vector<float> all;
  for (int y = 0; y < FH; ++y)
    for (int x = 0; x < FW; ++x)
      for (int a = 0; a < A; ++a) {
        float b[4];
        for (int k = 0; k < 4; ++k) b[k] = base[a * 4 + k] + (k % 2 ? y : x) * 16.f + (U(rng) - 0.5f) * 4.f;
        b[0] = std::max(b[0], 0.f); b[1] = std::max(b[1], 0.f);
        b[2] = std::min(b[2], 1332.f); b[3] = std::min(b[3], 799.f);
        sc.push_back({U(rng), (int)all.size() / 4});
        all.insert(all.end(), b, b + 4);
      }
  std::sort(sc.begin(), sc.end(), [](auto& a, auto& b) { return a.first > b.first; });
  std::vector<float> boxes(P * 4), scores(P), ru(post);
  for (int i = 0; i < P; ++i) {
    for (int k = 0; k < 4; ++k) boxes[i * 4 + k] = all[sc[i].second * 4 + k];
    scores[i] = sc[i].first;
  }
  for (auto& u : ru) u = U(rng);
  float *d_boxes, *d_scores, *d_ru, *d_rois, *d_os;
  int32_t *d_nv, *d_nk;
  int64_t* d_keep;
  uint64_t* d_mask;
  const int nb = (P + 63) / 64;
  CK(hipMalloc(&d_boxes, P * 16)); CK(hipMalloc(&d_scores, P * 4)); CK(hipMalloc(&d_ru, post * 4));
  CK(hipMalloc(&d_rois, post * 20)); CK(hipMalloc(&d_os, post * 4)); CK(hipMalloc(&d_nv, 4));
  CK(hipMalloc(&d_nk, 4)); CK(hipMalloc(&d_keep, post * 8));
  CK(hipMalloc(&d_mask, mxr::nms_mask_words(1, P) * 8));
  CK(hipMemcpy(d_boxes, boxes.data(), P * 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_scores, scores.data(), P * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_ru, ru.data(), post * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_nv, &P, 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1, e2;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2));
  float tm = 0, tr = 0;
  const int iters = 20;
  for (int it = 0; it < iters + 3; ++it) {
    CK(hipEventRecord(e0, 0));
    mxr::nms_mask(d_boxes, d_nv, 1, P, thresh, d_mask, 0);
    CK(hipEventRecord(e1, 0));
    mxr::nms_reduce(d_boxes, d_scores, d_nv, d_mask, 1, P, post, d_ru, d_rois, d_os, d_keep, d_nk, 0);
    CK(hipEventRecord(e2, 0));
    CK(hipEventSynchronize(e2));
    float a, b;
    CK(hipEventElapsedTime(&a, e0, e1)); CK(hipEventElapsedTime(&b, e1, e2));
    if (it >= 3) { tm += a; tr += b; }
  }
  int nk;
  CK(hipMemcpy(&nk, d_nk, 4, hipMemcpyDeviceToHost));
  // CPU greedy check of the kept count
  std::vector<char> rem(P, 0);
  int nk_ref = 0;
  for (int i = 0; i < P && nk_ref < post; ++i) {
    if (rem[i]) continue;
    ++nk_ref;
    const float* a = &boxes[i * 4];
    const float aa = (a[2] - a[0] + 1) * (a[3] - a[1] + 1);
    for (int j = i + 1; j < P; ++j) {
      if (rem[j]) continue;
      const float* c = &boxes[j * 4];
      const float ca = (c[2] - c[0] + 1) * (c[3] - c[1] + 1);
      const float iw = std::min(a[2], c[2]) - std::max(a[0], c[0]) + 1, ih = std::min(a[3], c[3]) - std::max(a[1], c[1]) + 1;
      if (iw > 0 && ih > 0 && iw * ih / (aa + ca - iw * ih) > thresh) rem[j] = 1;
    }
  }
  printf("P=%d post=%d  mask %.1f us  reduce %.1f us  n_keep %d (cpu %d)\n", P, post, tm / iters * 1e3,
         tr / iters * 1e3, nk, nk_ref);

  return 0;
}
