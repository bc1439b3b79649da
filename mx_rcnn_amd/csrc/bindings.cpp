// Python bindings for the gfx950 kernels.  Thin: validate shapes/dtypes/devices, allocate
// outputs through the PyTorch caching allocator, launch on the current HIP stream.  All
// launches are graph-capturable (no host sync, no allocation inside the launchers).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <tuple>
#include <mutex>
#include <string>
#include <torch/extension.h>
#include <ATen/Parallel.h>
#include <ATen/hip/HIPGeneratorImpl.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include "host_ops.h"
#include "kernels.h"

// a rejected launch (e.g. an LDS request over budget) must raise here, not leave the outputs
// uninitialised for a later gather to fault on
#define LAUNCH_CHECK(what)                                                                       \
  do {                                                                                           \
    const hipError_t e_ = hipGetLastError();                                                     \
    TORCH_CHECK(e_ == hipSuccess || e_ == hipErrorNotReady, what, ": kernel launch failed: ",     \
                hipGetErrorString(e_));                                                          \
  } while (0)

namespace {

using at::Tensor;

// PyTorch-ROCm registers its HIP runtime under the "cuda" device type, so tensors report
// device type CUDA: guard with the generic DeviceGuard and fetch the HIP stream by index.
thread_local c10::Device g_dev(c10::DeviceType::CUDA, 0);
hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream(g_dev.index()).stream(); }
struct DevGuard {
  c10::DeviceGuard guard;
  explicit DevGuard(const c10::Device& d) : guard(d) { g_dev = d; }
};

// Self-cleaning workspaces: a zeroed int32 buffer per (device, tag, size), allocated once and kept
// for the process; the kernels that use it leave it zeroed again at the end of their chain (the
// topk write kernel re-zeroes its histograms, the anchor output kernel the gt-max / histogram words,
// the next call's first assignment kernel the mark words), so the captured step carries no fill.
// A capture that meets a size for the first time gets a per-call zeroed tensor (never cached: it
// would live in the graph's private pool).  One chain at a time per buffer: the training step runs
// one proposal top-k and one anchor sampling per replay, in stream order.
// `layout` joins the key: a chain leaves only the words of ITS layout clean (the anchor chain's mark
// words are re-zeroed by the next call's first pass at that call's offset), so two calls with the
// same total size but different region boundaries must not share a buffer.
static Tensor clean_ws(const at::TensorOptions& o, const char* tag, int64_t n, int64_t layout = 0) {
  static std::mutex mu;
  static auto* cache = new std::map<std::tuple<int, std::string, int64_t, int64_t>, Tensor>();  // leaked: outlives exit
  const auto key = std::make_tuple((int)o.device().index(), std::string(tag), n, layout);
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache->find(key);
  if (it != cache->end()) return it->second;
  Tensor t = at::zeros({n}, o);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  const bool capturing = hipStreamIsCapturing(c10::hip::getCurrentHIPStream(o.device().index()).stream(), &cs) !=
                             hipSuccess || cs != hipStreamCaptureStatusNone;
  if (!capturing) cache->emplace(key, t);
  return t;
}

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be float32")
#define CHECK_I32(t) TORCH_CHECK((t).scalar_type() == at::kInt, #t " must be int32")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")

// 16-bit storage code of the dtype-generic kernels: 0 fp32, 1 bf16, 2 fp16
// planes of a multi-plane fp32-mode flag: 0 off, 2 x2 pairs (True / 1 / 2), 3 x3 triples (common.h)
inline int npl(int64_t x2) { return x2 <= 0 ? 0 : (x2 == 3 ? 3 : 2); }
// the elementwise kernels' storage code of those planes (common.h: 3 x2, 4 x3)
inline int pcode(int64_t x2) { return npl(x2) == 3 ? 4 : 3; }

int dcode(const Tensor& t) {
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kFloat || t.scalar_type() == at::kHalf,
              "expected bf16, fp16 or fp32 tensor");
  return t.scalar_type() == at::kBFloat16 ? 1 : t.scalar_type() == at::kHalf ? 2 : 0;
}

int is_bf16(const Tensor& t) {
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kFloat, "expected bf16 or fp32 tensor");
  return t.scalar_type() == at::kBFloat16 ? 1 : 0;
}

// ---- proposal -------------------------------------------------------------------------
std::vector<Tensor> proposal_decode(const Tensor& cls, const Tensor& dlt, const Tensor& im_info,
                                    const Tensor& base_anchors, double feat_stride, double min_size,
                                    bool crop_to_im, bool is_prob) {
  CHECK_DEV(cls); CHECK_DEV(dlt); CHECK_DEV(im_info); CHECK_DEV(base_anchors);
  CHECK_F32(im_info); CHECK_F32(base_anchors); CHECK_CONTIG(im_info); CHECK_CONTIG(base_anchors);
  TORCH_CHECK(cls.dim() == 4 && dlt.dim() == 4, "cls/dlt must be (B, C, H, W)");
  const int A = (int)base_anchors.size(0);
  const int B = (int)cls.size(0), H = (int)cls.size(2), W = (int)cls.size(3);
  TORCH_CHECK(cls.size(1) == 2 * A, "cls channels must be 2A");
  TORCH_CHECK(dlt.size(0) == B && dlt.size(1) == 4 * A && dlt.size(2) == H && dlt.size(3) == W, "dlt shape");
  TORCH_CHECK(im_info.size(0) == B && im_info.size(1) == 3, "im_info must be (B, 3)");
  DevGuard g(cls.device());
  const int64_t N = (int64_t)H * W * A;
  auto opts = cls.options().dtype(at::kFloat);
  Tensor boxes = at::empty({B, N, 4}, opts);
  Tensor keys = at::empty({B, N}, opts);
  mxr::proposal_decode(cls.data_ptr(), dcode(cls), cls.stride(0), cls.stride(1), cls.stride(2), cls.stride(3),
                       dlt.data_ptr(), dcode(dlt), dlt.stride(0), dlt.stride(1), dlt.stride(2), dlt.stride(3),
                       is_prob ? 1 : 0, im_info.data_ptr<float>(), base_anchors.data_ptr<float>(), A, B, H, W,
                       (float)feat_stride, (float)min_size, crop_to_im ? 1 : 0, boxes.data_ptr<float>(),
                       keys.data_ptr<float>(), cur_stream());
  return {boxes, keys};
}

// NMS over score-sorted boxes; returns (rois (B,post,5), scores (B,post), keep (B,post) int64, n_keep (B))
std::vector<Tensor> nms_proposals(const Tensor& boxes, const Tensor& scores, const Tensor& n_valid, double thresh,
                                  int64_t post, const Tensor& rand_u, c10::optional<Tensor> mask_in,
                                  c10::optional<Tensor> fault) {
  CHECK_DEV(boxes); CHECK_F32(boxes); CHECK_CONTIG(boxes);
  CHECK_DEV(scores); CHECK_F32(scores); CHECK_CONTIG(scores);
  CHECK_DEV(n_valid); CHECK_I32(n_valid); CHECK_CONTIG(n_valid);
  CHECK_DEV(rand_u); CHECK_F32(rand_u); CHECK_CONTIG(rand_u);
  TORCH_CHECK(boxes.dim() == 3 && boxes.size(2) == 4, "boxes must be (B, P, 4)");
  const int B = (int)boxes.size(0), P = (int)boxes.size(1);
  TORCH_CHECK(scores.size(0) == B && scores.size(1) == P, "scores shape");
  TORCH_CHECK(n_valid.numel() == B, "n_valid shape");
  TORCH_CHECK(rand_u.numel() == (int64_t)B * post, "rand_u must hold B*post values");
  TORCH_CHECK(post > 0, "post must be > 0");
  TORCH_CHECK(P > 0, "NMS needs at least one box slot");
  DevGuard g(boxes.device());
  const int nb = (P + 63) / 64;
  TORCH_CHECK(nb <= 1024, "NMS supports at most 65536 pre-NMS boxes per image");
  auto st = cur_stream();
  Tensor mask;
  if (mask_in.has_value() && mask_in->defined()) {  // built by nms_mask_build (the two-phase path)
    mask = *mask_in;
    TORCH_CHECK(mask.scalar_type() == at::kLong && mask.is_contiguous() && mask.numel() == mxr::nms_mask_words(B, P),
                "mask: the nms_mask_build output for these boxes");
  } else {
    mask = at::empty({mxr::nms_mask_words(B, P)}, boxes.options().dtype(at::kLong));
    mxr::nms_mask(boxes.data_ptr<float>(), n_valid.data_ptr<int32_t>(), B, P, (float)thresh,
                  reinterpret_cast<uint64_t*>(mask.data_ptr<int64_t>()), st);
    LAUNCH_CHECK("nms_mask");
  }
  // the caller's give-up counter (int32 on the device): +1 per image whose multi-workgroup chain gave
  // up a poll and was redone by the serial fallback (observability; the output is valid either way)
  int32_t* fault_p = nullptr;
  if (fault.has_value() && fault->defined()) {
    CHECK_DEV(*fault); CHECK_I32(*fault);
    TORCH_CHECK(fault->numel() >= 1 && fault->device() == boxes.device(), "gave_up: an int32 counter on the boxes' device");
    fault_p = fault->data_ptr<int32_t>();
  }
  Tensor rois = at::empty({B, post, 5}, boxes.options());
  Tensor out_scores = at::empty({B, post}, boxes.options());
  Tensor keep = at::empty({B, post}, boxes.options().dtype(at::kLong));
  Tensor n_keep = at::empty({B}, boxes.options().dtype(at::kInt));
  Tensor keep_ws;  // keep list beyond the LDS budget (post = all boxes of a > 32K-box image)
  if (!mxr::nms_keep_in_lds(P, (int)post)) keep_ws = at::empty({B, post}, boxes.options().dtype(at::kInt));
  mxr::nms_reduce(boxes.data_ptr<float>(), scores.data_ptr<float>(), n_valid.data_ptr<int32_t>(),
                  reinterpret_cast<const uint64_t*>(mask.data_ptr<int64_t>()), B, P, (int)post,
                  rand_u.data_ptr<float>(), rois.data_ptr<float>(), out_scores.data_ptr<float>(),
                  keep.data_ptr<int64_t>(), n_keep.data_ptr<int32_t>(),
                  keep_ws.defined() ? keep_ws.data_ptr<int32_t>() : nullptr, st, fault_p);
  LAUNCH_CHECK("nms_reduce");
  return {rois, out_scores, keep, n_keep};
}

// phase 1 of nms_proposals alone: the suppression bitmask (a caller can order other work between
// the data-parallel mask and the serial reduce)
// (skeys, order) of a descending sort over (B, N) keys, boxes (B, N, 4) fp32 -> (keys (B, P), boxes (B, P, 4),
// n_valid (B) int32)
std::vector<Tensor> proposal_gather(const Tensor& skeys, const Tensor& order, const Tensor& boxes, int64_t P) {
  CHECK_DEV(skeys); CHECK_DEV(order); CHECK_DEV(boxes);
  TORCH_CHECK(skeys.scalar_type() == at::kFloat && skeys.dim() == 2 && skeys.is_contiguous(), "proposal_gather: skeys");
  TORCH_CHECK(order.scalar_type() == at::kLong && order.sizes() == skeys.sizes() && order.is_contiguous(),
              "proposal_gather: order (B, N) int64");
  const int64_t B = skeys.size(0), N = skeys.size(1);
  TORCH_CHECK(boxes.scalar_type() == at::kFloat && boxes.dim() == 3 && boxes.size(0) == B && boxes.size(1) == N &&
                  boxes.size(2) == 4 && boxes.is_contiguous(),
              "proposal_gather: boxes (B, N, 4) fp32");
  TORCH_CHECK(P > 0 && P <= N, "proposal_gather: 0 < P <= N");
  DevGuard g(skeys.device());
  Tensor ok = at::empty({B, P}, skeys.options());
  Tensor ob = at::empty({B, P, 4}, boxes.options());
  Tensor nv = at::empty({B}, skeys.options().dtype(at::kInt));
  mxr::proposal_gather(skeys.data_ptr<float>(), order.data_ptr<int64_t>(), boxes.data_ptr<float>(), (int)B, N, (int)P,
                       ok.data_ptr<float>(), ob.data_ptr<float>(), nv.data_ptr<int32_t>(), cur_stream());
  LAUNCH_CHECK("proposal_gather");
  return {ok, ob, nv};
}

// MXR_NMS_CHECK: recompute greedy NMS on the device with a plain flag loop and compare with the
// reducer's keep list; returns (B, 2) int32 {first differing keep position or -1, greedy kept count}
Tensor nms_check(const Tensor& boxes, const Tensor& n_valid, double thresh, int64_t post, const Tensor& keep,
                 const Tensor& n_keep) {
  CHECK_DEV(boxes); CHECK_F32(boxes); CHECK_CONTIG(boxes);
  CHECK_DEV(n_valid); CHECK_I32(n_valid); CHECK_CONTIG(n_valid);
  CHECK_DEV(n_keep); CHECK_I32(n_keep); CHECK_CONTIG(n_keep);
  TORCH_CHECK(boxes.dim() == 3 && boxes.size(2) == 4, "boxes must be (B, P, 4)");
  const int B = (int)boxes.size(0), P = (int)boxes.size(1);
  TORCH_CHECK(keep.scalar_type() == at::kLong && keep.is_contiguous() && keep.dim() == 2 && keep.size(0) == B &&
                  keep.size(1) == post, "keep must be (B, post) int64");
  TORCH_CHECK(n_valid.numel() == B && n_keep.numel() == B && P > 0 && P <= 65536, "nms_check: shape");
  DevGuard g(boxes.device());
  Tensor res = at::empty({B, 2}, boxes.options().dtype(at::kInt));
  mxr::nms_check(boxes.data_ptr<float>(), n_valid.data_ptr<int32_t>(), B, P, (float)thresh, (int)post,
                 keep.data_ptr<int64_t>(), n_keep.data_ptr<int32_t>(), res.data_ptr<int32_t>(), cur_stream());
  LAUNCH_CHECK("nms_check");
  return res;
}

Tensor nms_mask_build(const Tensor& boxes, const Tensor& n_valid, double thresh) {
  CHECK_DEV(boxes); CHECK_F32(boxes); CHECK_CONTIG(boxes);
  CHECK_DEV(n_valid); CHECK_I32(n_valid); CHECK_CONTIG(n_valid);
  TORCH_CHECK(boxes.dim() == 3 && boxes.size(2) == 4, "boxes must be (B, P, 4)");
  const int B = (int)boxes.size(0), P = (int)boxes.size(1);
  TORCH_CHECK(n_valid.numel() == B && P > 0 && (P + 63) / 64 <= 1024, "nms_mask_build: shape");
  DevGuard g(boxes.device());
  Tensor mask = at::empty({mxr::nms_mask_words(B, P)}, boxes.options().dtype(at::kLong));
  mxr::nms_mask(boxes.data_ptr<float>(), n_valid.data_ptr<int32_t>(), B, P, (float)thresh,
                reinterpret_cast<uint64_t*>(mask.data_ptr<int64_t>()), cur_stream());
  LAUNCH_CHECK("nms_mask");
  return mask;
}

// ---- fused target sampling ------------------------------------------------------------------
std::vector<Tensor> anchor_sample(const Tensor& label_pre, const Tensor& targets, const Tensor& keys, int64_t A,
                                  int64_t H, int64_t W, int64_t num_fg, int64_t batch, std::vector<double> inside_w,
                                  double pos_weight) {
  CHECK_DEV(label_pre); CHECK_I32(label_pre); CHECK_CONTIG(label_pre);
  CHECK_DEV(targets); CHECK_F32(targets); CHECK_CONTIG(targets);
  CHECK_DEV(keys); CHECK_F32(keys); CHECK_CONTIG(keys);
  const int B = (int)label_pre.size(0);
  const int64_t N = H * W * A;
  TORCH_CHECK(label_pre.numel() == B * N && targets.numel() == B * N * 4 && keys.numel() == B * N, "anchor_sample shapes");
  TORCH_CHECK(inside_w.size() == 4, "inside_w: 4 values");
  TORCH_CHECK(num_fg >= 0 && batch >= 0 && num_fg <= 1024 && batch <= 1024, "RPN batch must be <= 1024 anchors");
  DevGuard g(label_pre.device());
  auto o = targets.options();
  Tensor kept = at::empty({B, (N + 31) / 32}, o.dtype(at::kInt));
  Tensor meta = at::empty({B, 4}, o.dtype(at::kInt));
  Tensor label = at::empty({B, A * H * W}, o.dtype(at::kInt));
  Tensor bt = at::empty({B, 4 * A, H, W}, o);
  Tensor iw = at::empty({B, 4 * A, H, W}, o);
  Tensor ow = at::empty({B, 4 * A, H, W}, o);
  const float iwf[4] = {(float)inside_w[0], (float)inside_w[1], (float)inside_w[2], (float)inside_w[3]};
  mxr::anchor_sample(label_pre.data_ptr<int32_t>(), targets.data_ptr<float>(), keys.data_ptr<float>(), B, (int)A,
                     (int)H, (int)W, (int)num_fg, (int)batch, iwf, (float)pos_weight,
                     reinterpret_cast<uint32_t*>(kept.data_ptr<int32_t>()), meta.data_ptr<int32_t>(),
                     label.data_ptr<int32_t>(), bt.data_ptr<float>(), iw.data_ptr<float>(), ow.data_ptr<float>(),
                     cur_stream());
  return {label, bt, iw, ow, meta};
}

// Anchor assignment + subsampling + reference-layout outputs in four grid-wide launches (assign
// pass 1, pass 2 with the key histograms, mark with the last-workgroup boundary ranking, output):
// the same result as anchor_target_assign + anchor_sample, without the one-workgroup pass.
std::vector<Tensor> anchor_target_fused(const Tensor& base_anchors, int64_t H, int64_t W, double feat_stride,
                                        const Tensor& im_info, int64_t allowed_border, const Tensor& gt,
                                        const Tensor& n_gt, double neg_thresh, double pos_thresh, bool clobber,
                                        const Tensor& keys, int64_t num_fg, int64_t batch, std::vector<double> inside_w,
                                        double pos_weight) {
  CHECK_DEV(base_anchors); CHECK_F32(base_anchors); CHECK_CONTIG(base_anchors);
  CHECK_DEV(im_info); CHECK_F32(im_info); CHECK_CONTIG(im_info);
  CHECK_DEV(gt); CHECK_F32(gt); CHECK_CONTIG(gt);
  CHECK_DEV(n_gt); CHECK_I32(n_gt); CHECK_CONTIG(n_gt);
  CHECK_DEV(keys); CHECK_F32(keys); CHECK_CONTIG(keys);
  const int A = (int)base_anchors.size(0), B = (int)gt.size(0), G = (int)gt.size(1);
  const int64_t N = H * W * A;
  TORCH_CHECK(im_info.size(0) == B && n_gt.numel() == B && keys.numel() == B * N, "anchor_target_fused shapes");
  TORCH_CHECK(inside_w.size() == 4, "inside_w: 4 values");
  TORCH_CHECK(num_fg >= 0 && batch >= 0 && num_fg <= 1024 && batch <= 1024, "RPN batch must be <= 1024 anchors");
  DevGuard g(gt.device());
  auto o = gt.options();
  // one zeroed workspace: gt_max (B, G) | key histograms (B, 2, bins) | mark workspace
  const int64_t n_gm = (int64_t)B * std::max(G, 1), n_h = (int64_t)B * 2 * mxr::kSampleBins;
  Tensor ws = clean_ws(o.dtype(at::kInt), "anchor", n_gm + n_h + mxr::anchor_mark_ws_ints(B, N),
                       ((int64_t)B << 32) | (int64_t)std::max(G, 1));
  int32_t* wsp = ws.data_ptr<int32_t>();
  Tensor max_ov = at::empty({B, N}, o);
  Tensor argmax = at::empty({B, N}, o.dtype(at::kInt));
  Tensor label_pre = at::empty({B, N}, o.dtype(at::kInt));
  Tensor targets = at::empty({B, N, 4}, o);
  mxr::anchor_target_assign(base_anchors.data_ptr<float>(), A, (int)H, (int)W, (float)feat_stride,
                            im_info.data_ptr<float>(), (int)allowed_border, gt.data_ptr<float>(),
                            n_gt.data_ptr<int32_t>(), G, B, (float)neg_thresh, (float)pos_thresh, clobber ? 1 : 0,
                            max_ov.data_ptr<float>(), argmax.data_ptr<int32_t>(), reinterpret_cast<float*>(wsp),
                            label_pre.data_ptr<int32_t>(), targets.data_ptr<float>(), cur_stream(),
                            keys.data_ptr<float>(), wsp + n_gm, wsp + n_gm + n_h, mxr::anchor_mark_ws_ints(B, N));
  Tensor meta = at::empty({B, 4}, o.dtype(at::kInt));
  Tensor label = at::empty({B, A * H * W}, o.dtype(at::kInt));
  Tensor bt = at::empty({B, 4 * A, H, W}, o);
  Tensor iw = at::empty({B, 4 * A, H, W}, o);
  Tensor ow = at::empty({B, 4 * A, H, W}, o);
  const float iwf[4] = {(float)inside_w[0], (float)inside_w[1], (float)inside_w[2], (float)inside_w[3]};
  mxr::anchor_sample_hist(label_pre.data_ptr<int32_t>(), targets.data_ptr<float>(), keys.data_ptr<float>(),
                          wsp + n_gm, B, A, (int)H, (int)W, (int)num_fg, (int)batch, iwf, (float)pos_weight,
                          wsp + n_gm + n_h, meta.data_ptr<int32_t>(), label.data_ptr<int32_t>(), bt.data_ptr<float>(),
                          iw.data_ptr<float>(), ow.data_ptr<float>(), cur_stream(), wsp, n_gm + n_h);
  return {label, bt, iw, ow, meta};
}

std::vector<Tensor> proposal_sample(const Tensor& rois, const Tensor& gt, const Tensor& n_gt, const Tensor& max_ov,
                                    const Tensor& argmax, const Tensor& rnd, int64_t R, int64_t F, int64_t C,
                                    double fg_thresh, double bg_hi, double bg_lo, bool is_train, bool normalize,
                                    std::vector<double> means, std::vector<double> stds,
                                    std::vector<double> inside_w) {
  for (const Tensor* t : {&rois, &gt, &max_ov, &rnd}) {
    CHECK_DEV((*t)); CHECK_F32((*t)); CHECK_CONTIG((*t));
  }
  CHECK_DEV(n_gt); CHECK_I32(n_gt); CHECK_CONTIG(n_gt);
  CHECK_DEV(argmax); CHECK_I32(argmax); CHECK_CONTIG(argmax);
  TORCH_CHECK(rois.dim() == 3 && rois.size(2) == 5 && gt.dim() == 3 && gt.size(2) == 5, "rois (B,P,5), gt (B,G,5)");
  const int B = (int)rois.size(0), P = (int)rois.size(1), G = (int)gt.size(1);
  TORCH_CHECK(gt.size(0) == B && n_gt.numel() == B && max_ov.numel() == (int64_t)B * P && argmax.numel() == (int64_t)B * P,
              "proposal_sample batch shapes");
  TORCH_CHECK(rnd.numel() == (int64_t)B * (2 * (P + G) + R), "rnd must hold B * (2 (P + G) + R) draws");
  TORCH_CHECK(means.size() == 4 && stds.size() == 4 && inside_w.size() == 4, "means/stds/inside_w: 4 values");
  DevGuard g(rois.device());
  auto o = rois.options();
  Tensor out_rois = at::empty({(int64_t)B * R, 5}, o);
  Tensor label = at::empty({(int64_t)B * R}, o.dtype(at::kInt));
  Tensor bt = at::empty({(int64_t)B * R, 4 * C}, o);
  Tensor iw = at::empty({(int64_t)B * R, 4 * C}, o);
  Tensor ow = at::empty({(int64_t)B * R, 4 * C}, o);
  float mf[4], sf[4], wf[4];
  for (int q = 0; q < 4; ++q) { mf[q] = (float)means[q]; sf[q] = (float)stds[q]; wf[q] = (float)inside_w[q]; }
  const int r = mxr::proposal_sample(rois.data_ptr<float>(), gt.data_ptr<float>(), n_gt.data_ptr<int32_t>(),
                                     max_ov.data_ptr<float>(), argmax.data_ptr<int32_t>(), rnd.data_ptr<float>(), B, P,
                                     G, (int)R, (int)F, (int)C, (float)fg_thresh, (float)bg_hi, (float)bg_lo,
                                     is_train ? 1 : 0, normalize ? 1 : 0, mf, sf, wf, out_rois.data_ptr<float>(),
                                     label.data_ptr<int32_t>(), bt.data_ptr<float>(), iw.data_ptr<float>(),
                                     ow.data_ptr<float>(), cur_stream());
  TORCH_CHECK(r == 0, "proposal_sample: shape beyond the kernel plan (P + G <= 16384, R - F <= 1024)");
  return {out_rois, label, bt, iw, ow};
}

// ---- IoU / assignment ------------------------------------------------------------------
std::vector<Tensor> iou_max(const Tensor& boxes, int64_t off, const Tensor& gt, const Tensor& n_gt,
                            bool want_gt_max) {
  CHECK_DEV(boxes); CHECK_F32(boxes); CHECK_CONTIG(boxes);
  CHECK_DEV(gt); CHECK_F32(gt); CHECK_CONTIG(gt);
  CHECK_DEV(n_gt); CHECK_I32(n_gt); CHECK_CONTIG(n_gt);
  TORCH_CHECK(boxes.dim() == 3 && gt.dim() == 3 && gt.size(2) == 5, "boxes (B,N,bs), gt (B,G,5)");
  const int B = (int)boxes.size(0), N = (int)boxes.size(1), bs = (int)boxes.size(2), G = (int)gt.size(1);
  TORCH_CHECK(off + 4 <= bs, "box offset out of range");
  TORCH_CHECK(gt.size(0) == B && n_gt.numel() == B, "batch mismatch");
  DevGuard g(boxes.device());
  Tensor max_ov = at::empty({B, N}, boxes.options());
  Tensor argmax = at::empty({B, N}, boxes.options().dtype(at::kInt));
  Tensor gt_max = want_gt_max ? at::zeros({B, G}, boxes.options()) : Tensor();
  mxr::iou_max(boxes.data_ptr<float>(), bs, (int)off, B, N, gt.data_ptr<float>(), n_gt.data_ptr<int32_t>(), G,
               nullptr, max_ov.data_ptr<float>(), argmax.data_ptr<int32_t>(),
               want_gt_max ? gt_max.data_ptr<float>() : nullptr, cur_stream());
  if (want_gt_max) return {max_ov, argmax, gt_max};
  return {max_ov, argmax};
}

std::vector<Tensor> anchor_target_assign(const Tensor& base_anchors, int64_t H, int64_t W, double feat_stride,
                                         const Tensor& im_info, int64_t allowed_border, const Tensor& gt,
                                         const Tensor& n_gt, double neg_thresh, double pos_thresh, bool clobber) {
  CHECK_DEV(base_anchors); CHECK_F32(base_anchors); CHECK_CONTIG(base_anchors);
  CHECK_DEV(im_info); CHECK_F32(im_info); CHECK_CONTIG(im_info);
  CHECK_DEV(gt); CHECK_F32(gt); CHECK_CONTIG(gt);
  CHECK_DEV(n_gt); CHECK_I32(n_gt); CHECK_CONTIG(n_gt);
  const int A = (int)base_anchors.size(0), B = (int)gt.size(0), G = (int)gt.size(1);
  TORCH_CHECK(im_info.size(0) == B && n_gt.numel() == B, "batch mismatch");
  DevGuard g(gt.device());
  const int64_t N = H * W * A;
  auto o = gt.options();
  Tensor max_ov = at::empty({B, N}, o);
  Tensor argmax = at::empty({B, N}, o.dtype(at::kInt));
  Tensor gt_max = at::zeros({B, std::max(G, 1)}, o);
  Tensor label = at::empty({B, N}, o.dtype(at::kInt));
  Tensor targets = at::empty({B, N, 4}, o);
  mxr::anchor_target_assign(base_anchors.data_ptr<float>(), A, (int)H, (int)W, (float)feat_stride,
                            im_info.data_ptr<float>(), (int)allowed_border, gt.data_ptr<float>(),
                            n_gt.data_ptr<int32_t>(), G, B, (float)neg_thresh, (float)pos_thresh, clobber ? 1 : 0,
                            max_ov.data_ptr<float>(), argmax.data_ptr<int32_t>(), gt_max.data_ptr<float>(),
                            label.data_ptr<int32_t>(), targets.data_ptr<float>(), cur_stream());
  return {label, targets, max_ov, argmax};
}

// frozen BN + ReLU fused into a pooling kernel's store (kernels.h PostBn): post_bn is bn_affine's
// (2, C) [scale; shift]; none: off
static mxr::PostBn post_bn_args(const c10::optional<Tensor>& bn, int64_t C) {
  mxr::PostBn p;
  if (!bn) return p;
  TORCH_CHECK(bn->is_cuda() && bn->scalar_type() == at::kFloat && bn->is_contiguous() && bn->dim() == 2 &&
                  bn->size(0) == 2 && bn->size(1) == C,
              "post_bn: fp32 (2, C) [scale; shift] device tensor from bn_affine");
  p.scale = bn->data_ptr<float>();
  p.shift = p.scale + C;
  return p;
}

Tensor bn_affine(const Tensor& gamma, const Tensor& beta, const Tensor& mean, const Tensor& var, double eps,
                 bool fix_gamma) {
  const int64_t C = var.numel();
  for (auto* t : {&gamma, &beta, &mean, &var})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == C,
                "bn_affine: fp32 (C,) device tensors");
  DevGuard g(var.device());
  Tensor out = at::empty({2, C}, var.options());
  mxr::bn_affine(gamma.data_ptr<float>(), beta.data_ptr<float>(), mean.data_ptr<float>(), var.data_ptr<float>(),
                 (float)eps, fix_gamma ? 1 : 0, (int)C, out.data_ptr<float>(), cur_stream());
  return out;
}

// ---- RoI pooling -----------------------------------------------------------------------
// feat must be channels-last in memory: logical (B, C, H, W) with NHWC strides.
// x2: feat is a (2B, C, H, W) hi / lo pair, the pooled output (2R, C, PH, PW) a pair too
std::vector<Tensor> roi_pool_fwd(const Tensor& feat, const Tensor& rois, int64_t PH, int64_t PW, double scale, int64_t x2,
                                 bool need_argmax, c10::optional<Tensor> post_bn) {
  CHECK_DEV(feat); CHECK_DEV(rois); CHECK_F32(rois); CHECK_CONTIG(rois);
  TORCH_CHECK(feat.dim() == 4 && feat.is_contiguous(at::MemoryFormat::ChannelsLast),
              "feat must be (B,C,H,W) channels_last");
  TORCH_CHECK(rois.dim() == 2 && rois.size(1) == 5, "rois must be (R, 5)");
  TORCH_CHECK(!x2 || (feat.scalar_type() == at::kBFloat16 && feat.size(0) % npl(x2) == 0 && feat.size(1) % 4 == 0),
              "x2: bf16 (2B, C, H, W) pairs, C % 4 == 0");
  const int B = (int)(x2 ? feat.size(0) / npl(x2) : feat.size(0)), C = (int)feat.size(1), H = (int)feat.size(2),
            W = (int)feat.size(3);
  const int R = (int)rois.size(0);
  TORCH_CHECK(!(post_bn && need_argmax), "roi_pool_fwd: post_bn is inference-only (no argmax)");
  const mxr::PostBn post = post_bn_args(post_bn, C);
  DevGuard g(feat.device());
  Tensor out = at::empty({x2 ? npl(x2) * R : R, C, PH, PW}, feat.options().memory_format(at::MemoryFormat::ChannelsLast));
  // inference skips the argmax map (4 B per output element: at batch 8 x 300 RoIs x 1024 channels
  // x 49 bins, 480 MB of writes that nothing reads)
  Tensor argmax = need_argmax ? at::empty({R, C, PH, PW}, feat.options().dtype(at::kInt).memory_format(
                                                              at::MemoryFormat::ChannelsLast))
                              : at::empty({0}, feat.options().dtype(at::kInt));
  mxr::roi_pool_fwd(feat.data_ptr(), x2 ? pcode(x2) : dcode(feat), B, H, W, C, rois.data_ptr<float>(), R, (int)PH, (int)PW,
                    (float)scale, out.data_ptr(), need_argmax ? argmax.data_ptr<int32_t>() : nullptr, cur_stream(), post);
  return {out, argmax};
}

Tensor roi_pool_bwd(const Tensor& grad_out, const Tensor& argmax, const Tensor& rois, int64_t B, int64_t H,
                    int64_t W, c10::optional<Tensor> grad_add, int64_t x2) {
  CHECK_DEV(grad_out); CHECK_DEV(argmax); CHECK_I32(argmax); CHECK_DEV(rois); CHECK_F32(rois);
  const int R = (int)(x2 ? grad_out.size(0) / npl(x2) : grad_out.size(0)), C = (int)grad_out.size(1),
            PH = (int)grad_out.size(2), PW = (int)grad_out.size(3);
  TORCH_CHECK(!x2 || (grad_out.scalar_type() == at::kBFloat16 && grad_out.size(0) % npl(x2) == 0 && argmax.size(0) == R),
              "x2: bf16 (2R, C, PH, PW) gradient pairs");
  Tensor go = grad_out.contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(argmax.is_contiguous(at::MemoryFormat::ChannelsLast), "argmax must be channels_last");
  DevGuard g(grad_out.device());
  auto st = cur_stream();
  static const bool lds_path = [] {
    const char* e = std::getenv("MXR_ROIPOOL_BWD_LDS");
    return e == nullptr || e[0] != '0';
  }();
  const bool add = grad_add.has_value() && grad_add->defined();
  if (add)
    TORCH_CHECK(grad_add->scalar_type() == grad_out.scalar_type() && grad_add->dim() == 4 &&
                    grad_add->size(0) == (x2 ? npl(x2) * B : B) &&
                    grad_add->size(1) == C && grad_add->size(2) == H && grad_add->size(3) == W &&
                    grad_add->is_contiguous(at::MemoryFormat::ChannelsLast),
                "grad_add: channels_last (B, C, H, W) of the gradient dtype");
  if (lds_path || x2) {
    Tensor gin = at::empty({x2 ? npl(x2) * B : B, C, H, W}, grad_out.options().memory_format(at::MemoryFormat::ChannelsLast));
    if (mxr::roi_pool_bwd_lds(go.data_ptr(), x2 ? pcode(x2) : dcode(go), argmax.data_ptr<int32_t>(),
                              rois.contiguous().data_ptr<float>(), R, PH, PW, (int)B, (int)H, (int)W, C, gin.data_ptr(),
                              st, add ? grad_add->data_ptr() : nullptr) == 0)
      return gin;
    TORCH_CHECK(!x2, "roi_pool_bwd: x2 needs the LDS slab kernel (H x W too large)");
  }
  // NOTE: at::zeros ignores a memory_format carried in TensorOptions (returns NCHW); allocate
  // the NHWC buffer explicitly and view it as logical NCHW.
  Tensor gin32 = at::zeros({B, H, W, C}, grad_out.options().dtype(at::kFloat)).permute({0, 3, 1, 2});
  mxr::roi_pool_bwd(go.data_ptr(), is_bf16(go), argmax.data_ptr<int32_t>(), rois.contiguous().data_ptr<float>(), R,
                    PH, PW, (int)B, (int)H, (int)W, C, gin32.data_ptr<float>(), st);
  if (add) gin32.add_(*grad_add);
  if (grad_out.scalar_type() == at::kFloat) return gin32;
  Tensor gin = at::empty({B, C, H, W}, grad_out.options().memory_format(at::MemoryFormat::ChannelsLast));
  mxr::cast_f32(gin32.data_ptr<float>(), gin.data_ptr(), 1, gin.numel(), st);
  return gin;
}

// ---- losses ----------------------------------------------------------------------------
// returns (grad like logits, loss_sum (1,), prob_fg (B, H*W*A) in (h, w, a) order)
// Persistent ticket counters of the grid-reduction losses (losses.hip), one slot per call site;
// zero at allocation and re-armed by the kernels.  Deliberately leaked (no destructor after
// the HIP runtime has gone at exit).
static unsigned* loss_ticket(const at::Device& dev, int64_t slot) {
  static auto* bufs = new std::map<int, Tensor>();
  TORCH_CHECK(slot >= 0 && slot < 64, "loss ticket slot out of range");
  auto it = bufs->find(dev.index());
  if (it == bufs->end())
    it = bufs->emplace(dev.index(), at::zeros({64}, at::TensorOptions().device(dev).dtype(at::kInt))).first;
  return reinterpret_cast<unsigned*>(it->second.data_ptr<int32_t>()) + slot;
}

// returns (grad like logits, loss (1,) already normalised[, prob_fg])
std::vector<Tensor> rpn_softmax_ce(const Tensor& logits, const Tensor& label, c10::optional<Tensor> norm,
                                   double grad_scale, bool want_prob, c10::optional<Tensor> meta) {
  CHECK_DEV(logits); CHECK_DEV(label); CHECK_I32(label); CHECK_CONTIG(label);
  const int B = (int)logits.size(0), C2 = (int)logits.size(1), H = (int)logits.size(2), W = (int)logits.size(3);
  TORCH_CHECK(C2 % 2 == 0, "logits channels must be 2A");
  const int A = C2 / 2;
  TORCH_CHECK(label.numel() == (int64_t)B * A * H * W, "label must be (B, A*H*W)");
  const bool has_meta = meta.has_value() && meta->defined();
  if (has_meta) {
    CHECK_DEV((*meta)); CHECK_I32((*meta)); CHECK_CONTIG((*meta));
    TORCH_CHECK(meta->numel() == (int64_t)B * 4, "meta must be (B, 4)");
  } else {
    TORCH_CHECK(norm.has_value() && norm->defined(), "rpn_softmax_ce: norm or meta required");
    CHECK_DEV((*norm)); CHECK_F32((*norm));
  }
  DevGuard g(logits.device());
  Tensor grad = at::empty_like(logits);
  TORCH_CHECK(grad.strides() == logits.strides(), "grad layout must match logits");
  Tensor loss = at::empty({1}, logits.options().dtype(at::kFloat));
  Tensor partials = at::empty({mxr::loss_blocks_rpn((int64_t)B * A * H * W)}, logits.options().dtype(at::kFloat));
  Tensor prob = want_prob ? at::empty({B, (int64_t)H * W * A}, logits.options().dtype(at::kFloat)) : Tensor();
  mxr::rpn_softmax_ce(logits.data_ptr(), is_bf16(logits), logits.stride(0), logits.stride(1), logits.stride(2),
                      logits.stride(3), label.data_ptr<int32_t>(), B, A, H, W,
                      has_meta ? nullptr : norm->data_ptr<float>(), has_meta ? meta->data_ptr<int32_t>() : nullptr,
                      (float)grad_scale, grad.data_ptr(), partials.data_ptr<float>(),
                      loss_ticket(logits.device(), 0), loss.data_ptr<float>(),
                      want_prob ? prob.data_ptr<float>() : nullptr, cur_stream());
  if (want_prob) return {grad, loss, prob};
  return {grad, loss};
}

// returns (grad (R,C) like logits, prob (R,C) fp32, loss (1,) = sum / norm)
std::vector<Tensor> row_softmax_ce(const Tensor& logits, const Tensor& label, double norm, double grad_scale,
                                   bool want_grad) {
  CHECK_DEV(logits); CHECK_CONTIG(logits); CHECK_DEV(label); CHECK_I32(label); CHECK_CONTIG(label);
  TORCH_CHECK(logits.dim() == 2, "logits must be (R, C)");
  const int R = (int)logits.size(0), C = (int)logits.size(1);
  TORCH_CHECK(label.numel() == R, "label must be (R,)");
  DevGuard g(logits.device());
  Tensor grad = want_grad ? at::empty_like(logits) : Tensor();
  Tensor prob = at::empty({R, C}, logits.options().dtype(at::kFloat));
  Tensor loss = R > 0 ? at::empty({1}, logits.options().dtype(at::kFloat))
                      : at::zeros({1}, logits.options().dtype(at::kFloat));  // R == 0 launches nothing
  Tensor partials = at::empty({std::max(mxr::loss_blocks_row(R), 1)}, logits.options().dtype(at::kFloat));
  mxr::row_softmax_ce(logits.data_ptr(), is_bf16(logits), R, C, label.data_ptr<int32_t>(), (float)norm,
                      (float)grad_scale, want_grad ? grad.data_ptr() : nullptr, prob.data_ptr<float>(),
                      partials.data_ptr<float>(), loss_ticket(logits.device(), 1), loss.data_ptr<float>(),
                      cur_stream());
  if (want_grad) return {grad, prob, loss};
  return {prob, loss};
}

// pred (n0,n1,n2,n3) any strides; tgt/in_w/out_w contiguous fp32 of the same logical shape.
// returns (grad like pred, loss (1,) = sum); `slot`: ticket slot of the call site (2..63)
std::vector<Tensor> smooth_l1(const Tensor& pred, const Tensor& tgt, const Tensor& in_w, const Tensor& out_w,
                              double sigma, double grad_scale, int64_t slot) {
  CHECK_DEV(pred); CHECK_DEV(tgt); CHECK_F32(tgt); CHECK_CONTIG(tgt);
  CHECK_F32(in_w); CHECK_CONTIG(in_w); CHECK_F32(out_w); CHECK_CONTIG(out_w);
  TORCH_CHECK(pred.dim() <= 4, "pred rank must be <= 4");
  TORCH_CHECK(slot >= 2, "smooth_l1: ticket slots 0/1 belong to the CE losses");
  Tensor p4 = pred;
  while (p4.dim() < 4) p4 = p4.unsqueeze(0);
  TORCH_CHECK(tgt.numel() == p4.numel() && in_w.numel() == p4.numel() && out_w.numel() == p4.numel(),
              "target/weights must match pred");
  DevGuard g(pred.device());
  Tensor grad = at::empty_like(pred);
  Tensor g4 = grad;
  while (g4.dim() < 4) g4 = g4.unsqueeze(0);
  TORCH_CHECK(g4.strides() == p4.strides(), "grad layout must match pred");
  Tensor loss = p4.numel() > 0 ? at::empty({1}, pred.options().dtype(at::kFloat))
                               : at::zeros({1}, pred.options().dtype(at::kFloat));  // empty: no launch
  Tensor partials = at::empty({std::max(mxr::loss_blocks_rpn(p4.numel()), 1)}, pred.options().dtype(at::kFloat));
  mxr::smooth_l1(p4.data_ptr(), is_bf16(p4), p4.stride(0), p4.stride(1), p4.stride(2), p4.stride(3), (int)p4.size(0),
                 (int)p4.size(1), (int)p4.size(2), (int)p4.size(3), tgt.data_ptr<float>(), in_w.data_ptr<float>(),
                 out_w.data_ptr<float>(), (float)sigma, (float)grad_scale, g4.data_ptr(), partials.data_ptr<float>(),
                 loss_ticket(pred.device(), slot), loss.data_ptr<float>(), cur_stream());
  return {grad, loss};
}

// x *= s[0] in place
Tensor scale_by_scalar_(Tensor x, const Tensor& s) {
  CHECK_DEV(x); CHECK_DEV(s); CHECK_F32(s);
  TORCH_CHECK(x.is_contiguous() || x.is_contiguous(at::MemoryFormat::ChannelsLast), "x must be dense");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat, "bf16 / fp32 only");
  TORCH_CHECK(s.numel() == 1, "scalar expected");
  DevGuard g(x.device());
  mxr::scale_by_scalar(x.data_ptr(), is_bf16(x), x.numel(), s.data_ptr<float>(), cur_stream());
  return x;
}

// (total, weighted objective) of scalar fp32 loss terms in one launch; nonfinite (int32, 1) += !isfinite(obj)
Tensor loss_combine(std::vector<Tensor> terms, std::vector<double> weights, c10::optional<Tensor> nonfinite) {
  TORCH_CHECK(!terms.empty() && terms.size() <= 8 && weights.size() == terms.size(), "1..8 terms with weights");
  mxr::LossTerms t;
  t.n = (int)terms.size();
  for (int i = 0; i < t.n; ++i) {
    CHECK_DEV(terms[i]); CHECK_F32(terms[i]);
    TORCH_CHECK(terms[i].numel() == 1, "scalar terms");
    t.p[i] = terms[i].data_ptr<float>();
    t.w[i] = (float)weights[i];
  }
  if (nonfinite.has_value() && nonfinite->defined()) {
    CHECK_DEV((*nonfinite)); CHECK_I32((*nonfinite));
  }
  DevGuard g(terms[0].device());
  Tensor out = at::empty({2}, terms[0].options());
  mxr::loss_combine(t, out.data_ptr<float>(), nonfinite.has_value() && nonfinite->defined() ? nonfinite->data_ptr<int32_t>() : nullptr,
                    cur_stream());
  return out;
}

// ---- optimizer -------------------------------------------------------------------------
void sgd_momentum(Tensor w, Tensor mom, const Tensor& grad, const Tensor& lr, double momentum, double wd,
                  double rescale, double clip, c10::optional<Tensor> w_bf16, int64_t planes,
                  c10::optional<Tensor> zero, int64_t plane_stride) {
  CHECK_DEV(w); CHECK_F32(w); CHECK_CONTIG(w); CHECK_DEV(mom); CHECK_F32(mom); CHECK_CONTIG(mom);
  CHECK_DEV(grad); CHECK_CONTIG(grad); CHECK_DEV(lr); CHECK_F32(lr);
  TORCH_CHECK(w.numel() == mom.numel() && w.numel() == grad.numel(), "size mismatch");
  uint16_t* wb = nullptr;
  int64_t x2_plane = 0;
  if (w_bf16.has_value() && w_bf16->defined()) {
    // planes 2 / 3: the shadow is the x2 pair / x3 triple of the fp32 modes (common.h), its planes
    // numel / planes elements apart (>= n, a multiple of 8 so every plane's rows stay 16-B aligned)
    if (plane_stride > 0 && planes > 1) {
      // a bucket slice of a store's shadow: plane k at [k * plane_stride, + numel) of the view
      TORCH_CHECK(w_bf16->scalar_type() == at::kBFloat16 && w_bf16->is_contiguous() && planes <= 3 &&
                      w_bf16->numel() >= (planes - 1) * plane_stride + w.numel() && plane_stride >= w.numel(),
                  "w_bf16 slice: bf16 view reaching (planes - 1) * plane_stride + numel elements");
      wb = reinterpret_cast<uint16_t*>(w_bf16->data_ptr());
      x2_plane = plane_stride;
    } else {
      TORCH_CHECK(w_bf16->scalar_type() == at::kBFloat16 && w_bf16->is_contiguous() && planes >= 1 && planes <= 3 &&
                      w_bf16->numel() % planes == 0 && w_bf16->numel() / planes >= w.numel() &&
                      (planes == 1 || (w_bf16->numel() / planes) % 8 == 0),
                  "w_bf16 must be contiguous bf16 of `planes` planes of >= numel elements (multiples of 8)");
      wb = reinterpret_cast<uint16_t*>(w_bf16->data_ptr());
      if (planes > 1) x2_plane = w_bf16->numel() / planes;
    }
  }
  void* zp = nullptr;
  int zb = 0;
  if (zero.has_value() && zero->defined()) {  // the gradient buffer to clear once consumed
    TORCH_CHECK(zero->is_contiguous() && zero->numel() == w.numel() && zero->device() == w.device() &&
                    (zero->scalar_type() == at::kFloat || zero->scalar_type() == at::kBFloat16),
                "zero: contiguous fp32 / bf16 of numel elements");
    zp = zero->data_ptr();
    zb = is_bf16(*zero);
  }
  DevGuard g(w.device());
  mxr::sgd_momentum(w.data_ptr<float>(), mom.data_ptr<float>(), grad.data_ptr(), is_bf16(grad), w.numel(),
                    lr.data_ptr<float>(), (float)momentum, (float)wd, (float)rescale, (float)clip, wb, cur_stream(),
                    x2_plane, planes == 3 ? 1 : 0, zp, zb);
}

// ---- BN + ReLU -------------------------------------------------------------------------
Tensor bn_relu_fwd(const Tensor& x, const Tensor& gamma, const Tensor& beta, const Tensor& mean, const Tensor& var,
                   double eps, bool fix_gamma, bool relu, int64_t x2) {
  CHECK_DEV(x);
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast), "x must be channels_last 4-D");
  TORCH_CHECK(!x2 || (x.scalar_type() == at::kBFloat16 && x.size(0) % npl(x2) == 0 && x.size(1) % 4 == 0),
              "bn_relu x2: bf16 (2N, C, H, W) pairs, C % 4 == 0");
  const int C = (int)x.size(1);
  TORCH_CHECK(C <= 4096 || C % 4 == 0, "C must be a multiple of 4 or <= 4096");
  for (auto* t : {&gamma, &beta, &mean, &var}) {
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == C, "BN params fp32 (C,)");
  }
  DevGuard g(x.device());
  Tensor y = at::empty_like(x, x.options(), at::MemoryFormat::ChannelsLast);
  mxr::bn_relu_fwd(x.data_ptr(), x2 ? pcode(x2) : dcode(x), x.numel() / C / (x2 ? npl(x2) : 1), C, gamma.data_ptr<float>(),
                   beta.data_ptr<float>(),
                   mean.data_ptr<float>(), var.data_ptr<float>(), (float)eps, fix_gamma ? 1 : 0, relu ? 1 : 0,
                   y.data_ptr(), cur_stream());
  return y;
}

std::vector<Tensor> bn_relu_bwd(const Tensor& x, const Tensor& dy, const Tensor& gamma, const Tensor& beta,
                                const Tensor& mean, const Tensor& var, double eps, bool fix_gamma, bool relu,
                                bool need_dx, bool need_params, c10::optional<Tensor> dgamma_out,
                                c10::optional<Tensor> dbeta_out, c10::optional<Tensor> dres, int64_t x2) {
  CHECK_DEV(x); CHECK_DEV(dy);
  TORCH_CHECK(!x2 || (x.scalar_type() == at::kBFloat16 && x.size(0) % npl(x2) == 0 && x.size(1) % 4 == 0),
              "bn_relu_bwd x2: bf16 (2N, C, H, W) pairs, C % 4 == 0");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), "x must be channels_last");
  Tensor g = dy.contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(g.scalar_type() == x.scalar_type(), "dy dtype must match x");
  const int C = (int)x.size(1);
  DevGuard guard(x.device());
  Tensor dx = need_dx ? at::empty_like(x, x.options(), at::MemoryFormat::ChannelsLast) : Tensor();
  const bool vec = (C % 4 == 0);
  // accumulate directly into caller-provided fp32 gradients (flat-buffer views) when given
  const bool acc = vec && dgamma_out.has_value() && dgamma_out->defined() && dbeta_out.has_value() &&
                   dbeta_out->defined();
  Tensor dgamma, dbeta;
  if (acc) {
    dgamma = *dgamma_out;
    dbeta = *dbeta_out;
    TORCH_CHECK(dgamma.scalar_type() == at::kFloat && dbeta.scalar_type() == at::kFloat && dgamma.is_contiguous() &&
                    dbeta.is_contiguous() && dgamma.numel() == C && dbeta.numel() == C,
                "dgamma_out/dbeta_out must be contiguous fp32 (C,)");
  } else if (need_params) {
    dgamma = vec ? at::empty({C}, x.options().dtype(at::kFloat)) : at::zeros({C}, x.options().dtype(at::kFloat));
    dbeta = vec ? at::empty({C}, x.options().dtype(at::kFloat)) : at::zeros({C}, x.options().dtype(at::kFloat));
  }
  need_params = need_params || acc;
  Tensor rd;
  if (dres.has_value() && dres->defined()) {
    TORCH_CHECK(vec && need_dx, "dres needs C % 4 == 0 and need_dx");
    rd = dres->contiguous(at::MemoryFormat::ChannelsLast);
    TORCH_CHECK(rd.scalar_type() == x.scalar_type() && rd.sizes() == x.sizes(), "dres must match x");
  }
  Tensor ws;
  const int64_t M = x.numel() / C / (x2 ? npl(x2) : 1);
  if (need_params && vec) ws = at::empty({mxr::bn_bwd_workspace_floats(M, C)}, x.options().dtype(at::kFloat));
  mxr::bn_relu_bwd(x.data_ptr(), g.data_ptr(), x2 ? pcode(x2) : dcode(x), M, C, gamma.data_ptr<float>(),
                   beta.data_ptr<float>(), mean.data_ptr<float>(), var.data_ptr<float>(), (float)eps,
                   fix_gamma ? 1 : 0, relu ? 1 : 0, need_dx ? dx.data_ptr() : nullptr,
                   rd.defined() ? rd.data_ptr() : nullptr, need_params ? dgamma.data_ptr<float>() : nullptr, need_params ? dbeta.data_ptr<float>() : nullptr,
                   ws.defined() ? ws.data_ptr<float>() : nullptr, acc ? 1 : 0, cur_stream());
  return {dx, dgamma, dbeta};
}

// ---- implicit-GEMM conv ----------------------------------------------------------------

// ---- per-shape conv autotune (MIOpen-find style, MI355X-measured) ------------------------------
// The best tile configuration of the implicit-GEMM conv depends on the grid's fit to 256 CUs,
// K depth and output width (tools/microbench/conv_tiles.py, profiles/r2_conv_tiles.txt): e.g. the
// 128-RoI stage-4 convs run 1.3-1.5x faster on the 16-wave 128x128 ring, the stage-3 1x1s 5-15 %
// faster on 8-wave tiles.  The first call of a shape (and epilogue kind) times every candidate
// into scratch outputs on the current stream (hipEvents, 3 runs each) and caches the fastest;
// graph capture never tunes (a capturing stream uses the cache or the static plan).  All
// candidates accumulate each output in the same K order, so the choice never changes results.
// MXR_CONV_TUNE=0 disables it.
namespace {
std::mutex g_tune_mu;
std::map<std::string, std::pair<int, int>> g_tune;

bool conv_tune_enabled() {
  static const bool on = [] {
    const char* e = getenv("MXR_CONV_TUNE");
    return e == nullptr || e[0] != '0';
  }();
  return on;
}

bool stream_capturing(hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) return true;  // unknown: be safe
  return cs != hipStreamCaptureStatusNone;
}
}  // namespace

std::vector<std::tuple<std::string, int64_t, int64_t>> conv_tune_table() {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  std::vector<std::tuple<std::string, int64_t, int64_t>> out;
  for (const auto& kv : g_tune) out.emplace_back(kv.first, kv.second.first, kv.second.second);
  return out;
}

// torch.rand(..).uniform_ semantics on the GPU without a torch distribution kernel: the draw uses the
// default generator's graph-safe Philox state (advanced like torch's own kernels advance it)
Tensor philox_uniform_(Tensor out) {
  CHECK_DEV(out); CHECK_F32(out);
  TORCH_CHECK(out.is_contiguous(), "philox_uniform_: contiguous fp32 output");
  DevGuard g(out.device());
  auto* gen = at::check_generator<at::CUDAGeneratorImpl>(at::cuda::detail::getDefaultCUDAGenerator(out.device().index()));
  at::PhiloxCudaState ps;
  {
    std::lock_guard<std::mutex> lock(gen->mutex_);
    ps = gen->philox_cuda_state(4);
  }
  mxr::PhiloxArgs a;
  a.captured = ps.captured_ ? 1 : 0;
  a.seed = ps.captured_ ? (uint64_t)reinterpret_cast<uintptr_t>(ps.seed_.ptr) : ps.seed_.val;
  a.offset = ps.captured_ ? (uint64_t)reinterpret_cast<uintptr_t>(ps.offset_.ptr) : ps.offset_.val;
  a.intra = ps.captured_ ? ps.offset_intragraph_ : 0;
  mxr::philox_fill(out.data_ptr<float>(), out.numel(), a, cur_stream());
  return out;
}

void counter_add_(Tensor c, int64_t v) {
  CHECK_DEV(c);
  TORCH_CHECK(c.scalar_type() == at::kLong && c.numel() >= 1 && c.is_contiguous(), "counter_add_: int64 counter");
  DevGuard g(c.device());
  mxr::counter_add(c.data_ptr<int64_t>(), v, cur_stream());
}

Tensor image_prep(const Tensor& img, const Tensor& im_info, std::vector<double> means, bool out_bf16) {
  CHECK_DEV(img); CHECK_DEV(im_info); CHECK_F32(im_info);
  TORCH_CHECK(img.scalar_type() == at::kByte && img.dim() == 4 && img.size(3) == 3 && img.is_contiguous(),
              "image_prep: contiguous uint8 (B, H, W, 3) images");
  TORCH_CHECK(im_info.dim() == 2 && im_info.size(0) == img.size(0) && im_info.size(1) >= 3 && im_info.is_contiguous(),
              "image_prep: im_info (B, 3)");
  TORCH_CHECK(means.size() == 3, "image_prep: three means");
  const int64_t B = img.size(0), H = img.size(1), W = img.size(2);
  Tensor out = at::empty({B, 3, H, W}, img.options().dtype(out_bf16 ? at::kBFloat16 : at::kFloat),
                         at::MemoryFormat::ChannelsLast);
  mxr::image_prep(img.data_ptr<uint8_t>(), im_info.data_ptr<float>(), (int)B, (int)H, (int)W, means.data(),
                  out_bf16 ? 1 : 0, out.data_ptr(), cur_stream());
  return out;
}

// Preload / override autotune choices (a persisted plan file, or rank 0's plan under data
// parallelism: ops/tune_plan.py).  A key present here is never re-timed.
int64_t conv_tune_set(const std::vector<std::tuple<std::string, int64_t, int64_t>>& entries, bool replace) {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  if (replace) g_tune.clear();
  for (const auto& e : entries) g_tune[std::get<0>(e)] = {(int)std::get<1>(e), (int)std::get<2>(e)};
  return (int64_t)g_tune.size();
}

// dadd either shaped like y, or the stride-s subsampled grid (N, C, ceil(Ho/s), ceil(Wo/s)) of an
// unmapped launch (a strided projection shortcut's gradient): sets ep.dadd / ep.dadd_s
void set_dadd(mxr::ConvEpi& ep, const Tensor& dadd, const Tensor& y, int Ho, int Wo, bool mapped) {
  TORCH_CHECK(dadd.scalar_type() == at::kBFloat16 && dadd.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  dadd.dim() == 4 && dadd.size(0) == y.size(0) && dadd.size(1) == y.size(1),
              "dadd must be a channels_last bf16 (N, C, ., .) tensor like y");
  ep.dadd = reinterpret_cast<const uint16_t*>(dadd.data_ptr());
  if (dadd.sizes() == y.sizes()) return;
  TORCH_CHECK(!mapped, "a subsampled dadd needs an unmapped launch");
  for (int s = 2; s <= 8; ++s) {
    if (dadd.size(2) == (Ho + s - 1) / s && dadd.size(3) == (Wo + s - 1) / s) {
      ep.dadd_s = s;
      ep.dadd_gh = Ho;
      ep.dadd_gw = Wo;
      return;
    }
  }
  TORCH_CHECK(false, "dadd must be shaped like y or its stride-s subsampled grid");
}

// ReLU (+ dropout) backward: dy * [y > 0] * scale; x2: dy (2N, ...) pairs, y the ReLU output pair
Tensor relu_mask_bwd(const Tensor& dy, const Tensor& y, double scale, int64_t x2) {
  CHECK_DEV(dy); CHECK_DEV(y);
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && y.scalar_type() == at::kBFloat16 && dy.sizes() == y.sizes() &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast) && y.is_contiguous(at::MemoryFormat::ChannelsLast),
              "relu_mask_bwd: bf16 channels_last dy / y of one shape");
  const int64_t n = x2 ? dy.numel() / npl(x2) : dy.numel();
  TORCH_CHECK(n % 8 == 0 && (!x2 || dy.size(0) % npl(x2) == 0), "relu_mask_bwd: numel % 8 (pairs: 2N rows)");
  DevGuard g(dy.device());
  Tensor out = at::empty_like(dy, dy.options(), at::MemoryFormat::ChannelsLast);
  // the sign of a multi-plane value is its hi plane's: plane 0 of a pair, plane 1 of a triple
  mxr::relu_mask(reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                 reinterpret_cast<const uint16_t*>(y.data_ptr()) + (npl(x2) == 3 ? n : 0),
                 reinterpret_cast<uint16_t*>(out.data_ptr()), n, x2 ? n : 0, (float)scale, cur_stream(),
                 x2 ? npl(x2) : 1);
  return out;
}

// conv_igemm_fwd(x, w, bias, stride, pad, relu, tile, splits, residual, bn, bn_eps, bn_fix_gamma, act_relu)
//   -> [y] or, when bn = (gamma, beta, mean, var) is given, [y, act(bn(y))]  (see ConvEpi)
std::vector<Tensor> conv_igemm_fwd(const Tensor& x, const Tensor& w, c10::optional<Tensor> bias, int64_t stride,
                                   int64_t pad, bool relu, int64_t tile, int64_t splits,
                                   c10::optional<Tensor> residual, c10::optional<std::vector<Tensor>> bn,
                                   double bn_eps, bool bn_fix_gamma, bool act_relu, c10::optional<Tensor> bnb_x,
                                   c10::optional<Tensor> dadd, c10::optional<Tensor> dgamma_out,
                                   c10::optional<Tensor> dbeta_out, double drop_p, int64_t drop_seed,
                                   c10::optional<Tensor> drop_step, int64_t pad_w, c10::optional<Tensor> out,
                                   c10::optional<std::vector<int64_t>> out_map, c10::optional<Tensor> stat_shift,
                                   c10::optional<Tensor> bnb_part, int64_t bnb_row0, int64_t x2, int64_t w_plane,
                                   bool out_f32, bool bt, c10::optional<Tensor> rmask, double rmask_scale) {
  CHECK_DEV(x); CHECK_DEV(w);
  TORCH_CHECK((x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf) && w.scalar_type() == x.scalar_type(),
              "conv_igemm: bf16 or fp16 activations and weights of the same dtype");
  const bool f16 = x.scalar_type() == at::kHalf;
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast), "x must be channels_last (N,C,H,W)");
  TORCH_CHECK(w.dim() == 4 && w.is_contiguous(at::MemoryFormat::ChannelsLast), "w must be channels_last (O,I,kh,kw)");
  // x2 (fp32-class): x / y / residual / bnb_x / dadd are (2N, ...) hi / lo plane pairs, w's lo plane
  // sits w_plane elements after it (the flat shadow or the dgrad cache); out_f32: fp32 (N, ...) output
  TORCH_CHECK(!x2 || (!f16 && x.size(0) % npl(x2) == 0 && w_plane >= w.numel()), "x2: bf16 pairs (2N, ...) and w_plane");
  TORCH_CHECK(!out_f32 || x2, "out_f32 needs x2");
  const int NB = (int)(x2 ? x.size(0) / npl(x2) : x.size(0)), Cin = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  // bt: a data gradient reading the forward filter w (Cout_f, Cin_f, kh, kw) directly -- this launch's
  // input channels are the filter's outputs and its outputs the filter's inputs (taps flipped in-kernel)
  const int Cout = (int)(bt ? w.size(1) : w.size(0)), KH = (int)w.size(2), KW = (int)w.size(3);
  TORCH_CHECK((bt ? w.size(0) : w.size(1)) == Cin, "channel mismatch");
  TORCH_CHECK(Cin % 64 == 0, "conv_igemm requires Cin % 64 == 0");
  TORCH_CHECK(!bt || (!f16 && stride == 1 && Cout % 8 == 0), "bt: bf16 stride-1 data gradient, Cout % 8 == 0");
  const int padw = pad_w >= 0 ? (int)pad_w : (int)pad;
  int Ho = (H + 2 * (int)pad - KH) / (int)stride + 1, Wo = (W + 2 * padw - KW) / (int)stride + 1;
  mxr::ConvEpi ep;
  ep.relu = relu ? 1 : 0;
  ep.f16 = f16 ? 1 : 0;
  ep.bt = bt ? 1 : 0;
  ep.pad_w = pad_w >= 0 ? (int)pad_w : -1;
  const bool mapped = out_map.has_value();
  if (mapped) {
    // out_map = (Ho, Wo, o_H, o_W, o_sh, o_sw, o_ph, o_pw): this launch computes an Ho x Wo grid and
    // scatters it into `out` (N, Cout, o_H, o_W) at rows (i*o_sh + o_ph, j*o_sw + o_pw)
    const auto& om = *out_map;
    TORCH_CHECK(om.size() == 8, "out_map = (Ho, Wo, o_H, o_W, o_sh, o_sw, o_ph, o_pw)");
    Ho = (int)om[0];
    Wo = (int)om[1];
    ep.omap = 1;
    ep.o_H = (int)om[2]; ep.o_W = (int)om[3]; ep.o_sh = (int)om[4]; ep.o_sw = (int)om[5];
    ep.o_ph = (int)om[6]; ep.o_pw = (int)om[7];
    TORCH_CHECK(Ho > 0 && Wo > 0 && (Ho - 1) * ep.o_sh + ep.o_ph < ep.o_H && (Wo - 1) * ep.o_sw + ep.o_pw < ep.o_W,
                "out_map: the grid does not fit the output map");
    TORCH_CHECK(out.has_value() && out->defined(), "out_map needs out");
  }
  Tensor b;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->numel() == Cout, "bias size");
    if (bias->scalar_type() == x.scalar_type() && bias->is_contiguous()) {
      ep.bias_h = reinterpret_cast<const uint16_t*>(bias->data_ptr());  // no per-call fp32 cast kernel
    } else {
      b = bias->to(at::kFloat).contiguous();
      ep.bias = b.data_ptr<float>();
    }
  }
  DevGuard g(x.device());
  Tensor y;
  const int NY = x2 && !out_f32 ? npl(x2) * NB : NB;  // leading dim of y (pairs: 2N, triples: 3N)
  if (mapped) {
    y = *out;
    TORCH_CHECK(!out_f32 && y.scalar_type() == at::kBFloat16 && y.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                    y.dim() == 4 && y.size(0) == NY && y.size(1) == Cout && y.size(2) == ep.o_H && y.size(3) == ep.o_W,
                "out must be a channels_last bf16 (N, Cout, o_H, o_W) tensor (2N: pairs)");
  } else {
    y = at::empty({NY, Cout, Ho, Wo},
                  x.options().dtype(out_f32 ? at::kFloat : x.scalar_type()).memory_format(at::MemoryFormat::ChannelsLast));
  }
  if (x2) {
    ep.x2 = 1;
    ep.x3 = npl(x2) == 3 ? 1 : 0;
    ep.x2_pa = (uint32_t)(x.numel() / npl(x2) * 2);
    ep.x2_pb = (uint32_t)(w_plane * 2);
    TORCH_CHECK(x.numel() < (int64_t)0x40000000 && (npl(x2) - 1) * w_plane + w.numel() < (int64_t)0x40000000,
                "x2: operand planes beyond 2 GB (buffer records)");
    if (out_f32) ep.yf = y.data_ptr<float>();
    else ep.x2_py = y.numel() / npl(x2);
  }
  if (drop_p > 0.0) {
    TORCH_CHECK(drop_p < 1.0, "dropout p must be < 1");
    TORCH_CHECK(drop_step.has_value() && drop_step->defined() && drop_step->scalar_type() == at::kLong &&
                    drop_step->is_cuda() && drop_step->numel() >= 1,
                "dropout needs drop_step: an int64 device tensor holding the step");
    ep.drop_p = (float)drop_p;
    ep.drop_seed = (uint32_t)drop_seed;
    ep.drop_step = drop_step->data_ptr<int64_t>();
  }
  if (residual.has_value() && residual->defined()) {
    const Tensor& r = *residual;
    TORCH_CHECK(r.scalar_type() == x.scalar_type() && r.sizes() == y.sizes() &&
                    r.is_contiguous(at::MemoryFormat::ChannelsLast),
                "residual must be a channels_last tensor of the activation dtype shaped like the output");
    ep.residual = reinterpret_cast<const uint16_t*>(r.data_ptr());
  }
  if (rmask.has_value() && rmask->defined()) {  // ReLU / dropout backward of the layer below (ConvEpi::rmask)
    const Tensor& r = *rmask;
    TORCH_CHECK(!f16 && !out_f32 && r.scalar_type() == at::kBFloat16 && r.sizes() == y.sizes() &&
                    r.is_contiguous(at::MemoryFormat::ChannelsLast),
                "rmask: a channels_last bf16 tensor shaped like the output (pairs in x2)");
    // the hi plane carries the sign: plane 0 of a pair, plane 1 of a triple
    ep.rmask = reinterpret_cast<const uint16_t*>(r.data_ptr()) + (ep.x3 ? r.numel() / 3 : 0);
    ep.rmask_s = (float)rmask_scale;
  }
  Tensor y2;
  std::vector<Tensor> bnf;
  if (bn.has_value()) {
    TORCH_CHECK(bn->size() == 4, "bn = (gamma, beta, mean, var)");
    for (const auto& t : *bn) {
      TORCH_CHECK(t.numel() == Cout, "bn parameter size");
      bnf.push_back(t.to(at::kFloat).contiguous());
    }
    ep.bn_gamma = bnf[0].data_ptr<float>();
    ep.bn_beta = bnf[1].data_ptr<float>();
    ep.bn_mean = bnf[2].data_ptr<float>();
    ep.bn_var = bnf[3].data_ptr<float>();
    ep.bn_eps = (float)bn_eps;
    ep.bn_fix_gamma = bn_fix_gamma ? 1 : 0;
    ep.act_relu = act_relu ? 1 : 0;
  }
  const bool bwd_mode = bnb_x.has_value() && bnb_x->defined();
  Tensor dgm, dbt;
  if (bwd_mode) {
    TORCH_CHECK(bn.has_value(), "bnb_x needs bn = (gamma, beta, mean, var)");
    const Tensor& bx = *bnb_x;
    TORCH_CHECK(bx.scalar_type() == at::kBFloat16 && bx.sizes() == y.sizes() &&
                    bx.is_contiguous(at::MemoryFormat::ChannelsLast), "bnb_x must be channels_last bf16 like y");
    ep.bnb_x = reinterpret_cast<const uint16_t*>(bx.data_ptr());
    if (dadd.has_value() && dadd->defined()) set_dadd(ep, *dadd, y, Ho, Wo, mapped);
    if (x2 && ep.dadd) ep.x2_pd = dadd->numel() / npl(x2);
    const bool det = bnb_part.has_value() && bnb_part->defined();
    if (det) {
      // deterministic column sums: 64-row tiles (tile 23) write rows bnb_row0 .. + ceil(M / 64)
      const int64_t rows = ((int64_t)NB * Ho * Wo + 63) / 64;
      TORCH_CHECK(bnb_part->scalar_type() == at::kFloat && bnb_part->is_contiguous() && Cout % 8 == 0 &&
                      bnb_part->numel() >= (bnb_row0 + rows) * 2 * Cout && bnb_row0 >= 0,
                  "bnb_part: contiguous fp32 with (bnb_row0 + ceil(M / 64)) * 2 * Cout elements");
      ep.bnb_part = bnb_part->data_ptr<float>();
      ep.bnb_row0 = (int)bnb_row0;
    } else if (dgamma_out.has_value() && dgamma_out->defined()) {
      dgm = *dgamma_out;
      dbt = *dbeta_out;
      TORCH_CHECK(dgm.scalar_type() == at::kFloat && dbt.scalar_type() == at::kFloat && dgm.is_contiguous() &&
                      dbt.is_contiguous() && dgm.numel() == Cout && dbt.numel() == Cout,
                  "dgamma_out/dbeta_out must be contiguous fp32 (C,)");
    } else {
      dgm = at::zeros({Cout}, x.options().dtype(at::kFloat));
      dbt = at::zeros({Cout}, x.options().dtype(at::kFloat));
    }
    if (!det) {
      ep.bnb_dgamma = dgm.data_ptr<float>();
      ep.bnb_dbeta = dbt.data_ptr<float>();
    }
  } else if (bn.has_value()) {
    y2 = at::empty_like(y, y.options(), at::MemoryFormat::ChannelsLast);
    ep.y2 = reinterpret_cast<uint16_t*>(y2.data_ptr());
  }
  // training-BN statistics of y in the epilogue (ConvEpi::st_part): partial rows for the smallest
  // row tile any candidate uses (32), the used tile's rows are returned as a view
  const bool stats = stat_shift.has_value() && stat_shift->defined();
  Tensor part;
  if (stats) {
    TORCH_CHECK(!bwd_mode && !bn.has_value() && !mapped && Cout % 8 == 0, "stat_shift: plain forward epilogue only");
    TORCH_CHECK(stat_shift->scalar_type() == at::kFloat && stat_shift->is_contiguous() && stat_shift->numel() == Cout,
                "stat_shift: fp32 (Cout,)");
    const int64_t Mr = (int64_t)NB * Ho * Wo;
    part = at::empty({((Mr + 31) / 32) * 2 + 1, Cout}, x.options().dtype(at::kFloat));
    ep.st_part = part.data_ptr<float>();
    ep.st_shift = stat_shift->data_ptr<float>();
  }
  int auto_splits = 1;
  int t = mxr::conv_igemm_plan(NB, Ho, Wo, Cin, Cout, KH, KW, (int)tile, &auto_splits);
  // fp32 triples: the 64x64 tile's ring depth in the plan (MXR_X3_FWD_S=2: tile 30, 48 KB, three
  // workgroups per CU instead of two; A/B knob, the autotune also times tile 30)
  static const int x3_fwd_s = [] {
    const char* e = getenv("MXR_X3_FWD_S");
    return e != nullptr && e[0] == '2' ? 2 : 3;
  }();
  if (ep.x3 && tile <= 0 && t == 23 && x3_fwd_s == 2) t = 30;
  // BN-backward epilogue: no split-K by default (the statistics are reduced in-tile instead)
  int sp = splits > 0 ? (int)splits : ((bwd_mode || stats) ? 1 : auto_splits);
  if (stats) {
    TORCH_CHECK(sp == 1, "stat_shift: no split-K");
    if (!(t == 21 || t == 22 || t == 23 || t >= 100)) t = 23;
  }
  if (ep.bnb_part) {  // the caller sized the partial rows for 64-row tiles (the autotune keeps to them)
    if (mxr::conv_tile_bm(t) != 64 || t < 21) t = 23;
    sp = 1;
  }
  if (f16 && !(t == 21 || t == 22 || t == 23 || t >= 100)) t = 23;  // fp16 MFMA: buffer / ring kernels
  if (mapped || ep.pad_w >= 0) {  // geometry extensions: buffer / ring kernels, no split-K
    if (!(t == 22 || t == 23 || t >= 100)) t = 23;
    sp = 1;
  }
  // fp32-class pairs: a grid of about one 64-row tile per CU (the batch-1 stage-3 convs) leaves each
  // CU latency-bound on its operand ring; MXR_X2_SPLITK=s splits K s ways while the grid has fewer
  // than two tiles per CU (A/B knob)
  static const int x2_split = [] {
    const char* e = getenv("MXR_X2_SPLITK");
    return e != nullptr ? std::max(1, atoi(e)) : 1;
  }();
  if (x2 && x2_split > 1 && tile <= 0 && splits <= 0 && !bwd_mode && !stats && !mapped && ep.pad_w < 0 &&
      Cout % 4 == 0) {
    const int bm = t == 22 ? 128 : 64;
    const int64_t blocks = (((int64_t)NB * Ho * Wo + bm - 1) / bm) * ((Cout + 63) / 64);
    if (blocks < 512 && KH * KW * Cin / 32 >= 8 * x2_split) sp = std::max(sp, x2_split);
  }
  if (tile <= 0 && splits <= 0 && !mapped && ep.pad_w < 0 && conv_tune_enabled()) {
    char kb[256];
    snprintf(kb, sizeof(kb), "%d,%d,%d,%d,%d,%d,%d,%d,%d|%d%d%d%d%d%d%d%d%d%d%d", NB, H, W, Cin, Cout, KH, KW,
             (int)stride, (int)pad, ep.residual != nullptr, ep.y2 != nullptr || bn.has_value(), bwd_mode,
             ep.dadd != nullptr, ep.relu, ep.bias != nullptr || ep.bias_h != nullptr,
             (ep.drop_p > 0.f ? 1 : 0) + (stats ? 2 : 0), ep.bt, ep.rmask != nullptr, ep.x2 + ep.x3 + (f16 ? 8 : 0),
             ep.bnb_part != nullptr);  // (f16: the K-group and some ring tiles are bf16-only)
    const std::string key(kb);
    std::unique_lock<std::mutex> lk(g_tune_mu);
    auto it = g_tune.find(key);
    if (it != g_tune.end()) {
      t = it->second.first;
      sp = it->second.second;
    } else if (!stream_capturing(cur_stream())) {
      // time the candidates into scratch outputs (no in-place aliasing, no statistics updates)
      std::vector<std::pair<int, int>> cands = {{t, sp}};
      for (int c : {23, 22, 30, 101, 104, 105, 106, 108, 109, 110, 111})
        if (c != t || sp != 1) cands.push_back({c, 1});
      // K groups (conv_kg.hip): 2-4 four-wave groups per 64x64 tile, each over a slice of K
      if (!f16 && Cout % 8 == 0 && getenv("MXR_NO_KG") == nullptr)
        for (int c : {27, 28, 29}) cands.push_back({c, 1});
      // fp32-class pairs: the wide-stage kernel (64 channels of both planes per LDS stage) is an
      // A/B candidate only (MXR_X2W=1): 13-26 % faster in isolation on the stage-3/4 and RPN convs,
      // but the headline step measured 1 % slower with it in the autotune (same-box interleaved)
      if (ep.x2 && getenv("MXR_X2W") != nullptr) cands.push_back({26, 1});
      // large grids: the 256-row tiles of conv_big.hip (512 threads, 4-tile LDS ring)
      if ((int64_t)NB * Ho * Wo >= 16384 && !ep.x2 && getenv("MXR_NO_BIG") == nullptr)
        for (int c : {200, 201, 202, 203, 204}) cands.push_back({c, 1});
      // grids far below one tile per CU (the FC head: M = 128 RoIs, K up to 25088): split K
      const int64_t Mrows = (int64_t)NB * Ho * Wo;
      const int nkk = KH * KW * (Cin / 64);
      if (!bwd_mode && !stats && Cout % 4 == 0 && ((Mrows + 63) / 64) * ((Cout + 63) / 64) < 128) {
        for (int c : {23, 22, 106, 109})
          for (int spl : {2, 4, 8})
            if (nkk / spl >= 4 && !(c == t && spl == sp)) cands.push_back({c, spl});
      } else if (!bwd_mode && !stats && Cout % 4 == 0 && nkk >= 64 && getenv("MXR_TUNE_DEEPK") == nullptr &&
                 ((Mrows + 63) / 64) * ((Cout + 63) / 64) <= 1024) {
        // deep K (the RPN 3x3 over 1024 channels: K = 9216) on about one tile per CU: K slices give
        // each CU several workgroups to overlap (fp32-class RPN conv 219 -> 179 us at split 8,
        // tools/microbench/conv_x2_tiles.py)
        for (int c : {23, 22})
          for (int spl : {2, 4, 8})
            if (!(c == t && spl == sp)) cands.push_back({c, spl});
      }
      int max_sp = sp;
      for (const auto& c : cands) max_sp = std::max(max_sp, c.second);
      mxr::ConvEpi et = ep;
      Tensor ys = at::empty_like(y, y.options(), at::MemoryFormat::ChannelsLast);
      Tensor y2s, dg2, db2;
      if (et.y2) {
        y2s = at::empty_like(y, y.options(), at::MemoryFormat::ChannelsLast);
        et.y2 = reinterpret_cast<uint16_t*>(y2s.data_ptr());
      }
      if (bwd_mode) {
        dg2 = at::zeros({Cout}, x.options().dtype(at::kFloat));
        db2 = at::zeros({Cout}, x.options().dtype(at::kFloat));
        et.bnb_dgamma = dg2.data_ptr<float>();
        et.bnb_dbeta = db2.data_ptr<float>();
      }
      Tensor slab_t;
      if (max_sp > 1) slab_t = at::empty({(int64_t)max_sp * NB * Ho * Wo * Cout}, x.options().dtype(at::kFloat));
      hipStream_t st = cur_stream();
      // time in isolation: work still queued on other streams (the side-stream weight gradients)
      // would otherwise share the CUs with the candidates and randomise the choice
      hipDeviceSynchronize();
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      float best = 1e30f, plan_ms = 1e30f;
      std::pair<int, int> pick = {t, sp};
      for (const auto& c : cands) {
        // deterministic BN-backward sums: 64-row tiles, whole K (the partial rows are per 64 rows)
        if (ep.bnb_part && (c.second != 1 || c.first < 21 || mxr::conv_tile_bm(c.first) != 64)) continue;
        float* sl = c.second > 1 ? slab_t.data_ptr<float>() : nullptr;
        auto run = [&]() {
          return mxr::conv_igemm_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                     reinterpret_cast<const uint16_t*>(w.data_ptr()),
                                     reinterpret_cast<uint16_t*>(ys.data_ptr()), NB, H, W, Cin, Ho, Wo, Cout, KH, KW,
                                     (int)stride, (int)pad, et, c.first, c.second, sl, st);
        };
        if (run() != c.first) continue;  // fell back to another variant: not this candidate
        hipEventRecord(e0, st);
        for (int r = 0; r < 5; ++r) run();
        hipEventRecord(e1, st);
        hipEventSynchronize(e1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        if (c == cands[0]) plan_ms = ms;
        if (ms < best) {
          best = ms;
          pick = c;
        }
      }
      // leave the static plan only for a clear win: near ties measured in isolation did not
      // survive the concurrent streams of the real step (profiles/r2_conv_tune_choices.txt)
      static const float margin = [] {  // A/B knob MXR_TUNE_MARGIN (default 0.9: a 10 % win)
        const char* e = getenv("MXR_TUNE_MARGIN");
        return e != nullptr ? (float)atof(e) : 0.9f;
      }();
      if (best > margin * plan_ms) pick = cands[0];
      hipEventDestroy(e0);
      hipEventDestroy(e1);
      g_tune[key] = pick;
      t = pick.first;
      sp = pick.second;
    }
  }
  Tensor slab;
  if (sp > 1) slab = at::empty({(int64_t)sp * NB * Ho * Wo * Cout}, x.options().dtype(at::kFloat));
  int used = mxr::conv_igemm_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                 reinterpret_cast<const uint16_t*>(w.data_ptr()),
                                 out_f32 ? nullptr : reinterpret_cast<uint16_t*>(y.data_ptr()), NB, H, W, Cin, Ho, Wo,
                                 Cout, KH, KW, (int)stride, (int)pad, ep, t, sp,
                                 sp > 1 ? slab.data_ptr<float>() : nullptr, cur_stream());
  if (used <= 0 && tile <= 0 && t != 23 && !(sp > 1)) {  // a cached choice this epilogue cannot take: the plan tile
    used = mxr::conv_igemm_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                               reinterpret_cast<const uint16_t*>(w.data_ptr()),
                               out_f32 ? nullptr : reinterpret_cast<uint16_t*>(y.data_ptr()), NB, H, W, Cin, Ho, Wo,
                               Cout, KH, KW, (int)stride, (int)pad, ep, 23, 1, nullptr, cur_stream());
  }
  TORCH_CHECK(used > 0, "conv_igemm: unsupported shape");
  if (stats) {
    const int bm = mxr::conv_tile_bm(used);
    TORCH_CHECK(bm >= 32, "stat_shift: unexpected tile");
    const int64_t nparts = ((int64_t)NB * Ho * Wo + bm - 1) / bm;
    return {y, part.narrow(0, 0, nparts * 2 + 1)};
  }
  if (bwd_mode && ep.bnb_part) return {y};
  if (bwd_mode) return {y, dgm, dbt};
  if (y2.defined()) return {y, y2};
  return {y};
}

// Grouped backward of a stride-1 conv (conv_igemm.hip conv_dgrad_wgrad): the data gradient
// dgrad = conv(x = dY, w = flipped filter, pad) -- with the BN-ReLU backward epilogue when `bn` is
// given (bnb_x, optional dadd / residual, dgamma / dbeta fp32 accumulators), else plain (+residual)
// -- AND the weight gradient of (wg_dy, wg_x) accumulated into wg_out, in one launch.  With
// `defer` the weight gradient's split-K reduce is not launched: the returned slab (and wg_out)
// go to the NEXT grouped launch as prev_slab / prev_out, whose first workgroups run it.
// Returns [dx, dgamma, dbeta, slab] (dgamma / dbeta / slab empty when unused).
std::vector<Tensor> conv_dgrad_wgrad(const Tensor& x, const Tensor& w, int64_t pad, c10::optional<Tensor> residual,
                                     c10::optional<std::vector<Tensor>> bn, double bn_eps, bool bn_fix_gamma,
                                     c10::optional<Tensor> bnb_x, c10::optional<Tensor> dadd,
                                     c10::optional<Tensor> dgamma, c10::optional<Tensor> dbeta, const Tensor& wg_dy,
                                     const Tensor& wg_x, int64_t KH, int64_t KW, int64_t wg_stride, int64_t wg_pad,
                                     Tensor wg_out, bool defer, c10::optional<Tensor> prev_slab,
                                     c10::optional<Tensor> prev_out, c10::optional<Tensor> bnb_part, int64_t x2,
                                     int64_t w_plane, bool bt, c10::optional<Tensor> rmask, double rmask_scale) {
  CHECK_DEV(x); CHECK_DEV(w); CHECK_DEV(wg_dy); CHECK_DEV(wg_x); CHECK_DEV(wg_out);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast) && w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_dgrad_wgrad: channels_last bf16 x / w");
  // x2: dY / x / residual / bnb_x / dadd / wg_x are (2N, ...) pairs, w's lo plane w_plane elements on,
  // the weight gradient wg_out fp32
  TORCH_CHECK(!x2 || (x.size(0) % npl(x2) == 0 && w_plane >= w.numel()), "x2: (2N, ...) pairs and w_plane");
  const int NB = (int)(x2 ? x.size(0) / npl(x2) : x.size(0)), Cin = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  // bt: the dgrad reads the forward filter w (Cin, Cout, kh, kw) directly (see conv_igemm_fwd)
  const int Cout = (int)(bt ? w.size(1) : w.size(0)), kh = (int)w.size(2), kw = (int)w.size(3);
  TORCH_CHECK((bt ? w.size(0) : w.size(1)) == Cin && Cin % 64 == 0 && Cout % 8 == 0, "conv_dgrad_wgrad: dgrad channels");
  const int Ho = H + 2 * (int)pad - kh + 1, Wo = W + 2 * (int)pad - kw + 1;
  mxr::ConvEpi ep;
  ep.bt = bt ? 1 : 0;
  Tensor y = at::empty({x2 ? npl(x2) * NB : NB, Cout, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  if (x2) {
    TORCH_CHECK(x.numel() < (int64_t)0x40000000 && w_plane + w.numel() < (int64_t)0x40000000,
                "x2: operand planes beyond 2 GB (buffer records)");
    ep.x2 = 1;
    ep.x3 = npl(x2) == 3 ? 1 : 0;
    ep.x2_pa = (uint32_t)(x.numel() / npl(x2) * 2);
    ep.x2_pb = (uint32_t)(w_plane * 2);
    ep.x2_py = y.numel() / npl(x2);
  }
  if (residual.has_value() && residual->defined()) {
    TORCH_CHECK(residual->scalar_type() == at::kBFloat16 && residual->sizes() == y.sizes() &&
                    residual->is_contiguous(at::MemoryFormat::ChannelsLast), "residual like y");
    ep.residual = reinterpret_cast<const uint16_t*>(residual->data_ptr());
  }
  if (rmask.has_value() && rmask->defined()) {  // ReLU / dropout backward of the layer below (ConvEpi::rmask)
    TORCH_CHECK(!bn.has_value() && rmask->scalar_type() == at::kBFloat16 && rmask->sizes() == y.sizes() &&
                    rmask->is_contiguous(at::MemoryFormat::ChannelsLast),
                "rmask: channels_last bf16 like y, no BN epilogue");
    ep.rmask = reinterpret_cast<const uint16_t*>(rmask->data_ptr()) + (ep.x3 ? rmask->numel() / 3 : 0);
    ep.rmask_s = (float)rmask_scale;
  }
  std::vector<Tensor> bnf;
  Tensor dgm, dbt;
  if (bn.has_value()) {
    TORCH_CHECK(bn->size() == 4, "bn = (gamma, beta, mean, var)");
    for (const auto& t : *bn) {
      TORCH_CHECK(t.numel() == Cout, "bn parameter size");
      bnf.push_back(t.to(at::kFloat).contiguous());
    }
    ep.bn_gamma = bnf[0].data_ptr<float>();
    ep.bn_beta = bnf[1].data_ptr<float>();
    ep.bn_mean = bnf[2].data_ptr<float>();
    ep.bn_var = bnf[3].data_ptr<float>();
    ep.bn_eps = (float)bn_eps;
    ep.bn_fix_gamma = bn_fix_gamma ? 1 : 0;
    ep.act_relu = 1;
    TORCH_CHECK(bnb_x.has_value() && bnb_x->defined() && bnb_x->scalar_type() == at::kBFloat16 &&
                    bnb_x->sizes() == y.sizes() && bnb_x->is_contiguous(at::MemoryFormat::ChannelsLast),
                "bn needs bnb_x like y");
    ep.bnb_x = reinterpret_cast<const uint16_t*>(bnb_x->data_ptr());
    if (dadd.has_value() && dadd->defined()) set_dadd(ep, *dadd, y, Ho, Wo, false);
    if (x2 && ep.dadd) ep.x2_pd = dadd->numel() / npl(x2);
    if (bnb_part.has_value() && bnb_part->defined()) {  // deterministic sums, 64-row dgrad tiles
      TORCH_CHECK(bnb_part->scalar_type() == at::kFloat && bnb_part->is_contiguous() &&
                      bnb_part->numel() >= (((int64_t)NB * Ho * Wo + 63) / 64) * 2 * Cout,
                  "bnb_part: contiguous fp32 with ceil(M / 64) * 2 * Cout elements");
      ep.bnb_part = bnb_part->data_ptr<float>();
    } else {
      TORCH_CHECK(dgamma.has_value() && dbeta.has_value() && dgamma->scalar_type() == at::kFloat &&
                      dbeta->scalar_type() == at::kFloat && dgamma->is_contiguous() && dbeta->is_contiguous() &&
                      dgamma->numel() == Cout && dbeta->numel() == Cout,
                  "dgamma / dbeta: contiguous fp32 (C,)");
      dgm = *dgamma;
      dbt = *dbeta;
      ep.bnb_dgamma = dgm.data_ptr<float>();
      ep.bnb_dbeta = dbt.data_ptr<float>();
    }
  }
  // weight-gradient role
  TORCH_CHECK(wg_dy.scalar_type() == at::kBFloat16 && wg_x.scalar_type() == at::kBFloat16 &&
                  wg_dy.is_contiguous(at::MemoryFormat::ChannelsLast) && wg_x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_dgrad_wgrad: channels_last bf16 wg_dy / wg_x");
  TORCH_CHECK(!x2 || (wg_x.size(0) % npl(x2) == 0 && wg_dy.size(0) % npl(x2) == 0), "x2: wg_dy / wg_x pairs");
  const int gNB = (int)(x2 ? wg_x.size(0) / npl(x2) : wg_x.size(0)), gCin = (int)wg_x.size(1), gH = (int)wg_x.size(2),
            gW = (int)wg_x.size(3);
  const int gCout = (int)wg_dy.size(1), gHo = (int)wg_dy.size(2), gWo = (int)wg_dy.size(3);
  TORCH_CHECK(wg_dy.size(0) == wg_x.size(0) && gCin % 64 == 0 && gCout % 8 == 0, "conv_dgrad_wgrad: wgrad channels");
  TORCH_CHECK(gHo == (gH + 2 * wg_pad - KH) / wg_stride + 1 && gWo == (gW + 2 * wg_pad - KW) / wg_stride + 1,
              "conv_dgrad_wgrad: wgrad geometry");
  const auto gdt = x2 ? at::kFloat : at::kBFloat16;
  TORCH_CHECK(wg_out.scalar_type() == gdt && wg_out.size(0) == gCout && wg_out.size(1) == gCin &&
                  wg_out.size(2) == KH && wg_out.size(3) == KW && wg_out.is_contiguous(at::MemoryFormat::ChannelsLast),
              "wg_out: channels_last (Cout, Cin, KH, KW), bf16 (fp32 for x2)");
  mxr::WgradX2 wx2;
  if (x2) {
    wx2.x2 = 1;
    wx2.x3 = npl(x2) == 3 ? 1 : 0;
    wx2.pdy = (uint32_t)(wg_dy.numel() / npl(x2) * 2);
    wx2.px = (uint32_t)(wg_x.numel() / npl(x2) * 2);
    wx2.dwf = wg_out.data_ptr<float>();
  }
  const float* pslab = nullptr;
  uint16_t* pout = nullptr;
  float* poutf = nullptr;
  int psplits = 0;
  int64_t pn = 0;
  if (prev_slab.has_value() && prev_slab->defined() && prev_slab->numel() > 0) {
    TORCH_CHECK(prev_out.has_value() && prev_out->defined() && prev_out->scalar_type() == gdt &&
                    prev_slab->scalar_type() == at::kFloat && prev_slab->numel() % prev_out->numel() == 0,
                "prev_slab (splits * n fp32) / prev_out (n, the gradient dtype)");
    pn = prev_out->numel();
    psplits = (int)(prev_slab->numel() / pn);
    pslab = prev_slab->data_ptr<float>();
    if (x2) poutf = prev_out->data_ptr<float>();
    else pout = reinterpret_cast<uint16_t*>(prev_out->data_ptr());
  }
  DevGuard g(x.device());
  int sp = 1;
  mxr::conv_wgrad_plan(gNB, gHo, gWo, gCin, gCout, (int)KH, (int)KW, &sp, (int)x2);
  Tensor slab = at::empty({sp > 1 ? (int64_t)sp * gCout * KH * KW * gCin : 1}, x.options().dtype(at::kFloat));
  const int r = mxr::conv_dgrad_wgrad(
      reinterpret_cast<const uint16_t*>(x.data_ptr()), reinterpret_cast<const uint16_t*>(w.data_ptr()),
      reinterpret_cast<uint16_t*>(y.data_ptr()), NB, H, W, Cin, Ho, Wo, Cout, kh, kw, (int)pad, ep,
      reinterpret_cast<const uint16_t*>(wg_dy.data_ptr()), reinterpret_cast<const uint16_t*>(wg_x.data_ptr()),
      x2 ? nullptr : reinterpret_cast<uint16_t*>(wg_out.data_ptr()), slab.data_ptr<float>(), gNB, gH, gW, gCin, gHo,
      gWo, gCout, (int)KH, (int)KW, (int)wg_stride, (int)wg_pad, sp, 1, cur_stream(), defer ? 1 : 0, pslab, psplits,
      pn, pout, wx2, poutf);
  TORCH_CHECK(r == 0, "conv_dgrad_wgrad: unsupported shape");
  const Tensor none = at::empty({0}, x.options().dtype(at::kFloat));
  return {y, dgm.defined() ? dgm : none, dbt.defined() ? dbt : none, (defer && sp > 1) ? slab : none};
}

// split-K reduce of a deferred grouped weight gradient: out (bf16, n) += sum of slab's splits
void wgrad_reduce_run(const Tensor& slab, Tensor out) {
  CHECK_DEV(slab); CHECK_DEV(out);
  const bool f32 = out.scalar_type() == at::kFloat;
  TORCH_CHECK(slab.scalar_type() == at::kFloat && (f32 || out.scalar_type() == at::kBFloat16) && out.numel() % 4 == 0 &&
                  slab.numel() % out.numel() == 0, "wgrad_reduce_run: slab (splits * n fp32), out (n bf16 / fp32)");
  DevGuard g(out.device());
  mxr::wgrad_reduce_run(slab.data_ptr<float>(), (int)(slab.numel() / out.numel()), out.numel(),
                        f32 ? nullptr : reinterpret_cast<uint16_t*>(out.data_ptr()), cur_stream(),
                        f32 ? out.data_ptr<float>() : nullptr);
}

// ---- pooling ---------------------------------------------------------------------------------
std::vector<Tensor> maxpool_fwd(const Tensor& x, int64_t k, int64_t s, int64_t p, int64_t x2, bool need_arg,
                                c10::optional<Tensor> post_bn) {
  CHECK_DEV(x);
  TORCH_CHECK((x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf) && x.dim() == 4 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "maxpool: x must be channels_last bf16 / fp16 (N,C,H,W)");
  TORCH_CHECK(!x2 || (x.scalar_type() == at::kBFloat16 && x.size(0) % npl(x2) == 0), "maxpool x2: bf16 (2N, ...) pairs");
  const int N = (int)(x2 ? x.size(0) / npl(x2) : x.size(0)), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  TORCH_CHECK(C % 8 == 0, "maxpool needs C % 8 == 0");
  const int Ho = (H + 2 * (int)p - (int)k) / (int)s + 1, Wo = (W + 2 * (int)p - (int)k) / (int)s + 1;
  TORCH_CHECK(Ho > 0 && Wo > 0, "maxpool: empty output");
  TORCH_CHECK(!(post_bn && need_arg), "maxpool_fwd: post_bn is inference-only (no taps)");
  const mxr::PostBn post = post_bn_args(post_bn, C);
  DevGuard g(x.device());
  Tensor y = at::empty({x2 ? npl(x2) * N : N, C, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor arg = need_arg ? at::empty({N, C, Ho, Wo}, x.options().dtype(at::kByte).memory_format(at::MemoryFormat::ChannelsLast))
                        : at::empty({0}, x.options().dtype(at::kByte));  // inference: no taps written
  const int rc = mxr::maxpool_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()), reinterpret_cast<uint16_t*>(y.data_ptr()),
                                  need_arg ? arg.data_ptr<uint8_t>() : nullptr, N, H, W, C, Ho, Wo, (int)k, (int)s, (int)p,
                                  x2 ? pcode(x2) : dcode(x), cur_stream(), post);
  TORCH_CHECK(rc == 0, "maxpool_fwd: unsupported shape");
  return {y, arg};
}

Tensor maxpool_bwd(const Tensor& dy, const Tensor& arg, int64_t H, int64_t W, int64_t k, int64_t s, int64_t p,
                   int64_t x2) {
  CHECK_DEV(dy); CHECK_DEV(arg);
  TORCH_CHECK((dy.scalar_type() == at::kBFloat16 || dy.scalar_type() == at::kHalf) &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast) && arg.scalar_type() == at::kByte &&
                  arg.size(0) * (x2 ? npl(x2) : 1) == dy.size(0) && arg.size(1) == dy.size(1) && arg.size(2) == dy.size(2) &&
                  arg.size(3) == dy.size(3) && arg.is_contiguous(at::MemoryFormat::ChannelsLast),
              "maxpool_bwd: channels_last bf16 dy (2N: x2 pairs) + byte arg (N, ...)");
  const int N = (int)arg.size(0), C = (int)dy.size(1), Ho = (int)dy.size(2), Wo = (int)dy.size(3);
  TORCH_CHECK((H + 2 * p - k) / s + 1 == Ho && (W + 2 * p - k) / s + 1 == Wo, "maxpool_bwd: shape mismatch");
  DevGuard g(dy.device());
  Tensor dx = at::empty({x2 ? npl(x2) * N : N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int rc = mxr::maxpool_bwd(reinterpret_cast<const uint16_t*>(dy.data_ptr()), arg.data_ptr<uint8_t>(),
                                  reinterpret_cast<uint16_t*>(dx.data_ptr()), N, (int)H, (int)W, C, Ho, Wo, (int)k,
                                  (int)s, (int)p, x2 ? pcode(x2) : dcode(dy), cur_stream());
  TORCH_CHECK(rc == 0, "maxpool_bwd: unsupported shape");
  return dx;
}

Tensor avgpool_fwd(const Tensor& x, int64_t x2) {
  CHECK_DEV(x);
  TORCH_CHECK((x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf) && x.dim() == 4 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "avgpool: x must be channels_last bf16 / fp16 (N,C,H,W)");
  TORCH_CHECK(!x2 || (x.scalar_type() == at::kBFloat16 && x.size(0) % npl(x2) == 0), "avgpool x2: bf16 (2N, ...) pairs");
  const int N = (int)(x2 ? x.size(0) / npl(x2) : x.size(0)), C = (int)x.size(1), HW = (int)(x.size(2) * x.size(3));
  DevGuard g(x.device());
  Tensor y = at::empty({x2 ? npl(x2) * N : N, C}, x.options());
  TORCH_CHECK(mxr::avgpool_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()), reinterpret_cast<uint16_t*>(y.data_ptr()),
                               N, HW, C, x2 ? pcode(x2) : dcode(x), cur_stream()) == 0, "avgpool_fwd: C % 8 != 0");
  return y;
}

Tensor avgpool_bwd(const Tensor& dy, int64_t H, int64_t W, int64_t x2) {
  CHECK_DEV(dy);
  TORCH_CHECK((dy.scalar_type() == at::kBFloat16 || dy.scalar_type() == at::kHalf) && dy.dim() == 2 && dy.is_contiguous(),
              "avgpool_bwd: dy (N, C) bf16 / fp16");
  TORCH_CHECK(!x2 || (dy.scalar_type() == at::kBFloat16 && dy.size(0) % npl(x2) == 0), "avgpool_bwd x2: bf16 (2N, C) pairs");
  const int N = (int)(x2 ? dy.size(0) / npl(x2) : dy.size(0)), C = (int)dy.size(1);
  DevGuard g(dy.device());
  Tensor dx = at::empty({x2 ? npl(x2) * N : N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  TORCH_CHECK(mxr::avgpool_bwd(reinterpret_cast<const uint16_t*>(dy.data_ptr()), reinterpret_cast<uint16_t*>(dx.data_ptr()),
                               N, (int)(H * W), C, x2 ? pcode(x2) : dcode(dy), cur_stream()) == 0, "avgpool_bwd: C % 8 != 0");
  return dx;
}

// ---- stem conv (stem.hip) ------------------------------------------------------------------------
Tensor stem_conv(const Tensor& x, const Tensor& w, const std::vector<Tensor>& in_bn, double in_eps, bool in_fixg,
                 const std::vector<Tensor>& out_bn, double out_eps, bool out_fixg, const c10::optional<Tensor>& bias,
                 int64_t KH, int64_t KW, int64_t stride, int64_t pad, bool relu) {
  CHECK_DEV(x); CHECK_DEV(w);
  // fp32 modes: an fp32 image, the packed filter an x2 pair (128, KP) / x3 triple (192, KP) in the
  // logical plane order (hi, lo) / (hi, mid, lo), and the output x2 pairs / x3 triples
  const bool x2 = x.scalar_type() == at::kFloat;
  const int sp = x2 ? (w.size(0) == 192 ? 3 : 2) : 1;
  TORCH_CHECK((x2 || x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf) && x.dim() == 4 &&
                  x.size(1) == 3 && x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem_conv: x must be channels_last fp32 / bf16 / fp16 (N,3,H,W)");
  const int64_t KP = (KH * KW * 3 + 31) / 32 * 32;
  TORCH_CHECK(w.scalar_type() == (x2 ? at::kBFloat16 : x.scalar_type()) && w.dim() == 2 &&
                  w.size(0) == 64 * sp && w.size(1) == KP && w.is_contiguous(),
              "stem_conv: w must be the packed contiguous (64, KP) filter of x's dtype ((128, KP) x2 pair for fp32)");
  mxr::StemArgs a{};
  TORCH_CHECK(in_bn.empty() || in_bn.size() == 4, "stem_conv: in_bn = [] or [gamma, beta, mean, var]");
  TORCH_CHECK(out_bn.empty() || out_bn.size() == 4, "stem_conv: out_bn = [] or [gamma, beta, mean, var]");
  for (const Tensor& t : in_bn) {
    CHECK_DEV(t);
    TORCH_CHECK(t.scalar_type() == at::kFloat && t.numel() == 3 && t.is_contiguous(), "stem_conv: in_bn fp32 (3)");
  }
  for (const Tensor& t : out_bn) {
    CHECK_DEV(t);
    TORCH_CHECK(t.scalar_type() == at::kFloat && t.numel() == 64 && t.is_contiguous(), "stem_conv: out_bn fp32 (64)");
  }
  if (!in_bn.empty()) {
    a.in_g = in_bn[0].data_ptr<float>(); a.in_b = in_bn[1].data_ptr<float>();
    a.in_m = in_bn[2].data_ptr<float>(); a.in_v = in_bn[3].data_ptr<float>();
  }
  a.in_eps = (float)in_eps; a.in_fixg = in_fixg ? 1 : 0;
  if (!out_bn.empty()) {
    a.out_g = out_bn[0].data_ptr<float>(); a.out_b = out_bn[1].data_ptr<float>();
    a.out_m = out_bn[2].data_ptr<float>(); a.out_v = out_bn[3].data_ptr<float>();
  }
  a.out_eps = (float)out_eps; a.out_fixg = out_fixg ? 1 : 0;
  if (bias.has_value() && bias->defined()) {
    CHECK_DEV((*bias));
    TORCH_CHECK(bias->numel() == 64 && bias->is_contiguous(), "stem_conv: bias (64)");
    a.bias = bias->data_ptr();
    a.bias_code = dcode(*bias);
  }
  TORCH_CHECK(pad >= 0 && pad < KH && pad < KW, "stem_conv: pad");
  const int N = (int)x.size(0), H = (int)x.size(2), W = (int)x.size(3);
  const int Ho = (int)((H + 2 * pad - KH) / stride + 1), Wo = (int)((W + 2 * pad - KW) / stride + 1);
  TORCH_CHECK(Ho > 0 && Wo > 0, "stem_conv: empty output");
  DevGuard g(x.device());
  Tensor y = at::empty({sp * N, 64, Ho, Wo},
                       x.options().dtype(x2 ? at::kBFloat16 : x.scalar_type()).memory_format(at::MemoryFormat::ChannelsLast));
  const int rc = mxr::stem_conv(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                reinterpret_cast<const uint16_t*>(w.data_ptr()), a,
                                reinterpret_cast<uint16_t*>(y.data_ptr()), N, H, W, Ho, Wo, (int)KH, (int)KW,
                                (int)stride, (int)pad, relu ? 1 : 0, x2 ? (sp == 3 ? 4 : 3) : dcode(x), cur_stream());
  TORCH_CHECK(rc == 0, "stem_conv: unsupported geometry (7x7/2 and 3x3/1 only) or grid too large");
  LAUNCH_CHECK("stem_conv");
  return y;
}

// ---- small-head backward / channel sum (head_bwd.hip) --------------------------------------------
bool al16(const Tensor& t) { return (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0; }

// x (M, K) bf16 rows shared by 1-2 heads; dys[h] (M, N_h), ws[h] (N_h, K), dws[h] (N_h, K) bf16 targets
// (accumulated when dw_acc[h]); dbs[h] (N_h) fp32 / bf16 targets (accumulated when db_acc[h]) or
// empty (skipped).  Returns dx (M, K), ReLU-masked by x > 0 when relu_mask (empty unless need_dx).
Tensor head_bwd(const Tensor& x, const std::vector<Tensor>& dys, const std::vector<Tensor>& ws,
                const std::vector<Tensor>& dws, const std::vector<bool>& dw_acc, const std::vector<Tensor>& dbs,
                const std::vector<bool>& db_acc, bool need_dx, bool relu_mask, int64_t x2,
                const std::vector<int64_t>& w_planes, double mask_scale) {
  CHECK_DEV(x);
  const int nh = (int)dys.size();
  TORCH_CHECK(nh >= 1 && nh <= 2 && (int)ws.size() == nh && (int)dws.size() == nh && (int)dw_acc.size() == nh &&
                  (int)dbs.size() == nh && (int)db_acc.size() == nh, "head_bwd: 1 or 2 heads, one entry per head");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.is_contiguous() && al16(x),
              "head_bwd: x must be a contiguous 16-B aligned bf16 (M, K) matrix");
  // x2 (fp32-class): x (2M, K) and dx are hi / lo pairs, each w_h a pair with its lo plane
  // w_planes[h] elements on, dy / dw fp32
  TORCH_CHECK(!x2 || (x.size(0) % npl(x2) == 0 && (int)w_planes.size() == nh), "head_bwd x2: (2M, K) x and w_planes");
  const int M = (int)(x2 ? x.size(0) / npl(x2) : x.size(0)), K = (int)x.size(1);
  TORCH_CHECK(K % 64 == 0, "head_bwd: K % 64 == 0");
  mxr::HeadBwdArgs a;
  a.nheads = nh;
  a.x2 = x2 ? 1 : 0;
  a.x3 = npl(x2) == 3 ? 1 : 0;
  const auto adt = x2 ? at::kFloat : at::kBFloat16;  // dy / dw dtype
  for (int h = 0; h < nh; ++h) {
    const Tensor &dy = dys[h], &w = ws[h], &dw = dws[h], &db = dbs[h];
    CHECK_DEV(dy); CHECK_DEV(w); CHECK_DEV(dw);
    TORCH_CHECK(dy.scalar_type() == adt && dy.dim() == 2 && dy.size(0) == M && dy.is_contiguous(),
                "head_bwd: dy must be contiguous (M, N), bf16 (fp32 for x2)");
    const int N = (int)dy.size(1);
    TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.numel() == (int64_t)N * K && al16(w),
                "head_bwd: w must be a contiguous 16-B aligned bf16 (N, K) matrix");
    TORCH_CHECK(dw.scalar_type() == adt && dw.is_contiguous() && dw.numel() == (int64_t)N * K && al16(dw),
                "head_bwd: dw must be a contiguous 16-B aligned (N, K) matrix, bf16 (fp32 for x2)");
    if (x2) {
      TORCH_CHECK(w_planes[h] >= (int64_t)N * K && w_planes[h] % 8 == 0, "head_bwd: w plane");
      a.dyf[h] = dy.data_ptr<float>();
      a.dwf[h] = dw.data_ptr<float>();
      a.w_plane[h] = w_planes[h];
    } else {
      a.dy[h] = reinterpret_cast<const uint16_t*>(dy.data_ptr());
      a.dw[h] = reinterpret_cast<uint16_t*>(dw.data_ptr());
    }
    a.w[h] = reinterpret_cast<const uint16_t*>(w.data_ptr());
    a.N[h] = N;
    a.dw_acc[h] = dw_acc[h] ? 1 : 0;
    if (db.defined() && db.numel() > 0) {
      CHECK_DEV(db);
      TORCH_CHECK(db.numel() == N && db.is_contiguous(), "head_bwd: db must be contiguous (N,)");
      a.db[h] = db.data_ptr();
      a.db_code[h] = dcode(db);
      a.db_acc[h] = db_acc[h] ? 1 : 0;
    }
  }
  DevGuard g(x.device());
  Tensor dx;
  if (need_dx) {
    dx = at::empty({x2 ? npl(x2) * M : M, K}, x.options());
    a.dx = reinterpret_cast<uint16_t*>(dx.data_ptr());
    a.relu_mask = relu_mask ? 1 : 0;
    a.mask_scale = (float)mask_scale;
  }
  a.rs = mxr::head_bwd_splits(M, K, a.N, nh);
  Tensor wsp;
  if (a.rs > 1) {
    int64_t tot = 0;
    for (int h = 0; h < nh; ++h) tot += (int64_t)a.rs * a.N[h] * (K + 1);
    wsp = at::empty({tot}, x.options().dtype(at::kFloat));
    float* p = wsp.data_ptr<float>();
    for (int h = 0; h < nh; ++h) {
      a.ws_dw[h] = p;
      p += (int64_t)a.rs * a.N[h] * K;
      a.ws_db[h] = p;
      p += (int64_t)a.rs * a.N[h];
    }
  }
  TORCH_CHECK(mxr::head_bwd(reinterpret_cast<const uint16_t*>(x.data_ptr()), M, K, a, cur_stream()) == 0,
              "head_bwd: unsupported shape");
  return dx;
}

// per-channel sum of a channels_last map or (M, C) matrix into out (C,) fp32 / bf16 (+= when accumulate)
void chan_sum(const Tensor& x, Tensor out, bool accumulate, int64_t x2) {
  CHECK_DEV(x); CHECK_DEV(out);
  TORCH_CHECK(!x2 || (x.scalar_type() == at::kBFloat16 && x.size(0) % npl(x2) == 0), "chan_sum x2: bf16 (2N, ...) pairs");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf, "chan_sum: bf16 / fp16 input");
  int64_t C;
  if (x.dim() == 4) {
    TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), "chan_sum: 4-D input must be channels_last");
    C = x.size(1);
  } else {
    TORCH_CHECK(x.dim() == 2 && x.is_contiguous(), "chan_sum: 2-D input must be contiguous");
    C = x.size(1);
  }
  TORCH_CHECK(C % 8 == 0 && al16(x), "chan_sum: C % 8 == 0 and 16-B aligned rows");
  TORCH_CHECK(out.numel() == C && out.is_contiguous(), "chan_sum: out (C,) contiguous");
  const int64_t M = x.numel() / C / (x2 ? npl(x2) : 1);
  DevGuard g(x.device());
  Tensor part = at::empty({(int64_t)mxr::chan_sum_chunks(M, (int)C) * C}, x.options().dtype(at::kFloat));
  TORCH_CHECK(mxr::chan_sum(reinterpret_cast<const uint16_t*>(x.data_ptr()), M, (int)C, x2 ? pcode(x2) : dcode(x),
                            part.data_ptr<float>(), out.data_ptr(), dcode(out), accumulate ? 1 : 0, cur_stream()) == 0,
              "chan_sum: unsupported shape");
}

// ---- DP interference probes (tools/dp_interference.py) -----------------------------------------
void cu_spin(int64_t nwg, double us) {
  mxr::cu_spin((int)nwg, (int64_t)(us * 100.0), cur_stream());  // s_memrealtime: 100 MHz
}

void cu_copy(const Tensor& src, Tensor dst, int64_t nwg) {
  CHECK_DEV(src); CHECK_DEV(dst);
  TORCH_CHECK(src.scalar_type() == at::kFloat && dst.scalar_type() == at::kFloat && src.is_contiguous() &&
                  dst.is_contiguous() && src.numel() == dst.numel() && src.numel() % 4 == 0,
              "cu_copy: contiguous fp32 src / dst of one size (multiple of 4)");
  mxr::cu_copy(src.data_ptr<float>(), dst.data_ptr<float>(), src.numel(), (int)nwg, cur_stream());
}

// ---- proposal top-k ----------------------------------------------------------------------------
std::vector<Tensor> proposal_topk(const Tensor& keys, const Tensor& boxes, int64_t P) {
  CHECK_DEV(keys); CHECK_DEV(boxes);
  TORCH_CHECK(keys.scalar_type() == at::kFloat && boxes.scalar_type() == at::kFloat && keys.is_contiguous() &&
                  boxes.is_contiguous() && keys.dim() == 2 && boxes.dim() == 3 && boxes.size(2) == 4 &&
                  boxes.size(0) == keys.size(0) && boxes.size(1) == keys.size(1),
              "proposal_topk: keys (B, N) and boxes (B, N, 4), contiguous fp32");
  const int B = (int)keys.size(0), N = (int)keys.size(1);
  TORCH_CHECK(P > 0 && P <= N, "proposal_topk: 0 < P <= N");
  DevGuard g(keys.device());
  auto o = keys.options();
  Tensor ws = clean_ws(o.dtype(at::kInt), "topk", mxr::proposal_topk_ws_words(B, N), B);  // histograms: atomics
  Tensor wk = at::empty({(int64_t)B * P}, o.dtype(at::kInt));
  Tensor wi = at::empty({(int64_t)B * P}, o.dtype(at::kInt));
  Tensor sk = at::empty({B, P}, o);
  Tensor sb = at::empty({B, P, 4}, o);
  Tensor nv = at::empty({B}, o.dtype(at::kInt));
  TORCH_CHECK(mxr::proposal_topk(keys.data_ptr<float>(), boxes.data_ptr<float>(), B, N, (int)P,
                                 reinterpret_cast<uint32_t*>(ws.data_ptr<int>()),
                                 reinterpret_cast<uint32_t*>(wk.data_ptr<int>()), wi.data_ptr<int>(),
                                 sk.data_ptr<float>(), sb.data_ptr<float>(), nv.data_ptr<int>(), cur_stream()) == 0,
              "proposal_topk failed");
  return {sk, sb, nv};
}

// ---- detection post-process -------------------------------------------------------------------
std::vector<Tensor> det_postprocess(const Tensor& rois, const Tensor& scores, const Tensor& deltas,
                                    const Tensor& im_info, double thresh, double nms_thresh, int64_t max_per,
                                    int64_t cap) {
  CHECK_DEV(rois); CHECK_DEV(scores); CHECK_DEV(deltas); CHECK_DEV(im_info);
  for (const Tensor* t : {&rois, &scores, &deltas, &im_info})
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous(), "det_postprocess: contiguous fp32 inputs");
  const int B = (int)im_info.size(0);
  const int64_t RB = rois.size(0);
  const int C = (int)scores.size(1);
  TORCH_CHECK(B > 0 && RB % B == 0, "rois must hold the same number of RoIs per image, grouped by image");
  const int R = (int)(RB / B);
  TORCH_CHECK(rois.size(1) == 5 && scores.size(0) == RB && deltas.size(0) == RB && deltas.size(1) == 4 * C,
              "det_postprocess: shape mismatch");
  TORCH_CHECK(R <= 1024 && C >= 2 && C <= 1025, "det_postprocess: at most 1024 RoIs per image and 1024 classes");
  DevGuard g(rois.device());
  auto fo = rois.options();
  Tensor ws_s = at::empty({(int64_t)B * (C - 1) * R}, fo);
  Tensor ws_b = at::empty({(int64_t)B * (C - 1) * R * 4}, fo);
  Tensor ws_n = at::empty({(int64_t)B * (C - 1)}, fo.dtype(at::kInt));
  Tensor dets = at::zeros({B, cap, 6}, fo);
  Tensor counts = at::empty({B}, fo.dtype(at::kInt));
  const int rc = mxr::det_postprocess(rois.data_ptr<float>(), scores.data_ptr<float>(), deltas.data_ptr<float>(),
                                      im_info.data_ptr<float>(), B, R, C, (float)thresh, (float)nms_thresh,
                                      (int)max_per, (int)cap, ws_s.data_ptr<float>(), ws_b.data_ptr<float>(),
                                      ws_n.data_ptr<int>(), dets.data_ptr<float>(), counts.data_ptr<int>(),
                                      cur_stream());
  TORCH_CHECK(rc == 0, "det_postprocess: unsupported shape");
  return {dets, counts};
}

Tensor nest_keep(const Tensor& dets, double thresh) {
  CHECK_DEV(dets);
  TORCH_CHECK(dets.scalar_type() == at::kFloat && dets.dim() == 2 && dets.size(1) >= 4 && dets.stride(1) == 1,
              "nest: dets (N, >=4) fp32 with unit column stride");
  DevGuard g(dets.device());
  Tensor keep = at::empty({dets.size(0)}, dets.options().dtype(at::kByte));
  mxr::nest_filter(dets.data_ptr<float>(), (int)dets.size(0), (int)dets.stride(0), (float)thresh,
                   keep.data_ptr<uint8_t>(), cur_stream());
  return keep;
}

Tensor philox_uniform_cpu(int64_t seed, int64_t step, int64_t n) {
  Tensor out = at::empty({n}, at::TensorOptions().dtype(at::kFloat));
  float* o = out.data_ptr<float>();
  at::parallel_for(0, n, 4096, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) o[i] = mxr::philox_uniform_host((uint32_t)seed, (uint64_t)step, (uint64_t)i);
  });
  return out;
}

// ---- training-mode BN ----------------------------------------------------------------------
std::vector<Tensor> bn_train_fwd(const Tensor& x, const Tensor& gamma, const Tensor& beta, Tensor rmean, Tensor rvar,
                                 double momentum, double eps, bool fix_gamma, bool relu, int64_t x2) {
  CHECK_DEV(x);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.is_contiguous(at::MemoryFormat::ChannelsLast), "x: bf16 NHWC");
  TORCH_CHECK(!x2 || x.size(0) % npl(x2) == 0, "x2: (2N, ...) pairs");
  const int C = (int)x.size(1);
  const int64_t M = x.numel() / C / (x2 ? npl(x2) : 1);
  TORCH_CHECK(C % 64 == 0, "bn_train needs C % 64 == 0");
  CHECK_F32(rmean); CHECK_F32(rvar); CHECK_CONTIG(rmean); CHECK_CONTIG(rvar);
  DevGuard g(x.device());
  Tensor gf = gamma.to(at::kFloat).contiguous(), bf = beta.to(at::kFloat).contiguous();
  Tensor y = at::empty_like(x, x.options(), at::MemoryFormat::ChannelsLast);
  // save rows: mean, invstd, var + eps
  Tensor save = at::empty({3, C}, x.options().dtype(at::kFloat));
  float* sv = save.data_ptr<float>();
  Tensor ws = at::empty({mxr::bn_train_workspace_floats(M, C)}, x.options().dtype(at::kFloat));
  const int r = mxr::bn_train_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()), M, C,
                                  gf.data_ptr<float>(), bf.data_ptr<float>(), rmean.data_ptr<float>(),
                                  rvar.data_ptr<float>(), (float)momentum, (float)eps, fix_gamma ? 1 : 0, relu ? 1 : 0,
                                  reinterpret_cast<uint16_t*>(y.data_ptr()), sv, sv + C, ws.data_ptr<float>(),
                                  cur_stream(), sv + 2 * C, x2 ? npl(x2) : 0);
  TORCH_CHECK(r == 0, "bn_train_fwd: unsupported shape");
  return {y, save};
}

// normalisation from conv-epilogue statistics partials (conv_igemm_fwd(..., stat_shift=rmean)[1])
std::vector<Tensor> bn_train_apply(const Tensor& x, const Tensor& part, const Tensor& gamma, const Tensor& beta,
                                   Tensor rmean, Tensor rvar, double momentum, double eps, bool fix_gamma, bool relu,
                                   int64_t x2) {
  CHECK_DEV(x); CHECK_DEV(part);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.is_contiguous(at::MemoryFormat::ChannelsLast), "x: bf16 NHWC");
  TORCH_CHECK(!x2 || x.size(0) % npl(x2) == 0, "x2: (2N, ...) pairs");
  const int C = (int)x.size(1);
  const int64_t M = x.numel() / C / (x2 ? npl(x2) : 1);
  TORCH_CHECK(C % 64 == 0, "bn_train needs C % 64 == 0");
  CHECK_F32(rmean); CHECK_F32(rvar); CHECK_CONTIG(rmean); CHECK_CONTIG(rvar);
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.is_contiguous() && part.dim() == 2 && part.size(1) == C &&
                  part.size(0) % 2 == 1 && part.size(0) >= 3, "part: fp32 (2 * nparts + 1, C)");
  DevGuard g(x.device());
  Tensor gf = gamma.to(at::kFloat).contiguous(), bf = beta.to(at::kFloat).contiguous();
  Tensor y = at::empty_like(x, x.options(), at::MemoryFormat::ChannelsLast);
  Tensor save = at::empty({3, C}, x.options().dtype(at::kFloat));
  const int r = mxr::bn_train_apply(reinterpret_cast<const uint16_t*>(x.data_ptr()), M, C,
                                    part.data_ptr<float>(), (int)((part.size(0) - 1) / 2), gf.data_ptr<float>(),
                                    bf.data_ptr<float>(), rmean.data_ptr<float>(), rvar.data_ptr<float>(),
                                    (float)momentum, (float)eps, fix_gamma ? 1 : 0, relu ? 1 : 0,
                                    reinterpret_cast<uint16_t*>(y.data_ptr()), save.data_ptr<float>(), cur_stream(),
                                    x2 ? npl(x2) : 0);
  TORCH_CHECK(r == 0, "bn_train_apply: unsupported shape");
  return {y, save};
}

// frozen-BN gamma / beta gradients from the conv epilogue's partial rows (ConvEpi::bnb_part,
// [nparts][sum g | sum g * xhat][C]): dbeta += fixed-order sum of the first halves, dgamma += of
// the second (deterministic; either output may be None)
void bnb_part_fold(const Tensor& part, int64_t nparts, int64_t C, c10::optional<Tensor> dgamma,
                   c10::optional<Tensor> dbeta) {
  CHECK_DEV(part);
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.is_contiguous() && nparts > 0 &&
                  part.numel() >= nparts * 2 * C, "part: fp32 with nparts * 2 * C elements");
  float* out[2] = {nullptr, nullptr};
  int i = 0;
  for (auto* p : {&dbeta, &dgamma}) {
    if (p->has_value() && (*p)->defined()) {
      TORCH_CHECK((*p)->scalar_type() == at::kFloat && (*p)->is_contiguous() && (*p)->numel() == C &&
                      (*p)->device() == part.device(), "dgamma / dbeta: fp32 (C,) on part's device");
      out[i] = (*p)->data_ptr<float>();
    }
    ++i;
  }
  DevGuard g(part.device());
  mxr::col_part_fold(part.data_ptr<float>(), (int)nparts, (int)C, out[0], out[1], cur_stream());
}

// many bnb_part_fold calls in as few launches as possible: entries (part, nparts, C, dgamma | None,
// dbeta | None), up to mxr::kMaxFolds per launch
void bnb_part_fold_multi(const std::vector<std::tuple<Tensor, int64_t, int64_t, c10::optional<Tensor>,
                                                      c10::optional<Tensor>>>& entries) {
  if (entries.empty()) return;
  DevGuard g(std::get<0>(entries[0]).device());
  mxr::FoldBatch fb{};
  auto flush = [&]() {
    if (fb.n > 0) mxr::bn_part_fold_multi(fb, cur_stream());
    fb.n = 0;
  };
  int blk = 0;
  for (const auto& en : entries) {
    const Tensor& part = std::get<0>(en);
    const int64_t np = std::get<1>(en), C = std::get<2>(en);
    CHECK_DEV(part);
    TORCH_CHECK(part.scalar_type() == at::kFloat && part.is_contiguous() && np > 0 && part.numel() >= np * 2 * C,
                "part: fp32 with nparts * 2 * C elements");
    float* out[2] = {nullptr, nullptr};
    const c10::optional<Tensor>* opts[2] = {&std::get<4>(en), &std::get<3>(en)};  // (dbeta, dgamma)
    for (int k = 0; k < 2; ++k) {
      const auto& o = *opts[k];
      if (o.has_value() && o->defined()) {
        TORCH_CHECK(o->scalar_type() == at::kFloat && o->is_contiguous() && o->numel() == C &&
                        o->device() == part.device(), "dgamma / dbeta: fp32 (C,) on part's device");
        out[k] = o->data_ptr<float>();
      }
    }
    if (!out[0] && !out[1]) continue;
    if (fb.n == mxr::kMaxFolds) {
      flush();
      blk = 0;
    }
    fb.e[fb.n++] = {part.data_ptr<float>(), out[0], out[1], (int)np, (int)C, blk};
    blk += (int)((2 * C + 63) / 64);
  }
  flush();
}

// finish of a training-BN backward whose BN-backward epilogue (a dgrad conv with bnb_x = x,
// bn = (gamma_eff, beta, save[0], save[2]), eps 0, bnb_part = part) produced o; nparts partial rows
Tensor bn_train_dx_apply(Tensor o, const Tensor& x, const Tensor& save, const Tensor& gamma_eff, const Tensor& part,
                         int64_t nparts, c10::optional<Tensor> dres, c10::optional<Tensor> dgamma,
                         c10::optional<Tensor> dbeta, int64_t x2) {
  CHECK_DEV(o); CHECK_DEV(x); CHECK_DEV(part);
  TORCH_CHECK(!x2 || x.size(0) % npl(x2) == 0, "x2: (2N, ...) pairs");
  const int C = (int)x.size(1);
  const int64_t M = x.numel() / C / (x2 ? npl(x2) : 1);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  o.scalar_type() == at::kBFloat16 && o.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  o.sizes() == x.sizes(), "o / x: bf16 NHWC of one shape");
  TORCH_CHECK(save.scalar_type() == at::kFloat && save.is_contiguous() && save.numel() == 3 * C, "save: fp32 (3, C)");
  TORCH_CHECK(gamma_eff.scalar_type() == at::kFloat && gamma_eff.is_contiguous() && gamma_eff.numel() == C,
              "gamma_eff: fp32 (C,)");
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.is_contiguous() && nparts > 0 &&
                  part.numel() >= nparts * 2 * C, "part: fp32 with nparts * 2 * C elements");
  const uint16_t* rp = nullptr;
  if (dres.has_value() && dres->defined()) {
    TORCH_CHECK(dres->scalar_type() == at::kBFloat16 && dres->is_contiguous(at::MemoryFormat::ChannelsLast) &&
                    dres->sizes() == x.sizes(), "dres: bf16 NHWC like x");
    rp = reinterpret_cast<const uint16_t*>(dres->data_ptr());
  }
  float* dg = nullptr;
  float* db = nullptr;
  for (auto* p : {&dgamma, &dbeta}) {
    if (p->has_value() && (*p)->defined())
      TORCH_CHECK((*p)->scalar_type() == at::kFloat && (*p)->is_contiguous() && (*p)->numel() == C,
                  "dgamma / dbeta: fp32 (C,)");
  }
  if (dgamma.has_value() && dgamma->defined()) dg = dgamma->data_ptr<float>();
  if (dbeta.has_value() && dbeta->defined()) db = dbeta->data_ptr<float>();
  DevGuard g(x.device());
  const int r = mxr::bn_train_dx_apply(reinterpret_cast<const uint16_t*>(o.data_ptr()),
                                       reinterpret_cast<const uint16_t*>(x.data_ptr()), M, C,
                                       part.data_ptr<float>(), (int)nparts, gamma_eff.data_ptr<float>(),
                                       save.data_ptr<float>(), rp, reinterpret_cast<uint16_t*>(o.data_ptr()), dg, db,
                                       cur_stream(), x2 ? npl(x2) : 0);
  TORCH_CHECK(r == 0, "bn_train_dx_apply: unsupported shape");
  return o;
}

std::vector<Tensor> bn_train_bwd(const Tensor& x, const Tensor& dy, const Tensor& gamma, const Tensor& beta,
                                 const Tensor& save_mean, const Tensor& save_invstd, bool fix_gamma, bool relu,
                                 bool need_dx, c10::optional<Tensor> dgamma_out, c10::optional<Tensor> dbeta_out,
                                 int64_t x2) {
  CHECK_DEV(x); CHECK_DEV(dy);
  TORCH_CHECK(!x2 || (x.size(0) % npl(x2) == 0 && dy.scalar_type() == at::kBFloat16 && dy.sizes() == x.sizes()),
              "x2: (2N, ...) bf16 pairs");
  const int C = (int)x.size(1);
  const int64_t M = x.numel() / C / (x2 ? npl(x2) : 1);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.is_contiguous(at::MemoryFormat::ChannelsLast), "x: bf16 NHWC");
  Tensor g = dy.to(at::kBFloat16).contiguous(at::MemoryFormat::ChannelsLast);
  DevGuard dg(x.device());
  Tensor gf = gamma.to(at::kFloat).contiguous(), bf = beta.to(at::kFloat).contiguous();
  Tensor dx = need_dx ? at::empty_like(x, x.options(), at::MemoryFormat::ChannelsLast) : Tensor();
  const bool acc = dgamma_out.has_value() && dgamma_out->defined() && dbeta_out.has_value() && dbeta_out->defined();
  Tensor dgm, dbt;
  if (acc) {
    dgm = *dgamma_out;
    dbt = *dbeta_out;
    TORCH_CHECK(dgm.scalar_type() == at::kFloat && dbt.scalar_type() == at::kFloat && dgm.is_contiguous() &&
                    dbt.is_contiguous() && dgm.numel() == C && dbt.numel() == C, "dgamma/dbeta out: fp32 (C,)");
  } else {
    dgm = at::zeros({C}, x.options().dtype(at::kFloat));
    dbt = at::zeros({C}, x.options().dtype(at::kFloat));
  }
  TORCH_CHECK(C % 64 == 0, "bn_train needs C % 64 == 0");
  Tensor ws = at::empty({mxr::bn_train_workspace_floats(M, C)}, x.options().dtype(at::kFloat));
  const int r = mxr::bn_train_bwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                  reinterpret_cast<const uint16_t*>(g.data_ptr()), M, C,
                                  gf.data_ptr<float>(), bf.data_ptr<float>(), save_mean.data_ptr<float>(),
                                  save_invstd.data_ptr<float>(), fix_gamma ? 1 : 0, relu ? 1 : 0,
                                  need_dx ? reinterpret_cast<uint16_t*>(dx.data_ptr()) : nullptr,
                                  dgm.data_ptr<float>(), dbt.data_ptr<float>(), acc ? 1 : 0, ws.data_ptr<float>(),
                                  cur_stream(), x2 ? npl(x2) : 0);
  TORCH_CHECK(r == 0, "bn_train_bwd: unsupported shape");
  return {dx, dgm, dbt};
}

// dgrad filter cache: table of (src, dst) filters -> device byte tensor, built once
std::vector<int64_t> wt_flip_table_info(const std::vector<Tensor>& srcs) {
  int64_t tiles = 0;
  for (const auto& s : srcs) tiles += (int64_t)s.size(2) * s.size(3) * ((s.size(0) + 63) / 64) * ((s.size(1) + 63) / 64);
  return {(int64_t)srcs.size(), tiles};
}

// subs (optional, one list per entry): (buffer, row taps, col taps) parity sub-filters of the flipped
// filter -- the (I, O, |rows|, |cols|) channels_last slice at those taps (ops/conv.py sub_filter)
Tensor wt_flip_build(const std::vector<Tensor>& srcs, const std::vector<Tensor>& dsts,
                     const std::vector<std::vector<std::tuple<Tensor, std::vector<int64_t>, std::vector<int64_t>>>>&
                         subs) {
  TORCH_CHECK(srcs.size() == dsts.size() && !srcs.empty(), "srcs/dsts mismatch");
  TORCH_CHECK(subs.empty() || subs.size() == srcs.size(), "subs: one list per entry");
  std::vector<mxr::WtFlipEntry> ents(srcs.size());
  std::memset(ents.data(), 0, ents.size() * sizeof(mxr::WtFlipEntry));
  int tiles = 0;
  for (size_t k = 0; k < srcs.size(); ++k) {
    const Tensor &s = srcs[k], &d = dsts[k];
    CHECK_DEV(s); CHECK_DEV(d);
    TORCH_CHECK(s.scalar_type() == at::kBFloat16 && d.scalar_type() == at::kBFloat16, "bf16 filters only");
    TORCH_CHECK(s.is_contiguous(at::MemoryFormat::ChannelsLast) && d.is_contiguous(at::MemoryFormat::ChannelsLast),
                "filters must be channels_last");
    const int O = (int)s.size(0), I = (int)s.size(1), KH = (int)s.size(2), KW = (int)s.size(3);
    TORCH_CHECK(d.size(0) == I && d.size(1) == O && d.size(2) == KH && d.size(3) == KW, "dst must be (I, O, KH, KW)");
    TORCH_CHECK(O % 8 == 0 && I % 8 == 0, "filter flip needs O % 8 == 0 and I % 8 == 0");
    ents[k].src = reinterpret_cast<const uint16_t*>(s.data_ptr());
    ents[k].dst = reinterpret_cast<uint16_t*>(d.data_ptr());
    ents[k].O = O; ents[k].I = I; ents[k].KH = KH; ents[k].KW = KW;
    ents[k].tile_begin = tiles;
    if (!subs.empty() && !subs[k].empty()) {
      TORCH_CHECK(KH <= 8 && KW <= 8, "sub-filters: KH, KW <= 8");
      // classes are numbered by first appearance along each axis
      std::vector<std::vector<int64_t>> rsets, csets;
      auto cls_of = [](std::vector<std::vector<int64_t>>& sets, const std::vector<int64_t>& taps) {
        for (size_t q = 0; q < sets.size(); ++q)
          if (sets[q] == taps) return (int)q;
        sets.push_back(taps);
        return (int)sets.size() - 1;
      };
      for (int q = 0; q < 8; ++q) ents[k].rcls[q] = ents[k].ccls[q] = ents[k].ridx[q] = ents[k].cidx[q] = 0;
      for (const auto& sb : subs[k]) {
        const Tensor& buf = std::get<0>(sb);
        const auto& rt = std::get<1>(sb);
        const auto& ct = std::get<2>(sb);
        const int rc = cls_of(rsets, rt), cc = cls_of(csets, ct);
        TORCH_CHECK(rc < 2 && cc < 2, "sub-filters: at most two parity classes per axis");
        CHECK_DEV(buf);
        TORCH_CHECK(buf.scalar_type() == at::kBFloat16 && buf.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                        buf.size(0) == I && buf.size(1) == O && buf.size(2) == (int64_t)rt.size() &&
                        buf.size(3) == (int64_t)ct.size(),
                    "sub-filter buffer must be a channels_last bf16 (I, O, |rows|, |cols|) tensor");
        ents[k].sub[2 * rc + cc] = reinterpret_cast<uint16_t*>(buf.data_ptr());
        ents[k].rcnt[rc] = (int8_t)rt.size();
        ents[k].ccnt[cc] = (int8_t)ct.size();
        for (size_t j = 0; j < rt.size(); ++j) {
          TORCH_CHECK(rt[j] >= 0 && rt[j] < KH, "sub-filter row tap out of range");
          ents[k].rcls[rt[j]] = (int8_t)rc; ents[k].ridx[rt[j]] = (int8_t)j;
        }
        for (size_t j = 0; j < ct.size(); ++j) {
          TORCH_CHECK(ct[j] >= 0 && ct[j] < KW, "sub-filter col tap out of range");
          ents[k].ccls[ct[j]] = (int8_t)cc; ents[k].cidx[ct[j]] = (int8_t)j;
        }
      }
      // every flipped tap must land in exactly one registered class pair, or the kernel would write
      // a tap into a sub-filter it does not belong to: require a full partition
      int covered = 0;
      for (const auto& r : rsets) covered += (int)r.size();
      TORCH_CHECK(covered == KH, "sub-filters must partition the row taps");
      covered = 0;
      for (const auto& c : csets) covered += (int)c.size();
      TORCH_CHECK(covered == KW, "sub-filters must partition the col taps");
      for (size_t rc = 0; rc < rsets.size(); ++rc)
        for (size_t cc = 0; cc < csets.size(); ++cc)
          TORCH_CHECK(ents[k].sub[2 * rc + cc] != nullptr, "sub-filters: every (row, col) class pair is needed");
    }
    tiles += KH * KW * ((O + 63) / 64) * ((I + 63) / 64);
  }
  Tensor host = at::empty({(int64_t)(ents.size() * sizeof(mxr::WtFlipEntry))}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(host.data_ptr(), ents.data(), ents.size() * sizeof(mxr::WtFlipEntry));
  return host.to(srcs[0].device());
}

void wt_flip_run(const Tensor& table, int64_t n_entries, int64_t total_tiles) {
  CHECK_DEV(table);
  TORCH_CHECK((int64_t)table.numel() == n_entries * (int64_t)sizeof(mxr::WtFlipEntry), "table size");
  DevGuard g(table.device());
  mxr::conv_wt_flip_multi(reinterpret_cast<const mxr::WtFlipEntry*>(table.data_ptr()), (int)n_entries,
                          (int)total_tiles, cur_stream());
}

Tensor conv_wgrad(const Tensor& dy, const Tensor& x, int64_t KH, int64_t KW, int64_t stride, int64_t pad,
                  int64_t splits, c10::optional<Tensor> out, int64_t variant, int64_t x2) {
  CHECK_DEV(dy); CHECK_DEV(x);
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16, "bf16 only");
  TORCH_CHECK(dy.is_contiguous(at::MemoryFormat::ChannelsLast) && x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "dy/x must be channels_last");
  // x2: dy / x are (2N, ...) pairs and the gradient is fp32
  TORCH_CHECK(!x2 || x.size(0) % npl(x2) == 0, "x2: (2N, ...) pairs");
  const int NB = (int)(x2 ? x.size(0) / npl(x2) : x.size(0)), Cin = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int Cout = (int)dy.size(1), Ho = (int)dy.size(2), Wo = (int)dy.size(3);
  TORCH_CHECK(dy.size(0) == x.size(0), "batch mismatch");
  TORCH_CHECK(Cin % 64 == 0 && Cout % 8 == 0, "conv_wgrad requires Cin % 64 == 0 and Cout % 8 == 0");
  TORCH_CHECK(Ho == (H + 2 * pad - KH) / stride + 1 && Wo == (W + 2 * pad - KW) / stride + 1, "geometry mismatch");
  DevGuard g(x.device());
  int sp = 1;
  mxr::conv_wgrad_plan(NB, Ho, Wo, Cin, Cout, (int)KH, (int)KW, &sp, (int)x2);
  static const int max_sp = [] {  // A/B knob: cap the pixel split (fewer reduce launches)
    const char* e = std::getenv("MXR_WGRAD_MAX_SPLITS");
    return e ? std::max(1, std::atoi(e)) : 1 << 30;
  }();
  sp = std::min(sp, max_sp);
  if (splits > 0) sp = (int)splits;
  Tensor dw;
  const bool acc = out.has_value() && out->defined();
  const auto gdt = x2 ? at::kFloat : at::kBFloat16;
  if (acc) {
    dw = *out;
    TORCH_CHECK(dw.scalar_type() == gdt && dw.size(0) == Cout && dw.size(1) == Cin && dw.size(2) == KH &&
                    dw.size(3) == KW && dw.is_contiguous(at::MemoryFormat::ChannelsLast),
                "out must be a channels_last (Cout, Cin, KH, KW) tensor, bf16 (fp32 for x2)");
  } else {
    dw = at::empty({Cout, Cin, KH, KW}, x.options().dtype(gdt).memory_format(at::MemoryFormat::ChannelsLast));
  }
  mxr::WgradX2 wx2;
  if (x2) {
    TORCH_CHECK(x.numel() < (int64_t)0x40000000 && dy.numel() < (int64_t)0x40000000, "x2: planes beyond 2 GB");
    wx2.x2 = 1;
    wx2.x3 = npl(x2) == 3 ? 1 : 0;
    wx2.pdy = (uint32_t)(dy.numel() / npl(x2) * 2);
    wx2.px = (uint32_t)(x.numel() / npl(x2) * 2);
    wx2.dwf = dw.data_ptr<float>();
  }
  Tensor slab = at::empty({(int64_t)sp * Cout * KH * KW * Cin}, x.options().dtype(at::kFloat));
  const int r = mxr::conv_wgrad(reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                                reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                x2 ? nullptr : reinterpret_cast<uint16_t*>(dw.data_ptr()), slab.data_ptr<float>(), NB, H,
                                W, Cin, Ho, Wo, Cout, (int)KH, (int)KW, (int)stride, (int)pad, sp, acc ? 1 : 0,
                                cur_stream(), (int)variant, wx2);
  TORCH_CHECK(r > 0, "conv_wgrad: unsupported shape");
  return dw;
}

// Weight gradient of (dy, x) applied at once as an SGD-momentum update of the parameter (w / mom
// fp32 flat views, `shadow` its bf16 copy or x2 / x3 planes `plane_stride` apart) -- the gradient
// is never stored (the VGG16 FC weights: ops/vgg_fused.py, core/params.py fused_sgd).  grad_bf16:
// round the gradient as the unfused bf16 path stores it.
void conv_wgrad_sgd(const Tensor& dy, const Tensor& x, int64_t KH, int64_t KW, int64_t stride, int64_t pad, int64_t x2,
                    Tensor w, Tensor mom, c10::optional<Tensor> shadow, int64_t planes, int64_t plane_stride,
                    const Tensor& lr, double momentum, double wd, double rescale, double clip, bool grad_bf16) {
  CHECK_DEV(dy); CHECK_DEV(x); CHECK_DEV(w); CHECK_DEV(mom); CHECK_DEV(lr);
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16, "bf16 only");
  TORCH_CHECK(dy.is_contiguous(at::MemoryFormat::ChannelsLast) && x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "dy/x must be channels_last");
  TORCH_CHECK(!x2 || x.size(0) % npl(x2) == 0, "x2: (2N, ...) pairs");
  const int NB = (int)(x2 ? x.size(0) / npl(x2) : x.size(0)), Cin = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int Cout = (int)dy.size(1), Ho = (int)dy.size(2), Wo = (int)dy.size(3);
  TORCH_CHECK(dy.size(0) == x.size(0), "batch mismatch");
  TORCH_CHECK(Ho == (H + 2 * pad - KH) / stride + 1 && Wo == (W + 2 * pad - KW) / stride + 1, "geometry mismatch");
  const int64_t n = (int64_t)Cout * KH * KW * Cin;
  TORCH_CHECK(w.scalar_type() == at::kFloat && mom.scalar_type() == at::kFloat && w.is_contiguous() &&
                  mom.is_contiguous() && w.numel() == n && mom.numel() == n,
              "w / mom: contiguous fp32 of Cout * KH * KW * Cin elements");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(mom.data_ptr()) % 16 == 0,
              "w / mom: 16-B aligned");
  TORCH_CHECK(lr.scalar_type() == at::kFloat && lr.numel() >= 1, "lr: fp32 device scalar");
  mxr::WgradSgd sg;
  sg.w = w.data_ptr<float>();
  sg.mom = mom.data_ptr<float>();
  sg.lr = lr.data_ptr<float>();
  sg.mu = (float)momentum;
  sg.wd = (float)wd;
  sg.rescale = (float)rescale;
  sg.clip = (float)clip;
  sg.gbf16 = grad_bf16 ? 1 : 0;
  if (shadow.has_value() && shadow->defined()) {
    TORCH_CHECK(shadow->scalar_type() == at::kBFloat16 && shadow->is_contiguous() && planes >= 1 && planes <= 3,
                "shadow: contiguous bf16, 1-3 planes");
    if (planes > 1) {
      TORCH_CHECK(plane_stride >= n && plane_stride % 4 == 0 && shadow->numel() >= (planes - 1) * plane_stride + n &&
                      reinterpret_cast<uintptr_t>(shadow->data_ptr()) % 8 == 0,
                  "shadow planes: 8-B aligned, plane_stride >= numel and a multiple of 4");
      sg.plane = plane_stride;
      sg.x3 = planes == 3 ? 1 : 0;
    } else {
      TORCH_CHECK(shadow->numel() >= n && reinterpret_cast<uintptr_t>(shadow->data_ptr()) % 16 == 0,
                  "shadow: 16-B aligned bf16 of numel elements");
    }
    sg.wb = reinterpret_cast<uint16_t*>(shadow->data_ptr());
  }
  mxr::WgradX2 wx2;
  if (x2) {
    TORCH_CHECK(x.numel() < (int64_t)0x40000000 && dy.numel() < (int64_t)0x40000000, "x2: planes beyond 2 GB");
    wx2.x2 = 1;
    wx2.x3 = npl(x2) == 3 ? 1 : 0;
    wx2.pdy = (uint32_t)(dy.numel() / npl(x2) * 2);
    wx2.px = (uint32_t)(x.numel() / npl(x2) * 2);
  }
  DevGuard g(x.device());
  const int r = mxr::conv_wgrad_sgd(reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                                    reinterpret_cast<const uint16_t*>(x.data_ptr()), NB, H, W, Cin, Ho, Wo, Cout,
                                    (int)KH, (int)KW, (int)stride, (int)pad, cur_stream(), wx2, sg);
  TORCH_CHECK(r > 0, "conv_wgrad_sgd: unsupported shape (Cin % 64, Cout % 8, 32-bit buffer offsets)");
  LAUNCH_CHECK("conv_wgrad_sgd");
}

}  // namespace

// ---- CPU twin of the proposal NMS (host C++, the CPU configuration and the test oracle's
// fast path): greedy over score-sorted boxes, suppress j when IoU(i, j) > thresh with +1-pixel
// areas, stop after max_keep kept (<= 0: no cap).  Returns kept positions (int64).
Tensor nms_cpu(const Tensor& boxes_in, int64_t n_valid, double thresh, int64_t max_keep, bool fp32) {
  TORCH_CHECK(!boxes_in.is_cuda(), "nms_cpu takes CPU boxes");
  TORCH_CHECK(boxes_in.dim() == 2 && boxes_in.size(1) == 4, "boxes must be (P, 4)");
  const Tensor boxes = boxes_in.to(fp32 ? at::kFloat : at::kDouble).contiguous();
  const int64_t n = std::min<int64_t>(n_valid, boxes.size(0));
  std::vector<int64_t> keep;
  if (fp32) mxr::host::nms_greedy(boxes.data_ptr<float>(), n, thresh, max_keep, keep);
  else mxr::host::nms_greedy(boxes.data_ptr<double>(), n, thresh, max_keep, keep);
  Tensor out = at::empty({(int64_t)keep.size()}, at::TensorOptions().dtype(at::kLong));
  std::copy(keep.begin(), keep.end(), out.data_ptr<int64_t>());
  return out;
}

// ---- CPU twin of the RoI max-pool forward (MXNet ROIPooling semantics, as roi_pool.hip):
// roundf RoI corners, float32 bin edges with floor / ceil, first maximum in row-major order
// (strict '>'), empty bins -> 0 with argmax -1.  feat (B, C, H, W) fp32, rois (R, 5).
std::vector<Tensor> roi_pool_fwd_cpu(const Tensor& feat_in, const Tensor& rois_in, int64_t PH, int64_t PW,
                                     double spatial_scale) {
  TORCH_CHECK(!feat_in.is_cuda() && feat_in.dim() == 4, "feat must be a CPU (B, C, H, W) tensor");
  const Tensor feat = feat_in.to(at::kFloat).contiguous();
  const Tensor rois = rois_in.to(at::kFloat).contiguous();
  TORCH_CHECK(rois.dim() == 2 && rois.size(1) == 5, "rois must be (R, 5)");
  const int64_t B = feat.size(0), C = feat.size(1), H = feat.size(2), W = feat.size(3), R = rois.size(0);
  Tensor out = at::zeros({R, C, PH, PW}, feat.options());
  Tensor arg = at::full({R, C, PH, PW}, -1, feat.options().dtype(at::kInt));
  const float* f = feat.data_ptr<float>();
  const float* ro = rois.data_ptr<float>();
  float* o = out.data_ptr<float>();
  int32_t* a = arg.data_ptr<int32_t>();
  const float sc = (float)spatial_scale;
  at::parallel_for(0, R, 1, [&](int64_t r0, int64_t r1) {
    mxr::host::roi_pool_range(f, B, C, H, W, ro, r0, r1, PH, PW, sc, o, a);
  });
  return {out, arg};
}

// ---- CPU twin of the RoI max-pool backward: scatter gout through the forward's argmax,
// parallel over channels (no atomics, per-channel sums in RoI order).  Returns fp32 (B, C, H, W).
Tensor roi_pool_bwd_cpu(const Tensor& gout_in, const Tensor& arg_in, const Tensor& rois_in, int64_t B, int64_t H,
                        int64_t W) {
  TORCH_CHECK(!gout_in.is_cuda() && gout_in.dim() == 4, "gout must be a CPU (R, C, PH, PW) tensor");
  const Tensor gout = gout_in.to(at::kFloat).contiguous();
  const Tensor arg = arg_in.to(at::kInt).contiguous();
  const Tensor rois = rois_in.to(at::kFloat).contiguous();
  TORCH_CHECK(arg.sizes() == gout.sizes(), "arg must match gout");
  const int64_t R = gout.size(0), C = gout.size(1), PHW = gout.size(2) * gout.size(3);
  TORCH_CHECK(rois.dim() == 2 && rois.size(0) == R && rois.size(1) == 5, "rois must be (R, 5)");
  Tensor gin = at::zeros({B, C, H, W}, gout.options());
  const float* g = gout.data_ptr<float>();
  const int32_t* a = arg.data_ptr<int32_t>();
  const float* ro = rois.data_ptr<float>();
  float* o = gin.data_ptr<float>();
  at::parallel_for(0, C, 1, [&](int64_t c0, int64_t c1) {
    mxr::host::roi_pool_bwd_channels(g, a, ro, R, B, C, H, W, PHW, c0, c1, o);
  });
  return gin;
}

// ---- CPU twin of the fused proposal decode (proposal.hip): per image, softmax fg + anchors +
// decode + clip + min-size; rows (h, w, a).  cls (B, 2A, H, W), dlt (B, 4A, H, W), im_info
// (B, 3), base (A, 4).  Returns boxes (B, N, 4) and keys (B, N) (-inf = filtered).
std::vector<Tensor> proposal_decode_cpu(const Tensor& cls_in, const Tensor& dlt_in, const Tensor& im_info_in,
                                        const Tensor& base_in, double stride, double min_size, bool crop,
                                        bool is_prob) {
  TORCH_CHECK(!cls_in.is_cuda() && cls_in.dim() == 4 && dlt_in.dim() == 4, "cls / dlt must be CPU NCHW tensors");
  const Tensor cls = cls_in.to(at::kFloat).contiguous();
  const Tensor dlt = dlt_in.to(at::kFloat).contiguous();
  const Tensor im_info = im_info_in.to(at::kFloat).contiguous();
  const Tensor base = base_in.to(at::kFloat).contiguous();
  const int64_t B = cls.size(0), A = cls.size(1) / 2, H = cls.size(2), W = cls.size(3), N = H * W * A;
  TORCH_CHECK(cls.size(1) == 2 * A && dlt.size(0) == B && dlt.size(1) == 4 * A && dlt.size(2) == H &&
                  dlt.size(3) == W, "dlt must be (B, 4A, H, W) with cls (B, 2A, H, W)");
  TORCH_CHECK(im_info.dim() == 2 && im_info.size(0) == B && im_info.size(1) >= 3, "im_info must be (B, 3)");
  TORCH_CHECK(base.numel() == 4 * A, "base must hold A anchors");
  Tensor boxes = at::empty({B, N, 4}, cls.options());
  Tensor keys = at::empty({B, N}, cls.options());
  const float* ii = im_info.data_ptr<float>();
  const int64_t ist = im_info.size(1);
  at::parallel_for(0, B, 1, [&](int64_t b0, int64_t b1) {
    for (int64_t b = b0; b < b1; ++b)
      mxr::host::proposal_decode_image(cls.data_ptr<float>() + b * 2 * A * H * W,
                                       dlt.data_ptr<float>() + b * 4 * A * H * W, A, H, W, ii[b * ist],
                                       ii[b * ist + 1], ii[b * ist + 2], base.data_ptr<float>(), (float)stride,
                                       (float)min_size, crop, is_prob, boxes.data_ptr<float>() + b * N * 4,
                                       keys.data_ptr<float>() + b * N);
  });
  return {boxes, keys};
}

// ---- CPU twin of the RPN anchor-target assignment (assign.hip, before subsampling): labels
// (B, N) int32 in {-1, 0, 1} and targets (B, N, 4), rows (h, w, a).  gt (B, G, >=4) padded
// past n_gt[b]; im_info (B, >=2).  Pass 1 per image, pass 2 parallel over anchor rows.
std::vector<Tensor> anchor_assign_cpu(const Tensor& base_in, int64_t H, int64_t W, double stride,
                                      const Tensor& im_info_in, int64_t border, const Tensor& gt_in,
                                      const Tensor& n_gt_in, double neg, double pos, bool clobber) {
  TORCH_CHECK(!gt_in.is_cuda() && gt_in.dim() == 3 && gt_in.size(2) >= 4, "gt must be a CPU (B, G, >=4) tensor");
  const Tensor base = base_in.to(at::kFloat).contiguous();
  const Tensor im_info = im_info_in.to(at::kFloat).contiguous();
  const Tensor gt = gt_in.to(at::kFloat).contiguous();
  const Tensor n_gt = n_gt_in.to(at::kLong).contiguous();
  const int64_t A = base.numel() / 4, B = gt.size(0), G = gt.size(1), gs = gt.size(2), N = H * W * A;
  TORCH_CHECK(base.numel() == 4 * A && im_info.size(0) == B && n_gt.numel() == B, "base / im_info / n_gt shapes");
  Tensor labels = at::empty({B, N}, gt.options().dtype(at::kInt));
  Tensor targets = at::empty({B, N, 4}, gt.options());
  const float* bs = base.data_ptr<float>();
  const float* ii = im_info.data_ptr<float>();
  const int64_t ist = im_info.size(1);
  std::vector<float> gmax(std::max<int64_t>(G, 1));
  for (int64_t b = 0; b < B; ++b) {
    const int64_t ng = std::min<int64_t>(std::max<int64_t>(n_gt.data_ptr<int64_t>()[b], 0), G);
    const float im_h = ii[b * ist], im_w = ii[b * ist + 1];
    const float* g = gt.data_ptr<float>() + b * G * gs;
    mxr::host::anchor_gt_max(bs, A, H, W, (float)stride, im_h, im_w, (int)border, g, gs, ng, gmax.data());
    int32_t* lb = labels.data_ptr<int32_t>() + b * N;
    float* tg = targets.data_ptr<float>() + b * N * 4;
    at::parallel_for(0, N, 2048, [&](int64_t n0, int64_t n1) {
      mxr::host::anchor_assign_range(bs, A, W, (float)stride, im_h, im_w, (int)border, g, gs, ng, gmax.data(),
                                     (float)neg, (float)pos, clobber, n0, n1, lb, tg);
    });
  }
  return {labels, targets};
}

// ---- CPU twin of iou_max (assign.hip): boxes (B, N, bs) rows [off, off+4), gt (B, G, >=4),
// n_gt (B,).  Returns max (B, N), argmax (B, N) int32 [, per-gt max over rows of max(IoU, 0)].
std::vector<Tensor> iou_max_cpu(const Tensor& boxes_in, int64_t off, const Tensor& gt_in, const Tensor& n_gt_in,
                                bool want_gt_max) {
  TORCH_CHECK(!boxes_in.is_cuda() && boxes_in.dim() == 3 && boxes_in.size(2) >= off + 4, "boxes must be CPU (B, N, >=off+4)");
  TORCH_CHECK(gt_in.dim() == 3 && gt_in.size(2) >= 4 && gt_in.size(0) == boxes_in.size(0), "gt must be (B, G, >=4)");
  const Tensor boxes = boxes_in.to(at::kFloat).contiguous();
  const Tensor gt = gt_in.to(at::kFloat).contiguous();
  const Tensor n_gt = n_gt_in.to(at::kLong).contiguous();
  const int64_t B = boxes.size(0), N = boxes.size(1), bs = boxes.size(2), G = gt.size(1), gs = gt.size(2);
  TORCH_CHECK(n_gt.numel() == B, "n_gt must be (B,)");
  Tensor mx = at::empty({B, N}, boxes.options());
  Tensor am = at::empty({B, N}, boxes.options().dtype(at::kInt));
  Tensor gm = at::zeros({B, G}, boxes.options());
  for (int64_t b = 0; b < B; ++b) {
    const int64_t ng = std::min<int64_t>(std::max<int64_t>(n_gt.data_ptr<int64_t>()[b], 0), G);
    const float* bx = boxes.data_ptr<float>() + b * N * bs;
    const float* g = gt.data_ptr<float>() + b * G * gs;
    at::parallel_for(0, N, 1024, [&](int64_t n0, int64_t n1) {
      mxr::host::iou_max_rows(bx, bs, off, n0, n1, g, gs, ng, mx.data_ptr<float>() + b * N,
                              am.data_ptr<int32_t>() + b * N);
    });
    if (want_gt_max) {
      float* gmb = gm.data_ptr<float>() + b * G;
      for (int64_t n = 0; n < N; ++n)
        for (int64_t j = 0; j < ng; ++j) gmb[j] = std::max(gmb[j], mxr::host::iou1(bx + n * bs + off, g + j * gs));
    }
  }
  if (want_gt_max) return {mx, am, gm};
  return {mx, am};
}

// ---- CPU twins of the fused losses (losses.hip): value and gradient in one pass.
std::vector<Tensor> rpn_softmax_ce_cpu(const Tensor& logits_in, const Tensor& label_in, double grad_scale) {
  TORCH_CHECK(!logits_in.is_cuda() && logits_in.dim() == 4 && logits_in.size(1) % 2 == 0, "logits must be CPU (B, 2A, H, W)");
  const Tensor logits = logits_in.to(at::kFloat).contiguous();
  const Tensor label = label_in.to(at::kInt).contiguous();
  const int64_t B = logits.size(0), AHW = logits.size(1) / 2 * logits.size(2) * logits.size(3);
  TORCH_CHECK(label.numel() == B * AHW, "label must hold B * A*H*W entries");
  Tensor grad = at::empty_like(logits);
  const float loss = mxr::host::rpn_softmax_ce(logits.data_ptr<float>(), label.data_ptr<int32_t>(), B, AHW,
                                               (float)grad_scale, grad.data_ptr<float>());
  return {grad, at::full({1}, loss, logits.options())};
}

std::vector<Tensor> smooth_l1_cpu(const Tensor& pred_in, const Tensor& tgt_in, const Tensor& iw_in,
                                  const Tensor& ow_in, double sigma, double grad_scale) {
  TORCH_CHECK(!pred_in.is_cuda(), "smooth_l1_cpu takes CPU tensors");
  const Tensor pred = pred_in.to(at::kFloat).contiguous();
  const Tensor tgt = tgt_in.to(at::kFloat).contiguous();
  const Tensor iw = iw_in.to(at::kFloat).contiguous();
  const Tensor ow = ow_in.to(at::kFloat).contiguous();
  TORCH_CHECK(tgt.numel() == pred.numel() && iw.numel() == pred.numel() && ow.numel() == pred.numel(),
              "pred / target / weights must have the same size");
  Tensor grad = at::empty_like(pred);
  const float loss = mxr::host::smooth_l1(pred.data_ptr<float>(), tgt.data_ptr<float>(), iw.data_ptr<float>(),
                                          ow.data_ptr<float>(), pred.numel(), (float)sigma, (float)grad_scale,
                                          grad.data_ptr<float>());
  return {grad, at::full({1}, loss, pred.options())};
}

// ---- CPU twin of the fused SGD-momentum update (sgd.hip), in place on fp32 w / mom.
void sgd_momentum_cpu(Tensor w, Tensor mom, const Tensor& grad_in, double lr, double momentum, double wd,
                      double rescale, double clip) {
  TORCH_CHECK(!w.is_cuda() && w.scalar_type() == at::kFloat && mom.scalar_type() == at::kFloat &&
                  w.is_contiguous() && mom.is_contiguous() && w.numel() == mom.numel(),
              "w / mom must be contiguous fp32 CPU tensors of one size");
  const Tensor grad = grad_in.to(at::kFloat).contiguous();
  TORCH_CHECK(grad.numel() == w.numel(), "grad size");
  float* wp = w.data_ptr<float>();
  float* mp = mom.data_ptr<float>();
  const float* gp = grad.data_ptr<float>();
  at::parallel_for(0, w.numel(), 1 << 16, [&](int64_t n0, int64_t n1) {
    mxr::host::sgd_momentum_range(wp, mp, gp, n0, n1, (float)lr, (float)momentum, (float)wd, (float)rescale,
                                  (float)clip);
  });
}

// ---- CPU twin of the head softmax-CE (row_softmax_ce in losses.hip).  Returns grad, prob,
// loss (1,) = sum over valid rows of -log p / norm; per-chunk partial sums are added in chunk
// order, so the value does not depend on the thread count's scheduling.
std::vector<Tensor> row_softmax_ce_cpu(const Tensor& logits_in, const Tensor& label_in, double norm,
                                       double grad_scale) {
  TORCH_CHECK(!logits_in.is_cuda() && logits_in.dim() == 2, "logits must be a CPU (R, C) tensor");
  const Tensor logits = logits_in.to(at::kFloat).contiguous();
  const Tensor label = label_in.to(at::kInt).contiguous();
  const int64_t R = logits.size(0), C = logits.size(1);
  TORCH_CHECK(label.numel() == R && C > 0, "label must be (R,)");
  Tensor prob = at::empty_like(logits), grad = at::empty_like(logits);
  const int64_t grain = 64, chunks = (R + grain - 1) / grain;
  std::vector<double> part(std::max<int64_t>(chunks, 1), 0.0);
  at::parallel_for(0, chunks, 1, [&](int64_t c0, int64_t c1) {
    for (int64_t k = c0; k < c1; ++k)
      part[k] = mxr::host::row_softmax_ce_range(logits.data_ptr<float>(), label.data_ptr<int32_t>(), C, k * grain,
                                                std::min(R, (k + 1) * grain), (float)norm, (float)grad_scale,
                                                prob.data_ptr<float>(), grad.data_ptr<float>());
  });
  double loss = 0.0;
  for (double v : part) loss += v;
  return {grad, prob, at::full({1}, (float)(loss / norm), logits.options())};
}

// ---- CPU twin of the frozen BN+ReLU forward (bn_act.hip): keeps x's memory format
// (NCHW or channels_last), returns fp32.
Tensor bn_relu_fwd_cpu(const Tensor& x_in, const Tensor& gamma, const Tensor& beta, const Tensor& mean,
                       const Tensor& var, double eps, bool fix_gamma, bool relu) {
  TORCH_CHECK(!x_in.is_cuda() && x_in.dim() == 4, "x must be a CPU (N, C, H, W) tensor");
  const bool cl = !x_in.is_contiguous() && x_in.is_contiguous(at::MemoryFormat::ChannelsLast);
  const auto fmt = cl ? at::MemoryFormat::ChannelsLast : at::MemoryFormat::Contiguous;
  const Tensor x = x_in.to(at::kFloat).contiguous(fmt);
  const int64_t C = x.size(1), inner = cl ? 1 : x.size(2) * x.size(3);
  TORCH_CHECK(gamma.numel() == C && beta.numel() == C && mean.numel() == C && var.numel() == C, "per-channel params");
  const Tensor g = fix_gamma ? at::ones({C}, x.options()) : gamma.to(at::kFloat).contiguous();
  const Tensor scale = (g * at::rsqrt(var.to(at::kFloat) + eps)).contiguous();
  const Tensor shift = (beta.to(at::kFloat) - mean.to(at::kFloat) * scale).contiguous();
  Tensor y = at::empty_like(x);
  const float* xp = x.data_ptr<float>();
  float* yp = y.data_ptr<float>();
  at::parallel_for(0, x.numel(), 1 << 15, [&](int64_t n0, int64_t n1) {
    mxr::host::bn_frozen_range(xp, yp, n0, n1, C, inner, scale.data_ptr<float>(), shift.data_ptr<float>(), relu);
  });
  return y;
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "mx_rcnn_amd gfx950 kernels";
  m.def("proposal_decode", &proposal_decode);
  m.def("nms_proposals", &nms_proposals, py::arg("boxes"), py::arg("scores"), py::arg("n_valid"), py::arg("thresh"),
        py::arg("post"), py::arg("rand_u"), py::arg("mask") = py::none(), py::arg("fault") = py::none());
  m.def("nms_mask_build", &nms_mask_build);
  m.def("conv_wgrad_sgd", &conv_wgrad_sgd, py::arg("dy"), py::arg("x"), py::arg("KH"), py::arg("KW"), py::arg("stride"),
        py::arg("pad"), py::arg("x2"), py::arg("w"), py::arg("mom"), py::arg("shadow"), py::arg("planes"),
        py::arg("plane_stride"), py::arg("lr"), py::arg("momentum"), py::arg("wd"), py::arg("rescale"),
        py::arg("clip"), py::arg("grad_bf16"));
  m.def("nms_check", &nms_check);
  m.def("nms_cpu", &nms_cpu, py::arg("boxes"), py::arg("n_valid"), py::arg("thresh"), py::arg("max_keep"),
        py::arg("fp32") = false);
  m.def("roi_pool_fwd_cpu", &roi_pool_fwd_cpu);
  m.def("roi_pool_bwd_cpu", &roi_pool_bwd_cpu);
  m.def("proposal_decode_cpu", &proposal_decode_cpu);
  m.def("anchor_assign_cpu", &anchor_assign_cpu);
  m.def("iou_max_cpu", &iou_max_cpu);
  m.def("rpn_softmax_ce_cpu", &rpn_softmax_ce_cpu);
  m.def("smooth_l1_cpu", &smooth_l1_cpu);
  m.def("sgd_momentum_cpu", &sgd_momentum_cpu);
  m.def("row_softmax_ce_cpu", &row_softmax_ce_cpu);
  m.def("bn_relu_fwd_cpu", &bn_relu_fwd_cpu);
  m.def("iou_max", &iou_max);
  m.def("anchor_sample", &anchor_sample);
  m.def("anchor_target_fused", &anchor_target_fused);
  m.def("proposal_sample", &proposal_sample);
  m.def("anchor_target_assign", &anchor_target_assign);
  m.def("roi_pool_fwd", &roi_pool_fwd, py::arg("feat"), py::arg("rois"), py::arg("PH"), py::arg("PW"),
        py::arg("scale"), py::arg("x2") = 0, py::arg("need_argmax") = true, py::arg("post_bn") = py::none());
  m.def("roi_pool_bwd", &roi_pool_bwd, py::arg("grad_out"), py::arg("argmax"), py::arg("rois"), py::arg("B"),
        py::arg("H"), py::arg("W"), py::arg("grad_add") = py::none(), py::arg("x2") = 0);
  m.def("rpn_softmax_ce", &rpn_softmax_ce, py::arg("logits"), py::arg("label"), py::arg("norm"), py::arg("grad_scale"),
        py::arg("want_prob"), py::arg("meta") = py::none());
  m.def("row_softmax_ce", &row_softmax_ce);
  m.def("smooth_l1", &smooth_l1, py::arg("pred"), py::arg("tgt"), py::arg("in_w"), py::arg("out_w"), py::arg("sigma"),
        py::arg("grad_scale"), py::arg("slot") = 2);
  m.def("scale_by_scalar_", &scale_by_scalar_);
  m.def("loss_combine", &loss_combine, py::arg("terms"), py::arg("weights"), py::arg("nonfinite") = py::none());
  m.def("sgd_momentum", &sgd_momentum, py::arg("w"), py::arg("mom"), py::arg("grad"), py::arg("lr"),
        py::arg("momentum"), py::arg("wd"), py::arg("rescale"), py::arg("clip"), py::arg("w_bf16") = py::none(),
        py::arg("planes") = 1, py::arg("zero") = py::none(), py::arg("plane_stride") = 0);
  m.def("bn_relu_fwd", &bn_relu_fwd, py::arg("x"), py::arg("gamma"), py::arg("beta"), py::arg("mean"), py::arg("var"),
        py::arg("eps"), py::arg("fix_gamma"), py::arg("relu"), py::arg("x2") = 0);
  m.def("bn_relu_bwd", &bn_relu_bwd, py::arg("x"), py::arg("dy"), py::arg("gamma"), py::arg("beta"),
        py::arg("mean"), py::arg("var"), py::arg("eps"), py::arg("fix_gamma"), py::arg("relu"), py::arg("need_dx"),
        py::arg("need_params"), py::arg("dgamma_out") = py::none(), py::arg("dbeta_out") = py::none(),
        py::arg("dres") = py::none(), py::arg("x2") = 0);
  m.def("philox_uniform_", &philox_uniform_, py::arg("out"),
        "fill a contiguous fp32 GPU tensor with U[0,1) from the default generator's graph-safe Philox state");
  m.def("counter_add_", &counter_add_, py::arg("counter"), py::arg("v") = 1, "counter[0] += v on the device");
  m.def("image_prep", &image_prep, py::arg("img"), py::arg("im_info"), py::arg("means"), py::arg("out_bf16"),
        "uint8 BGR (B,H,W,3) -> channels_last (B,3,H,W) RGB minus means, 0 outside im_info's (h, w)");
  m.def("conv_tune_table", &conv_tune_table, "per-shape conv autotune choices: [(key, tile, splits)]");
  m.def("conv_tune_set", &conv_tune_set, py::arg("entries"), py::arg("replace") = false,
        "set autotune choices [(key, tile, splits)] (replace: drop the current table first); returns the table size");
  m.def("conv_igemm_fwd", &conv_igemm_fwd, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("stride"),
        py::arg("pad"), py::arg("relu"), py::arg("tile") = 0, py::arg("splits") = 0, py::arg("residual") = py::none(),
        py::arg("bn") = py::none(), py::arg("bn_eps") = 2e-5, py::arg("bn_fix_gamma") = false,
        py::arg("act_relu") = true, py::arg("bnb_x") = py::none(), py::arg("dadd") = py::none(),
        py::arg("dgamma_out") = py::none(), py::arg("dbeta_out") = py::none(), py::arg("drop_p") = 0.0,
        py::arg("drop_seed") = 0, py::arg("drop_step") = py::none(), py::arg("pad_w") = -1,
        py::arg("out") = py::none(), py::arg("out_map") = py::none(), py::arg("stat_shift") = py::none(),
        py::arg("bnb_part") = py::none(), py::arg("bnb_row0") = 0, py::arg("x2") = 0, py::arg("w_plane") = 0,
        py::arg("out_f32") = false, py::arg("bt") = false, py::arg("rmask") = py::none(), py::arg("rmask_scale") = 1.0);
  m.def("relu_mask_bwd", &relu_mask_bwd, py::arg("dy"), py::arg("y"), py::arg("scale") = 1.0, py::arg("x2") = 0);
  m.def("proposal_topk", &proposal_topk, py::arg("keys"), py::arg("boxes"), py::arg("P"));
  m.def("conv_dgrad_wgrad", &conv_dgrad_wgrad, py::arg("x"), py::arg("w"), py::arg("pad"), py::arg("residual"),
        py::arg("bn"), py::arg("bn_eps"), py::arg("bn_fix_gamma"), py::arg("bnb_x"), py::arg("dadd"), py::arg("dgamma"),
        py::arg("dbeta"), py::arg("wg_dy"), py::arg("wg_x"), py::arg("KH"), py::arg("KW"), py::arg("wg_stride"),
        py::arg("wg_pad"), py::arg("wg_out"), py::arg("defer") = false, py::arg("prev_slab") = py::none(),
        py::arg("prev_out") = py::none(), py::arg("bnb_part") = py::none(), py::arg("x2") = 0,
        py::arg("w_plane") = 0, py::arg("bt") = false, py::arg("rmask") = py::none(), py::arg("rmask_scale") = 1.0);
  m.def("wgrad_reduce_run", &wgrad_reduce_run, py::arg("slab"), py::arg("out"));
  m.def("head_bwd", &head_bwd, py::arg("x"), py::arg("dys"), py::arg("ws"), py::arg("dws"), py::arg("dw_acc"),
        py::arg("dbs"), py::arg("db_acc"), py::arg("need_dx"), py::arg("relu_mask"), py::arg("x2") = 0,
        py::arg("w_planes") = std::vector<int64_t>(), py::arg("mask_scale") = 1.0);
  m.def("cu_spin", &cu_spin, py::arg("nwg"), py::arg("us"));
  m.def("cu_copy", &cu_copy, py::arg("src"), py::arg("dst"), py::arg("nwg"));
  m.def("chan_sum", &chan_sum, py::arg("x"), py::arg("out"), py::arg("accumulate"), py::arg("x2") = 0);
  m.def("det_postprocess", &det_postprocess, py::arg("rois"), py::arg("scores"), py::arg("deltas"),
        py::arg("im_info"), py::arg("thresh"), py::arg("nms_thresh"), py::arg("max_per"), py::arg("cap"));
  m.def("nest_keep", &nest_keep, py::arg("dets"), py::arg("thresh"));
  m.def("maxpool_fwd", &maxpool_fwd, py::arg("x"), py::arg("k"), py::arg("s"), py::arg("p"), py::arg("x2") = 0,
        py::arg("need_arg") = true, py::arg("post_bn") = py::none());
  m.def("bn_affine", &bn_affine, py::arg("gamma"), py::arg("beta"), py::arg("mean"), py::arg("var"), py::arg("eps"),
        py::arg("fix_gamma"));
  m.def("maxpool_bwd", &maxpool_bwd, py::arg("dy"), py::arg("arg"), py::arg("H"), py::arg("W"), py::arg("k"),
        py::arg("s"), py::arg("p"), py::arg("x2") = 0);
  m.def("avgpool_fwd", &avgpool_fwd, py::arg("x"), py::arg("x2") = 0);
  m.def("avgpool_bwd", &avgpool_bwd, py::arg("dy"), py::arg("H"), py::arg("W"), py::arg("x2") = 0);
  m.def("proposal_gather", &proposal_gather);
  m.def("stem_conv", &stem_conv, py::arg("x"), py::arg("w"), py::arg("in_bn"), py::arg("in_eps"), py::arg("in_fixg"),
        py::arg("out_bn"), py::arg("out_eps"), py::arg("out_fixg"), py::arg("bias"), py::arg("KH"), py::arg("KW"),
        py::arg("stride"), py::arg("pad"), py::arg("relu"));
  m.def("philox_uniform", &philox_uniform_cpu, py::arg("seed"), py::arg("step"), py::arg("n"),
        "host twin of the fused-dropout generator: uniforms of elements 0..n-1 (CPU float tensor)");
  m.def("bn_train_fwd", &bn_train_fwd, py::arg("x"), py::arg("gamma"), py::arg("beta"), py::arg("rmean"),
        py::arg("rvar"), py::arg("momentum"), py::arg("eps"), py::arg("fix_gamma"), py::arg("relu"),
        py::arg("x2") = 0);
  m.def("bn_train_apply", &bn_train_apply, py::arg("x"), py::arg("part"), py::arg("gamma"), py::arg("beta"),
        py::arg("rmean"), py::arg("rvar"), py::arg("momentum"), py::arg("eps"), py::arg("fix_gamma"), py::arg("relu"),
        py::arg("x2") = 0);
  m.def("bnb_part_fold", &bnb_part_fold, py::arg("part"), py::arg("nparts"), py::arg("C"),
        py::arg("dgamma") = py::none(), py::arg("dbeta") = py::none());
  m.def("bnb_part_fold_multi", &bnb_part_fold_multi, py::arg("entries"));
  m.def("bn_train_dx_apply", &bn_train_dx_apply, py::arg("o"), py::arg("x"), py::arg("save"), py::arg("gamma_eff"),
        py::arg("part"), py::arg("nparts"), py::arg("dres") = py::none(), py::arg("dgamma") = py::none(),
        py::arg("dbeta") = py::none(), py::arg("x2") = 0);
  m.def("bn_train_bwd", &bn_train_bwd, py::arg("x"), py::arg("dy"), py::arg("gamma"), py::arg("beta"),
        py::arg("save_mean"), py::arg("save_invstd"), py::arg("fix_gamma"), py::arg("relu"), py::arg("need_dx"),
        py::arg("dgamma_out") = py::none(), py::arg("dbeta_out") = py::none(), py::arg("x2") = 0);
  m.def("wt_flip_table_info", &wt_flip_table_info);
  m.def("wt_flip_build", &wt_flip_build, py::arg("srcs"), py::arg("dsts"),
        py::arg("subs") = std::vector<std::vector<std::tuple<Tensor, std::vector<int64_t>, std::vector<int64_t>>>>());
  m.def("wt_flip_run", &wt_flip_run);
  m.def("conv_wgrad", &conv_wgrad, py::arg("dy"), py::arg("x"), py::arg("kh"), py::arg("kw"), py::arg("stride"),
        py::arg("pad"), py::arg("splits") = 0, py::arg("out") = py::none(), py::arg("variant") = 0,
        py::arg("x2") = 0);
  m.attr("arch") = "gfx950";
}
