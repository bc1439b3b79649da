// Launcher declarations for the hand-written gfx950 kernels.
// Every launcher is asynchronous on the given HIP stream, never allocates,
// never synchronises (so a caller may capture it into a hipGraph).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace mxr {

// ---- proposal (proposal.hip) ----------------------------------------------
// Fused RPN fg-softmax + anchor enumeration + delta decode + clip + min-size.
// cls  : logits, element (b, c, h, w) at cls[b*cs0 + c*cs1 + h*cs2 + w*cs3], c in [0, 2A)
// dlt  : deltas, element (b, c, h, w) at dlt[b*ds0 + ...], c in [0, 4A)
// is_prob: cls already holds softmax probabilities (test graph) instead of logits.
// Writes boxes (B, N, 4) and keys (B, N) where N = Hc*Wc*A, order (h*Wc+w)*A+a.
// Filtered boxes get key = -inf.  Hc/Wc are per-image crops (device arrays, may be null).
// skeys / order (B, N) from a descending sort, boxes (B, N, 4) -> out_keys (B, P), out_boxes (B, P, 4),
// n_valid (B) = number of finite keys among the first P
void proposal_gather(const float* skeys, const int64_t* order, const float* boxes, int B, int64_t N, int P,
                     float* out_keys, float* out_boxes, int32_t* n_valid, hipStream_t st);
void proposal_decode(const void* cls, int cls_bf16, int64_t cs0, int64_t cs1, int64_t cs2, int64_t cs3,
                     const void* dlt, int dlt_bf16, int64_t ds0, int64_t ds1, int64_t ds2, int64_t ds3,
                     int is_prob, const float* im_info, const float* base_anchors, int A,
                     int B, int H, int W, float feat_stride, float min_size,
                     int crop_to_im, float* boxes, float* keys, hipStream_t st);

// ---- NMS (nms.hip) ----------------------------------------------------------
// boxes (B, P, 4) sorted by descending score, n_valid (B) int32 on device.
// mask workspace: nms_mask_words(B, P) uint64 (transposed, column blocks paired: [B][nb][ceil(nb/2)*128], nb = ceil(P/64)),
// followed by the multi-workgroup reducer's block records [B][nb][2] and exit counters [B].
int64_t nms_mask_words(int B, int P);
size_t nms_reduce_lds(int P, int post);
// the reducer keeps its keep list in LDS when this holds, else in a (B, post) int32 global workspace
bool nms_keep_in_lds(int P, int post);
void nms_mask(const float* boxes, const int32_t* n_valid, int B, int P, float thresh,
              uint64_t* mask, hipStream_t st);
// Greedy reduction + output assembly: keep up to `post` boxes per image; slots
// beyond the kept count are filled with keep[floor(u * n_keep)] (rand u in [0,1)).
// rois (B, post, 5) = [b, x1, y1, x2, y2], out_scores (B, post), n_keep (B).  An image whose
// multi-workgroup chain gives up a poll is redone by the serial reducer launched behind it (same
// result), which adds 1 to *gave_up (if given) per image redone.
void nms_reduce(const float* boxes, const float* scores, const int32_t* n_valid, const uint64_t* mask,
                int B, int P, int post, const float* rand_u, float* rois, float* out_scores,
                int64_t* keep_idx, int32_t* n_keep, int32_t* keep_ws, hipStream_t st, int32_t* gave_up = nullptr);
// device greedy-NMS oracle (MXR_NMS_CHECK): result (B, 2) int32 = {first differing keep position or -1, kept count}
void nms_check(const float* boxes, const int32_t* n_valid, int B, int P, float thresh, int post,
               const int64_t* keep_idx, const int32_t* n_keep, int32_t* result, hipStream_t st);

// ---- IoU / target assignment (assign.hip) ----------------------------------
// boxes (B, N, bs) with box at [off..off+4), gt (B, G, 5) padded with -1 rows, n_gt (B).
// max_ov (B, N) fp32, argmax (B, N) int32 (0 when no gt), gt_max (B, G) fp32 (may be null,
// must be zeroed by caller; filled by atomicMax over rows where row_mask != 0 or row_mask null).
void iou_max(const float* boxes, int bs, int off, int B, int N, const float* gt, const int32_t* n_gt, int G,
             const uint8_t* row_mask, float* max_ov, int32_t* argmax, float* gt_max, hipStream_t st);

// Anchor target labels (pre-sampling) + regression targets for all anchors of a (H, W, A) grid.
// label (B, N) int32 in {-1, 0, 1}, N = H*W*A in (h, w, a) order; targets (B, N, 4).
void anchor_target_assign(const float* base_anchors, int A, int H, int W, float feat_stride,
                          const float* im_info, int allowed_border,
                          const float* gt, const int32_t* n_gt, int G, int B,
                          float neg_thresh, float pos_thresh, int clobber_positives,
                          float* max_ov, int32_t* argmax, float* gt_max,
                          int32_t* label, float* targets, hipStream_t st, const float* keys = nullptr,
                          int32_t* hist = nullptr, int32_t* zero_ws = nullptr, int64_t zero_n = 0);
// (zero_ws: [0, zero_n) zeroed by the first kernel -- the self-cleaning sampling workspace, bindings.cpp)

// ---- fused target sampling (sample.hip) ------------------------------------
// RPN: label_pre (B, N=H*W*A) in (h, w, a) order from anchor_target_assign, targets (B, N, 4), keys
// (B, N) uniform [0,1).  Workspaces: kept (B, ceil(N/32)) uint32, meta (B, 4) int32.  Outputs in the
// reference layout: label (B, A*H*W), bbox_target / inside / outside (B, 4A, H, W).
void anchor_sample(const int32_t* label_pre, const float* targets, const float* keys, int B, int A, int H, int W,
                   int num_fg, int batch, const float* inside_w, float pos_weight, uint32_t* kept_ws,
                   int32_t* meta_ws, int32_t* label, float* bbox_target, float* inside, float* outside,
                   hipStream_t st);
// Multi-workgroup form of anchor_sample (the same selection: the k smallest (key, index) of each
// pool): `hist` (B, 2, kSampleBins) key histograms of the fg / bg pools from anchor_target_assign's
// second pass (keys + hist given); `ws`: anchor_mark_ws_ints(B, N) zeroed int32 (kept bitmap,
// boundary lists, counters).  Launches the mark kernel (its last workgroup per image ranks the
// boundary bin) and the output kernel.
constexpr int kSampleBins = 4096;
__host__ __device__ inline int sample_bin(float key) {
  const int b = (int)(key * (float)kSampleBins);
  return b < 0 ? 0 : (b >= kSampleBins ? kSampleBins - 1 : b);
}
int64_t anchor_mark_ws_ints(int B, int64_t N);
void anchor_sample_hist(const int32_t* label_pre, const float* targets, const float* keys, const int32_t* hist,
                        int B, int A, int H, int W, int num_fg, int batch, const float* inside_w, float pos_weight,
                        int32_t* ws, int32_t* meta, int32_t* label, float* bbox_target, float* inside, float* outside,
                        hipStream_t st, int32_t* clean_ws = nullptr, int64_t clean_n = 0);
// (clean_ws: [0, clean_n) -- the gt-max / histogram words the earlier kernels consumed -- zeroed by
// the output kernel, so a persistent workspace is left clean for the next call)
// R-CNN: rois (B, P, 5), gt (B, G, 5), n_gt (B), max_ov / argmax (B, P) vs gt, rnd (B, 2(P+G)+R).
// Returns -1 when the shape exceeds the kernel's LDS plan.
size_t proposal_sample_lds(int P, int G, int R, int F);
int proposal_sample(const float* rois, const float* gt, const int32_t* n_gt, const float* max_ov, const int32_t* argmax,
                    const float* rnd, int B, int P, int G, int R, int F, int C, float fg_thresh, float bg_hi,
                    float bg_lo, int is_train, int normalize, const float* means, const float* stds,
                    const float* inside_w, float* out_rois, int32_t* out_label, float* bbox_target, float* inside,
                    float* outside, hipStream_t st);

// Frozen BatchNorm + ReLU applied to a pooling output in the pooling kernel (inference: the next
// pre-activation unit's bn1, whose input nothing else reads): relu(v * scale[c] + shift[c]) with the
// per-channel coefficients from bn_affine (bn_act.hip, the same arithmetic as bn_relu_fwd).
// scale == nullptr: off.
struct PostBn {
  const float* scale = nullptr;
  const float* shift = nullptr;
};
// (scale, shift) of a frozen BN into out[0..C) / out[C..2C)
void bn_affine(const float* gamma, const float* beta, const float* mean, const float* var, float eps, int fix_gamma,
               int C, float* out, hipStream_t st);

// ---- RoI pooling (roi_pool.hip) -------------------------------------------
// feat NHWC (B, H, W, C) bf16 or fp32; rois (R, 5); out (R, PH, PW, C); argmax (R, PH, PW, C) int32
// holding h*W + w (or -1).  post: relu(bn(out)) written instead of out (argmax must be null)
void roi_pool_fwd(const void* feat, int bf16, int B, int H, int W, int C, const float* rois, int R,
                  int PH, int PW, float spatial_scale, void* out, int32_t* argmax, hipStream_t st,
                  PostBn post = PostBn());
// grad_in fp32 NHWC (B, H, W, C), must be zeroed; grad_out (R, PH, PW, C) bf16/fp32.
// LDS-accumulated backward straight into grad_in (B, H, W, C) of the grad_out dtype (code: 0 fp32,
// 1 bf16, 2 fp16); -1 when the H x W slab does not fit LDS (use roi_pool_bwd)
// grad_add (nullable, NHWC like grad_in): another gradient of the feature map, added in the kernel
void col_part_fold(const float* part, int nparts, int C, float* out0, float* out1, hipStream_t st);
// batched col_part_fold (passed by value: kernel arguments, graph-capture safe)
constexpr int kMaxFolds = 32;
struct FoldEntry {
  const float* part;
  float* out0;
  float* out1;
  int nparts, C, blk0;  // blk0: first workgroup of this entry
};
struct FoldBatch {
  FoldEntry e[kMaxFolds];
  int n;
};
void bn_part_fold_multi(const FoldBatch& fb, hipStream_t st);
int roi_pool_bwd_lds(const void* grad_out, int code, const int32_t* argmax, const float* rois, int R, int PH, int PW,
                     int B, int H, int W, int C, void* grad_in, hipStream_t st, const void* grad_add = nullptr);
void roi_pool_bwd(const void* grad_out, int bf16, const int32_t* argmax, const float* rois, int R,
                  int PH, int PW, int B, int H, int W, int C, float* grad_in, hipStream_t st);
// fp32 -> bf16 / fp32 copy-convert helper (n elements)
void cast_f32(const float* in, void* out, int out_bf16, int64_t n, hipStream_t st);

// ---- uniform draws from PyTorch's graph-safe Philox state (rng.hip) ------------------
// seed / offset are values, or (captured) device pointers to int64 values, offset += intra
struct PhiloxArgs {
  uint64_t seed, offset, intra;
  int captured;
};
void philox_fill(float* out, int64_t n, const PhiloxArgs& a, hipStream_t st);
void counter_add(int64_t* p, int64_t v, hipStream_t st);  // p[0] += v (one lane)

// ---- image preparation (image.hip) ---------------------------------------------
// uint8 BGR (B, H, W, 3) -> channels_last (B, 3, H, W) fp32 / bf16 (NHWC memory): RGB, minus means
// (RGB order), 0 outside im_info[b, 0:2] (the valid resized height / width)
void image_prep(const uint8_t* in, const float* im_info, int B, int H, int W, const double* means, int out_bf16,
                void* out, hipStream_t st);

// ---- losses (losses.hip) ---------------------------------------------------
// Every loss kernel writes its final (normalised) value to loss_out[0] itself: blocks store
// partial sums into `partials` (>= loss_blocks_* floats) and the last block to take a ticket
// (a persistent counter, zero between launches, re-armed by that block) reduces them.
// RPN 2-class softmax CE with ignore label -1 ("valid" normalisation).
// logits (B, 2A, H, W) strided; label (B, A*H*W) int32 in (a, h, w) order.
// grad written with the same strides as logits.  Divisor: the sampled counts meta (B, 4) =
// [all_fg, all_bg, n_fg, n_bg] of anchor_sample when given, else *norm (device float).
int loss_blocks_rpn(int64_t total);
void rpn_softmax_ce(const void* logits, int bf16, int64_t s0, int64_t s1, int64_t s2, int64_t s3,
                    const int32_t* label, int B, int A, int H, int W, const float* norm, const int32_t* meta,
                    float grad_scale, void* grad, float* partials, unsigned* ticket, float* loss_out,
                    float* prob_fg, hipStream_t st);
// Row softmax CE for (R, C) logits, labels int32 (R), ignore < 0; normalisation divisor `norm`.
int loss_blocks_row(int R);
void row_softmax_ce(const void* logits, int bf16, int R, int C, const int32_t* label, float norm,
                    float grad_scale, void* grad, float* prob, float* partials, unsigned* ticket, float* loss_out,
                    hipStream_t st);
// Weighted smooth-L1: out_w * f(in_w * (pred - tgt)), sigma; grad = gs * out_w * f'(.) * in_w.
// pred strided 4-D (n0, n1, n2, n3); tgt/in_w/out_w contiguous 4-D of the same logical shape.
// loss_out[0] = sum (blocks: loss_blocks_rpn(n0*n1*n2*n3)).
void smooth_l1(const void* pred, int bf16, int64_t s0, int64_t s1, int64_t s2, int64_t s3,
               int n0, int n1, int n2, int n3, const float* tgt, const float* in_w, const float* out_w,
               float sigma, float grad_scale, void* grad, float* partials, unsigned* ticket, float* loss_out,
               hipStream_t st);
// x[i] *= s[0] (device scalar), bf16 or fp32, in place.
void scale_by_scalar(void* x, int bf16, int64_t n, const float* s, hipStream_t st);
// total / weighted objective of up to 8 scalar loss terms, plus the non-finite step counter.
struct LossTerms {
  const float* p[8];
  float w[8];
  int n;
};
void loss_combine(const LossTerms& t, float* out, int32_t* nonfinite, hipStream_t st);

// ---- optimizer (sgd.hip) ---------------------------------------------------
// MXNet SGD semantics: g = clip(rescale*g, +-clip) (clip<=0: off); mom = mu*mom - lr*(g + wd*w); w += mom.
// grad fp32 or bf16; lr read from device pointer; optional bf16 shadow copy of w.
void sgd_momentum(float* w, float* mom, const void* grad, int grad_bf16, int64_t n, const float* lr,
                  float momentum, float wd, float rescale, float clip, uint16_t* w_bf16, hipStream_t st,
                  int64_t x2_plane = 0,   // x2_plane > 0: w_bf16 is an x2 hi / lo pair, lo x2_plane elements on
                  int x3 = 0,             // with x2_plane: an x3 triple (mid, hi, lo) x2_plane apart
                  void* zero = nullptr,   // cleared after reading (the consumed gradient buffer, n elements)
                  int zero_bf16 = 0);

// ---- frozen BN + ReLU (bn_act.hip) -----------------------------------------
// NHWC x (M rows, C channels) bf16/fp32; y = relu((x-mean)*rsqrt(var+eps)*gamma + beta).
void bn_relu_fwd(const void* x, int bf16, int64_t M, int C, const float* gamma, const float* beta,
                 const float* mean, const float* var, float eps, int fix_gamma, int relu, void* y,
                 hipStream_t st);
// dx = dy * [y>0] * s;  dgamma = sum(dy*[y>0]*xhat), dbeta = sum(dy*[y>0]) (fp32; written, not
// accumulated, on the vector path; the scalar C%4 path accumulates into zeroed buffers).
// workspace: bn_bwd_workspace_floats(M, C) floats (per-block partial rows, no atomics).
int bn_bwd_workspace_floats(int64_t M, int C);
void bn_relu_bwd(const void* x, const void* dy, int bf16, int64_t M, int C, const float* gamma,
                 const float* beta, const float* mean, const float* var, float eps, int fix_gamma, int relu,
                 void* dx, const void* dres, float* dgamma, float* dbeta, float* workspace, int accumulate,
                 hipStream_t st);

// ---- implicit-GEMM convolution (conv_igemm.hip) ------------------------------
// NHWC bf16 x (NB, H, W, Cin), weight (Cout, KH, KW, Cin) bf16, bias fp32 (Cout) or null,
// y (NB, Ho, Wo, Cout) bf16.  tile: 0 = auto, 1 = 128x128, 2 = 128x64, 3 = 64x64.
// conv_igemm_plan picks (tile, splits); splits > 1 needs an fp32 slab of splits*M*Cout floats.
// Returns the tile used, or -1 if the shape is unsupported (Cin % 64 != 0).
int conv_igemm_plan(int NB, int Ho, int Wo, int Cin, int Cout, int KH, int KW, int tile, int* splits_out);
// Fused epilogue of the implicit-GEMM conv (all fields optional):
//   v  = acc + bias[n] + residual[m][n];  if relu: v = max(v, 0);  y[m][n] = bf16(v)
//   if y2: y2[m][n] = bf16(act(v * s[n] + t[n])) with the frozen-BN affine
//          s = gamma * rsqrt(var + eps) (gamma := 1 when fix_gamma), t = beta - mean * s,
//          act = ReLU when act_relu.  (Conv -> frozen BN -> ReLU of a pre-activation ResNet unit,
//          keeping the raw conv output y for the BN backward.)
struct ConvEpi {
  const float* bias = nullptr;
  const uint16_t* bias_h = nullptr;  // bias in the activation dtype (bf16 / fp16), instead of `bias`
  const uint16_t* residual = nullptr;
  int relu = 0;
  const float* bn_gamma = nullptr;
  const float* bn_beta = nullptr;
  const float* bn_mean = nullptr;
  const float* bn_var = nullptr;
  float bn_eps = 2e-5f;
  int bn_fix_gamma = 0;
  int act_relu = 1;
  uint16_t* y2 = nullptr;
  // BN-ReLU BACKWARD mode (the conv is a dgrad producing d(act) of a frozen BN + ReLU whose
  // input was bnb_x): v = acc + dadd; g = v * [bn(bnb_x) > 0]; y = g * s + residual;
  // dgamma += sum_rows g * xhat, dbeta += sum_rows g (fp32 atomics; may be null).
  const uint16_t* bnb_x = nullptr;
  const uint16_t* dadd = nullptr;
  // dadd_s > 1: dadd is the stride-dadd_s subsampled grid (ceil(Ho/s) x ceil(Wo/s)) of this
  // launch's Ho x Wo grid and adds only at rows (img, i*s, j*s) -- a strided projection
  // shortcut's gradient, without scattering it into a zero-filled full-size map first
  int dadd_s = 0;
  int dadd_gh = 0, dadd_gw = 0;  // the launch grid (Ho, Wo) the subsampled dadd refers to
  float* bnb_dgamma = nullptr;
  float* bnb_dbeta = nullptr;
  // inverted dropout AFTER bias/residual/ReLU (the FC head's ReLU -> Dropout, rcnn/symbol.py:98,102):
  // element e of step s is kept iff philox_uniform(drop_seed, s, e) >= drop_p, kept values are
  // scaled by 1 / (1 - drop_p).  The step is read from device memory (graph replay safe).
  float drop_p = 0.f;
  uint32_t drop_seed = 0;
  const int64_t* drop_step = nullptr;
  // geometry extensions (ring / buffer kernels only, no split-K): width padding different from the
  // height padding, and an output row map that scatters output pixel (img, i, j) of the Ho x Wo
  // grid to row (img, i*o_sh + o_ph, j*o_sw + o_pw) of an o_H x o_W map -- the parity classes of
  // a strided data gradient each write their own positions of dx (ops/conv.py strided_dgrad)
  int pad_w = -1;
  int omap = 0;
  int o_H = 0, o_W = 0, o_sh = 1, o_sw = 1, o_ph = 0, o_pw = 0;
  // fp16 activations / weights (inference): MFMA f16 operands, fp16 epilogue loads / stores
  int f16 = 0;
  // batch statistics of the STORED output for a training-mode BN that consumes it (LDS-epilogue
  // kernels, no split-K): row tile t writes sum(y - shift) / sum((y - shift)^2) of its rows to
  // st_part[t][0][:] / st_part[t][1][:]; row tile 0 also copies the shift to st_part[tiles_m][0][:]
  // (the bn_train.hip partial layout, folded by bn_train_apply)
  float* st_part = nullptr;
  const float* st_shift = nullptr;
  // BN-backward mode, deterministic sums (batch-statistics BNs, whose dx needs them): instead of
  // atomics into bnb_dgamma / bnb_dbeta, row tile t writes [sum g | sum g * xhat] of its rows to
  // bnb_part[bnb_row0 + t][0 / 1][:] (LDS-epilogue kernels, no split-K)
  float* bnb_part = nullptr;
  int bnb_row0 = 0;
  // fp32-class mode (common.h "x2"): every 16-bit operand and output is a hi / lo bf16 plane pair.
  // The main loop runs three K phases (A_hi B_hi, A_hi B_lo, A_lo B_hi) with the lo planes reached
  // through plane byte offsets; the epilogue reads pairs and stores pairs (buffer kernels 22 / 23
  // and the grouped launch only)
  // x3 (the fp32 mode, common.h): operands are (mid, hi, lo) triples with x2 = 1 and the x2_* plane
  // offsets one plane apart; the main loops run their K range twice, first with every operand base
  // one plane further on (products hh + hl + lh), then at the base (mm + mh + hm); the epilogues read
  // and store triples (x2_py / x2_pd are then the plane spacings)
  int x2 = 0;
  int x3 = 0;
  uint32_t x2_pa = 0, x2_pb = 0;  // lo-plane offsets of the A (activation) / B (filter) operands, bytes
  int64_t x2_py = 0;              // lo-plane offset of y, y2, residual and bnb_x, elements
  int64_t x2_pd = 0;              // lo-plane offset of dadd, elements
  float* yf = nullptr;            // fp32 output instead of y (no y2): the x2 mode's prediction heads
  // data gradient straight from the forward filter (Cin, KH, KW, Cout) -- no flipped / transposed
  // copy; the launch's Cin / Cout are the dgrad's (the filter's output / input channels), the taps
  // are flipped in-kernel (buffer kernels 22 / 23 and the grouped launch)
  int bt = 0;
  // ReLU (+ inverted dropout) backward fused into a data gradient: y = v * [rmask > 0] * rmask_s, where
  // rmask (shaped like y, bf16; x2 / x3: its hi plane) is the ReLU / dropout OUTPUT of the previous layer,
  // i.e. this data gradient's forward input (plain epilogue only: no bnb_x / y2)
  const uint16_t* rmask = nullptr;
  float rmask_s = 1.f;
};
// counter-based uniform in [0, 1) (Philox-4x32-10, key = (seed, 0x9E3779B9), counter = (e, s))
float philox_uniform_host(uint32_t seed, uint64_t step, uint64_t e);
// output rows per workgroup tile (BM) of a tile code
int conv_tile_bm(int tile);
// K-group kernels (conv_kg.hip), tile codes 27-29; returns the tile or -1 (unsupported)
int conv_igemm_kg(int tile, const uint16_t* x, const uint16_t* w, uint16_t* y, int NB, int H, int W, int Cin, int Ho,
                  int Wo, int Cout, int KH, int KW, int stride, int pad, const ConvEpi& ep, int splits, float* slab,
                  hipStream_t st);
// large-tile conv (conv_big.hip): tile 200 = 256x256, 201 = 256x128, 512 threads, bf16 / fp16, plain
// epilogues (bias, residual, ReLU, frozen-BN second output); -1 when unsupported
int conv_big_fwd(const uint16_t* x, const uint16_t* w, uint16_t* y, int NB, int H, int W, int Cin, int Ho, int Wo,
                 int Cout, int KH, int KW, int stride, int pad, const ConvEpi& ep, int tile, hipStream_t st);
int conv_igemm_fwd(const uint16_t* x, const uint16_t* w, uint16_t* y, int NB, int H, int W, int Cin, int Ho, int Wo,
                   int Cout, int KH, int KW, int stride, int pad, const ConvEpi& ep, int tile, int splits, float* slab,
                   hipStream_t st);
// ---- training-mode BatchNorm (bn_train.hip) -----------------------------------------------
// (x2 = 1 or 2: every bf16 (M, C) operand is an x2 hi / lo pair, lo plane M * C elements on; 3: an
// x3 triple, planes M * C apart)
// x/y/dy/dx NHWC bf16 (M rows x C), C % 64 == 0.  fwd updates the running stats in place
// (moving = momentum * moving + (1 - momentum) * batch, unbiased var) and saves mean / invstd.
// workspace: bn_train_workspace_floats(M, C) floats.
int bn_train_workspace_floats(int64_t M, int C);
int bn_train_fwd(const uint16_t* x, int64_t M, int C, const float* gamma, const float* beta, float* rmean,
                 float* rvar, float momentum, float eps, int fix_gamma, int relu, uint16_t* y, float* save_mean,
                 float* save_invstd, float* workspace, hipStream_t st, float* save_veps = nullptr, int x2 = 0);
// the same normalisation from statistics partials produced elsewhere (a conv epilogue's
// ConvEpi::st_part, nparts row tiles + the shift row).  save: [3][C] = mean, invstd, var + eps
int bn_train_apply(const uint16_t* x, int64_t M, int C, const float* part, int nparts, const float* gamma,
                   const float* beta, float* rmean, float* rvar, float momentum, float eps, int fix_gamma, int relu,
                   uint16_t* y, float* save, hipStream_t st, int x2 = 0);
// BN-ReLU backward finish after a BN-backward conv epilogue wrote o = g * s and the partial rows
// part[nparts][sum g | sum g * xhat][C] (ConvEpi::bnb_part): dx = o - s * (mean g + xhat *
// mean(g xhat)) (+ dres); o may alias dx; dgamma / dbeta (nullable) += the folded sums.
// gamma: the effective gamma (ones under fix_gamma)
int bn_train_dx_apply(const uint16_t* o, const uint16_t* x, int64_t M, int C, const float* part, int nparts,
                      const float* gamma, const float* save, const uint16_t* dres, uint16_t* dx, float* dgamma,
                      float* dbeta, hipStream_t st, int x2 = 0);
// dgamma/dbeta: written (accumulate = 0) or added to (accumulate = 1); may be null.
int bn_train_bwd(const uint16_t* x, const uint16_t* dy, int64_t M, int C, const float* gamma, const float* beta,
                 const float* save_mean, const float* save_invstd, int fix_gamma, int relu, uint16_t* dx,
                 float* dgamma, float* dbeta, int accumulate, float* workspace, hipStream_t st, int x2 = 0);

// ---- pooling (pool.hip): NHWC bf16, C % 8 == 0 ------------------------------------------------
// arg: one byte per output element, the winning tap (i * k + j) of its window
// post: relu(bn(y)) written instead of y (inference; the taps in arg still index the max)
int maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* arg, int N, int H, int W, int C, int Ho, int Wo, int k,
                int s, int p, int code, hipStream_t st, PostBn post = PostBn());
int maxpool_bwd(const uint16_t* dy, const uint8_t* arg, uint16_t* dx, int N, int H, int W, int C, int Ho, int Wo,
                int k, int s, int p, int code, hipStream_t st);
int avgpool_fwd(const uint16_t* x, uint16_t* y, int N, int HW, int C, int code, hipStream_t st);
int avgpool_bwd(const uint16_t* dy, uint16_t* dx, int N, int HW, int C, int code, hipStream_t st);
// stem conv (stem.hip): x (N,H,W,3) 16-bit NHWC, w the packed (64, KP) filter, k = (fr*KW+fc)*3+c,
// zero-padded to KP = roundup(3*KH*KW, 32);
// y (N,Ho,Wo,64) = relu?(conv(in_bn(x)) -> out_bn | + bias).  Geometries 7x7/2, 3x3/1.
struct StemArgs {
  const float *in_g, *in_b, *in_m, *in_v;    // frozen input BN (in_m == nullptr: identity)
  float in_eps;
  int in_fixg;
  const float *out_g, *out_b, *out_m, *out_v;  // frozen output BN (out_m == nullptr: bias or none)
  float out_eps;
  int out_fixg;
  const void* bias;                          // per-channel bias (bias_code: 0 fp32, 1 bf16, 2 fp16)
  int bias_code;
};
int stem_conv(const uint16_t* x, const uint16_t* w, const StemArgs& a, uint16_t* y, int N, int H, int W, int Ho,
              int Wo, int KH, int KW, int stride, int pad, int relu, int code, hipStream_t st);

// ---- proposal pre-NMS top-k (topk.hip): keys (B, N), boxes (B, N, 4) -> the P best in stable
// descending order; ws: proposal_topk_ws_words(B, N) ZEROED words, ws_key / ws_idx: B * P each
int64_t proposal_topk_ws_words(int B, int N);
int proposal_topk(const float* keys, const float* boxes, int B, int N, int P, uint32_t* ws, uint32_t* ws_key,
                  int* ws_idx, float* skeys, float* sboxes, int* n_valid, hipStream_t st);

// ---- test-time detection post-process (det_post.hip) ------------------------------------------
// rois (B*R, 5) grouped by image, scores (B*R, C), deltas (B*R, 4C), im_info (B, 3), all fp32.
// ws_*: (B, C-1, R) kept scores, (B, C-1, R, 4) kept boxes, (B, C-1) kept counts.
// dets (B, cap, 6) [x1 y1 x2 y2 score class] in original-image pixels, counts (B,).
int det_postprocess(const float* rois, const float* scores, const float* deltas, const float* im_info, int B, int R,
                    int C, float thresh, float nms_thresh, int max_per, int cap, float* ws_scores, float* ws_boxes,
                    int* ws_counts, float* dets, int* counts, hipStream_t st);
// keep[i] = 0 when box i lies inside another box by more than `thresh` of its own area
int nest_filter(const float* dets, int n, int stride, float thresh, uint8_t* keep, hipStream_t st);

// Flip + transpose many conv filters in ONE launch (dgrad operand cache):
//   dst[i][r][s][o] = src[o][KH-1-r][KW-1-s][i]   (both channels_last, i.e. (O,KH,KW,I) rows)
struct WtFlipEntry {
  const uint16_t* src;
  uint16_t* dst;
  int O, I, KH, KW;
  int tile_begin;  // prefix sum of 64x64 tiles (per tap) over entries
  // parity sub-filters of the flipped filter (strided data gradient, ops/conv.py sub_filter):
  // flipped tap (r, c) also goes to sub[2 * rcls[r] + ccls[c]] (I, O, rcnt, ccnt channels_last)
  // at sub-tap (ridx[r], cidx[c]); a null sub entry is skipped
  uint16_t* sub[4];
  int8_t rcls[8], ridx[8], ccls[8], cidx[8];
  int8_t rcnt[2], ccnt[2];
};
void conv_wt_flip_multi(const WtFlipEntry* entries, int n_entries, int total_tiles, hipStream_t st);

// ---- MFMA weight gradient (conv_wgrad.hip) -------------------------------------
// dy (NB, Ho, Wo, Cout) bf16, x (NB, H, W, Cin) bf16 -> dw (Cout, KH, KW, Cin) bf16.
// slab: splits * Cout * KH*KW*Cin floats.  Requires Cin % 64 == 0, Cout % 8 == 0.
int conv_wgrad_plan(int NB, int Ho, int Wo, int Cin, int Cout, int KH, int KW, int* splits_out, int planes = 0);
// fp32-class (x2) weight gradient: dY / X are hi / lo plane pairs (lo planes pdy / px bytes after the
// hi ones), the gradient dwf is fp32 (dw unused)
struct WgradX2 {
  int x2 = 0;
  int x3 = 0;  // x3 triples (common.h): pdy / px are the plane spacings, K (pixels) runs twice
  uint32_t pdy = 0, px = 0;
  float* dwf = nullptr;
};
// Grouped launch (conv_igemm.hip): the stride-1 implicit-GEMM conv (x, w) -> y with epilogue `ep`
// (64x64 buffer kernel, no split) AND the weight gradient (wg_*: as conv_wgrad) in ONE launch, plus
// the wgrad split-K reduce when wg_splits > 1.  Returns 0, or -1 when a role's shape is unsupported.
int conv_dgrad_wgrad(const uint16_t* x, const uint16_t* w, uint16_t* y, int NB, int H, int W, int Cin, int Ho, int Wo,
                     int Cout, int KH, int KW, int pad, const ConvEpi& ep, const uint16_t* wg_dy,
                     const uint16_t* wg_x, uint16_t* dw, float* slab, int wg_NB, int wg_H, int wg_W, int wg_Cin,
                     int wg_Ho, int wg_Wo, int wg_Cout, int wg_KH, int wg_KW, int wg_stride, int wg_pad, int wg_splits,
                     int accumulate, hipStream_t st, int defer_reduce = 0, const float* prev_slab = nullptr,
                     int prev_splits = 0, int64_t prev_n = 0, uint16_t* prev_dw = nullptr,
                     const WgradX2& wx2 = WgradX2(), float* prev_dwf = nullptr);
// standalone split-K reduce of a deferred grouped weight gradient (accumulates into dw, or dwf)
void wgrad_reduce_run(const float* slab, int splits, int64_t n, uint16_t* dw, hipStream_t st, float* dwf = nullptr);
int conv_wgrad(const uint16_t* dy, const uint16_t* x, uint16_t* dw, float* slab, int NB, int H, int W, int Cin,
               int Ho, int Wo, int Cout, int KH, int KW, int stride, int pad, int splits, int accumulate,
               hipStream_t st, int variant = 0, const WgradX2& x2 = WgradX2());
// Weight gradient with a fused SGD-momentum update (no split, one pass): the gradient of every
// (Cout, KH*KW*Cin) element updates w / mom / the shadow wb (bf16, or x2 / x3 planes `plane`
// elements apart) in place with the SGD kernel's arithmetic; gbf16: the gradient rounds to bf16
// first (what the unfused bf16 path stores).  Every row must start 16-B aligned (w, mom) and the
// planes 8-B aligned.  Returns 1, or -1 when the shape is unsupported.
struct WgradSgd {
  float* w = nullptr;
  float* mom = nullptr;
  uint16_t* wb = nullptr;
  int64_t plane = 0;
  int x3 = 0, gbf16 = 0;
  const float* lr = nullptr;
  float mu = 0.f, wd = 0.f, rescale = 1.f, clip = -1.f;
};
int conv_wgrad_sgd(const uint16_t* dy, const uint16_t* x, int NB, int H, int W, int Cin, int Ho, int Wo, int Cout, int KH,
                   int KW, int stride, int pad, hipStream_t st, const WgradX2& x2, const WgradSgd& sgd);

// ---- small-head backward (head_bwd.hip) ---------------------------------------------------------
// One or two heads y_h = X W_h^T (+b_h) over the same X (M, K) bf16, K % 64 == 0, dY_h (M, N_h):
// dX (optional, ReLU-masked by X > 0 when relu_mask), dW_h (N_h, K) bf16 (+= when dw_acc), db_h (N_h)
// fp32 / bf16 by db_code (+= when db_acc; null: skipped).  rs > 1 splits the dW rows M and needs
// ws_dw[h] (rs * N_h * K floats) and ws_db[h] (rs * N_h floats).
struct HeadBwdArgs {
  const uint16_t* dy[2] = {nullptr, nullptr};
  const uint16_t* w[2] = {nullptr, nullptr};
  int N[2] = {0, 0};
  uint16_t* dw[2] = {nullptr, nullptr};
  int dw_acc[2] = {0, 0};
  void* db[2] = {nullptr, nullptr};
  int db_code[2] = {0, 0};
  int db_acc[2] = {0, 0};
  float* ws_dw[2] = {nullptr, nullptr};
  float* ws_db[2] = {nullptr, nullptr};
  uint16_t* dx = nullptr;
  int relu_mask = 0;
  float mask_scale = 1.f;  // kept dX values are scaled (inverted dropout after the masked ReLU)
  int nheads = 1;
  int rs = 1;
  // fp32-class mode: X / W / dX are x2 hi / lo pairs (X's and dX's lo planes M * K on, W_h's w_plane[h]
  // on), dY is fp32 (dyf), dW fp32 (dwf); products hi*hi + hi*lo + lo*hi on the bf16 MFMA
  // x3 (the fp32 mode): X / W / dX are (mid, hi, lo) triples, six products
  int x2 = 0;
  int x3 = 0;
  const float* dyf[2] = {nullptr, nullptr};
  float* dwf[2] = {nullptr, nullptr};
  int64_t w_plane[2] = {0, 0};
};
// DP interference probes (probe.hip): k workgroups spinning on the real-time counter / copying
void cu_spin(int nwg, int64_t ticks, hipStream_t st);
void cu_copy(const float* src, float* dst, int64_t n, int nwg, hipStream_t st);
// out = dy * [y > 0] * scale (bf16, n % 8 == 0; planes: y is the output's hi plane, dy / out hold
// np planes `plane` = n apart)
void relu_mask(const uint16_t* dy, const uint16_t* y, uint16_t* out, int64_t n, int64_t plane, float scale,
               hipStream_t st, int np = 1);
int head_bwd_splits(int M, int K, const int* N, int nheads);
int head_bwd(const uint16_t* x, int M, int K, const HeadBwdArgs& a, hipStream_t st);
// per-channel sum of x (M, C) (bf16 / fp16 by code) into out (C) fp32 / bf16 by out_code (+= when
// accumulate); part: chan_sum_chunks(M, C) * C floats
int chan_sum_chunks(int64_t M, int C);
int chan_sum(const uint16_t* x, int64_t M, int C, int code, float* part, void* out, int out_code, int accumulate,
             hipStream_t st);

}  // namespace mxr
