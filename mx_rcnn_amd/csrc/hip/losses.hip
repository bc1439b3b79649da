// Fused loss kernels: each computes the loss value AND its input gradient in one pass
// (SURVEY kernels K15/K16; MXNet SoftmaxOutput / smooth_l1 / MakeLoss semantics, reference
// `rcnn/symbol.py:194-200,372-378`, `rcnn/resnet.py:96-100,173-181`).  Because SoftmaxOutput
// and MakeLoss ignore the head gradient, the gradient is final at forward time and the
// autograd backward is a scale of the stored buffer -- no second pass over the logits.
#include "common.h"
#include "../kernels.h"

namespace mxr {

__device__ __forceinline__ void block_accumulate(float v, float* dst) {
  __shared__ float part[16];
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) part[wid] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += part[i];
    if (s != 0.f) atomicAdd(dst, s);
  }
}

// RPN: logits (B, 2A, H, W) viewed as (B, 2, A*H, W): channel a = bg, A+a = fg of anchor a.
// Thread order (b, h, w, a) with a fastest so channels-last logits are read contiguously.
__global__ void __launch_bounds__(256)
rpn_softmax_ce_kernel(const void* __restrict__ logits, int bf16, int64_t s0, int64_t s1, int64_t s2, int64_t s3,
                      const int32_t* __restrict__ label, int B, int A, int H, int W, const float* __restrict__ norm,
                      float grad_scale, void* __restrict__ grad, float* __restrict__ loss_sum,
                      float* __restrict__ prob_fg) {
  const int64_t total = (int64_t)B * H * W * A;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float loss = 0.f;
  if (t < total) {
    const int a = (int)(t % A);
    int64_t rest = t / A;
    const int w = (int)(rest % W); rest /= W;
    const int h = (int)(rest % H);
    const int b = (int)(rest / H);
    const int64_t base = (int64_t)b * s0 + (int64_t)h * s2 + (int64_t)w * s3;
    const int64_t ibg = base + (int64_t)a * s1, ifg = base + (int64_t)(A + a) * s1;
    const float zb = ld(logits, ibg, bf16), zf = ld(logits, ifg, bf16);
    const float m = fmaxf(zb, zf);
    const float eb = __expf(zb - m), ef = __expf(zf - m);
    const float inv = 1.f / (eb + ef);
    const float pb = eb * inv, pf = ef * inv;
    const int lab = label[(int64_t)b * A * H * W + ((int64_t)a * H + h) * W + w];
    float gb = 0.f, gf = 0.f;
    if (lab >= 0) {
      const float sc = grad_scale / fmaxf(*norm, 1.f);
      gb = (pb - (lab == 0 ? 1.f : 0.f)) * sc;
      gf = (pf - (lab == 1 ? 1.f : 0.f)) * sc;
      loss = -logf(fmaxf(lab == 1 ? pf : pb, 1e-14f));
    }
    st(grad, ibg, gb, bf16);
    st(grad, ifg, gf, bf16);
    if (prob_fg) prob_fg[t] = pf;
  }
  if (loss_sum) block_accumulate(loss, loss_sum);
}

void rpn_softmax_ce(const void* logits, int bf16, int64_t s0, int64_t s1, int64_t s2, int64_t s3, const int32_t* label,
                    int B, int A, int H, int W, const float* norm, float grad_scale, void* grad, float* loss_sum,
                    float* prob_fg, hipStream_t st) {
  const int64_t total = (int64_t)B * H * W * A;
  if (total == 0) return;
  rpn_softmax_ce_kernel<<<div_up(total, 256), 256, 0, st>>>(logits, bf16, s0, s1, s2, s3, label, B, A, H, W, norm,
                                                            grad_scale, grad, loss_sum, prob_fg);
}

// Row softmax CE: one wave per row, lanes over classes.
__global__ void __launch_bounds__(256)
row_softmax_ce_kernel(const void* __restrict__ logits, int bf16, int R, int C, const int32_t* __restrict__ label,
                      float norm, float grad_scale, void* __restrict__ grad, float* __restrict__ prob,
                      float* __restrict__ loss_sum) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  float loss = 0.f;
  if (row < R) {
    const int64_t rb = (int64_t)row * C;
    float m = -FLT_MAX;
    for (int c = lane; c < C; c += 64) m = fmaxf(m, ld(logits, rb + c, bf16));
    m = wave_max(m);
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += __expf(ld(logits, rb + c, bf16) - m);
    s = wave_sum(s);
    const float inv = 1.f / s;
    const int lab = label[row];
    const float sc = grad_scale / norm;
    for (int c = lane; c < C; c += 64) {
      const float p = __expf(ld(logits, rb + c, bf16) - m) * inv;
      if (prob) prob[rb + c] = p;
      if (grad) st(grad, rb + c, lab >= 0 ? (p - (c == lab ? 1.f : 0.f)) * sc : 0.f, bf16);
      if (c == lab) loss = -logf(fmaxf(p, 1e-14f));
    }
  }
  if (loss_sum) block_accumulate(loss, loss_sum);
}

void row_softmax_ce(const void* logits, int bf16, int R, int C, const int32_t* label, float norm, float grad_scale,
                    void* grad, float* prob, float* loss_sum, hipStream_t st) {
  if (R == 0) return;
  row_softmax_ce_kernel<<<div_up(R, 4), 256, 0, st>>>(logits, bf16, R, C, label, norm, grad_scale, grad, prob,
                                                      loss_sum);
}

// Weighted smooth-L1 (MXNet smooth_l1(scalar=sigma) wrapped in outside * f(inside * diff)).
__global__ void __launch_bounds__(256)
smooth_l1_kernel(const void* __restrict__ pred, int bf16, int64_t s0, int64_t s1, int64_t s2, int64_t s3, int n1,
                 int n2, int n3, int64_t total, const float* __restrict__ tgt, const float* __restrict__ in_w,
                 const float* __restrict__ out_w, float sigma2, float grad_scale, void* __restrict__ grad,
                 float* __restrict__ loss_sum) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float loss = 0.f;
  if (t < total) {
    const int i3 = (int)(t % n3);
    int64_t rest = t / n3;
    const int i2 = (int)(rest % n2); rest /= n2;
    const int i1 = (int)(rest % n1);
    const int i0 = (int)(rest / n1);
    const int64_t pi = (int64_t)i0 * s0 + (int64_t)i1 * s1 + (int64_t)i2 * s2 + (int64_t)i3 * s3;
    const float iw = in_w[t], ow = out_w[t];
    const float x = iw * (ld(pred, pi, bf16) - tgt[t]);
    const float ax = fabsf(x);
    float f, d;
    if (ax < 1.f / sigma2) { f = 0.5f * sigma2 * x * x; d = sigma2 * x; }
    else { f = ax - 0.5f / sigma2; d = x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }
    loss = ow * f;
    if (grad) st(grad, pi, grad_scale * ow * d * iw, bf16);
  }
  if (loss_sum) block_accumulate(loss, loss_sum);
}

void smooth_l1(const void* pred, int bf16, int64_t s0, int64_t s1, int64_t s2, int64_t s3, int n0, int n1, int n2,
               int n3, const float* tgt, const float* in_w, const float* out_w, float sigma, float grad_scale,
               void* grad, float* loss_sum, hipStream_t st) {
  const int64_t total = (int64_t)n0 * n1 * n2 * n3;
  if (total == 0) return;
  smooth_l1_kernel<<<div_up(total, 256), 256, 0, st>>>(pred, bf16, s0, s1, s2, s3, n1, n2, n3, total, tgt, in_w,
                                                       out_w, sigma * sigma, grad_scale, grad, loss_sum);
}

}  // namespace mxr
