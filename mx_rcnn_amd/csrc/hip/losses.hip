// Fused loss kernels: each computes the loss value AND its input gradient in one pass
// (SURVEY kernels K15/K16; MXNet SoftmaxOutput / smooth_l1 / MakeLoss semantics, reference
// `rcnn/symbol.py:194-200,372-378`, `rcnn/resnet.py:96-100,173-181`).  Because SoftmaxOutput
// and MakeLoss ignore the head gradient, the gradient is final at forward time and the
// autograd backward is a scale of the stored buffer -- no second pass over the logits.
#include <algorithm>

#include "common.h"
#include "../kernels.h"

namespace mxr {

// Grid-wide sum without a pre-zeroed accumulator: every block writes its partial, takes a ticket,
// and the last block to finish sums the partials (device-scope loads, past L1), writes the final
// value * scale and re-arms the ticket for the next launch (graph-replay safe).  Replaces the
// zero-fill + atomicAdd + divide kernels around every loss.
__device__ __forceinline__ void block_reduce_final(float v, float* __restrict__ partials, unsigned* __restrict__ ticket,
                                                   float scale, float* __restrict__ out) {
  __shared__ float part[16];
  __shared__ int last;
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (int)(blockDim.x >> 6);
  if (lane == 0) part[wid] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < nw; ++i) s += part[i];
    __hip_atomic_store(partials + blockIdx.x, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __threadfence();
    last = atomicAdd(ticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  float acc = 0.f;
  for (int i = threadIdx.x; i < (int)gridDim.x; i += blockDim.x)
    acc += __hip_atomic_load(partials + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  acc = wave_sum(acc);
  __syncthreads();
  if (lane == 0) part[wid] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < nw; ++i) s += part[i];
    *out = s * scale;
    *ticket = 0u;
  }
}

// normaliser of the RPN loss ('valid'): the labels >= 0, i.e. the sampled fg + bg counts the
// anchor-sampling kernel recorded per image (meta (B, 4) = [all_fg, all_bg, n_fg, n_bg]), or a
// precomputed count
__device__ __forceinline__ float rpn_norm(const float* __restrict__ norm, const int32_t* __restrict__ meta, int B) {
  if (!meta) return fmaxf(*norm, 1.f);
  int n = 0;
  for (int b = 0; b < B; ++b) n += meta[b * 4 + 2] + meta[b * 4 + 3];
  return fmaxf((float)n, 1.f);
}

// RPN: logits (B, 2A, H, W) viewed as (B, 2, A*H, W): channel a = bg, A+a = fg of anchor a.
// Thread order (b, h, w, a) with a fastest so channels-last logits are read contiguously.
__global__ void __launch_bounds__(256)
rpn_softmax_ce_kernel(const void* __restrict__ logits, int bf16, int64_t s0, int64_t s1, int64_t s2, int64_t s3,
                      const int32_t* __restrict__ label, int B, int A, int H, int W, const float* __restrict__ norm,
                      const int32_t* __restrict__ meta, float grad_scale, void* __restrict__ grad,
                      float* __restrict__ partials, unsigned* __restrict__ ticket, float* __restrict__ loss_out,
                      float* __restrict__ prob_fg) {
  const int64_t total = (int64_t)B * H * W * A;
  const float nrm = rpn_norm(norm, meta, B);
  float loss = 0.f;
  // grid-stride over a capped grid (loss_blocks_rpn): fewer partials / ticket arrivals to fold
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
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
      const float sc = grad_scale / nrm;
      gb = (pb - (lab == 0 ? 1.f : 0.f)) * sc;
      gf = (pf - (lab == 1 ? 1.f : 0.f)) * sc;
      loss += -logf(fmaxf(lab == 1 ? pf : pb, 1e-14f));
    }
    st(grad, ibg, gb, bf16);
    st(grad, ifg, gf, bf16);
    if (prob_fg) prob_fg[t] = pf;
  }
  block_reduce_final(loss, partials, ticket, 1.f / nrm, loss_out);
}

// grid of the element-wise grid-reduction losses: at most 128 blocks (a few elements per thread
// at RPN sizes), so the last-block fold and the ticket see 128 arrivals, not ~800
int loss_blocks_rpn(int64_t total) { return (int)std::min<int64_t>(div_up(total, 256), 128); }

void rpn_softmax_ce(const void* logits, int bf16, int64_t s0, int64_t s1, int64_t s2, int64_t s3, const int32_t* label,
                    int B, int A, int H, int W, const float* norm, const int32_t* meta, float grad_scale, void* grad,
                    float* partials, unsigned* ticket, float* loss_out, float* prob_fg, hipStream_t st) {
  const int64_t total = (int64_t)B * H * W * A;
  if (total == 0) return;
  rpn_softmax_ce_kernel<<<loss_blocks_rpn(total), 256, 0, st>>>(logits, bf16, s0, s1, s2, s3, label, B, A, H, W, norm, meta,
                                                            grad_scale, grad, partials, ticket, loss_out, prob_fg);
}

// Row softmax CE: one wave per row, lanes over classes.
__global__ void __launch_bounds__(256)
row_softmax_ce_kernel(const void* __restrict__ logits, int bf16, int R, int C, const int32_t* __restrict__ label,
                      float norm, float grad_scale, void* __restrict__ grad, float* __restrict__ prob,
                      float* __restrict__ partials, unsigned* __restrict__ ticket, float* __restrict__ loss_out) {
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
  block_reduce_final(loss, partials, ticket, 1.f / norm, loss_out);
}

int loss_blocks_row(int R) { return div_up(R, 4); }

void row_softmax_ce(const void* logits, int bf16, int R, int C, const int32_t* label, float norm, float grad_scale,
                    void* grad, float* prob, float* partials, unsigned* ticket, float* loss_out, hipStream_t st) {
  if (R == 0) return;
  row_softmax_ce_kernel<<<div_up(R, 4), 256, 0, st>>>(logits, bf16, R, C, label, norm, grad_scale, grad, prob,
                                                      partials, ticket, loss_out);
}

// Weighted smooth-L1 (MXNet smooth_l1(scalar=sigma) wrapped in outside * f(inside * diff)).
__global__ void __launch_bounds__(256)
smooth_l1_kernel(const void* __restrict__ pred, int bf16, int64_t s0, int64_t s1, int64_t s2, int64_t s3, int n1,
                 int n2, int n3, int64_t total, const float* __restrict__ tgt, const float* __restrict__ in_w,
                 const float* __restrict__ out_w, float sigma2, float grad_scale, void* __restrict__ grad,
                 float* __restrict__ partials, unsigned* __restrict__ ticket, float* __restrict__ loss_out) {
  float loss = 0.f;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
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
    loss += ow * f;
    if (grad) st(grad, pi, grad_scale * ow * d * iw, bf16);
  }
  block_reduce_final(loss, partials, ticket, 1.f, loss_out);
}

void smooth_l1(const void* pred, int bf16, int64_t s0, int64_t s1, int64_t s2, int64_t s3, int n0, int n1, int n2,
               int n3, const float* tgt, const float* in_w, const float* out_w, float sigma, float grad_scale,
               void* grad, float* partials, unsigned* ticket, float* loss_out, hipStream_t st) {
  const int64_t total = (int64_t)n0 * n1 * n2 * n3;
  if (total == 0) return;
  smooth_l1_kernel<<<loss_blocks_rpn(total), 256, 0, st>>>(pred, bf16, s0, s1, s2, s3, n1, n2, n3, total, tgt, in_w,
                                                       out_w, sigma * sigma, grad_scale, grad, partials, ticket,
                                                       loss_out);
}

// --- small fused tails ------------------------------------------------------------------------
// x *= s[0] in place (bf16 or fp32): the backward of every loss above (the stored gradient times
// the incoming scalar) without a cast kernel and a new buffer
__global__ void __launch_bounds__(256)
scale_by_scalar_kernel(void* __restrict__ x, int bf16, int64_t n, const float* __restrict__ s) {
  const float f = *s;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    st(x, i, ld(x, i, bf16) * f, bf16);
}

void scale_by_scalar(void* x, int bf16, int64_t n, const float* s, hipStream_t st) {
  if (n == 0) return;
  scale_by_scalar_kernel<<<(int)std::min<int64_t>(div_up(n, 256), 1024), 256, 0, st>>>(x, bf16, n, s);
}

// out[0] = sum_i terms[i]; out[1] = sum_i w[i] * terms[i]; nonfinite[0] += !isfinite(out[1])
__global__ void loss_combine_kernel(const LossTerms t, float* __restrict__ out, int32_t* __restrict__ nonfinite) {
  if (threadIdx.x != 0) return;
  float a = 0.f, b = 0.f;
  for (int i = 0; i < t.n; ++i) {
    const float v = *t.p[i];
    a += v;
    b += t.w[i] * v;
  }
  out[0] = a;
  out[1] = b;
  if (nonfinite && !isfinite(b)) nonfinite[0] += 1;
}

void loss_combine(const LossTerms& t, float* out, int32_t* nonfinite, hipStream_t st) {
  loss_combine_kernel<<<1, 64, 0, st>>>(t, out, nonfinite);
}

}  // namespace mxr
