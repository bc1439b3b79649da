// Uniform [0, 1) draws for the sampling ops (anchor / RoI subsets, the proposal random pad) from
// PyTorch's graph-safe Philox state: the host takes (seed, offset) from the default HIP generator
// (CUDAGeneratorImpl::philox_cuda_state), which under hipGraph capture hands out POINTERS to the
// seed / offset that every replay advances, so a replayed step draws fresh numbers exactly like
// torch.rand would -- but through this kernel (the Philox-4x32-10 of the fused dropout, common.h),
// not a torch distribution kernel in the captured step.
#include "common.h"
#include "../kernels.h"

namespace mxr {

__global__ void __launch_bounds__(256)
philox_fill_kernel(float* __restrict__ out, int64_t n, PhiloxArgs a) {
  const uint64_t seed = a.captured ? (uint64_t)*reinterpret_cast<const int64_t*>(a.seed) : a.seed;
  const uint64_t off = (a.captured ? (uint64_t)*reinterpret_cast<const int64_t*>(a.offset) : a.offset) + a.intra;
  const uint32_t key = (uint32_t)seed ^ (uint32_t)(seed >> 32);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = philox_uniform(key, off, (uint64_t)i);
}

void philox_fill(float* out, int64_t n, const PhiloxArgs& a, hipStream_t st) {
  if (n <= 0) return;
  const int blocks = (int)std::min<int64_t>(div_up(n, 256), 1024);
  philox_fill_kernel<<<blocks, 256, 0, st>>>(out, n, a);
}

// The training step's Philox counter (the fused dropout's step, ops/fc.py) advances inside the
// captured step with this one-lane kernel instead of a host fill before every replay.
__global__ void counter_add_kernel(int64_t* __restrict__ p, int64_t v) {
  if (threadIdx.x == 0) p[0] += v;
}

void counter_add(int64_t* p, int64_t v, hipStream_t st) { counter_add_kernel<<<1, 64, 0, st>>>(p, v); }

}  // namespace mxr
