// Interference probes for the data-parallel design (tools/dp_interference.py): kernels that hold k
// compute units for a set time beside a graph-replayed training step, the way an RCCL ring
// all-reduce's k channel workgroups would while a gradient bucket reduces.
//   cu_spin: k workgroups of 512 threads that spin on the 100 MHz real-time counter for `ticks`
//            (the occupancy of channels waiting on flags / the link)
//   cu_copy: k workgroups streaming a buffer copy (the HBM traffic of a channel's reduce + copy)
#include "common.h"
#include "../kernels.h"

namespace mxr {

__global__ void __launch_bounds__(512) cu_spin_kernel(int64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) < ticks) __builtin_amdgcn_s_sleep(8);
}

__global__ void __launch_bounds__(512) cu_copy_kernel(const float4* __restrict__ src, float4* __restrict__ dst,
                                                      int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) dst[i] = src[i];
}

void cu_spin(int nwg, int64_t ticks, hipStream_t st) {
  if (nwg > 0) cu_spin_kernel<<<nwg, 512, 0, st>>>(ticks);
}

void cu_copy(const float* src, float* dst, int64_t n, int nwg, hipStream_t st) {
  if (nwg > 0 && n >= 4)
    cu_copy_kernel<<<nwg, 512, 0, st>>>(reinterpret_cast<const float4*>(src), reinterpret_cast<float4*>(dst), n / 4);
}

}  // namespace mxr
