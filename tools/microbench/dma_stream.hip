// Per-CU LDS-DMA streaming rate of the implicit-GEMM operand pattern (no MFMA): each workgroup
// streams `nk` stages of R rows x 128 B (8 rows x 128 B per wave-instruction, buffer_load ... lds)
// through an S-deep LDS ring with counted vmcnt waits and a raw barrier -- the conv buffer
// kernel's load loop alone.  Sharing model of a 64x64-tile GEMM: A panel = blk / 4 (four column
// tiles share a row panel), B panel = blk % 4; `mode` 1: every block reads ONE shared panel pair
// (L2-resident), 2: every block its own panels (no reuse), 3: contiguous 1 KB per wave-instruction.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/dma_stream tools/microbench/dma_stream.hip && /tmp/dma_stream
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);         \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int R, int S, int RD = 0, int NMF = 0>
__global__ void __launch_bounds__(256) stream_kernel(const char* __restrict__ a, const char* __restrict__ b, int nk,
                                                     int rowbytes, int mode, int nwg, float* sink) {
  constexpr int PER = R / 32;  // wave-instructions per stage per wave (4 waves x 8 rows each)
  __shared__ __attribute__((aligned(16))) char lds[S * R * 128];
  const int bid = blockIdx.x;
  const int q = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
  const int wg = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + bid / 8;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int pa = wg / 4, pb = wg % 4;
  if (mode == 1) pa = pb = 0;
  if (mode == 2) pa = pb = wg;
  const int64_t a_span = (int64_t)64 * rowbytes;
  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc((void*)a, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc((void*)b, (short)0, 0x7fffffff, 0x00020000);
  uint32_t off[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int row = 32 * (i % (PER / 2)) + 8 * wid + (lane >> 3);  // row within the 64-row panel
    const int slot = lane & 7;
    if (mode == 3)
      off[i] = (uint32_t)((i < PER / 2 ? pa : pb) * a_span + (int64_t)((i % (PER / 2)) * 4 + wid) * 1024 + lane * 16);
    else
      off[i] = (uint32_t)((i < PER / 2 ? pa : pb) * a_span + (int64_t)row * rowbytes + (slot ^ ((row >> 1) & 7)) * 16);
  }
  auto issue = [&](int k, int buf) {
    const uint32_t so = (uint32_t)(mode == 3 ? k * (R / 2) * 128 : k * 128);
#pragma unroll
    for (int i = 0; i < PER; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(i < PER / 2 ? ar : br,
                                               (__attribute__((address_space(3))) void*)(lds + (buf * R + 32 * i + 8 * wid) * 128),
                                               16, (int)off[i], (int)so, 0, 0);
  };
  float acc = 0.f;
  f32x4 c[4] = {};
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) issue(s, s);
  for (int k = 0; k < nk; ++k) {
    const int ahead = min(S - 2, nk - 1 - k);
    if (ahead >= 4) wait_vm<4 * PER>();
    else if (ahead == 3) wait_vm<3 * PER>();
    else if (ahead == 2) wait_vm<2 * PER>();
    else if (ahead == 1) wait_vm<PER>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    if (k + S - 1 < nk) issue(k + S - 1, (k + S - 1) % S);
    if constexpr (RD == 0) {
      acc += *reinterpret_cast<const float*>(lds + ((k % S) * R + (tid & (R - 1))) * 128 + (tid & 7) * 16);
    } else {
      // the conv's fragment reads: RD ds_read_b128 per wave (16 rows x 16 B chunks), then NMF MFMAs
      bf16x8 f[RD];
#pragma unroll
      for (int i = 0; i < RD; ++i) {
        const int row = (i * 16 + (lane & 15)) & (R - 1);
        f[i] = *reinterpret_cast<const bf16x8*>(lds + ((k % S) * R + row) * 128 + (((lane >> 4) + 4 * (i & 1)) ^ ((row >> 1) & 7)) * 16);
      }
#pragma unroll
      for (int j = 0; j < NMF; ++j) c[j % 4] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[j % RD], f[(j + 1) % RD], c[j % 4], 0, 0, 0);
    }
  }
  if constexpr (RD > 0) acc += c[0][0] + c[1][1] + c[2][2] + c[3][3];
  if (acc == 12345.f) sink[bid] = acc;
}

template <int R, int S, int RD = 0, int NMF = 0>
static void run(const char* a, const char* b, int nwg, int nk, int rowbytes, int mode, float* sink) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) stream_kernel<R, S, RD, NMF><<<nwg, 256>>>(a, b, nk, rowbytes, mode, nwg, sink);
  CK(hipEventRecord(e0));
  const int it = 20;
  for (int w = 0; w < it; ++w) stream_kernel<R, S, RD, NMF><<<nwg, 256>>>(a, b, nk, rowbytes, mode, nwg, sink);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / it;
  const double per_wg = (double)R * 128 * nk;
  printf("{\"RD\": %d, \"NMF\": %d, \"R\": %d, \"S\": %d, \"nwg\": %d, \"nk\": %d, \"rowbytes\": %d, \"mode\": %d, \"us\": %.2f, "
         "\"GBps_per_wg\": %.1f, \"TBps_chip\": %.2f}\n",
         RD, NMF, R, S, nwg, nk, rowbytes, mode, us, per_wg / us / 1e3, per_wg * nwg / us / 1e6);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main() {
  const size_t bytes = (size_t)512 << 20;
  char *a, *b;
  float* sink;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&sink, 1 << 20));
  CK(hipMemset(a, 1, bytes));
  CK(hipMemset(b, 1, bytes));
  // bisection toward the conv main loop (64x64 tile, 4 waves: 8 fragment reads, 8 (bf16) / 12 (x2) MFMAs per stage)
  // vs double-depth stages (R = 256 rows of 128 B = the 64x64 tile's 256-B stage rows: 16 reads, 24 x2 MFMAs)
  run<128, 3, 8, 12>(a, b, 264, 32, 4096, 0, sink);
  run<256, 3, 16, 24>(a, b, 264, 16, 4096, 0, sink);
  run<256, 2, 16, 24>(a, b, 264, 16, 4096, 0, sink);
  run<256, 4, 16, 24>(a, b, 264, 16, 4096, 0, sink);
  run<512, 2, 32, 48>(a, b, 264, 8, 4096, 0, sink);
  run<128, 3, 8, 8>(a, b, 264, 16, 2048, 0, sink);
  run<256, 3, 16, 16>(a, b, 264, 8, 2048, 0, sink);
  run<256, 3, 16, 0>(a, b, 264, 16, 4096, 0, sink);
  run<256, 3, 16, 12>(a, b, 264, 16, 4096, 0, sink);
  run<128, 3, 8, 12>(a, b, 264, 72, 4096 * 9 / 4, 0, sink);
  run<256, 3, 16, 24>(a, b, 264, 36, 4096 * 9 / 4, 0, sink);
  CK(hipDeviceSynchronize());
  return 0;
}
