// Large-M GEMM main loop, wave layout study on the batch-8 stage-3 reduce (M = 33600, K = 1024,
// N = 256, bf16, NT operands: both K-contiguous): conv_big's loop (LDS-DMA ring of NBUF K tiles of
// 32 channels, one barrier per K tile, ds_read_b128 fragments with the chunk ^ ((row >> 2) & 3)
// swizzle, v_mfma_f32_16x16x32_bf16) with WGM x WGN waves, each owning a (BM/WGM) x (BN/WGN) block.
// Fewer, larger wave blocks read fewer LDS bytes per MFMA (profiles/r6_load_paths.jsonl: the
// fragment reads, not the loads or the MFMAs, are what the 8-wave 160 x 256 loop pays for).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/microbench/_bin/big_tile tools/microbench/big_tile.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
constexpr int BK = 32;

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BM, int BN, int WGM, int WGN, int NBUF>
__global__ void __launch_bounds__(64 * WGM * WGN) gemm_kernel(const uint16_t* __restrict__ a, const uint16_t* __restrict__ b,
                                                              float* __restrict__ c, int M, int K, int N) {
  constexpr int NT = 64 * WGM * WGN, ROWS = BM + BN, RPI = NT / 4;  // LDS rows per DMA instruction round
  constexpr int LPT_HI = (ROWS + RPI - 1) / RPI, LPT_LO = ROWS / RPI;
  constexpr int WM = BM / WGM, WN = BN / WGN, TM = WM / 16, TN = WN / 16;
  static_assert(ROWS % 16 == 0 && BM % 16 == 0, "16-row DMA blocks");
  __shared__ __attribute__((aligned(16))) uint16_t lds[NBUF * ROWS * BK];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WGN, wn = wid % WGN;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc((void*)a, (short)0, M * K * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc((void*)b, (short)0, N * K * 2, 0x00020000);
  constexpr int NHI = (ROWS % RPI) / 16;  // waves issuing the extra partial round
  const int lpt = wid < NHI ? LPT_HI : LPT_LO;
  uint32_t off[LPT_HI];
#pragma unroll
  for (int i = 0; i < LPT_HI; ++i) {
    const int row = i * RPI + (tid >> 2);
    const int lc = (tid & 3) ^ ((row >> 2) & 3);
    off[i] = 0x80000000u;
    if (row < BM) {
      if (m0 + row < M) off[i] = (uint32_t)(((m0 + row) * K + lc * 8) * 2);
    } else if (row < ROWS) {
      off[i] = (uint32_t)(((n0 + row - BM) * K + lc * 8) * 2);
    }
  }
  const int nk = K / BK;
  auto issue = [&](int kt, int buf) {
    uint16_t* base = lds + (buf * ROWS + wid * 16) * BK;
#pragma unroll
    for (int i = 0; i < LPT_HI; ++i) {
      const int row0 = i * RPI + wid * 16;
      if (row0 >= ROWS) continue;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(row0 < BM ? ar : br,
                                               (__attribute__((address_space(3))) void*)(base + i * RPI * BK), 16,
                                               (int)off[i], kt * BK * 2, 0, 0);
    }
  };
  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NBUF - 1; ++s)
    if (s < nk) issue(s, s);
  const int fr = lane & 15, fc = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(NBUF - 2, nk - 1 - kt);
    if (ahead >= 2) {
      if (lpt == LPT_LO) wait_vm<2 * LPT_LO>(); else wait_vm<2 * LPT_HI>();
    } else if (ahead == 1) {
      if (lpt == LPT_LO) wait_vm<LPT_LO>(); else wait_vm<LPT_HI>();
    } else {
      wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    if (kt + NBUF - 1 < nk) issue(kt + NBUF - 1, (kt + NBUF - 1) % NBUF);
    const uint16_t* T = lds + (kt % NBUF) * ROWS * BK;
    uint4 bf[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = BM + wn * WN + j * 16 + fr;
      bf[j] = *reinterpret_cast<const uint4*>(T + row * BK + ((fc ^ ((row >> 2) & 3)) << 3));
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * WM + i * 16 + fr;
      const uint4 af = *reinterpret_cast<const uint4*>(T + row * BK + ((fc ^ ((row >> 2) & 3)) << 3));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af),
                                                            __builtin_bit_cast(bf16x8_t, bf[j]), acc[i][j], 0, 0, 0);
    }
  }
  // checksum only (the study times the main loop; the kernel's epilogue is conv_big's)
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) s += acc[i][j][0] + acc[i][j][3];
  if (s == 12345.f) c[blockIdx.x] = s;
}

template <int BM, int BN, int WGM, int WGN, int NBUF>
static void run(const uint16_t* a, const uint16_t* b, float* c, int M, int K, int N) {
  dim3 grid((M + BM - 1) / BM, N / BN);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) gemm_kernel<BM, BN, WGM, WGN, NBUF><<<grid, 64 * WGM * WGN>>>(a, b, c, M, K, N);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  const int it = 20;
  CK(hipEventRecord(e0));
  for (int w = 0; w < it; ++w) gemm_kernel<BM, BN, WGM, WGN, NBUF><<<grid, 64 * WGM * WGN>>>(a, b, c, M, K, N);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / it;
  printf("{\"BM\": %d, \"BN\": %d, \"waves\": \"%dx%d\", \"nbuf\": %d, \"wgs\": %d, \"us\": %.2f, \"TFs\": %.0f}\n", BM, BN,
         WGM, WGN, NBUF, grid.x * grid.y, us, 2.0 * M * N * K / us / 1e6);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main() {
  const int M = 33600, K = 1024, N = 256;
  uint16_t *a, *b;
  float* c;
  CK(hipMalloc(&a, (size_t)M * K * 2));
  CK(hipMalloc(&b, (size_t)N * K * 2));
  CK(hipMalloc(&c, 1 << 20));
  CK(hipMemset(a, 0x3c, (size_t)M * K * 2));
  CK(hipMemset(b, 0x3c, (size_t)N * K * 2));
  run<160, 256, 2, 4, 4>(a, b, c, M, K, N);  // conv_big t204
  run<256, 256, 2, 4, 4>(a, b, c, M, K, N);  // conv_big t200
  run<128, 256, 2, 4, 4>(a, b, c, M, K, N);  // conv_big t203
  run<256, 256, 2, 2, 4>(a, b, c, M, K, N);  // 4 waves, 128 x 128 each
  run<256, 256, 2, 2, 3>(a, b, c, M, K, N);
  run<160, 256, 2, 2, 4>(a, b, c, M, K, N);  // 4 waves, 80 x 128
  run<128, 256, 2, 2, 4>(a, b, c, M, K, N);  // 4 waves, 64 x 128
  run<128, 256, 1, 4, 4>(a, b, c, M, K, N);  // 4 waves, 128 x 64
  run<256, 256, 4, 2, 4>(a, b, c, M, K, N);  // 8 waves, 64 x 128
  CK(hipDeviceSynchronize());
  return 0;
}
