// Operand load paths of the large-M GEMM, per CU, on the batch-8 stage-3 reduce shape (A: M = 33600
// rows x K = 1024 bf16 channels, each workgroup its own 160-row panel; B: 256 rows x K shared by
// all, L2-resident), no MFMA:
//   mode 0 "dma":  buffer_load_dwordx4 ... lds straight into an NBUF-deep LDS ring (conv_big.hip's
//                  loop: counted vmcnt, one barrier per 32-channel K tile)
//   mode 1 "reg":  buffer_load_dwordx4 into VGPRs PF K tiles ahead, then ds_write_b128 into a
//                  two-deep LDS ring (the classic register-staged pipeline), one barrier per K tile
//   mode 2 "vmem": buffer_load_dwordx4 into VGPRs only (no LDS): the raw VMEM rate
// The A copies rotate over `ncopy` buffers so a launch does not find its panel in the 256 MB
// infinity cache left by the previous one (ncopy = 1: cache-warm).
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/load_paths tools/microbench/load_paths.hip && /tmp/load_paths
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

constexpr int BM = 160, BN = 256, ROWS = BM + BN, BK = 32;  // 64-B rows per K tile
constexpr int NT = 512;

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// every thread owns LPT row-chunks per K tile: chunk c = tid + NT * i of the ROWS x 4 chunk grid
constexpr int CHUNKS = ROWS * 4;                // 1664
constexpr int LPT = (CHUNKS + NT - 1) / NT;     // 4 (the last partial)

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

template <int MODE, int NBUF, int PF, int RD = 0, int MF = 0, int PRIO = 1>
__global__ void __launch_bounds__(NT) load_kernel(const char* __restrict__ a, const char* __restrict__ b, int K,
                                                  int M, float* sink) {
  __shared__ __attribute__((aligned(16))) char lds[NBUF * ROWS * BK * 2];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int m0 = blockIdx.x * BM;
  const int rowbytes = K * 2;
  const __amdgpu_buffer_rsrc_t ar =
      __builtin_amdgcn_make_buffer_rsrc((void*)a, (short)0, (int)((int64_t)M * rowbytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc((void*)b, (short)0, BN * rowbytes, 0x00020000);
  const int nk = K / BK;
  float acc = 0.f;
  f32x4_t cacc[5][4] = {};
  if constexpr (MODE == 0) {
    // conv_big layout: instruction i of wave w -> rows i*128 + 16w + lane/4, chunk lane & 3
    uint32_t off[LPT];
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int row = i * 128 + (tid >> 2);
      off[i] = row < BM ? (uint32_t)((m0 + row) * rowbytes + (tid & 3) * 16)
                        : (uint32_t)((row - BM) * rowbytes + (tid & 3) * 16);
    }
    const int lpt = wid < (ROWS % 128) / 16 ? LPT : ROWS / 128;
    auto issue = [&](int k, int buf) {
#pragma unroll
      for (int i = 0; i < LPT; ++i) {
        const int row0 = i * 128 + wid * 16;
        if (row0 >= ROWS) continue;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(row0 < BM ? ar : br,
                                                 (__attribute__((address_space(3))) void*)(lds + (buf * ROWS + row0) * BK * 2),
                                                 16, (int)off[i], k * BK * 2, 0, 0);
      }
    };
    for (int s = 0; s < NBUF - 1; ++s) issue(s, s);
    for (int k = 0; k < nk; ++k) {
      const int ahead = min(NBUF - 2, nk - 1 - k);
      if (ahead >= 2) {
        if (lpt == LPT) wait_vm<2 * LPT>(); else wait_vm<2 * (LPT - 1)>();
      } else if (ahead == 1) {
        if (lpt == LPT) wait_vm<LPT>(); else wait_vm<LPT - 1>();
      } else {
        wait_vm<0>();
      }
      __builtin_amdgcn_s_barrier();
      if (k + NBUF - 1 < nk) issue(k + NBUF - 1, (k + NBUF - 1) % NBUF);
      if constexpr (RD == 0 && MF == 0) {
        acc += *reinterpret_cast<const float*>(lds + ((k % NBUF) * ROWS + (tid % ROWS)) * BK * 2 + (lane & 15) * 4);
      } else {
        // conv_big t204 fragments: wave (wm, wn) = (wid / 4, wid % 4), A rows wm*80 + 16i, B rows BM + wn*64 + 16j
        const char* T = lds + (k % NBUF) * ROWS * BK * 2;
        const int wm = wid >> 2, wn = wid & 3, fr = lane & 15, fc = lane >> 4;
        uint4 af[5], bfr[4];
        if constexpr (RD) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = BM + wn * 64 + j * 16 + fr;
            bfr[j] = *reinterpret_cast<const uint4*>(T + row * BK * 2 + ((fc ^ ((row >> 2) & 3)) << 4));
          }
#pragma unroll
          for (int i = 0; i < 5; ++i) {
            const int row = wm * 80 + i * 16 + fr;
            af[i] = *reinterpret_cast<const uint4*>(T + row * BK * 2 + ((fc ^ ((row >> 2) & 3)) << 4));
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) bfr[j] = make_uint4(k + j, lane, 1, 2);
#pragma unroll
          for (int i = 0; i < 5; ++i) af[i] = make_uint4(k + i, lane, 3, 4);
        }
        if constexpr (MF) {
          if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int i = 0; i < 5; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              cacc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[i]),
                                                                   __builtin_bit_cast(bf16x8_t, bfr[j]), cacc[i][j], 0, 0, 0);
          if (PRIO) __builtin_amdgcn_s_setprio(0);
        } else {
#pragma unroll
          for (int i = 0; i < 5; ++i) acc += __builtin_bit_cast(float, af[i].x);
#pragma unroll
          for (int j = 0; j < 4; ++j) acc += __builtin_bit_cast(float, bfr[j].y);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc += cacc[i][j][0];
  } else {
    // chunk c = tid + NT*i: row c / 4, 16-B chunk c % 4 (4 lanes per 64-B row: coalesced)
    uint32_t off[LPT];
    bool isb[LPT], ok[LPT];
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int c = tid + NT * i, row = c >> 2;
      ok[i] = row < ROWS;
      isb[i] = row >= BM;
      off[i] = row < BM ? (uint32_t)((m0 + row) * rowbytes + (c & 3) * 16) : (uint32_t)((row - BM) * rowbytes + (c & 3) * 16);
    }
    uint4 rg[PF][LPT];
    auto load = [&](int k, uint4(&r)[LPT]) {
#pragma unroll
      for (int i = 0; i < LPT; ++i) {
        if (!ok[i]) continue;
        r[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(isb[i] ? br : ar, off[i], k * BK * 2, 0));
      }
    };
#pragma unroll
    for (int p = 0; p < PF; ++p)
      if (p < nk) load(p, rg[p]);
    for (int k0 = 0; k0 < nk; k0 += PF) {
#pragma unroll
      for (int p = 0; p < PF; ++p) {
        const int k = k0 + p;
        if (k >= nk) break;
        if constexpr (MODE == 1) {
          char* dst = lds + (k & 1) * ROWS * BK * 2;
#pragma unroll
          for (int i = 0; i < LPT; ++i) {
            if (!ok[i]) continue;
            const int c = tid + NT * i;
            *reinterpret_cast<uint4*>(dst + (c >> 2) * BK * 2 + (c & 3) * 16) = rg[p][i];
          }
          if (k + PF < nk) load(k + PF, rg[p]);
          __syncthreads();
          acc += *reinterpret_cast<const float*>(dst + (tid % ROWS) * BK * 2 + (lane & 15) * 4);
        } else {
#pragma unroll
          for (int i = 0; i < LPT; ++i)
            if (ok[i]) acc += __builtin_bit_cast(float, rg[p][i].x);
          if (k + PF < nk) load(k + PF, rg[p]);
        }
      }
    }
  }
  if (acc == 12345.f) sink[blockIdx.x] = acc;
}

template <int MODE, int NBUF, int PF, int RD = 0, int MF = 0, int PRIO = 1>
static void run(char** a, int ncopy, const char* b, int M, int K, float* sink, const char* name) {
  const int nwg = M / BM;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) load_kernel<MODE, NBUF, PF, RD, MF, PRIO><<<nwg, NT>>>(a[w % ncopy], b, K, M, sink);
  CK(hipDeviceSynchronize());
  const int it = 24;
  CK(hipEventRecord(e0));
  for (int w = 0; w < it; ++w) load_kernel<MODE, NBUF, PF, RD, MF, PRIO><<<nwg, NT>>>(a[w % ncopy], b, K, M, sink);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / it;
  const double per_wg = (double)ROWS * K * 2;  // bytes a workgroup pulls into the CU
  const double hbm = (double)M * K * 2;        // unique A bytes
  printf("{\"path\": \"%s\", \"rd\": %d, \"mf\": %d, \"mode\": %d, \"nbuf\": %d, \"pf\": %d, \"ncopy\": %d, \"nwg\": %d, \"us\": %.2f, "
         "\"GBps_per_cu\": %.1f, \"A_TBps\": %.2f}\n",
         name, RD, MF, MODE, NBUF, PF, ncopy, nwg, us, per_wg / us / 1e3, hbm / us / 1e6);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main() {
  const int M = 33600, K = 1024;
  const size_t abytes = (size_t)M * K * 2;
  const int ncopy = 8;  // 8 x 69 MB: past the infinity cache
  char* a[ncopy];
  for (int i = 0; i < ncopy; ++i) {
    CK(hipMalloc(&a[i], abytes));
    CK(hipMemset(a[i], 1, abytes));
  }
  char* b;
  float* sink;
  CK(hipMalloc(&b, (size_t)BN * K * 2));
  CK(hipMemset(b, 1, (size_t)BN * K * 2));
  CK(hipMalloc(&sink, 1 << 20));
  for (int nc : {1, ncopy}) {
    run<0, 4, 1, 1, 0>(a, nc, b, M, K, sink, "dma4 + frag reads");
    run<0, 4, 1, 0, 1>(a, nc, b, M, K, sink, "dma4 + mfma (register operands)");
    run<0, 4, 1, 1, 1>(a, nc, b, M, K, sink, "dma4 + reads + mfma (conv_big t204 loop)");
    run<0, 4, 1, 1, 1, 0>(a, nc, b, M, K, sink, "dma4 + reads + mfma, no setprio");
    run<0, 3, 1, 1, 1>(a, nc, b, M, K, sink, "dma3 + reads + mfma");
    run<0, 4, 1>(a, nc, b, M, K, sink, "dma nbuf4");
    run<0, 3, 1>(a, nc, b, M, K, sink, "dma nbuf3");
    run<1, 2, 1>(a, nc, b, M, K, sink, "reg pf1");
    run<1, 2, 2>(a, nc, b, M, K, sink, "reg pf2");
    run<1, 2, 3>(a, nc, b, M, K, sink, "reg pf3");
    run<2, 2, 2>(a, nc, b, M, K, sink, "vmem pf2");
    run<2, 2, 4>(a, nc, b, M, K, sink, "vmem pf4");
  }
  CK(hipDeviceSynchronize());
  return 0;
}
