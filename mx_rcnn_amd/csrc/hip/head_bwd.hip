// Backward of a pair of small "heads" that read the same input X (SURVEY K12 / K3 backward):
// the RPN's rpn_cls_score + rpn_bbox_pred 1x1 convs over the ReLU'd 3x3 conv map
// (`rcnn/symbol.py:165-172`, M = H*W pixels, K = 512, N = 2A / 4A) and the detector's
// cls_score + bbox_pred FullyConnected layers over the pooled RoI feature (`rcnn/symbol.py:108-111`,
// `rcnn/resnet.py:167-171`, M = 128 RoIs, K = 2048 / 4096, N = C / 4C).  N is far below one
// 64-wide tile and not a multiple of 8, which the conv / wgrad kernels need, so without this
// kernel each head's backward was a hipBLASLt dgrad + dW, a torch column sum for db, dtype casts
// and autograd adds (~14 launches, ~70 us serial per pair).  One launch here computes
//
//   dX[m][k]     = mask(m, k) * sum_h sum_n dY_h[m][n] W_h[n][k]    (mask = X[m][k] > 0 when relu_mask:
//                                                                    the ReLU backward of X's producer)
//   dW_h[n][k] (+)= sum_m dY_h[m][n] X[m][k]
//   db_h[n]    (+)= sum_m dY_h[m][n]
//
// as 64x64 MFMA tiles (v_mfma_f32_16x16x32_bf16, fp32 accumulation).  Workgroup roles by index:
// dX tiles (reduction over both heads' N), then dW tiles of head 0 and head 1, each split RS ways
// over the rows M (the RPN's M = 4200 would leave 16 workgroups otherwise); the dW tile of column
// block 0 also sums db.  With RS > 1 the fp32 row-split partials go to a workspace that a second
// launch folds into the (accumulated) bf16 dW / fp32-or-bf16 db -- deterministic, no atomics.
//
// Operands are staged through LDS as [row][32 reduction elements] (+8 pad) with plain loads: the
// heads' dY rows are N = 24 ... 324 elements, not 16-B aligned, so no LDS-DMA; the next step's
// global values are loaded into registers while the MFMAs of the current step run.
#include "common.h"
#include "../kernels.h"

namespace mxr {

typedef __bf16 hb16x8 __attribute__((ext_vector_type(8)));
typedef float hf32x4 __attribute__((ext_vector_type(4)));

constexpr int HB_R = 32;        // reduction elements per step
constexpr int HB_LD = HB_R + 8; // LDS row (uint16), 80 B

struct HeadStep {
  int h, r0;  // head, first reduction index of this step
};

// NP = 2: the bf16x3 variant (HeadBwdArgs::x2): dY fp32 split into hi / lo in registers, X / W
// read as hi / lo planes, both halves staged in LDS, three MFMAs per fragment pair.  NP = 3: the
// fp32 mode (HeadBwdArgs::x3): (hi, mid, lo) -- LDS planes in that logical order, memory planes
// (mid, hi, lo) (common.h) -- and six MFMAs per fragment pair
template <int NP>
__global__ void __launch_bounds__(256)
head_bwd_kernel(const uint16_t* __restrict__ x, int M, int K, HeadBwdArgs a) {
  constexpr bool X2 = NP >= 2, X3 = NP == 3;
  // memory plane (in units of the plane spacing) of logical plane lp
  auto mpl = [](int lp) -> int64_t { return X3 ? (lp == 0 ? 1 : lp == 1 ? 0 : 2) : lp; };
  __shared__ __attribute__((aligned(16))) uint16_t As[NP][64 * HB_LD];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[NP][64 * HB_LD];
  __shared__ __attribute__((aligned(16))) float T[64 * 68];
  const int64_t xplane = (int64_t)M * K;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tk_n = K / 64;
  const int tm_n = (M + 63) / 64;
  const int n_dx = a.dx ? tm_n * tk_n : 0;
  int t = blockIdx.x;

  // ---- role -------------------------------------------------------------------------------
  bool dx_role = t < n_dx;
  int h = 0, i0 = 0, k0 = 0, split = 0, rb = 0, re = 0;
  if (dx_role) {
    i0 = (t / tk_n) * 64;
    k0 = (t % tk_n) * 64;
  } else {
    t -= n_dx;
    for (h = 0; h < a.nheads; ++h) {
      const int cnt = ((a.N[h] + 63) / 64) * tk_n * a.rs;
      if (t < cnt) break;
      t -= cnt;
    }
    if (h >= a.nheads) return;  // (grid is sized exactly; defensive)
    split = t % a.rs;
    t /= a.rs;
    i0 = (t / tk_n) * 64;  // head-output (n) block
    k0 = (t % tk_n) * 64;
    const int per = (M + a.rs - 1) / a.rs;
    rb = split * per;
    re = min(M, rb + per);
  }
  // reduction steps: dX runs over head 0's N then head 1's; dW over rows [rb, re)
  const int s0 = dx_role ? (a.N[0] + HB_R - 1) / HB_R : 0;
  const int nsteps = dx_role ? s0 + (a.nheads > 1 ? (a.N[1] + HB_R - 1) / HB_R : 0) : (re - rb + HB_R - 1) / HB_R;
  auto step_of = [&](int s) -> HeadStep {
    HeadStep st;
    if (dx_role) {
      st.h = s < s0 ? 0 : 1;
      st.r0 = (s < s0 ? s : s - s0) * HB_R;
    } else {
      st.h = h;
      st.r0 = rb + s * HB_R;
    }
    return st;
  };

  // ---- register stage: 8 A values + one 16-B B vector per thread (per plane) ---------------
  uint16_t ra[NP][8];
  uint4 rbv[NP];
  // dY element (m, n) of head h as (hi, lo) or (hi, mid, lo) bf16 (unused planes 0)
  auto dy_at = [&](int hh, int Nh, int64_t idx, uint16_t& hi, uint16_t& lo, uint16_t& l2) {
    l2 = 0;
    if constexpr (X3) {
      split3_bf16(a.dyf[hh][idx], hi, lo, l2);
    } else if constexpr (X2) {
      split_bf16(a.dyf[hh][idx], hi, lo);
    } else {
      hi = a.dy[hh][idx];
      lo = 0;
    }
  };
  auto load = [&](int s) {
    const HeadStep st = step_of(s);
    const int Nh = a.N[st.h];
    if (dx_role) {
      // A(i = m, r = n) = dY[m][n]: thread -> row i, 8 consecutive r
      const int i = tid >> 2, rq = (tid & 3) * 8;
      const int m = i0 + i;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int n = st.r0 + rq + e;
        uint16_t hi = 0, lo = 0, l2 = 0;
        if (m < M && n < Nh) dy_at(st.h, Nh, (int64_t)m * Nh + n, hi, lo, l2);
        ra[0][e] = hi;
        if constexpr (X2) ra[1][e] = lo;
        if constexpr (X3) ra[2][e] = l2;
      }
      // B(r = n, j = k) = W[n][k]
      const int r = tid >> 3, jq = (tid & 7) * 8;
      const int n = st.r0 + r;
#pragma unroll
      for (int pl = 0; pl < NP; ++pl)
        rbv[pl] = n < Nh ? *reinterpret_cast<const uint4*>(a.w[st.h] + mpl(pl) * a.w_plane[st.h] + (int64_t)n * K + k0 + jq)
                         : make_uint4(0, 0, 0, 0);
    } else {
      // A(i = n, r = m) = dY[m][n]: thread -> row r, 8 consecutive i
      const int r = tid >> 3, iq = (tid & 7) * 8;
      const int m = st.r0 + r;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int n = i0 + iq + e;
        uint16_t hi = 0, lo = 0, l2 = 0;
        if (m < re && n < Nh) dy_at(st.h, Nh, (int64_t)m * Nh + n, hi, lo, l2);
        ra[0][e] = hi;
        if constexpr (X2) ra[1][e] = lo;
        if constexpr (X3) ra[2][e] = l2;
      }
      // B(r = m, j = k) = X[m][k]
#pragma unroll
      for (int pl = 0; pl < NP; ++pl)
        rbv[pl] = m < re ? *reinterpret_cast<const uint4*>(x + mpl(pl) * xplane + (int64_t)m * K + k0 + (tid & 7) * 8)
                         : make_uint4(0, 0, 0, 0);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int pl = 0; pl < NP; ++pl) {
      if (dx_role) {
        const int i = tid >> 2, rq = (tid & 3) * 8;
        uint4 v;
        v.x = (uint32_t)ra[pl][0] | ((uint32_t)ra[pl][1] << 16);
        v.y = (uint32_t)ra[pl][2] | ((uint32_t)ra[pl][3] << 16);
        v.z = (uint32_t)ra[pl][4] | ((uint32_t)ra[pl][5] << 16);
        v.w = (uint32_t)ra[pl][6] | ((uint32_t)ra[pl][7] << 16);
        *reinterpret_cast<uint4*>(As[pl] + i * HB_LD + rq) = v;
      } else {
        const int r = tid >> 3, iq = (tid & 7) * 8;
#pragma unroll
        for (int e = 0; e < 8; ++e) As[pl][(iq + e) * HB_LD + r] = ra[pl][e];
      }
      const int r = tid >> 3, jq = (tid & 7) * 8;
      const uint32_t bw[4] = {rbv[pl].x, rbv[pl].y, rbv[pl].z, rbv[pl].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        Bs[pl][(jq + 2 * e) * HB_LD + r] = (uint16_t)(bw[e] & 0xffffu);
        Bs[pl][(jq + 2 * e + 1) * HB_LD + r] = (uint16_t)(bw[e] >> 16);
      }
    }
  };

  hf32x4 acc[2][2];
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int q = 0; q < 2; ++q) acc[p][q] = hf32x4{0.f, 0.f, 0.f, 0.f};
  if (nsteps > 0) load(0);
  for (int s = 0; s < nsteps; ++s) {
    __syncthreads();  // the previous step's fragment reads are done
    store();
    __syncthreads();
    if (s + 1 < nsteps) load(s + 1);  // in flight during the MFMAs
    const int kc = (lane >> 4) * 8;
    hb16x8 af[NP][2], bf[NP][2];
#pragma unroll
    for (int pl = 0; pl < NP; ++pl) {
#pragma unroll
      for (int p = 0; p < 2; ++p)
        af[pl][p] = *reinterpret_cast<const hb16x8*>(As[pl] + (wm * 32 + p * 16 + (lane & 15)) * HB_LD + kc);
#pragma unroll
      for (int q = 0; q < 2; ++q)
        bf[pl][q] = *reinterpret_cast<const hb16x8*>(Bs[pl] + (wn * 32 + q * 16 + (lane & 15)) * HB_LD + kc);
    }
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        acc[p][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][p], bf[0][q], acc[p][q], 0, 0, 0);
        if constexpr (X2) {
          acc[p][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][p], bf[1][q], acc[p][q], 0, 0, 0);
          acc[p][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1][p], bf[0][q], acc[p][q], 0, 0, 0);
        }
        if constexpr (X3) {  // (hi, lo), (lo, hi), (mid, mid)
          acc[p][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][p], bf[2][q], acc[p][q], 0, 0, 0);
          acc[p][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[2][p], bf[0][q], acc[p][q], 0, 0, 0);
          acc[p][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1][p], bf[1][q], acc[p][q], 0, 0, 0);
        }
      }
  }

  // ---- epilogue through LDS: T[i][j] fp32, then 8-wide rows ---------------------------------
  // C/D layout of the 16x16 MFMA: lane holds rows (lane >> 4) * 4 + v, column lane & 15
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int v = 0; v < 4; ++v)
        T[(wm * 32 + p * 16 + (lane >> 4) * 4 + v) * 68 + wn * 32 + q * 16 + (lane & 15)] = acc[p][q][v];
  __syncthreads();
  const int Nh = a.N[h];
#pragma unroll
  for (int vv = 0; vv < 2; ++vv) {
    const int e = tid + vv * 256, row = e >> 3, cv = (e & 7) * 8;
    const int i = i0 + row;
    const float4 p0 = *reinterpret_cast<const float4*>(T + row * 68 + cv);
    const float4 p1 = *reinterpret_cast<const float4*>(T + row * 68 + cv + 4);
    float v8[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
    if (dx_role) {
      if (i >= M) continue;
      const int64_t o = (int64_t)i * K + k0 + cv;
      if (a.relu_mask) {
        float xv[8];
        if constexpr (X2) ld8x(x + o, xplane, xv, X3);
        else ld8_bf16(x + o, xv);
#pragma unroll
        for (int q = 0; q < 8; ++q) v8[q] = xv[q] > 0.f ? v8[q] * a.mask_scale : 0.f;
      }
      if constexpr (X2) st8x(a.dx + o, xplane, v8, v8, X3);
      else st8_bf16(a.dx + o, v8);
    } else {
      if (i >= Nh) continue;
      const int64_t o = (int64_t)i * K + k0 + cv;
      if (a.rs > 1) {
        float* wp = a.ws_dw[h] + (int64_t)split * Nh * K + o;
        *reinterpret_cast<float4*>(wp) = p0;
        *reinterpret_cast<float4*>(wp + 4) = p1;
      } else if constexpr (X2) {  // fp32 dW
        float4* d = reinterpret_cast<float4*>(a.dwf[h] + o);
        if (a.dw_acc[h]) {
          const float4 q0 = d[0], q1 = d[1];
          d[0] = make_float4(p0.x + q0.x, p0.y + q0.y, p0.z + q0.z, p0.w + q0.w);
          d[1] = make_float4(p1.x + q1.x, p1.y + q1.y, p1.z + q1.z, p1.w + q1.w);
        } else {
          d[0] = p0;
          d[1] = p1;
        }
      } else {
        if (a.dw_acc[h]) {
          float prev[8];
          ld8_bf16(a.dw[h] + o, prev);
#pragma unroll
          for (int q = 0; q < 8; ++q) v8[q] += prev[q];
        }
        st8_bf16(a.dw[h] + o, v8);
      }
    }
  }
  // ---- db: the column-block-0 dW tile of each (head, n block, split) --------------------------
  if (dx_role || k0 != 0 || a.db[h] == nullptr) return;
  {
    float* red = T;  // reuse: [4][64]
    __syncthreads();
    const int i = tid & 63, qq = tid >> 6;
    const int n = i0 + i;
    float s = 0.f;
    if (n < Nh)
      for (int m = rb + qq; m < re; m += 4) {
        if constexpr (X2) s += a.dyf[h][(int64_t)m * Nh + n];
        else s += bf16_to_f32(a.dy[h][(int64_t)m * Nh + n]);
      }
    red[qq * 64 + i] = s;
    __syncthreads();
    if (tid < 64 && n < Nh) {
      const float tot = red[i] + red[64 + i] + red[128 + i] + red[192 + i];
      if (a.rs > 1) {
        a.ws_db[h][(int64_t)split * Nh + n] = tot;
      } else {
        const float prev = a.db_acc[h] ? ld(a.db[h], n, a.db_code[h]) : 0.f;
        st(a.db[h], n, prev + tot, a.db_code[h]);
      }
    }
  }
}

// rs > 1: fold the row-split partials of head h into dW (bf16, accumulated when asked) and db
__global__ void __launch_bounds__(256)
head_bwd_fold_kernel(int K, HeadBwdArgs a, int h) {
  const int Nh = a.N[h];
  const int64_t nw = (int64_t)Nh * K;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < nw) {
    float s = 0.f;
#pragma unroll 8
    for (int r = 0; r < a.rs; ++r) s += a.ws_dw[h][(int64_t)r * nw + e];
    if (a.x2) {
      if (a.dw_acc[h]) s += a.dwf[h][e];
      a.dwf[h][e] = s;
    } else {
      if (a.dw_acc[h]) s += bf16_to_f32(a.dw[h][e]);
      a.dw[h][e] = f32_to_bf16(s);
    }
  } else if (e < nw + Nh && a.db[h] != nullptr) {
    const int n = (int)(e - nw);
    float s = 0.f;
#pragma unroll 8
    for (int r = 0; r < a.rs; ++r) s += a.ws_db[h][(int64_t)r * Nh + n];
    if (a.db_acc[h]) s += ld(a.db[h], n, a.db_code[h]);
    st(a.db[h], n, s, a.db_code[h]);
  }
}

int head_bwd_splits(int M, int K, const int* N, int nheads) {
  if (M <= 256) return 1;
  int tiles = 0;
  for (int h = 0; h < nheads; ++h) tiles += ((N[h] + 63) / 64) * (K / 64);
  int rs = 1;
  while (tiles * rs * 2 <= 512 && M / (rs * 2) >= 64) rs *= 2;
  return rs;
}

int head_bwd(const uint16_t* x, int M, int K, const HeadBwdArgs& a, hipStream_t st) {
  if (K % 64 != 0 || M <= 0 || a.nheads < 1 || a.nheads > 2 || a.rs < 1) return -1;
  const int tk_n = K / 64;
  int64_t nwg = a.dx ? (int64_t)((M + 63) / 64) * tk_n : 0;
  for (int h = 0; h < a.nheads; ++h) {
    if (a.N[h] <= 0) return -1;
    nwg += (int64_t)((a.N[h] + 63) / 64) * tk_n * a.rs;
  }
  if (a.x3) head_bwd_kernel<3><<<(unsigned)nwg, 256, 0, st>>>(x, M, K, a);
  else if (a.x2) head_bwd_kernel<2><<<(unsigned)nwg, 256, 0, st>>>(x, M, K, a);
  else head_bwd_kernel<1><<<(unsigned)nwg, 256, 0, st>>>(x, M, K, a);
  if (a.rs > 1)
    for (int h = 0; h < a.nheads; ++h)
      head_bwd_fold_kernel<<<div_up((int64_t)a.N[h] * K + a.N[h], 256), 256, 0, st>>>(K, a, h);
  return 0;
}

// ---- per-channel sum of an NHWC map (conv bias gradient) -------------------------------------
// Two launches, deterministic: row-chunk partials of 64-channel blocks (grid >= ~512 workgroups
// for the RPN's 4200 x 512 map, where torch's reduction ran on 2 workgroups, 10-15 us), then the
// fold into the (accumulated) fp32 / bf16 bias gradient.
__global__ void __launch_bounds__(256)
chan_sum_part_kernel(const uint16_t* __restrict__ x, int64_t M, int C, int rows, int code, float* __restrict__ part) {
  __shared__ float red[32][65];
  const int cg = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c0 = blockIdx.x * 64 + cg * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rows;
  const int64_t r1 = r0 + rows < M ? r0 + rows : M;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < C)
    for (int64_t r = r0 + rl; r < r1; r += 32) {
      float v[8];
      ld8c(x, r * C + c0, code, M * C, v);  // code 3 / 4: x2 / x3 planes M * C apart
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += v[k];
    }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[rl][cg * 8 + k] = s[k];
  __syncthreads();
  if (threadIdx.x < 64) {
    float t = 0.f;
    for (int r = 0; r < 32; ++r) t += red[r][threadIdx.x];
    const int c = blockIdx.x * 64 + threadIdx.x;
    if (c < C) part[(int64_t)blockIdx.y * C + c] = t;
  }
}

// one workgroup per 64 channels, 4 threads per channel over interleaved chunks (loads in flight
// instead of one thread walking ~100 dependent L2 loads)
__global__ void __launch_bounds__(256)
chan_sum_fold_kernel(const float* __restrict__ part, int nchunks, int C, void* __restrict__ out, int out_code,
                     int accumulate) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float s = 0.f;
  if (c < C) {
#pragma unroll 8
    for (int i = q; i < nchunks; i += 4) s += part[(int64_t)i * C + c];
  }
  red[q][cl] = s;
  __syncthreads();
  if (q == 0 && c < C) {
    float t = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
    if (accumulate) t += ld(out, c, out_code);
    st(out, c, t, out_code);
  }
}

int chan_sum_chunks(int64_t M, int C) {
  int rows = 256;
  while (rows > 32 && (int64_t)((C + 63) / 64) * ((M + rows - 1) / rows) < 512) rows >>= 1;
  return (int)((M + rows - 1) / rows);
}

int chan_sum(const uint16_t* x, int64_t M, int C, int code, float* part, void* out, int out_code, int accumulate,
             hipStream_t st) {
  if (C % 8 != 0 || M <= 0) return -1;
  const int nchunks = chan_sum_chunks(M, C);
  const int rows = (int)((M + nchunks - 1) / nchunks);
  chan_sum_part_kernel<<<dim3(div_up(C, 64), nchunks), 256, 0, st>>>(x, M, C, rows, code, part);
  chan_sum_fold_kernel<<<div_up(C, 64), 256, 0, st>>>(part, nchunks, C, out, out_code, accumulate);
  return 0;
}

}  // namespace mxr
