// KAN path: efficient-KAN `KANLinear` layers (kan.py:6-166):
//   A = [ SiLU(X) | B-spline bases of X ]   [N][9 in]   (grid 5, order 3)
//   Out = A W^T,  W = [ base_weight | spline_weight * spline_scaler ]  [out][9 in]
// and its autograd: dW = G^T A, dA = G W, dX = SiLU'(X) dA_base + sum_c B'_c(X) dA_spline_c.
//
// A and dA are never materialised (round 2; the first design wrote and re-read A / dA, 2.3 KB
// per coordinate each at width 64, ~26 KB of HBM per coordinate-step).  Three fused kernels
// recompute the bases of an (8-input x 64-row) chunk into LDS where they are consumed:
//   kan_fwd_fused  Out tile [64 rows][64 outs] = sum over input chunks of A_chunk W_chunk^T
//   kan_dw_fused   dW chunk [out][72] += G[rows]^T A_chunk[rows]   (split-K over rows, slabs)
//   kan_dx_fused   dA_chunk = G W_chunk (in LDS), contracted at once with the bases' derivatives
// Everything is fp32 like the reference.  The bases follow kan.py:94-104's Cox-de Boor
// recursion op for op (sub, div, mul, add; fp-contract off) on the layer's own `grid` buffer,
// so they are bit-identical to torch's CPU result; the derivative differentiates the same
// recursion.  The GEMMs are short (K = 9 in <= 2304, out <= 256): LDS-tiled VALU FMAs, not MFMA
// (SURVEY §8 f4).
#include "siren_common.h"
#include "siren_kernels.h"

namespace siren {

constexpr int KAN_NB = 8;       // grid_size + spline_order bases per input
constexpr int KAN_NG = 12;      // grid knots per input: grid_size + 2 * spline_order + 1
constexpr int KAN_K1 = 1 + KAN_NB;  // columns of A per input feature

// Cox-de Boor recursion of kan.py:94-104 for one x on one input's knots g[0..11]: order-0
// bases B[j] = (g[j] <= x < g[j+1]), then for k = 1..3
//   B[j] = ((x - g[j]) / (g[j+k] - g[j])) * B[j] + ((g[j+k+1] - x) / (g[j+k+1] - g[j+1])) * B[j+1]
// (each product rounded, then the sum: fp-contract off), and with DERIV the recursion
// differentiated in x.
// Evaluated on its support only.  An order-0 basis is 1 on at most one
// knot span s (g[s] <= x < g[s+1], the same predicate), so after step k only B[s-k .. s] can be
// non-zero; every other term of the full recursion is l*0 + r*0 = +-0 and, where it meets a
// non-zero term, x + (+-0) = x.  Computing the window terms with the same operations in the
// same order therefore gives the full recursion's values bit for bit (zeros up to sign), at 18
// instead of 54 divisions (36 instead of 108 with the derivative).  The knots are read through
// the pointer (a runtime-indexed register array would live in scratch).
// RCP (backward kernels): the knot-difference divisions become products with reciprocals
// inv[(k-1)*11 + j] = 1 / (g[j+k] - g[j]) precomputed per input (kf_fill_inv) -- within an ulp or
// two of the divisions, which only the weight / input gradients see (the forward keeps the exact
// divisions, so its bases stay bit-identical to torch's).
template <bool DERIV, bool RCP = false>
__device__ __forceinline__ void kan_bases_local(float x, const float* __restrict__ g, float* b, float* db,
                                                const float* __restrict__ inv = nullptr) {
#pragma unroll
  for (int j = 0; j < KAN_NB; ++j) b[j] = db[j] = 0.0f;
  int s = -1;
#pragma unroll
  for (int j = 0; j < KAN_NG - 1; ++j)
    if (x >= g[j] && x < g[j + 1]) s = j;
  if (s < 0) return;
  // window w[q] = B[s - 3 + q], q = 0..3, plus w[4] = B[s + 1] = 0
  float w[5] = {0.0f, 0.0f, 0.0f, 1.0f, 0.0f}, d[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int k = 1; k <= 3; ++k) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = s - 3 + q;
      if (q < 3 - k || j < 0 || j > KAN_NG - 2 - k) continue;  // outside the support / the array
      const float gj = g[j], gjk = g[j + k], gj1 = g[j + 1], gjk1 = g[j + k + 1];
      float il, ir, l, r;
      if constexpr (RCP) {
        il = inv[(k - 1) * 11 + j];
        ir = inv[(k - 1) * 11 + j + 1];
        l = (x - gj) * il;
        r = (gjk1 - x) * ir;
      } else {
        il = 1.0f / (gjk - gj);
        ir = 1.0f / (gjk1 - gj1);
        l = (x - gj) / (gjk - gj);
        r = (gjk1 - x) / (gjk1 - gj1);
      }
      if constexpr (DERIV) d[q] = il * w[q] + l * d[q] - ir * w[q + 1] + r * d[q + 1];
      w[q] = l * w[q] + r * w[q + 1];
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int j = s - 3 + q;
    if (j >= 0 && j < KAN_NB) {
      b[j] = w[q];
      if constexpr (DERIV) db[j] = d[q];
    }
  }
}

__device__ __forceinline__ float silu(float x) { return x / (1.0f + expf(-x)); }
__device__ __forceinline__ float silu_grad(float x) {
  const float s = 1.0f / (1.0f + expf(-x));
  return s * (1.0f + x * (1.0f - s));
}

// ---- fused layer kernels --------------------------------------------------------------------
// Chunk of IC inputs i0 .. i0+ic-1 (ic <= IC): local column kk < ic is the SiLU column of input
// i0+kk (combined-weight column k = i0+kk), kk = ic + 8 ii + c the spline basis c of input i0+ii
// (k = in + 8 (i0+ii) + c).
constexpr int KF_IC = 8, KF_KC = 9 * KF_IC, KF_R = 64, KF_O = 64;

__device__ __forceinline__ int kf_col(int kk, int ic, int i0, int in) {
  return kk < ic ? i0 + kk : in + 8 * i0 + (kk - ic);
}

// As[kk][r] (r < 64 rows of the tile, pad 4) = A columns of the chunk for rows r0 + r; rows past N
// are zero.  Every thread takes pairs (r, ii).
template <bool RCP = false>
__device__ __forceinline__ void kf_fill_a(float (*As)[KF_R + 4], const float* __restrict__ X,
                                          const float* __restrict__ grid, int64_t N, int in, int64_t r0, int i0,
                                          int ic, float (*inv)[33] = nullptr) {
  for (int p = threadIdx.x; p < KF_R * ic; p += blockDim.x) {
    const int r = p / ic, ii = p - r * ic;
    const int64_t n = r0 + r;
    float b[KAN_NB], unused[KAN_NB], sl = 0.f;
    if (n < N) {
      const float x = X[n * in + i0 + ii];
      kan_bases_local<false, RCP>(x, grid + (i0 + ii) * KAN_NG, b, unused, RCP ? inv[ii] : nullptr);
      sl = silu(x);
    } else {
#pragma unroll
      for (int c = 0; c < KAN_NB; ++c) b[c] = 0.f;
    }
    As[ii][r] = sl;
#pragma unroll
    for (int c = 0; c < KAN_NB; ++c) As[ic + 8 * ii + c][r] = b[c];
  }
}

// Y[n][o] = sum_k A[n][k] W[o][k]; grid (ceil(N/64), ceil(out/64)); 4x4 outputs per thread.
__global__ __launch_bounds__(256) void kan_fwd_fused_kernel(const float* __restrict__ X, const float* __restrict__ grid,
                                                            const float* __restrict__ W, int64_t N, int in, int out,
                                                            float* __restrict__ Y) {
  __shared__ __attribute__((aligned(16))) float As[KF_KC][KF_R + 4];
  __shared__ __attribute__((aligned(16))) float Ws[KF_KC][KF_O + 4];
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * KF_R;
  const int o0 = blockIdx.y * KF_O;
  const int tm = (tid >> 4) * 4, tn = (tid & 15) * 4;
  const int64_t K = (int64_t)KAN_K1 * in;
  float acc[4][4] = {};
  for (int i0 = 0; i0 < in; i0 += KF_IC) {
    const int ic = in - i0 < KF_IC ? in - i0 : KF_IC, kc = 9 * ic;
    kf_fill_a(As, X, grid, N, in, r0, i0, ic);
    for (int e = tid; e < KF_O * kc; e += blockDim.x) {
      const int o = e / kc, kk = e - o * kc;
      Ws[kk][o] = (o0 + o < out) ? W[(int64_t)(o0 + o) * K + kf_col(kk, ic, i0, in)] : 0.f;
    }
    __syncthreads();
    for (int kk = 0; kk < kc; ++kk) {
      const float4 a = *(const float4*)&As[kk][tm];
      const float4 w = *(const float4*)&Ws[kk][tn];
      const float av[4] = {a.x, a.y, a.z, a.w}, wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += av[i] * wv[j];
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t n = r0 + tm + i;
      const int o = o0 + tn + j;
      if (n < N && o < out) Y[n * out + o] = acc[i][j];
    }
}

// inv[ii][(k-1)*11 + j] = 1 / (g[j+k] - g[j]) for the knots of inputs i0 .. i0+ic-1 (RCP bases)
__device__ __forceinline__ void kf_fill_inv(float (*inv)[33], const float* __restrict__ grid, int i0, int ic) {
  for (int e = threadIdx.x; e < ic * 33; e += blockDim.x) {
    const int ii = e / 33, q = e - ii * 33, k = q / 11 + 1, j = q - (k - 1) * 11;
    const float* g = grid + (i0 + ii) * KAN_NG;
    inv[ii][q] = (j + k < KAN_NG) ? 1.0f / (g[j + k] - g[j]) : 0.0f;
  }
}

// ---- the last layer (out = 1): one wave per row, lane = input (strided by 64) -------------
// out[n] = sum_i SiLU(x_i) W[i] + sum_c B_c(x_i) W[in + 8 i + c], a fixed-order wave sum.
__global__ __launch_bounds__(256) void kan_head_fwd_kernel(const float* __restrict__ X, const float* __restrict__ grid,
                                                           const float* __restrict__ W, int64_t N, int in,
                                                           float* __restrict__ Y) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t n = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); n < N; n += nw) {
    float v = 0.f;
    for (int i = lane; i < in; i += 64) {
      const float x = X[n * in + i];
      float b[KAN_NB], unused[KAN_NB];
      kan_bases_local<false>(x, grid + i * KAN_NG, b, unused);
      v += silu(x) * W[i];
#pragma unroll
      for (int c = 0; c < KAN_NB; ++c) v += b[c] * W[in + KAN_NB * i + c];
    }
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) Y[n] = v;
  }
}

// Backward of the last layer for dLoss/dout = g: weight-gradient partials of this wave's rows
// (slab[wave][k], summed later in fixed order) and Gin[n][i] = g_n (SiLU'(x) W[i] + sum_c B'_c(x)
// W[in + 8 i + c]) -- dA = g W is a rank-1 product, so it is never formed.  Each wave takes a
// contiguous run of rows; lanes own inputs (in <= 64).
__global__ __launch_bounds__(256) void kan_head_bwd_kernel(const float* __restrict__ X, const float* __restrict__ grid,
                                                           const float* __restrict__ W, const float* __restrict__ g,
                                                           int64_t N, int in, int64_t rows_per_wave,
                                                           float* __restrict__ slab, float* __restrict__ Gin) {
  __shared__ float inv[64][33];
  kf_fill_inv(inv, grid, 0, in);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t wv = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t nb = wv * rows_per_wave;
  const int64_t ne = nb + rows_per_wave < N ? nb + rows_per_wave : N;
  const bool on = lane < in;
  float wb = 0.f, ws[KAN_NB] = {};
  if (on) {
    wb = W[lane];
#pragma unroll
    for (int c = 0; c < KAN_NB; ++c) ws[c] = W[in + KAN_NB * lane + c];
  }
  float ab = 0.f, as[KAN_NB] = {};
  for (int64_t n = nb; n < ne; ++n) {
    if (!on) continue;
    const float gn = g[n];
    const float x = X[n * in + lane];
    float b[KAN_NB], db[KAN_NB];
    kan_bases_local<true, true>(x, grid + lane * KAN_NG, b, db, inv[lane]);
    ab += gn * silu(x);
    float v = silu_grad(x) * wb;
#pragma unroll
    for (int c = 0; c < KAN_NB; ++c) {
      as[c] += gn * b[c];
      v += db[c] * ws[c];
    }
    Gin[n * in + lane] = gn * v;
  }
  if (on) {
    float* row = slab + wv * (int64_t)KAN_K1 * in;
    row[lane] = ab;
#pragma unroll
    for (int c = 0; c < KAN_NB; ++c) row[in + KAN_NB * lane + c] = as[c];
  }
}

// slab[z][o][k] = sum over rows of split z of G[n][o] A[n][k], for the chunk's columns k;
// grid (ceil(in/IC), ceil(out/64), splits).  Thread: 2 outputs x 9 chunk columns.
__global__ __launch_bounds__(256) void kan_dw_fused_kernel(const float* __restrict__ X, const float* __restrict__ grid,
                                                           const float* __restrict__ G, int64_t N, int in, int out,
                                                           int64_t rows_per_split, float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) float As[KF_KC][KF_R + 4];
  __shared__ __attribute__((aligned(16))) float Gs[KF_R][KF_O + 4];
  __shared__ float inv[KF_IC][33];
  const int tid = threadIdx.x;
  const int i0 = blockIdx.x * KF_IC, o0 = blockIdx.y * KF_O;
  const int ic = in - i0 < KF_IC ? in - i0 : KF_IC, kc = 9 * ic;
  kf_fill_inv(inv, grid, i0, ic);
  __syncthreads();
  const int64_t rb = (int64_t)blockIdx.z * rows_per_split;
  const int64_t re = rb + rows_per_split < N ? rb + rows_per_split : N;
  const int og = (tid & 31) * 2, kg = (tid >> 5) * 9;  // outs og, og+1; chunk columns kg .. kg+8
  float acc[2][9] = {};
  for (int64_t r0 = rb; r0 < re; r0 += KF_R) {
    kf_fill_a<true>(As, X, grid, re, in, r0, i0, ic, inv);
    for (int e = tid; e < KF_R * KF_O; e += blockDim.x) {
      const int r = e / KF_O, o = e - r * KF_O;
      Gs[r][o] = (r0 + r < re && o0 + o < out) ? G[(r0 + r) * out + o0 + o] : 0.f;
    }
    __syncthreads();
    if (kg < kc) {
      for (int r = 0; r < KF_R; ++r) {
        const float2 g = *(const float2*)&Gs[r][og];
#pragma unroll
        for (int j = 0; j < 9; ++j) {
          const float a = As[kg + j][r];
          acc[0][j] += g.x * a;
          acc[1][j] += g.y * a;
        }
      }
    }
    __syncthreads();
  }
  const int64_t K = (int64_t)KAN_K1 * in;
  float* out_slab = slab + (int64_t)blockIdx.z * out * K;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int o = o0 + og + h, kk = kg + j;
      if (o < out && kk < kc) out_slab[(int64_t)o * K + kf_col(kk, ic, i0, in)] = acc[h][j];
    }
}

// Gin[n][i] = SiLU'(x) dA[n][i] + sum_c B'_c(x) dA[n][in + 8 i + c], dA = Gout W (never stored);
// grid (ceil(N/64), ceil(in/IC)).  dA chunk: thread = 2 rows x 9 chunk columns, over out in chunks
// of 64.
__global__ __launch_bounds__(256) void kan_dx_fused_kernel(const float* __restrict__ X, const float* __restrict__ grid,
                                                           const float* __restrict__ Gout, const float* __restrict__ W,
                                                           int64_t N, int in, int out, float* __restrict__ Gin) {
  __shared__ __attribute__((aligned(16))) float Gs[KF_O][KF_R + 4];   // [o][r]
  __shared__ __attribute__((aligned(16))) float Ws[KF_O][KF_KC + 4];  // [o][kk]
  __shared__ __attribute__((aligned(16))) float dAs[KF_R][KF_KC + 1];
  __shared__ float inv[KF_IC][33];
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * KF_R;
  const int i0 = blockIdx.y * KF_IC;
  const int ic = in - i0 < KF_IC ? in - i0 : KF_IC, kc = 9 * ic;
  kf_fill_inv(inv, grid, i0, ic);
  const int64_t K = (int64_t)KAN_K1 * in;
  const int rg = (tid & 31) * 2, kg = (tid >> 5) * 9;  // rows rg, rg+1; chunk columns kg .. kg+8
  float acc[2][9] = {};
  for (int oc = 0; oc < out; oc += KF_O) {
    const int on = out - oc < KF_O ? out - oc : KF_O;
    for (int e = tid; e < KF_R * on; e += blockDim.x) {
      const int r = e / on, o = e - r * on;
      Gs[o][r] = (r0 + r < N) ? Gout[(r0 + r) * out + oc + o] : 0.f;
    }
    for (int e = tid; e < on * kc; e += blockDim.x) {
      const int o = e / kc, kk = e - o * kc;
      Ws[o][kk] = W[(int64_t)(oc + o) * K + kf_col(kk, ic, i0, in)];
    }
    __syncthreads();
    if (kg < kc) {
      for (int o = 0; o < on; ++o) {
        const float2 g = *(const float2*)&Gs[o][rg];
#pragma unroll
        for (int j = 0; j < 9; ++j) {
          const float w = Ws[o][kg + j];
          acc[0][j] += g.x * w;
          acc[1][j] += g.y * w;
        }
      }
    }
    __syncthreads();
  }
  if (kg < kc) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 9; ++j) dAs[rg + h][kg + j] = acc[h][j];
  }
  __syncthreads();
  for (int p = tid; p < KF_R * ic; p += blockDim.x) {
    const int r = p / ic, ii = p - r * ic;
    const int64_t n = r0 + r;
    if (n >= N) continue;
    const float x = X[n * in + i0 + ii];
    float b[KAN_NB], db[KAN_NB];
    kan_bases_local<true, true>(x, grid + (i0 + ii) * KAN_NG, b, db, inv[ii]);
    float v = silu_grad(x) * dAs[r][ii];
#pragma unroll
    for (int c = 0; c < KAN_NB; ++c) v += db[c] * dAs[r][ic + 8 * ii + c];
    Gin[n * in + i0 + ii] = v;
  }
}

// W[o][i] = base_w[o][i];  W[o][in + 8 i + c] = spline_w[o][i][c] * scaler[o][i]  (kan.py:145-151)
__global__ void kan_combine_kernel(const float* __restrict__ base_w, const float* __restrict__ spline_w,
                                   const float* __restrict__ scaler, int out, int in, float* __restrict__ W) {
  const int total = out * in;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int o = e / in, i = e - o * in;
    float* row = W + (int64_t)o * KAN_K1 * in;
    row[i] = base_w[e];
    const float s = scaler[e];
#pragma unroll
    for (int c = 0; c < KAN_NB; ++c) row[in + KAN_NB * i + c] = spline_w[(int64_t)e * KAN_NB + c] * s;
  }
}

// Parameter gradients from dW = dLoss/dW_combined (the autograd of kan_combine):
//   d base_w = dW_base;  d spline_w = dW_spline * scaler;  d scaler = sum_c dW_spline * spline_w
__global__ void kan_param_grads_kernel(const float* __restrict__ dW, const float* __restrict__ spline_w,
                                       const float* __restrict__ scaler, int out, int in, int accumulate,
                                       float* __restrict__ g_base, float* __restrict__ g_spline,
                                       float* __restrict__ g_scaler) {
  const int total = out * in;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int o = e / in, i = e - o * in;
    const float* row = dW + (int64_t)o * KAN_K1 * in;
    const float s = scaler[e];
    float gs = 0.f;
#pragma unroll
    for (int c = 0; c < KAN_NB; ++c) {
      const float d = row[in + KAN_NB * i + c];
      const int64_t k = (int64_t)e * KAN_NB + c;
      const float v = d * s;
      g_spline[k] = accumulate ? g_spline[k] + v : v;
      gs += d * spline_w[k];
    }
    g_base[e] = accumulate ? g_base[e] + row[i] : row[i];
    g_scaler[e] = accumulate ? g_scaler[e] + gs : gs;
  }
}

// ---- strided fp32 GEMM:  C[m][n] = sum_k A(m, k) B(k, n) --------------------------------
// A(m, k) = A[m*sam + k*sak], B(k, n) = B[k*sbk + n*sbn]; 64x64 tile, BK 16, 256 threads,
// 4x4 outputs per thread; split-K over blockIdx.z writes slab z of C (C + z*M*N) which
// kan_slab_reduce sums in fixed order.  Bounds-checked (zero fill) for any M, N, K.
constexpr int KG_T = 64, KG_BK = 16;

__global__ __launch_bounds__(256) void kan_gemm_kernel(const float* __restrict__ A, int64_t sam, int64_t sak,
                                                       const float* __restrict__ B, int64_t sbk, int64_t sbn,
                                                       float* __restrict__ C, int M, int N, int64_t K,
                                                       int64_t kchunk) {
  __shared__ float As[KG_BK][KG_T + 4];
  __shared__ float Bs[KG_BK][KG_T + 4];
  const int tid = threadIdx.x;
  const int m0 = blockIdx.y * KG_T, n0 = blockIdx.x * KG_T;
  const int64_t kb = (int64_t)blockIdx.z * kchunk;
  const int64_t ke = (kb + kchunk < K) ? kb + kchunk : K;
  C += (int64_t)blockIdx.z * M * N;
  const int tm = (tid / 16) * 4, tn = (tid % 16) * 4;
  float acc[4][4] = {};
  // loader index -> (k, m) with the unit-stride dimension fastest across threads (coalesced)
  const bool a_k_fast = (sak == 1), b_k_fast = (sbk == 1);
  for (int64_t k0 = kb; k0 < ke; k0 += KG_BK) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int idx = tid + r * 256;
      int kk, mm;
      if (a_k_fast) { kk = idx % KG_BK; mm = idx / KG_BK; } else { kk = idx / KG_T; mm = idx % KG_T; }
      const int64_t k = k0 + kk;
      const int m = m0 + mm;
      As[kk][mm] = (k < ke && m < M) ? A[(int64_t)m * sam + k * sak] : 0.f;
      int nn;
      if (b_k_fast) { kk = idx % KG_BK; nn = idx / KG_BK; } else { kk = idx / KG_T; nn = idx % KG_T; }
      const int64_t kq = k0 + kk;
      const int n = n0 + nn;
      Bs[kk][nn] = (kq < ke && n < N) ? B[kq * sbk + (int64_t)n * sbn] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < KG_BK; ++kk) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[kk][tm + i];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = Bs[kk][tn + j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += a[i] * b[j];
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + tm + i, n = n0 + tn + j;
      if (m < M && n < N) C[(int64_t)m * N + n] = acc[i][j];
    }
}

__global__ void kan_slab_reduce_kernel(const float* __restrict__ slab, int splits, int64_t mn,
                                       float* __restrict__ out) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < mn; e += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int z = 0; z < splits; ++z) s += slab[z * mn + e];
    out[e] = s;
  }
}

static inline int ew_grid(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}

hipError_t kan_fwd_fused(const float* X, const float* grid, const float* W, int64_t N, int in, int out, float* Y,
                         hipStream_t s) {
  if (N <= 0 || in <= 0 || out <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kan_fwd_fused_kernel, dim3((unsigned)((N + KF_R - 1) / KF_R), (out + KF_O - 1) / KF_O), dim3(256),
                     0, s, X, grid, W, N, in, out, Y);
  return hipGetLastError();
}

int64_t kan_dw_slab_floats(int in, int out, int splits) { return (int64_t)splits * out * KAN_K1 * in; }

hipError_t kan_head_fwd(const float* X, const float* grid, const float* W, int64_t N, int in, float* Y, hipStream_t s) {
  if (N <= 0 || in <= 0) return hipErrorInvalidValue;
  const int64_t blocks = (N + 3) / 4;
  hipLaunchKernelGGL(kan_head_fwd_kernel, dim3((unsigned)(blocks < 16384 ? blocks : 16384)), dim3(256), 0, s, X, grid, W,
                     N, in, Y);
  return hipGetLastError();
}

// out = 1 layer backward: `waves` waves of contiguous rows (waves <= slab rows), partial weight
// gradients summed in fixed order into dW
hipError_t kan_head_bwd(const float* X, const float* grid, const float* W, const float* g, int64_t N, int in, int waves,
                        float* slab, float* dW, float* Gin, hipStream_t s) {
  if (N <= 0 || in <= 0 || in > 64 || waves < 4) return hipErrorInvalidValue;
  const int blocks = waves / 4;
  int64_t rpw = (N + (int64_t)blocks * 4 - 1) / ((int64_t)blocks * 4);
  if (rpw < 1) rpw = 1;
  hipLaunchKernelGGL(kan_head_bwd_kernel, dim3(blocks), dim3(256), 0, s, X, grid, W, g, N, in, rpw, slab, Gin);
  const int64_t mn = (int64_t)KAN_K1 * in;
  hipLaunchKernelGGL(kan_slab_reduce_kernel, dim3(ew_grid(mn)), dim3(256), 0, s, (const float*)slab, blocks * 4, mn, dW);
  return hipGetLastError();
}

// dW[o][k] = sum_n G[n][o] A[n][k]: `splits` row slices into slabs, then the fixed-order slab sum
hipError_t kan_dw_fused(const float* X, const float* grid, const float* G, int64_t N, int in, int out, int splits,
                        float* slab, float* dW, hipStream_t s) {
  if (N <= 0 || in <= 0 || out <= 0 || splits < 1) return hipErrorInvalidValue;
  int64_t rps = (N + splits - 1) / splits;
  rps = (rps + KF_R - 1) / KF_R * KF_R;
  const int z = (int)((N + rps - 1) / rps);
  hipLaunchKernelGGL(kan_dw_fused_kernel, dim3((in + KF_IC - 1) / KF_IC, (out + KF_O - 1) / KF_O, z), dim3(256), 0, s,
                     X, grid, G, N, in, out, rps, slab);
  const int64_t mn = (int64_t)out * KAN_K1 * in;
  hipLaunchKernelGGL(kan_slab_reduce_kernel, dim3(ew_grid(mn)), dim3(256), 0, s, (const float*)slab, z, mn, dW);
  return hipGetLastError();
}

hipError_t kan_dx_fused(const float* X, const float* grid, const float* Gout, const float* W, int64_t N, int in,
                        int out, float* Gin, hipStream_t s) {
  if (N <= 0 || in <= 0 || out <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kan_dx_fused_kernel, dim3((unsigned)((N + KF_R - 1) / KF_R), (in + KF_IC - 1) / KF_IC), dim3(256),
                     0, s, X, grid, Gout, W, N, in, out, Gin);
  return hipGetLastError();
}

hipError_t kan_combine(const float* base_w, const float* spline_w, const float* scaler, int out, int in, float* W,
                       hipStream_t s) {
  hipLaunchKernelGGL(kan_combine_kernel, dim3(ew_grid((int64_t)out * in)), dim3(256), 0, s, base_w, spline_w,
                     scaler, out, in, W);
  return hipGetLastError();
}

hipError_t kan_param_grads(const float* dW, const float* spline_w, const float* scaler, int out, int in,
                           int accumulate, float* g_base, float* g_spline, float* g_scaler, hipStream_t s) {
  hipLaunchKernelGGL(kan_param_grads_kernel, dim3(ew_grid((int64_t)out * in)), dim3(256), 0, s, dW, spline_w,
                     scaler, out, in, accumulate, g_base, g_spline, g_scaler);
  return hipGetLastError();
}

// splits > 1: `C` must hold splits * M * N floats (slabs), reduced into `out`
hipError_t kan_gemm(const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk, int64_t sbn, int M,
                    int N, int64_t K, int splits, float* C, float* out, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0 || splits < 1) return hipErrorInvalidValue;
  int64_t kchunk = (K + splits - 1) / splits;
  kchunk = (kchunk + KG_BK - 1) / KG_BK * KG_BK;
  const int z = (int)((K + kchunk - 1) / kchunk);
  dim3 grid((N + KG_T - 1) / KG_T, (M + KG_T - 1) / KG_T, z);
  hipLaunchKernelGGL(kan_gemm_kernel, grid, dim3(256), 0, s, A, sam, sak, B, sbk, sbn, z > 1 ? C : out, M, N, K,
                     kchunk);
  if (z > 1)
    hipLaunchKernelGGL(kan_slab_reduce_kernel, dim3(ew_grid((int64_t)M * N)), dim3(256), 0, s, C, z,
                       (int64_t)M * N, out);
  return hipGetLastError();
}

}  // namespace siren
