// KAN path: efficient-KAN `KANLinear` layers (kan.py:6-166) as
//   expand   A = [ SiLU(X) | B-spline bases of X ]            [N][9 in]   (grid 5, order 3)
//   GEMM     Out = A W^T,  W = [ base_weight | spline_weight * spline_scaler ]  [out][9 in]
// and its autograd: dW = G^T A (split-K over coordinates, fixed-order slab reduction),
// dA = G W, dX = SiLU'(X) dA_base + sum_c B'_c(X) dA_spline_c.
//
// Everything is fp32 like the reference.  The bases follow kan.py:94-104's Cox-de Boor
// recursion op for op (sub, div, mul, add; fp-contract off) on the layer's own `grid` buffer,
// so they are bit-identical to torch's CPU result; the derivative differentiates the same
// recursion.  KAN is VALU / HBM-bound at the reference's widths (K = 9 * in <= 2304), so the
// GEMM is an LDS-tiled VALU kernel, not MFMA.
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
template <bool DERIV>
__device__ __forceinline__ void kan_bases_local(float x, const float* __restrict__ g, float* b, float* db) {
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
      const float l = (x - gj) / (gjk - gj);
      const float r = (gjk1 - x) / (gjk1 - gj1);
      if constexpr (DERIV)
        d[q] = (1.0f / (gjk - gj)) * w[q] + l * d[q] - (1.0f / (gjk1 - gj1)) * w[q + 1] + r * d[q + 1];
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

// A[n][i] = SiLU(x), A[n][in + 8 i + c] = B_c(x)  with x = X[n][i]
__global__ void kan_expand_kernel(const float* __restrict__ X, const float* __restrict__ grid, int64_t N,
                                  int in, float* __restrict__ A) {
  const int64_t total = N * in;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = e / in;
    const int i = (int)(e - n * in);
    const float x = X[e];
    float b[KAN_NB], unused[KAN_NB];
    kan_bases_local<false>(x, grid + i * KAN_NG, b, unused);
    float* row = A + n * (int64_t)(KAN_K1 * in);
    row[i] = silu(x);
    float4* sp = (float4*)(row + in + KAN_NB * i);  // 32-B aligned: in % 4 == 0 or in == 1
    if ((in & 3) == 0) {
      sp[0] = float4{b[0], b[1], b[2], b[3]};
      sp[1] = float4{b[4], b[5], b[6], b[7]};
    } else {
#pragma unroll
      for (int c = 0; c < KAN_NB; ++c) row[in + KAN_NB * i + c] = b[c];
    }
  }
}

// dX[n][i] = SiLU'(x) dA[n][i] + sum_c B'_c(x) dA[n][in + 8 i + c]
__global__ void kan_contract_kernel(const float* __restrict__ X, const float* __restrict__ grid,
                                    const float* __restrict__ dA, int64_t N, int in, float* __restrict__ dX) {
  const int64_t total = N * in;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = e / in;
    const int i = (int)(e - n * in);
    const float x = X[e];
    float b[KAN_NB], db[KAN_NB];
    kan_bases_local<true>(x, grid + i * KAN_NG, b, db);
    const float* row = dA + n * (int64_t)(KAN_K1 * in);
    float acc = silu_grad(x) * row[i];
#pragma unroll
    for (int c = 0; c < KAN_NB; ++c) acc += db[c] * row[in + KAN_NB * i + c];
    dX[e] = acc;
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

hipError_t kan_expand(const float* X, const float* grid, int64_t N, int in, float* A, hipStream_t s) {
  hipLaunchKernelGGL(kan_expand_kernel, dim3(ew_grid(N * in)), dim3(256), 0, s, X, grid, N, in, A);
  return hipGetLastError();
}

hipError_t kan_contract(const float* X, const float* grid, const float* dA, int64_t N, int in, float* dX,
                        hipStream_t s) {
  hipLaunchKernelGGL(kan_contract_kernel, dim3(ew_grid(N * in)), dim3(256), 0, s, X, grid, dA, N, in, dX);
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
