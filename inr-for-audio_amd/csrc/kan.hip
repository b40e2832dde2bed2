// KAN path: efficient-KAN `KANLinear` layers (kan.py:6-166):
//   A = [ SiLU(X) | B-spline bases of X ]   [N][9 in]   (grid 5, order 3)
//   Out = A W^T,  W = [ base_weight | spline_weight * spline_scaler ]  [out][9 in]
// and its autograd: dW = G^T A, dA = G W, dX = SiLU'(X) dA_base + sum_c B'_c(X) dA_spline_c.
//
// A and dA are never materialised (round 2; the first design wrote and re-read A / dA, 2.3 KB
// per coordinate each at width 64, ~26 KB of HBM per coordinate-step).  Three fused kernels
// recompute the bases of a (16-input x 64-row) chunk into LDS where they are consumed:
//   kan_fwd_fused  Out tile [64 rows][64 outs] = sum over input chunks of A_chunk W_chunk^T
//   kan_dw_fused   dW chunk [out][144] += G[rows]^T A_chunk[rows]   (split-K over rows, slabs)
//   kan_dx_fused   dA_chunk = G W_chunk (in LDS), contracted at once with the bases' derivatives
//   kan_bwd_fused  both backward products of a chunk in one pass (out <= 64)
//   kan_head_train the last layer (out = 1): forward, MSE gradient and backward in one pass
// Everything is fp32 like the reference.  The bases follow kan.py:94-104's Cox-de Boor
// recursion op for op (sub, div, mul, add; fp-contract off) on the layer's own `grid` buffer,
// so they are bit-identical to torch's CPU result; the derivative differentiates the same
// recursion.  The chunk products run on the f32-input MFMA (exact f32); the last
// layer (out = 1) is a per-row dot product on the VALU (kan_head_*).
#include "siren_common.h"
#include "siren_kernels.h"

// KAN_ABL (measurement-only builds via tools/kan_ablate.py, never the product): bit 1 replaces
// the basis recursion by a trivial stand-in, bit 2 skips the chunk products.
#ifndef KAN_ABL
#define KAN_ABL 0
#endif
// knot window of the basis recursion (kan_bases_window): 1 = span by counting + an 8-knot gather
// from the LDS knot row (cfg5 2.249 -> 2.202 ms per step), 0 = per-span predicate with the window
// captured by selects (kept for the head kernels, whose lanes hold one input's knots throughout)
#ifndef KAN_WINDOW_GATHER
#define KAN_WINDOW_GATHER 1
#endif

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
// instead of 54 divisions (36 instead of 108 with the derivative).
// The span search also captures the lane's knot window kw[d] = g[s-3+d] (d = 0..7) with selects,
// so the recursion indexes registers statically: no per-lane knot gathers.  Terms whose knot
// index falls outside the array are computed on stale window entries and discarded by a select
// (the full recursion has no such term).
// Forward (RCP false): every quotient a / D is the correctly rounded one, without a division:
// with y = RN(1/D) from the per-input table inv[(k-1)*11 + j] = 1 / (g[j+k] - g[j]) (IEEE
// divisions, once per input: kf_fill_inv), q = RN(a y), r = a - D q (exact by fma) and
// q' = RN(q + r y) equals RN(a / D) (Markstein's theorem: y within half an ulp of 1/D, q within
// one ulp of a/D; no underflow or overflow on these knot grids), so the bases stay bit-identical
// to torch's (tests/test_gpu_kan.py::test_kan_forward_bases_bit_exact).
// RCP (backward kernels): the knot-difference divisions become products with v_rcp_f32
// reciprocals (within an ulp of the divisions; only the weight / input gradients see them).
__device__ __forceinline__ float kan_div(float a, float d, float y) {
  const float q = a * y;
  const float r = fmaf(-q, d, a);
  return fmaf(r, y, q);
}

// The recursion on the window: s (the span, -1 outside the grid), w[q] = B[s-3+q] and, with
// DERIV, d[q] = B'[s-3+q] (q = 0..3).
template <bool DERIV, bool RCP, bool GATHER = (KAN_WINDOW_GATHER != 0)>
__device__ __forceinline__ int kan_bases_window(float x, const float* __restrict__ g, float* w, float* d,
                                                const float* __restrict__ inv) {
  int s = -1;
  float kw[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
if constexpr (GATHER) {
  // span by counting: for non-decreasing knots, g[s] <= x < g[s+1] holds exactly for
  // s = #{j : g[j] <= x} - 1 when that count is 1 .. NG-1 (x below the first knot, at or past the
  // last one, or NaN: no span), the same s as the per-span predicate below.  The window is then
  // one gather of 8 knots from the LDS row g (indices clamped into the array; the entries a clamp
  // touches belong to terms the recursion discards)
  int cnt = 0;
#pragma unroll
  for (int j = 0; j < KAN_NG; ++j) cnt += (x >= g[j]) ? 1 : 0;
  s = (cnt >= 1 && cnt <= KAN_NG - 1) ? cnt - 1 : -1;
  {
    const int s0 = s < 0 ? 0 : s;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      int t = s0 - 3 + e;
      t = t < 0 ? 0 : (t > KAN_NG - 1 ? KAN_NG - 1 : t);
      kw[e] = g[t];
    }
  }
  } else {
  float kn[KAN_NG];
#pragma unroll
  for (int j = 0; j < KAN_NG; ++j) kn[j] = g[j];
#pragma unroll
  for (int j = 0; j < KAN_NG - 1; ++j) {
    const bool hit = x >= kn[j] && x < kn[j + 1];
    s = hit ? j : s;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int t = j - 3 + e;
      if (t >= 0 && t < KAN_NG) kw[e] = hit ? kn[t] : kw[e];
    }
  }
  }
  // window w[q] = B[s - 3 + q], q = 0..3, plus w[4] = B[s + 1] = 0
  float ww[5] = {0.0f, 0.0f, 0.0f, 1.0f, 0.0f}, dd[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int k = 1; k <= 3; ++k) {
#pragma unroll
    for (int q = 3 - k; q < 4; ++q) {
      const int j = s - 3 + q;
      const bool ok = j >= 0 && j <= KAN_NG - 2 - k;  // inside the support and the array
      const float gj = kw[q], gjk = kw[q + k], gj1 = kw[q + 1], gjk1 = kw[q + k + 1];
      float il, ir, l, r;
      if constexpr (RCP) {
        il = __builtin_amdgcn_rcpf(gjk - gj);
        ir = __builtin_amdgcn_rcpf(gjk1 - gj1);
        l = (x - gj) * il;
        r = (gjk1 - x) * ir;
      } else {
        const int jt = j < 0 ? 0 : (j > KAN_NG - 2 - k ? KAN_NG - 2 - k : j);  // in-table for discarded terms
        il = inv[(k - 1) * 11 + jt];
        ir = inv[(k - 1) * 11 + jt + 1];
        l = kan_div(x - gj, gjk - gj, il);
        r = kan_div(gjk1 - x, gjk1 - gj1, ir);
      }
      if constexpr (DERIV) {
        const float nd = il * ww[q] + l * dd[q] - ir * ww[q + 1] + r * dd[q + 1];
        dd[q] = ok ? nd : dd[q];
      }
      const float nw = l * ww[q] + r * ww[q + 1];
      ww[q] = ok ? nw : ww[q];
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    w[q] = ww[q];
    if constexpr (DERIV) d[q] = dd[q];
  }
  return s;
}

template <bool DERIV, bool RCP = false, bool GATHER = (KAN_WINDOW_GATHER != 0)>
__device__ __forceinline__ void kan_bases_local(float x, const float* __restrict__ g, float* b, float* db,
                                                const float* __restrict__ inv = nullptr) {
#pragma unroll
  for (int j = 0; j < KAN_NB; ++j) b[j] = db[j] = 0.0f;
  if constexpr ((KAN_ABL & 1) != 0) {
#pragma unroll
    for (int j = 0; j < KAN_NB; ++j) b[j] = db[j] = x * g[j];
    return;
  }
  float w[4], d[4];
  const int s = kan_bases_window<DERIV, RCP, GATHER>(x, g, w, d, inv);
  if (s < 0) return;
#pragma unroll
  for (int c = 0; c < KAN_NB; ++c) {
    // B[c] = w[c - s + 3] when that is a window slot
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool at = (c == s - 3 + q);
      b[c] = at ? w[q] : b[c];
      if constexpr (DERIV) db[c] = at ? d[q] : db[c];
    }
  }
}

__device__ __forceinline__ float silu(float x) { return x / (1.0f + expf(-x)); }
__device__ __forceinline__ float silu_grad(float x) {
  const float s = 1.0f / (1.0f + expf(-x));
  return s * (1.0f + x * (1.0f - s));
}
// silu(x) and silu_grad(x) on one exp: the same values as the two calls (same operations on the
// same 1 + exp(-x))
__device__ __forceinline__ void silu_and_grad(float x, float& sl, float& dsl) {
  const float d = 1.0f + expf(-x);
  sl = x / d;
  const float s = 1.0f / d;
  dsl = s * (1.0f + x * (1.0f - s));
}

// ---- fused layer kernels --------------------------------------------------------------------
// Chunk of IC inputs i0 .. i0+ic-1 (ic <= IC): local column kk < ic is the SiLU column of input
// i0+kk (combined-weight column k = i0+kk), kk = ic + 8 ii + c the spline basis c of input i0+ii
// (k = in + 8 (i0+ii) + c).  kc = 9 ic columns, padded to kpad (a multiple of 16) with zeros.
// The products run on v_mfma_f32_16x16x4_f32 (exact f32, a k-ordered fmaf chain; the same rate
// as the f32 VALU but one LDS operand per 2048 flops instead of per 2): lane l supplies
// A[l&15][k=l>>4] and B[k=l>>4][l&15]; D[row=(l>>4)*4+reg][col=l&15].
constexpr int KF_IC = 16, KF_KC = 9 * KF_IC, KF_R = 64, KF_O = 64;
constexpr int64_t kKanResidentBlocks = 512;     // 256 CUs x 2 (LDS-limited) for the fused kernels
constexpr int64_t kKanBwdResidentBlocks = 256;  // kan_bwd_fused: one 512-thread block per CU

__device__ __forceinline__ int kf_col(int kk, int ic, int i0, int in) {
  return kk < ic ? i0 + kk : in + 8 * i0 + (kk - ic);
}

__device__ __forceinline__ f32x4 kf_mfma(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Xs[r][ii] = X[r0 + r][i0 + ii] for rows < re (else 0): the chunk's inputs, read along the row
// (a full chunk with in % 4 == 0: one 16-byte load per thread).  All tile loaders below issue
// every load of the tile before the first LDS store, so a tile costs one memory latency.
__device__ __forceinline__ float4 ldg4(const float* p) { return *reinterpret_cast<const float4*>(p); }

__device__ __forceinline__ void kf_stage_x(float (*Xs)[KF_IC + 1], const float* __restrict__ X, int64_t re, int in,
                                           int64_t r0, int i0, int ic) {
  if (ic == KF_IC && (in & 3) == 0) {
    if (threadIdx.x < KF_R * KF_IC / 4) {
      const int r = threadIdx.x >> 2, i4 = (threadIdx.x & 3) * 4;
      float4 v = float4{0.f, 0.f, 0.f, 0.f};
      if (r0 + r < re) v = ldg4(X + (r0 + r) * in + i0 + i4);
      Xs[r][i4] = v.x;
      Xs[r][i4 + 1] = v.y;
      Xs[r][i4 + 2] = v.z;
      Xs[r][i4 + 3] = v.w;
    }
    return;
  }
  for (int e = threadIdx.x; e < KF_R * KF_IC; e += blockDim.x) {
    const int r = e / KF_IC, ii = e % KF_IC;
    const int64_t n = r0 + r;
    Xs[r][ii] = (n < re && ii < ic) ? X[n * in + i0 + ii] : 0.f;
  }
}

// gk[ii][j] = knot j of input i0 + ii.  The recursion reads knots at a per-row span index; from
// LDS those reads cost an LDS round trip, from global memory an L1/L2 one on every step.
constexpr int KF_GST = KAN_NG + 1;
__device__ __forceinline__ void kf_fill_knots(float (*gk)[KF_GST], const float* __restrict__ grid, int i0, int ic) {
  for (int e = threadIdx.x; e < ic * KAN_NG; e += blockDim.x) gk[e / KAN_NG][e % KAN_NG] = grid[i0 * KAN_NG + e];
}

// inv[ii][(k-1)*11 + j] = RN(1 / (g[j+k] - g[j])) for the knots of inputs i0 .. i0+ic-1 (IEEE
// divisions; the forward's exact quotients, kan_div)
constexpr int KF_VST = 33;
__device__ __forceinline__ void kf_fill_inv(float (*inv)[KF_VST], const float* __restrict__ grid, int i0, int ic) {
  for (int e = threadIdx.x; e < ic * 33; e += blockDim.x) {
    const int ii = e / 33, q = e - ii * 33, k = q / 11 + 1, j = q - (k - 1) * 11;
    const float* g = grid + (i0 + ii) * KAN_NG;
    inv[ii][q] = (j + k < KAN_NG) ? 1.0f / (g[j + k] - g[j]) : 0.0f;
  }
}

// As[kk][r] (pad 4) = A columns of the chunk for rows r0 + r (zero past re, and rows kc .. kpad-1
// zero).  A wave takes one input ii and 64 consecutive rows: its knots / reciprocals are uniform
// and the LDS writes are conflict-free.
template <bool RCP = false>
__device__ __forceinline__ void kf_fill_a(float (*As)[KF_R + 4], const float (*Xs)[KF_IC + 1],
                                          const float (*gk)[KF_GST], int64_t re, int64_t r0, int i0, int ic,
                                          int kpad) {
  for (int p = threadIdx.x; p < KF_R * ic; p += blockDim.x) {
    const int r = p & (KF_R - 1), ii = p >> 6;
    float b[KAN_NB], unused[KAN_NB], sl = 0.f;
    if (r0 + r < re) {
      const float x = Xs[r][ii];
      static_assert(RCP, "the exact forward bases need the reciprocal table (kf_put_pair)");
      kan_bases_local<false, RCP>(x, gk[ii], b, unused);
      sl = silu(x);
    } else {
#pragma unroll
      for (int c = 0; c < KAN_NB; ++c) b[c] = 0.f;
    }
    As[ii][r] = sl;
#pragma unroll
    for (int c = 0; c < KAN_NB; ++c) As[ic + 8 * ii + c][r] = b[c];
  }
  const int kc = 9 * ic;
  for (int e = threadIdx.x; e < (kpad - kc) * KF_R; e += blockDim.x) As[kc + e / KF_R][e % KF_R] = 0.f;
}

// Operand tiles are read with one ds_read_b128 per lane per 16-k group: lane group lk = l>>4
// supplies k = 16 g + 4 lk + t to the t-th MFMA of group g (a permutation of the summation index
// applied to both operands alike).  Row strides are 4 mod 32 floats, so each 8-lane phase of a
// b128 read covers the 32 banks once.  The next group's fragments are loaded while the current
// group's MFMAs issue.
constexpr int KF_AST = KF_KC + 4;  // [row][kk] tiles of the forward
constexpr int KF_CST = KF_R + 4;   // [*][row] / [*][o] tiles of the backward

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float f4(const float4& v, int t) { return t == 0 ? v.x : t == 1 ? v.y : t == 2 ? v.z : v.w; }

// acc[j] += sum over ng groups of 16 k: A(16 rows at ap) x B(16 cols at bp + j * bstride).
// Two accumulator sets (k-steps t = 0, 2 of a group into acc, t = 1, 3 into acc2, added at the
// end in that fixed order): 2 NJ independent MFMA chains per wave.  With NJ = 4 chains the f32
// MFMA's dependent-issue latency is exposed (tools/micro/mfma_f32_rate: 111 vs 146 TFLOP/s for 4
// vs 9 chains at two waves per SIMD).  SPLIT = false keeps one set (the forward: measured no gain,
// cfg5 kan_fwd 0.753 vs 0.778 ms per step; the backward products gain 4% of the step).
template <int NJ, int NA, bool SPLIT = true>
__device__ __forceinline__ void kf_mfma_groups(const float* ap, const float* bp, int bstride, int ng, f32x4 (&acc)[NA]) {
  static_assert(NJ <= NA, "more column tiles than accumulators");
  f32x4 acc2[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) acc2[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float4 a = ld4(ap), b[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) b[j] = ld4(bp + j * bstride);
  for (int g = 0; g < ng; ++g) {
    float4 an = a, bn[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) bn[j] = b[j];
    if (g + 1 < ng) {
      an = ld4(ap + 16 * (g + 1));
#pragma unroll
      for (int j = 0; j < NJ; ++j) bn[j] = ld4(bp + j * bstride + 16 * (g + 1));
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (SPLIT && (t & 1)) acc2[j] = kf_mfma(f4(a, t), f4(b[j], t), acc2[j]);
        else acc[j] = kf_mfma(f4(a, t), f4(b[j], t), acc[j]);
      }
    a = an;
#pragma unroll
    for (int j = 0; j < NJ; ++j) b[j] = bn[j];
  }
  if constexpr (SPLIT) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] += acc2[j];
  }
}

// the same with a run-time count of B column tiles (0 .. NA)
template <int NA>
__device__ __forceinline__ void kf_mfma_groups_n(int nj, const float* ap, const float* bp, int bstride, int ng,
                                                 f32x4 (&acc)[NA]) {
  switch (nj) {
#define KF_CASE(n)                                                      \
  case n:                                                               \
    if constexpr (n <= NA) kf_mfma_groups<n>(ap, bp, bstride, ng, acc); \
    break;
    KF_CASE(9) KF_CASE(8) KF_CASE(7) KF_CASE(6) KF_CASE(5) KF_CASE(4) KF_CASE(3) KF_CASE(2) KF_CASE(1)
#undef KF_CASE
    default: break;
  }
}

// As[r][ii] = SiLU(x), As[r][ic + 8 ii + c] = B_c(x) for the pair (r, ii) (zeros for rows past N)
__device__ __forceinline__ void kf_put_pair(float (*As)[KF_AST], int r, int ii, int ic, float x, bool valid,
                                            const float (*gk)[KF_GST], const float (*inv)[KF_VST]) {
  float b[KAN_NB], unused[KAN_NB], sl = 0.f;
  if (valid) {
    kan_bases_local<false>(x, gk[ii], b, unused, inv[ii]);
    sl = silu(x);
  } else {
#pragma unroll
    for (int c = 0; c < KAN_NB; ++c) b[c] = 0.f;
  }
  As[r][ii] = sl;
  float* d = &As[r][ic + 8 * ii];
  if ((ic & 3) == 0) {
    *reinterpret_cast<float4*>(d) = float4{b[0], b[1], b[2], b[3]};
    *reinterpret_cast<float4*>(d + 4) = float4{b[4], b[5], b[6], b[7]};
  } else {
#pragma unroll
    for (int c = 0; c < KAN_NB; ++c) d[c] = b[c];
  }
}

// Y[n][o] = sum_k A[n][k] W[o][k]; grid (ceil(N/64), ceil(out/64)).  Wave w: rows 16w .. 16w+15
// x 64 outs (4 accumulators), K = the chunk's kpad columns, summed over the chunks.
__global__ __launch_bounds__(256) void kan_fwd_fused_kernel(const float* __restrict__ X, const float* __restrict__ grid,
                                                            const float* __restrict__ W, int64_t N, int in, int out,
                                                            float* __restrict__ Y) {
  __shared__ __attribute__((aligned(16))) float As[KF_R][KF_AST];  // [row][kk]
  __shared__ __attribute__((aligned(16))) float Ws[KF_O][KF_AST];  // [o][kk]
  __shared__ float gk[KF_IC][KF_GST];
  __shared__ float inv[KF_IC][KF_VST];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, li = lane & 15, lk = lane >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * KF_R;
  const int o0 = blockIdx.y * KF_O;
  const int64_t K = (int64_t)KAN_K1 * in;
  const bool vec = (in & 3) == 0 && in % KF_IC == 0;  // every chunk full, 16-byte pieces
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // vec path: a chunk's W pieces (4 SiLU + 32 spline 16-byte pieces per out) and X piece, loaded
  // into registers one chunk ahead so their latency hides under the previous chunk's products
  const int xr = tid >> 2, xi = (tid & 3) * 4;
  float4 wv4[9], xv4 = float4{0.f, 0.f, 0.f, 0.f};
  auto load_chunk = [&](int i0) {
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      const int idx = tid + 256 * q, o = idx / 36, c4 = idx % 36;
      const int64_t col = c4 < 4 ? i0 + 4 * c4 : in + 8 * i0 + 4 * (c4 - 4);
      wv4[q] = o0 + o < out ? ldg4(W + (int64_t)(o0 + o) * K + col) : float4{0.f, 0.f, 0.f, 0.f};
    }
    xv4 = r0 + xr < N ? ldg4(X + (r0 + xr) * in + i0 + xi) : float4{0.f, 0.f, 0.f, 0.f};
  };
  if (vec) load_chunk(0);
  for (int i0 = 0; i0 < in; i0 += KF_IC) {
    const int ic = in - i0 < KF_IC ? in - i0 : KF_IC, kc = 9 * ic, kpad = (kc + 15) & ~15;
    kf_fill_knots(gk, grid, i0, ic);
    kf_fill_inv(inv, grid, i0, ic);
    if (vec) {
#pragma unroll
      for (int q = 0; q < 9; ++q) {
        const int idx = tid + 256 * q, o = idx / 36, c4 = idx % 36;
        *reinterpret_cast<float4*>(&Ws[o][4 * c4]) = wv4[q];
      }
    } else {
      for (int e = tid; e < KF_O * kpad; e += blockDim.x) {
        const int o = e / kpad, kk = e - o * kpad;
        Ws[o][kk] = (o0 + o < out && kk < kc) ? W[(int64_t)(o0 + o) * K + kf_col(kk, ic, i0, in)] : 0.f;
      }
      for (int e = tid; e < (kpad - kc) * KF_R; e += blockDim.x) As[e % KF_R][kc + e / KF_R] = 0.f;
    }
    __syncthreads();
    // A tile: the vec path's thread computes the 4 pairs whose x it loaded
    if (vec) {
      const bool valid = r0 + xr < N;
      kf_put_pair(As, xr, xi, ic, xv4.x, valid, gk, inv);
      kf_put_pair(As, xr, xi + 1, ic, xv4.y, valid, gk, inv);
      kf_put_pair(As, xr, xi + 2, ic, xv4.z, valid, gk, inv);
      kf_put_pair(As, xr, xi + 3, ic, xv4.w, valid, gk, inv);
    } else {
      for (int p = tid; p < KF_R * ic; p += blockDim.x) {
        const int r = p & (KF_R - 1), ii = p >> 6;
        const bool valid = r0 + r < N;
        kf_put_pair(As, r, ii, ic, valid ? X[(r0 + r) * in + i0 + ii] : 0.f, valid, gk, inv);
      }
    }
    __syncthreads();
    if (vec && i0 + KF_IC < in) load_chunk(i0 + KF_IC);
    if ((KAN_ABL & 2) == 0)
      kf_mfma_groups<4, 4, false>(&As[16 * wv + li][4 * lk], &Ws[li][4 * lk], 16 * KF_AST, kpad >> 4, acc);
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t n = r0 + 16 * wv + 4 * lk + q;
      const int o = o0 + 16 * j + li;
      if (n < N && o < out) Y[n * out + o] = acc[j][q];
    }
}

// ---- the last layer (out = 1, in <= 64): one wave per row, lane = input ----------------------
// out[n] = SiLU(x_lane) W[lane] + sum_c B_c(x_lane) W[in + 8 lane + c], summed over the wave in a
// fixed butterfly order.
__global__ __launch_bounds__(256) void kan_head_fwd_kernel(const float* __restrict__ X, const float* __restrict__ grid,
                                                           const float* __restrict__ W, int64_t N, int in,
                                                           float* __restrict__ Y) {
  __shared__ float gk[64][KF_GST];
  __shared__ float inv[64][KF_VST];
  kf_fill_knots(gk, grid, 0, in);
  kf_fill_inv(inv, grid, 0, in);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const bool on = lane < in;
  float wb = 0.f, ws[KAN_NB] = {};
  if (on) {
    wb = W[lane];
#pragma unroll
    for (int c = 0; c < KAN_NB; ++c) ws[c] = W[in + KAN_NB * lane + c];
  }
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t n = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); n < N; n += nw) {
    float v = 0.f;
    if (on) {
      const float x = X[n * in + lane];
      float b[KAN_NB], unused[KAN_NB];
      kan_bases_local<false, false, false>(x, gk[lane], b, unused, inv[lane]);  // lane-fixed knots: selects
      v = silu(x) * wb;
#pragma unroll
      for (int c = 0; c < KAN_NB; ++c) v += b[c] * ws[c];
    }
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) Y[n] = v;
  }
}

// Training step of the last layer (out = 1, in <= 64) in one pass over its rows.  Per row: the
// forward out = SiLU(x) W[i] + sum_c B_c(x) W[in + 8 i + c] with kan_head_fwd's exact bases and
// butterfly (so out is bit-identical to inference), the MSE gradient g = 2 (out - y) / N and the
// squared error (run.py:160-168; rows >= n_valid contribute nothing), then the backward: Gin[n][i]
// = g_n (SiLU'(x) W[i] + sum_c B'_c(x) W[in + 8 i + c]) (dA = g W is a rank-1 product, never
// formed) and the weight-gradient partials -- one basis evaluation per (row, input) for the
// forward and the backward, and no pass over X or out between them.  Blocks take >= 256 contiguous rows (one
// slab row and one squared-error partial each); their 4 waves take every 4th row.
__global__ __launch_bounds__(256) void kan_head_train_kernel(const float* __restrict__ X, const float* __restrict__ grid,
                                                             const float* __restrict__ W, const float* __restrict__ y,
                                                             int64_t N, int in, int64_t n_valid, float gfac,
                                                             int64_t rows_per_block, float* __restrict__ out,
                                                             float* __restrict__ g, float* __restrict__ sse_part,
                                                             float* __restrict__ slab, float* __restrict__ Gin) {
  __shared__ float gk[64][KF_GST];
  __shared__ float inv[64][KF_VST];
  __shared__ float part[4][KAN_K1][64];
  __shared__ float sse_w[4];
  kf_fill_knots(gk, grid, 0, in);
  kf_fill_inv(inv, grid, 0, in);
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t nb = (int64_t)blockIdx.x * rows_per_block;
  const int64_t ne = nb + rows_per_block < N ? nb + rows_per_block : N;
  const bool on = lane < in;
  float wb = 0.f, ws[KAN_NB] = {};
  if (on) {
    wb = W[lane];
#pragma unroll
    for (int c = 0; c < KAN_NB; ++c) ws[c] = W[in + KAN_NB * lane + c];
  }
  float ab = 0.f, as[KAN_NB] = {}, sse = 0.f;
  // the next row's x and y are loaded before this row's stores: vmcnt retires loads and stores in
  // issue order, so a load issued after the stores would wait for them too
  int64_t n = nb + wv;
  float xn = 0.f, yn = 0.f;
  if (n < ne) {
    if (on) xn = X[n * in + lane];
    if (n < n_valid) yn = y[n];
  }
  for (; n < ne; n += 4) {
    const float xc = xn, yc = yn;
    if (n + 4 < ne) {
      if (on) xn = X[(n + 4) * in + lane];
      if (n + 4 < n_valid) yn = y[n + 4];
    }
    float x = 0.f, v = 0.f, sl = 0.f, b[KAN_NB], db[KAN_NB];
    if (on) {
      x = xc;
      kan_bases_local<true, false, false>(x, gk[lane], b, db, inv[lane]);  // lane-fixed knots: selects
      sl = silu(x);
      v = sl * wb;
#pragma unroll
      for (int c = 0; c < KAN_NB; ++c) v += b[c] * ws[c];
    }
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const float o = (0.f + v) + 0.f;  // head_loss's accumulation of the one partial and the zero bias
    float gn = 0.f;
    if (n < n_valid) {
      const float err = o - yc;
      sse += err * err;
      gn = err * gfac;
    }
    if (lane == 0) {
      out[n] = o;
      g[n] = gn;
    }
    if (on) {
      ab += gn * sl;
      float d = silu_grad(x) * wb;
#pragma unroll
      for (int c = 0; c < KAN_NB; ++c) {
        as[c] += gn * b[c];
        d += db[c] * ws[c];
      }
      Gin[n * in + lane] = gn * d;
    }
  }
  part[wv][0][lane] = ab;
#pragma unroll
  for (int c = 0; c < KAN_NB; ++c) part[wv][1 + c][lane] = as[c];
  if (lane == 0) sse_w[wv] = sse;
  __syncthreads();
  if (wv == 0) {
    if (on) {
      float* row = slab + (int64_t)blockIdx.x * KAN_K1 * in;
#pragma unroll
      for (int t = 0; t < KAN_K1; ++t) {
        const float v = ((part[0][t][lane] + part[1][t][lane]) + part[2][t][lane]) + part[3][t][lane];
        row[t == 0 ? lane : in + KAN_NB * lane + (t - 1)] = v;
      }
    }
    if (lane == 0) sse_part[blockIdx.x] = ((sse_w[0] + sse_w[1]) + sse_w[2]) + sse_w[3];
  }
}

// slab[z][o][k] = sum over rows of split z of G[n][o] A[n][k], for the chunk's columns k.
// 1-D grid of nchunk * nout * zpad blocks (zpad = splits rounded up to 8), numbered so that the
// blocks of one split (which read the same rows of G and X) share an XCD: block L runs on XCD
// L % 8.  Wave w: outs 16w .. 16w+15 x the chunk's kpad columns (kpad/16 accumulators), K = rows.
__global__ __launch_bounds__(256) void kan_dw_fused_kernel(const float* __restrict__ X, const float* __restrict__ grid,
                                                           const float* __restrict__ G, int64_t N, int in, int out,
                                                           int64_t rows_per_split, int nchunk, int nout, int splits,
                                                           float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) float As[KF_KC][KF_CST];  // [kk][r]
  __shared__ __attribute__((aligned(16))) float Gt[KF_O][KF_CST];   // [o][r]
  __shared__ float Xs[KF_R][KF_IC + 1];
  __shared__ float gk[KF_IC][KF_GST];
  const int per = nchunk * nout, L = blockIdx.x, q8 = L >> 3;
  const int cid = q8 % per, z = (q8 / per) * 8 + (L & 7);
  if (z >= splits) return;  // whole block, before any barrier
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, li = lane & 15, lk = lane >> 4;
  const int i0 = (cid % nchunk) * KF_IC, o0 = (cid / nchunk) * KF_O;
  const int ic = in - i0 < KF_IC ? in - i0 : KF_IC, kc = 9 * ic, kpad = (kc + 15) & ~15, nkt = kpad >> 4;
  kf_fill_knots(gk, grid, i0, ic);
  const int64_t rb = (int64_t)z * rows_per_split;
  const int64_t re = rb + rows_per_split < N ? rb + rows_per_split : N;
  f32x4 acc[9];
#pragma unroll
  for (int j = 0; j < 9; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int64_t r0 = rb; r0 < re; r0 += KF_R) {
    kf_stage_x(Xs, X, re, in, r0, i0, ic);
    if ((out & 3) == 0 && o0 + KF_O <= out) {
      // lanes take consecutive rows (conflict-free transposed stores), 16 bytes of outs each
      float4 v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int idx = tid + 256 * q, o4 = idx >> 6, r = idx & 63;
        v[q] = r0 + r < re ? ldg4(G + (r0 + r) * out + o0 + 4 * o4) : float4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int idx = tid + 256 * q, o4 = idx >> 6, r = idx & 63;
        Gt[4 * o4][r] = v[q].x;
        Gt[4 * o4 + 1][r] = v[q].y;
        Gt[4 * o4 + 2][r] = v[q].z;
        Gt[4 * o4 + 3][r] = v[q].w;
      }
    } else {
      for (int e = tid; e < KF_R * KF_O; e += blockDim.x) {
        const int r = e / KF_O, o = e % KF_O;
        Gt[o][r] = (r0 + r < re && o0 + o < out) ? G[(r0 + r) * out + o0 + o] : 0.f;
      }
    }
    __syncthreads();
    kf_fill_a<true>(As, Xs, gk, re, r0, i0, ic, kpad);
    __syncthreads();
    if ((KAN_ABL & 2) == 0)
      kf_mfma_groups_n(nkt, &Gt[16 * wv + li][4 * lk], &As[li][4 * lk], 16 * KF_CST, KF_R / 16, acc);
    __syncthreads();
  }
  const int64_t K = (int64_t)KAN_K1 * in;
  float* out_slab = slab + (int64_t)z * out * K;
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int kk = 16 * j + li;
    if (j >= nkt || kk >= kc) continue;
    const int64_t col = kf_col(kk, ic, i0, in);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int o = o0 + 16 * wv + 4 * lk + q;
      if (o < out) out_slab[(int64_t)o * K + col] = acc[j][q];
    }
  }
}

// Gin[n][i] = SiLU'(x) dA[n][i] + sum_c B'_c(x) dA[n][in + 8 i + c], dA = Gout W (never stored;
// W is read through its transposed copy WT[k][o], written by kan_combine);
// grid ceil(N/64): a block takes 64 rows through every input chunk (its Gout rows stay in LDS
// when out <= 64).  Wave w: rows 16w .. 16w+15 x the chunk's columns (kpad/16 accumulators),
// K = outs; the dA tile then goes to LDS (over the W chunk) for the contraction with the bases'
// derivatives, whose results leave through the X tile as coalesced row segments.
constexpr int KF_DST = KF_KC + 1;  // dA row stride

__global__ __launch_bounds__(256) void kan_dx_fused_kernel(const float* __restrict__ X, const float* __restrict__ grid,
                                                           const float* __restrict__ Gout, const float* __restrict__ WT,
                                                           int64_t N, int in, int out, float* __restrict__ Gin) {
  __shared__ __attribute__((aligned(16))) float Gs[KF_R][KF_CST];   // [r][o]
  __shared__ __attribute__((aligned(16))) float WD[KF_KC * KF_CST];  // Wt[kk][o], then dAs[r][kk]
  __shared__ float Xs[KF_R][KF_IC + 1];
  __shared__ float gk[KF_IC][KF_GST];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, li = lane & 15, lk = lane >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * KF_R;
  const int64_t K = (int64_t)KAN_K1 * in;
  const bool g_once = out <= KF_O;
  for (int i0 = 0; i0 < in; i0 += KF_IC) {
    const int ic = in - i0 < KF_IC ? in - i0 : KF_IC, kc = 9 * ic, nkt = (kc + 15) >> 4;
    f32x4 acc[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    kf_fill_knots(gk, grid, i0, ic);
    kf_stage_x(Xs, X, N, in, r0, i0, ic);
    for (int oc = 0; oc < out; oc += KF_O) {
      const int on = out - oc < KF_O ? out - oc : KF_O, opad = (on + 15) & ~15;
      const bool vec = (out & 3) == 0 && on == KF_O;
      if (!g_once || i0 == 0) {
        if (vec) {
          float4 v[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int idx = tid + 256 * q, r = idx >> 4, o4 = idx & 15;
            v[q] = r0 + r < N ? ldg4(Gout + (r0 + r) * out + oc + 4 * o4) : float4{0.f, 0.f, 0.f, 0.f};
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int idx = tid + 256 * q, r = idx >> 4, o4 = idx & 15;
            *reinterpret_cast<float4*>(&Gs[r][4 * o4]) = v[q];
          }
        } else {
          for (int e = tid; e < KF_R * KF_O; e += blockDim.x) {
            const int r = e / KF_O, o = e % KF_O;
            Gs[r][o] = (r0 + r < N && o < on) ? Gout[(r0 + r) * out + oc + o] : 0.f;
          }
        }
      }
      // Wt[kk][o] = W[oc + o][col(kk)] from the transposed copy (rows along o: coalesced, no conflicts)
      if (vec && ic == KF_IC && (in & 3) == 0) {
        float4 v[9];
#pragma unroll
        for (int q = 0; q < 9; ++q) {
          const int idx = tid + 256 * q, kk = idx >> 4, o4 = idx & 15;
          v[q] = ldg4(WT + (int64_t)kf_col(kk, ic, i0, in) * out + oc + 4 * o4);
        }
#pragma unroll
        for (int q = 0; q < 9; ++q) {
          const int idx = tid + 256 * q, kk = idx >> 4, o4 = idx & 15;
          *reinterpret_cast<float4*>(&WD[kk * KF_CST + 4 * o4]) = v[q];
        }
      } else {
        for (int e = tid; e < kc * KF_O; e += blockDim.x) {
          const int kk = e / KF_O, o = e % KF_O;
          WD[kk * KF_CST + o] = o < on ? WT[(int64_t)kf_col(kk, ic, i0, in) * out + oc + o] : 0.f;
        }
      }
      __syncthreads();
      if ((KAN_ABL & 2) == 0)
        kf_mfma_groups_n(nkt, &Gs[16 * wv + li][4 * lk], &WD[li * KF_CST + 4 * lk], 16 * KF_CST, opad >> 4, acc);
      __syncthreads();
    }
    // columns kc .. 16 nkt - 1 of dA hold products with stale LDS: never read below
#pragma unroll
    for (int j = 0; j < 9; ++j)
      if (j < nkt)
#pragma unroll
        for (int q = 0; q < 4; ++q) WD[(16 * wv + 4 * lk + q) * KF_DST + 16 * j + li] = acc[j][q];
    __syncthreads();
    for (int p = tid; p < KF_R * ic; p += blockDim.x) {
      const int r = p & (KF_R - 1), ii = p >> 6;
      if (r0 + r >= N) continue;
      const float x = Xs[r][ii];
      float b[KAN_NB], db[KAN_NB];
      kan_bases_local<true, true>(x, gk[ii], b, db);
      const float* dA = WD + r * KF_DST;
      float v = silu_grad(x) * dA[ii];
#pragma unroll
      for (int c = 0; c < KAN_NB; ++c) v += db[c] * dA[ic + 8 * ii + c];
      Xs[r][ii] = v;  // same element this thread read: no barrier needed before the write
    }
    __syncthreads();
    for (int e = tid; e < KF_R * ic; e += blockDim.x) {
      const int r = e / ic, ii = e - r * ic;
      if (r0 + r < N) Gin[(r0 + r) * in + i0 + ii] = Xs[r][ii];
    }
    __syncthreads();  // Xs / gk / WD are refilled by the next chunk
  }
}

// ---- hidden layer backward in one pass (out <= 64) --------------------------------------------
// dW and dX of a layer share the bases of every (row, input) pair and the G rows; evaluating them
// once per pass halves the recursion (with its derivative) and the G reads of kan_dw_fused +
// kan_dx_fused.  1-D grid of nchunk x zpad blocks (XCD-grouped as kan_dw_fused), 512 threads:
// a block takes one 16-input chunk and walks the 64-row tiles of its row split:
//   X, G tile -> LDS (the next tile's loads are issued before this tile's products)
//   bases + derivatives -> As[kk][r] (derivatives stay in the registers of the pair's thread)
//   dW chunk += G^T A                    (acc_w; waves: 4 out groups x 2 column halves)
//   dA = G W_chunk (W chunk resident)    (acc_x; waves: 4 row groups x 2 column halves)
//   dA -> LDS over As; Gin = SiLU' dA_base + sum_c B'_c dA_c, out through the X tile.
constexpr int KB_THREADS = 512;

__global__ __launch_bounds__(KB_THREADS) void kan_bwd_fused_kernel(const float* __restrict__ X,
                                                                  const float* __restrict__ grid,
                                                                  const float* __restrict__ G,
                                                                  const float* __restrict__ WT, int64_t N, int in,
                                                                  int out, int64_t rows_per_split, int nchunk,
                                                                  int splits, float* __restrict__ slab,
                                                                  float* __restrict__ Gin) {
  __shared__ __attribute__((aligned(16))) float AD[KF_KC * KF_CST];  // As[kk][r], then dAs[r][kk]
  __shared__ __attribute__((aligned(16))) float GG[KF_O * KF_CST];   // Gt[o][r], then Gs[r][o]
  __shared__ __attribute__((aligned(16))) float Wt[KF_KC * KF_CST];  // W chunk [kk][o]
  __shared__ float Xs[KF_R][KF_IC + 1];
  __shared__ float gk[KF_IC][KF_GST];
  const int L = blockIdx.x, q8 = L >> 3;
  const int cid = q8 % nchunk, z = (q8 / nchunk) * 8 + (L & 7);
  if (z >= splits) return;  // whole block, before any barrier
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, li = lane & 15, lk = lane >> 4;
  const int wr = wv & 3, wh = wv >> 2;  // 16-row (or 16-out) group, column half
  const int i0 = cid * KF_IC;
  const int ic = in - i0 < KF_IC ? in - i0 : KF_IC, kc = 9 * ic, kpad = (kc + 15) & ~15, nkt = kpad >> 4;
  const int j0 = 5 * wh, nj = nkt - j0 < 0 ? 0 : (nkt - j0 > 5 ? 5 : nkt - j0);
  const int opad = (out + 15) & ~15;
  const int64_t K = (int64_t)KAN_K1 * in;
  const bool vec = ic == KF_IC && (in & 3) == 0 && out == KF_O;
  kf_fill_knots(gk, grid, i0, ic);
  // the chunk's W^T [kk][o] stays in LDS for the whole split
  for (int e = tid; e < kpad * KF_O; e += KB_THREADS) {
    const int kk = e / KF_O, o = e % KF_O;
    Wt[kk * KF_CST + o] = (kk < kc && o < out) ? WT[(int64_t)kf_col(kk, ic, i0, in) * out + o] : 0.f;
  }
  const int64_t rb = (int64_t)z * rows_per_split;
  const int64_t re = rb + rows_per_split < N ? rb + rows_per_split : N;
  f32x4 accw[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) accw[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // tile loads (vec path): X one float4 for threads < 256, G two float4 per thread
  const int xr = tid >> 2, xi = (tid & 3) * 4;
  auto load_x = [&](int64_t r0) {
    float4 v = float4{0.f, 0.f, 0.f, 0.f};
    if (tid < 256 && r0 + xr < re) v = ldg4(X + (r0 + xr) * in + i0 + xi);
    return v;
  };
  auto load_g = [&](int64_t r0, int q) {  // piece q: rows (tid + 512 q) & 63, outs 4 * ((tid + 512 q) >> 6)
    const int idx = tid + KB_THREADS * q, r = idx & 63, o4 = idx >> 6;
    float4 v = float4{0.f, 0.f, 0.f, 0.f};
    if (r0 + r < re) v = ldg4(G + (r0 + r) * out + 4 * o4);
    return v;
  };
  float4 xv = float4{0.f, 0.f, 0.f, 0.f}, gv0 = xv, gv1 = xv;
  if (vec && rb < re) {
    xv = load_x(rb);
    gv0 = load_g(rb, 0);
    gv1 = load_g(rb, 1);
  }
  for (int64_t r0 = rb; r0 < re; r0 += KF_R) {
    // ---- X and G^T tiles into LDS
    if (vec) {
      if (tid < 256) {
        Xs[xr][xi] = xv.x;
        Xs[xr][xi + 1] = xv.y;
        Xs[xr][xi + 2] = xv.z;
        Xs[xr][xi + 3] = xv.w;
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const float4 v = q ? gv1 : gv0;
        const int idx = tid + KB_THREADS * q, r = idx & 63, o4 = idx >> 6;
        GG[(4 * o4) * KF_CST + r] = v.x;
        GG[(4 * o4 + 1) * KF_CST + r] = v.y;
        GG[(4 * o4 + 2) * KF_CST + r] = v.z;
        GG[(4 * o4 + 3) * KF_CST + r] = v.w;
      }
    } else {
      kf_stage_x(Xs, X, re, in, r0, i0, ic);
      for (int e = tid; e < KF_R * KF_O; e += KB_THREADS) {
        const int o = e / KF_R, r = e % KF_R;
        GG[o * KF_CST + r] = (r0 + r < re && o < out) ? G[(r0 + r) * out + o] : 0.f;
      }
    }
    __syncthreads();
    // ---- bases (As) and derivatives (registers) of the pairs (r, ii) = (p & 63, p >> 6)
    float dsl[2], dbs[2][KAN_NB];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int p = tid + KB_THREADS * h, r = p & 63, ii = p >> 6;
      dsl[h] = 0.f;
#pragma unroll
      for (int c = 0; c < KAN_NB; ++c) dbs[h][c] = 0.f;
      if (ii < ic) {
        float b[KAN_NB], sl = 0.f;
#pragma unroll
        for (int c = 0; c < KAN_NB; ++c) b[c] = 0.f;
        if (r0 + r < re) {
          const float x = Xs[r][ii];
          kan_bases_local<true, true>(x, gk[ii], b, dbs[h]);
          silu_and_grad(x, sl, dsl[h]);
        }
        AD[ii * KF_CST + r] = sl;
#pragma unroll
        for (int c = 0; c < KAN_NB; ++c) AD[(ic + 8 * ii + c) * KF_CST + r] = b[c];
      }
    }
    for (int e = tid; e < (kpad - kc) * KF_R; e += KB_THREADS) AD[(kc + e / KF_R) * KF_CST + e % KF_R] = 0.f;
    __syncthreads();
    // ---- the next tile's loads go out under this tile's products
    float4 nxv = xv, ngv0 = gv0, ngv1 = gv1;
    if (vec && r0 + KF_R < re) {
      nxv = load_x(r0 + KF_R);
      ngv0 = load_g(r0 + KF_R, 0);
      ngv1 = load_g(r0 + KF_R, 1);
    }
    // ---- dW chunk += G^T A over the tile's rows
    if ((KAN_ABL & 2) == 0)
      kf_mfma_groups_n(nj, &GG[(16 * wr + li) * KF_CST + 4 * lk], &AD[(16 * j0 + li) * KF_CST + 4 * lk], 16 * KF_CST,
                       KF_R / 16, accw);
    __syncthreads();
    // ---- G rows [r][o] over G^T, then dA = G W_chunk
    if (vec) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int idx = tid + KB_THREADS * q, r = idx & 63, o4 = idx >> 6;
        *reinterpret_cast<float4*>(&GG[r * KF_CST + 4 * o4]) = q ? gv1 : gv0;
      }
    } else {
      for (int e = tid; e < KF_R * KF_O; e += KB_THREADS) {
        const int r = e / KF_O, o = e % KF_O;
        GG[r * KF_CST + o] = (r0 + r < re && o < out) ? G[(r0 + r) * out + o] : 0.f;
      }
    }
    __syncthreads();
    f32x4 accx[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) accx[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if ((KAN_ABL & 2) == 0)
      kf_mfma_groups_n(nj, &GG[(16 * wr + li) * KF_CST + 4 * lk], &Wt[(16 * j0 + li) * KF_CST + 4 * lk], 16 * KF_CST,
                       opad >> 4, accx);
    // dA tile over As (last read by the dW products, before the barrier above); columns past kc
    // hold products of zero-padded W rows and are never read
#pragma unroll
    for (int j = 0; j < 5; ++j)
      if (j < nj)
#pragma unroll
        for (int q = 0; q < 4; ++q) AD[(16 * wr + 4 * lk + q) * KF_DST + 16 * (j0 + j) + li] = accx[j][q];
    __syncthreads();
    // ---- Gin through the X tile
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int p = tid + KB_THREADS * h, r = p & 63, ii = p >> 6;
      if (ii < ic && r0 + r < re) {
        const float* dA = AD + r * KF_DST;
        float v = dsl[h] * dA[ii];
#pragma unroll
        for (int c = 0; c < KAN_NB; ++c) v += dbs[h][c] * dA[ic + 8 * ii + c];
        Xs[r][ii] = v;
      }
    }
    __syncthreads();
    for (int e = tid; e < KF_R * ic; e += KB_THREADS) {
      const int r = e / ic, ii = e - r * ic;
      if (r0 + r < re) Gin[(r0 + r) * in + i0 + ii] = Xs[r][ii];
    }
    xv = nxv;
    gv0 = ngv0;
    gv1 = ngv1;
    __syncthreads();  // Xs / GG / AD are refilled by the next tile
  }
  float* out_slab = slab + (int64_t)z * out * K;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int kk = 16 * (j0 + j) + li;
    if (j >= nj || kk >= kc) continue;
    const int64_t col = kf_col(kk, ic, i0, in);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int o = 16 * wr + 4 * lk + q;
      if (o < out) out_slab[(int64_t)o * K + col] = accw[j][q];
    }
  }
}

// W[o][i] = base_w[o][i];  W[o][in + 8 i + c] = spline_w[o][i][c] * scaler[o][i]  (kan.py:145-151)
__global__ void kan_combine_kernel(const float* __restrict__ base_w, const float* __restrict__ spline_w,
                                   const float* __restrict__ scaler, int out, int in, float* __restrict__ W,
                                   float* __restrict__ WT) {
  const int total = out * in;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int o = e / in, i = e - o * in;
    float* row = W + (int64_t)o * KAN_K1 * in;
    row[i] = base_w[e];
    if (WT) WT[(int64_t)i * out + o] = base_w[e];
    const float s = scaler[e];
#pragma unroll
    for (int c = 0; c < KAN_NB; ++c) {
      const float v = spline_w[(int64_t)e * KAN_NB + c] * s;
      row[in + KAN_NB * i + c] = v;
      if (WT) WT[(int64_t)(in + KAN_NB * i + c) * out + o] = v;
    }
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

// out[e] = sum_z slab[z][e] in a fixed order: a block takes C columns; its 256 / C thread groups
// sum every (256/C)-th slab row (4 loads in flight per thread), then the group partials add up
// in group order.  C = 64 for wide slabs; C = 16 (64-byte row segments, 16 groups) when there are
// few columns and many slab rows.
template <int C>
__global__ __launch_bounds__(256) void kan_slab_reduce_kernel(const float* __restrict__ slab, int splits, int64_t mn,
                                                              float* __restrict__ out) {
  constexpr int NG = 256 / C;
  __shared__ float part[NG][C];
  const int col = threadIdx.x % C, grp = threadIdx.x / C;
  const int64_t e = (int64_t)blockIdx.x * C + col;
  float acc = 0.f;
  if (e < mn) {
    int z = grp;
    for (; z + 3 * NG < splits; z += 4 * NG) {
      const float a0 = slab[(int64_t)z * mn + e], a1 = slab[(int64_t)(z + NG) * mn + e];
      const float a2 = slab[(int64_t)(z + 2 * NG) * mn + e], a3 = slab[(int64_t)(z + 3 * NG) * mn + e];
      acc = (((acc + a0) + a1) + a2) + a3;
    }
    for (; z < splits; z += NG) acc += slab[(int64_t)z * mn + e];
  }
  part[grp][col] = acc;
  __syncthreads();
  if (grp == 0 && e < mn) {
    float v = part[0][col];
#pragma unroll
    for (int g = 1; g < NG; ++g) v += part[g][col];
    out[e] = v;
  }
}

static hipError_t slab_reduce(const float* slab, int splits, int64_t mn, float* out, hipStream_t s) {
  if (mn < 64 * 256 && splits > 64)
    hipLaunchKernelGGL(kan_slab_reduce_kernel<16>, dim3((unsigned)((mn + 15) / 16)), dim3(256), 0, s, slab, splits, mn, out);
  else
    hipLaunchKernelGGL(kan_slab_reduce_kernel<64>, dim3((unsigned)((mn + 63) / 64)), dim3(256), 0, s, slab, splits, mn, out);
  return hipGetLastError();
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
  if (N <= 0 || in <= 0 || in > 64) return hipErrorInvalidValue;
  const int64_t blocks = (N + 3) / 4;
  hipLaunchKernelGGL(kan_head_fwd_kernel, dim3((unsigned)(blocks < 16384 ? blocks : 16384)), dim3(256), 0, s, X, grid, W,
                     N, in, Y);
  return hipGetLastError();
}

// the last layer's training pass (out = 1, in <= 64): returns the number of squared-error
// partials written (<= max_parts, one per block) in *nparts
hipError_t kan_head_train(const float* X, const float* grid, const float* W, const float* y, int64_t N, int in,
                          int64_t n_valid, float gfac, int64_t slots, int64_t max_parts, float* out, float* g,
                          float* sse_part, float* slab, float* dW, float* Gin, int* nparts, hipStream_t s) {
  if (N <= 0 || in <= 0 || in > 64 || slots < 1 || max_parts < 1 || !nparts) return hipErrorInvalidValue;
  int64_t blocks = (N + 255) / 256;
  if (blocks > slots) blocks = slots;
  if (blocks > max_parts) blocks = max_parts;
  const int64_t rpb = (N + blocks - 1) / blocks;
  blocks = (N + rpb - 1) / rpb;
  hipLaunchKernelGGL(kan_head_train_kernel, dim3((unsigned)blocks), dim3(256), 0, s, X, grid, W, y, N, in, n_valid, gfac,
                     rpb, out, g, sse_part, slab, Gin);
  *nparts = (int)blocks;
  return slab_reduce(slab, (int)blocks, (int64_t)KAN_K1 * in, dW, s);
}

// dW[o][k] = sum_n G[n][o] A[n][k]: `splits` row slices into slabs, then the fixed-order slab sum
hipError_t kan_dw_fused(const float* X, const float* grid, const float* G, int64_t N, int in, int out,
                        int64_t max_splits, float* slab, float* dW, hipStream_t s) {
  if (N <= 0 || in <= 0 || out <= 0 || max_splits < 1) return hipErrorInvalidValue;
  const int nchunk = (in + KF_IC - 1) / KF_IC, nout = (out + KF_O - 1) / KF_O;
  // one round of resident blocks (2 per CU x 256 CUs): every CU busy, no tail
  int64_t splits = kKanResidentBlocks / ((int64_t)nchunk * nout);
  if (splits < 1) splits = 1;
  if (splits > max_splits) splits = max_splits;
  int64_t rps = (N + splits - 1) / splits;
  rps = (rps + KF_R - 1) / KF_R * KF_R;
  const int z = (int)((N + rps - 1) / rps);
  const int64_t blocks = (int64_t)nchunk * nout * ((z + 7) / 8 * 8);
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kan_dw_fused_kernel, dim3((unsigned)blocks), dim3(256), 0, s, X, grid, G, N, in, out, rps, nchunk,
                     nout, z, slab);
  const int64_t mn = (int64_t)out * KAN_K1 * in;
  return slab_reduce(slab, z, mn, dW, s);
}

hipError_t kan_dx_fused(const float* X, const float* grid, const float* Gout, const float* WT, int64_t N, int in,
                        int out, float* Gin, hipStream_t s) {
  if (N <= 0 || in <= 0 || out <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kan_dx_fused_kernel, dim3((unsigned)((N + KF_R - 1) / KF_R)), dim3(256), 0, s, X, grid, Gout, WT,
                     N, in, out, Gin);
  return hipGetLastError();
}

// dW (split-K slabs + fixed-order sum) and Gin of a layer with out <= 64 in one pass
hipError_t kan_bwd_fused(const float* X, const float* grid, const float* G, const float* WT, int64_t N, int in, int out,
                         int64_t max_splits, float* slab, float* dW, float* Gin, hipStream_t s) {
  if (N <= 0 || in <= 0 || out <= 0 || out > KF_O || max_splits < 1) return hipErrorInvalidValue;
  const int nchunk = (in + KF_IC - 1) / KF_IC;
  int64_t splits = kKanBwdResidentBlocks / nchunk;  // one block per CU (LDS), one round
  if (splits < 1) splits = 1;
  if (splits > max_splits) splits = max_splits;
  int64_t rps = (N + splits - 1) / splits;
  rps = (rps + KF_R - 1) / KF_R * KF_R;
  const int z = (int)((N + rps - 1) / rps);
  const int64_t blocks = (int64_t)nchunk * ((z + 7) / 8 * 8);
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kan_bwd_fused_kernel, dim3((unsigned)blocks), dim3(KB_THREADS), 0, s, X, grid, G, WT, N, in, out,
                     rps, nchunk, z, slab, Gin);
  return slab_reduce(slab, z, (int64_t)out * KAN_K1 * in, dW, s);
}

hipError_t kan_combine(const float* base_w, const float* spline_w, const float* scaler, int out, int in, float* W,
                       float* WT, hipStream_t s) {
  hipLaunchKernelGGL(kan_combine_kernel, dim3(ew_grid((int64_t)out * in)), dim3(256), 0, s, base_w, spline_w,
                     scaler, out, in, W, WT);
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
  if (z > 1) return slab_reduce(C, z, (int64_t)M * N, out, s);
  return hipGetLastError();
}

}  // namespace siren
