// Memory-bound SIREN kernels: coordinate grid, fp32 first layer, head/MSE, column
// reductions, fused Adam, ReduceLROnPlateau and the h16 weight shadows.
#include <math.h>
#include "siren_common.h"
#include "siren_kernels.h"

namespace siren {

static inline int grid_for(int64_t n, int per_block, int cap = 8192) {
  int64_t g = (n + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

// ---------------------------------------------------------------------------------
// get_coord / torch.linspace(-1, 1, N) (utils.py:99-109), evaluated at global indices
// [offset, offset+rows): i < N/2 -> fma(step, i, -1), else fma(-step, N-1-i, 1), step = 2/(N-1)
// (the contracted form torch's CPU kernel computes; bit-exact with torch.linspace).
__global__ void coords_fill_kernel(float* t, int64_t rows, int64_t offset, int64_t n_total) {
  const float step = (n_total > 1) ? 2.0f / (float)(n_total - 1) : 0.f;
  const int64_t half = n_total / 2;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows;
       r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = offset + r;
    float v;
    if (i >= n_total) v = 0.f;  // padding rows
    else if (n_total == 1) v = -1.0f;
    else if (i < half) v = __builtin_fmaf(step, (float)i, -1.0f);
    else v = __builtin_fmaf(-step, (float)(n_total - 1 - i), 1.0f);
    t[r] = v;
  }
}

hipError_t coords_fill(float* t, int64_t rows, int64_t offset, int64_t n_total, hipStream_t s) {
  hipLaunchKernelGGL(coords_fill_kernel, dim3(grid_for(rows, 256)), dim3(256), 0, s, t, rows, offset,
                     n_total);
  return hipGetLastError();
}

// torch.linspace(-1, 1, n)[i] in fp32 (the same contracted form as coords_fill_kernel)
__device__ __forceinline__ float linspace_at(int64_t i, int64_t n) {
  if (n == 1) return -1.0f;
  const float step = 2.0f / (float)(n - 1);
  return (i < n / 2) ? __builtin_fmaf(step, (float)i, -1.0f) : __builtin_fmaf(-step, (float)(n - 1 - i), 1.0f);
}

// MultiWaveformFitting's (time, channel) grid (utils.py:211-220): row k of the height-major
// meshgrid is (linspace(-1,1,height)[k / width], linspace(-1,1,width)[k % width]), channel 0
// when width == 1 (linspace(0, 0, 1)).  One float2 per row, coalesced 8-B stores.
__global__ void coords_grid_kernel(float2* xy, int64_t rows, int64_t offset, int64_t height, int width) {
  const int64_t n = height * width;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows;
       r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = offset + r;
    float2 v = {0.f, 0.f};
    if (k < n) {
      const int64_t i = k / width;
      const int j = (int)(k - i * width);
      v.x = linspace_at(i, height);
      v.y = width == 1 ? 0.f : linspace_at(j, width);
    }
    xy[r] = v;
  }
}

hipError_t coords_fill_grid(float* xy, int64_t rows, int64_t offset, int64_t height, int width, hipStream_t s) {
  hipLaunchKernelGGL(coords_grid_kernel, dim3(grid_for(rows, 256)), dim3(256), 0, s, (float2*)xy, rows, offset,
                     height, width);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------
// First SineLayer (is_first=True, models.py:105-115): y0 = sin(omega0 * (t W0^T + b0)).
// Kept in fp32 end to end: |omega0*z| reaches ~4.4e4 rad at omega0 = 22000, so the
// pre-activation a is formed exactly as torch's CPU addmm rounds it (K=1: one fma;
// K=2: fma(t1, w1, t0*w0) + b), then reduced in revolutions with a two-part 1/(2*pi):
//   r = fma(a, inv2pi_hi, -n) + a * inv2pi_lo,  n = rint(a * inv2pi_hi)
// fma forms a*inv2pi_hi - n with one rounding (|r| <= 1/2: error <= 2^-25 rev), the low part
// adds < 2e-4 rev with 2^-24 relative error, so r is within ~4e-8 rev (2.5e-7 rad) of a/(2pi)
// mod 1 for every |a| < 2^17.  v_sin_f32 / v_cos_f32 take revolutions directly.  (OCML's
// sincosf with its large-argument reduction made this kernel VALU-bound at 2.1 ms.)
// (sincos_rev / first_preact live in siren_common.h.  A layer-0 dX epilogue that recomputed this
// cosine instead of reading C0 was measured in round 2 and removed: DESIGN §4.)
// Row-wise: each thread owns 8 columns (W0 / b0 in registers) and walks rows; a row is H/8
// threads, a 256-thread block covers 256/(H/8) rows per pass; Y0 / C0 go out as 16-B pieces.
// SNAKE (first_linear=True, models.py:330-333): Linear(in, H) + Snake(a0) --
// Y0 = z + sin^2(a z)/a, C0 = 1 + sin(2az) (dY/dz), E0 = (z sin(2az) - sin^2(az)/a)/a (dY/da)
template <bool STORE_C, bool SNAKE>
__global__ void first_fwd_kernel(const float* __restrict__ t, int in_dim, const float* __restrict__ W0,
                                 const float* __restrict__ b0, float omega0, int R, int H,
                                 h16* __restrict__ Y0, h16* __restrict__ C0, const float* __restrict__ a0,
                                 h16* __restrict__ E0, int ld) {
  const int tpr = H >> 3;
  const int rpb = blockDim.x / tpr;
  const int lt = threadIdx.x % tpr, lr = threadIdx.x / tpr;
  const int n = lt * 8;
  float w0[8], w1[8], bb[8], av[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    w0[r] = W0[(n + r) * in_dim];
    w1[r] = (in_dim > 1) ? W0[(n + r) * in_dim + 1] : 0.f;
    bb[r] = b0[n + r];
    av[r] = SNAKE ? a0[n + r] : 0.f;
  }
  // the next row's coordinates are loaded before this row's stores: vmcnt retires loads and
  // stores in issue order, so a load issued after the stores would wait for them too
  const int64_t stride = (int64_t)gridDim.x * rpb;
  int64_t m = (int64_t)blockIdx.x * rpb + lr;
  float t0n = 0.f, t1n = 0.f;
  if (m < R) {
    t0n = t[m * in_dim];
    if (in_dim > 1) t1n = t[m * in_dim + 1];
  }
  for (; m < R; m += stride) {
    const float t0 = t0n, t1 = t1n;
    if (m + stride < R) {
      t0n = t[(m + stride) * in_dim];
      if (in_dim > 1) t1n = t[(m + stride) * in_dim + 1];
    }
    float y[8], c[8], ev[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      if constexpr (SNAKE) {
        snake_epi(first_preact(in_dim, t0, t1, w0[r], w1[r], bb[r]), av[r], 1.0f / av[r], y[r], c[r], ev[r]);
        continue;
      }
      sincos_rev(omega0 * first_preact(in_dim, t0, t1, w0[r], w1[r], bb[r]), &y[r], &c[r]);
    }
    h16x8 yv, cv;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      yv[r] = (h16)y[r];
      cv[r] = (h16)c[r];
    }
    *(h16x8*)(Y0 + m * ld + n) = yv;
    if constexpr (STORE_C) *(h16x8*)(C0 + m * ld + n) = cv;
    if constexpr (SNAKE) {
      h16x8 evv;
#pragma unroll
      for (int r = 0; r < 8; ++r) evv[r] = (h16)ev[r];
      *(h16x8*)(E0 + m * ld + n) = evv;
    }
  }
}

hipError_t first_fwd(const float* t, int in_dim, const float* W0, const float* b0, float omega0,
                     int R, int H, h16* Y0, h16* C0, hipStream_t s, const float* a0, h16* E0) {
  // widths above 2048 run as launches over 1024-column windows (row stride H; every element's
  // arithmetic is its own column's, so the result is the one-launch result)
  const int win = H <= 2048 ? H : 1024;
  if (H < 8 || H % 8 || 256 % (win / 8) || H % win || in_dim < 1 || in_dim > 2) return hipErrorInvalidValue;
  if ((a0 != nullptr) != (E0 != nullptr) || (a0 && !C0)) return hipErrorInvalidValue;
  const int rpb = 256 / (win / 8);
  const dim3 grid(grid_for(R, rpb, 4096));
  auto off = [](auto* v, int nb) { return v ? v + nb : v; };
  for (int nb = 0; nb < H; nb += win) {
    const float* W0w = W0 + (size_t)nb * in_dim;
    // C0 == NULL: Y0 only (the cos is not needed); a0 != NULL: Linear + Snake first layer
    if (a0)
      hipLaunchKernelGGL((first_fwd_kernel<true, true>), grid, dim3(256), 0, s, t, in_dim, W0w, b0 + nb, omega0, R,
                         win, Y0 + nb, off(C0, nb), a0 + nb, off(E0, nb), H);
    else if (C0)
      hipLaunchKernelGGL((first_fwd_kernel<true, false>), grid, dim3(256), 0, s, t, in_dim, W0w, b0 + nb, omega0, R,
                         win, Y0 + nb, C0 + nb, a0, E0, H);
    else
      hipLaunchKernelGGL((first_fwd_kernel<false, false>), grid, dim3(256), 0, s, t, in_dim, W0w, b0 + nb, omega0, R,
                         win, Y0 + nb, C0, a0, E0, H);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// ---------------------------------------------------------------------------------
// Final nn.Linear(H,1) + MSELoss (models.py:374-381, run.py:125,168):
//   out = sum_j head_part[j][m] + b;  err = out - y;  g = err * (2/N_total) (0 on pad rows)
// plus per-block partial sums of err^2 (loss) and g (bias gradient), and per-block max |g|
// (for grad_scale).  loss_mode 1 = L1Loss (run.py:124, 161-163, loss_mode='mae'): the loss
// term is |err| and g = sign(err) * (1/N_total) (torch's sign: 0 at err == 0); the caller
// passes gfac = 1/N_total then.
__global__ void head_loss_kernel(const float* __restrict__ head_part, int nparts, int R,
                                 const float* __restrict__ b_head, const float* __restrict__ y,
                                 int n_valid, float gfac, float* __restrict__ out,
                                 float* __restrict__ g, float* __restrict__ sse_part,
                                 float* __restrict__ gsum_part, float* __restrict__ gmax_part,
                                 float head_omega, int loss_mode) {
  __shared__ float scratch[12];  // 3 x (256 / 64) (block_sum2_max)
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  float e2 = 0.f, gv = 0.f;
  if (m < R) {
    float o = 0.f;
    for (int j = 0; j < nparts; ++j) o += head_part[(size_t)j * R + m];
    o += b_head[0];
    // last_linear=False: the last layer is SineLayer(H, 1, omega) -- out = sin(omega * o) and
    // g is the gradient at the linear output o: 2(out - y)/N * cos(omega o) * omega
    const float a = head_omega * o;
    const float ov = head_omega > 0.f ? sinf(a) : o;
    out[m] = ov;
    if (m < n_valid) {
      const float err = ov - y[m];
      if (loss_mode == 1) {
        e2 = fabsf(err);
        gv = (err > 0.f ? 1.0f : (err < 0.f ? -1.0f : 0.f)) * gfac;
      } else {
        e2 = err * err;
        gv = err * gfac;
      }
      if (head_omega > 0.f) gv = (gv * cosf(a)) * head_omega;
    }
    g[m] = gv;
  }
  float se = e2, gs = gv, gm = fabsf(gv);
  block_sum2_max(se, gs, gm, scratch);
  if (threadIdx.x == 0) {
    sse_part[blockIdx.x] = se;
    gsum_part[blockIdx.x] = gs;
    if (gmax_part) gmax_part[blockIdx.x] = gm;
  }
}

hipError_t head_loss(const float* head_part, int nparts, int R, const float* b_head, const float* y,
                     int n_valid, float gfac, float* out, float* g, float* sse_part,
                     float* gsum_part, float* gmax_part, hipStream_t s, float head_omega, int loss_mode) {
  hipLaunchKernelGGL(head_loss_kernel, dim3((R + 255) / 256), dim3(256), 0, s, head_part, nparts, R,
                     b_head, y, n_valid, gfac, out, g, sse_part, gsum_part, gmax_part, head_omega, loss_mode);
  return hipGetLastError();
}

// last_linear=False in siren_backward: dLoss/dout -> dLoss/do at the final SineLayer's linear
// output o = sum head_part + b (kept from the forward): g *= cos(omega o) * omega
__global__ void head_sine_chain_kernel(const float* __restrict__ head_part, int nparts, int R,
                                       const float* __restrict__ b_head, float omega, float* __restrict__ g) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= R) return;
  float o = 0.f;
  for (int j = 0; j < nparts; ++j) o += head_part[(size_t)j * R + m];
  o += b_head[0];
  g[m] = (g[m] * cosf(omega * o)) * omega;
}

hipError_t head_sine_chain(const float* head_part, int nparts, int R, const float* b_head, float omega, float* g,
                           hipStream_t s) {
  hipLaunchKernelGGL(head_sine_chain_kernel, dim3((R + 255) / 256), dim3(256), 0, s, head_part, nparts, R, b_head,
                     omega, g);
  return hipGetLastError();
}

// Per-256-row-block max |g| of an externally supplied dLoss/dout (siren_backward).
__global__ void gmax_partials_kernel(const float* __restrict__ g, int R, float* __restrict__ gmax_part) {
  __shared__ float scratch[4];
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  const float gm = block_max(m < R ? fabsf(g[m]) : 0.f, scratch);
  if (threadIdx.x == 0) gmax_part[blockIdx.x] = gm;
}

hipError_t gmax_partials(const float* g, int R, float* gmax_part, hipStream_t s) {
  hipLaunchKernelGGL(gmax_partials_kernel, dim3((R + 255) / 256), dim3(256), 0, s, g, R, gmax_part);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------
// Backward gradient scale.  dZ is stored in fp16 (11-bit significand, the precision the
// forward needs -- DESIGN.md "Storage precision"), whose exponent range cannot hold raw
// MSE gradients (|g| ~ 2|err|/N reaches 1e-9 at N = 2^20).  The head backward therefore
// stores dZ * S with S = 2^k chosen so that its bound max|g| * max|w_head| * omega lands
// just under 2^6 (headroom for growth through the layers below), and every fp32 gradient
// reduced from a scaled dZ is multiplied by 1/S.  Powers of two: scaling is exact.
// gscale[0] = S, gscale[1] = 1/S.  One block.  The exponent target (6 above) comes from the
// range guard when one is given: siren_apply_update lowers it after an fp16 overflow.
__global__ void grad_scale_kernel(const float* __restrict__ gmax_part, int nparts,
                                  const float* __restrict__ w_head, int H, float omega,
                                  float* __restrict__ gscale, const GuardState* __restrict__ guard) {
  __shared__ float scratch[4];
  float gm = 0.f, wm = 0.f;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) gm = fmaxf(gm, gmax_part[i]);
  for (int i = threadIdx.x; i < H; i += blockDim.x) wm = fmaxf(wm, fabsf(w_head[i]));
  gm = block_max(gm, scratch);
  wm = block_max(wm, scratch);
  if (threadIdx.x == 0) {
    const float bound = gm * wm * fabsf(omega);
    int k = 0;
    if (bound > 0.f && bound < INFINITY) {
      int e;
      (void)frexpf(bound, &e);  // bound < 2^e
      k = (guard ? guard->headroom : kHeadroomDefault) - e;
      k = k < -100 ? -100 : (k > 100 ? 100 : k);
    }
    gscale[0] = ldexpf(1.0f, k);
    gscale[1] = ldexpf(1.0f, -k);
  }
}

// S for the fused head backward (NT_FWD_HB), fixed BEFORE the forward, so it cannot use the step's
// max|g|.  Instead it bounds it from quantities known then: MSE g = (out - y) * gfac with
// |out| <= sum|w_head| * max|Y_L| + |b_head| (max|Y_L| <= 1 for a sine / tanh last layer; 1 for
// the final sine of last_linear=False), L1 |g| <= gfac, times head_omega through the final sine.
// The bound is loose by ~sum|w_head| / max|out - y| (2^4-2^5 at H = 1024), which only moves
// dZ_L x S further below the fp16 maximum (scaling by a power of two is exact above fp16's
// normal minimum).  ymax_part: per-256-row max|target| partials (gmax_partials on the target).
__global__ void grad_scale_bound_kernel(const float* __restrict__ ymax_part, int nparts,
                                        const float* __restrict__ w_head, const float* __restrict__ b_head, int H,
                                        float gfac, float head_omega, int loss_mode, float act_bound,
                                        float* __restrict__ gscale, const GuardState* __restrict__ guard) {
  __shared__ float scratch[4];
  float ym = 0.f, wm = 0.f, ws = 0.f;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) ym = fmaxf(ym, ymax_part[i]);
  for (int i = threadIdx.x; i < H; i += blockDim.x) {
    const float a = fabsf(w_head[i]);
    wm = fmaxf(wm, a);
    ws += a;
  }
  ym = block_max(ym, scratch);
  wm = block_max(wm, scratch);
  ws = block_sum(ws, scratch);
  if (threadIdx.x == 0) {
    float gb = loss_mode == 1 ? gfac : gfac * ((head_omega > 0.f ? 1.0f : ws + fabsf(b_head[0])) + ym);
    if (head_omega > 0.f) gb *= head_omega;
    // 2^-10 of slack over the fp32 roundings of the bound itself
    const float bound = gb * wm * fabsf(act_bound) * (1.0f + 0x1p-10f);
    int k = 0;
    if (bound > 0.f && bound < INFINITY) {
      int e;
      (void)frexpf(bound, &e);
      k = (guard ? guard->headroom : kHeadroomDefault) - e;
      k = k < -100 ? -100 : (k > 100 ? 100 : k);
    }
    gscale[0] = ldexpf(1.0f, k);
    gscale[1] = ldexpf(1.0f, -k);
  }
}

hipError_t grad_scale_bound(const float* ymax_part, int nparts, const float* w_head, const float* b_head, int H,
                            float gfac, float head_omega, int loss_mode, float act_bound, float* gscale,
                            hipStream_t s, const GuardState* guard) {
  hipLaunchKernelGGL(grad_scale_bound_kernel, dim3(1), dim3(256), 0, s, ymax_part, nparts, w_head, b_head, H, gfac,
                     head_omega, loss_mode, act_bound, gscale, guard);
  return hipGetLastError();
}

hipError_t grad_scale(const float* gmax_part, int nparts, const float* w_head, int H, float omega,
                      float* gscale, hipStream_t s, const GuardState* guard) {
  hipLaunchKernelGGL(grad_scale_kernel, dim3(1), dim3(256), 0, s, gmax_part, nparts, w_head, H, omega,
                     gscale, guard);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------
// Backward through the head into the last hidden SineLayer:
//   dY[m][n] = g[m]*w[n];  dZ = (dY * cos) * omega;  db partial = sum_m dZ;
//   dw_head partial = sum_m g[m]*Y[m][n].     One block per 128 rows.
// A Snake / Tanh last layer passes its derivative as C with omega = 1; a Snake one also E
// (dY/da) and gets da partial = sum_m dY[m][n]*E[m][n].
// The partials are unscaled; the stored dZ carries the gradient scale S (grad_scale).
template <int V>  // columns per thread: 8 (16-B loads) when H allows, else 4
__global__ __launch_bounds__(256) void head_bwd_kernel(
    const h16* __restrict__ C, const h16* __restrict__ Y, const float* __restrict__ g,
    const float* __restrict__ w_head, float omega, int R, int H, const float* __restrict__ gscale,
    h16* __restrict__ dZ, float* __restrict__ db_part, float* __restrict__ dwh_part,
    const h16* __restrict__ E, float* __restrict__ da_part, int ld) {
  typedef _Float16 hv __attribute__((ext_vector_type(V)));
  __shared__ float red[3][256 * V];
  const float S = gscale ? gscale[0] : 1.0f;  // dZ storage scale (grad_scale)
  const int hq = H / V;                        // column groups (divides 256)
  const int cq = threadIdx.x % hq, rg = threadIdx.x / hq, nrg = blockDim.x / hq;
  const int n = cq * V;
  float wv[V], db[V], dw[V], da[V];
#pragma unroll
  for (int k = 0; k < V; ++k) {
    wv[k] = w_head[n + k];
    db[k] = dw[k] = da[k] = 0.f;
  }
  const int64_t m0 = (int64_t)blockIdx.x * 128;
  // rows rg, rg + nrg, ...: unrolled so that several rows' loads are in flight per thread
#pragma unroll 4
  for (int r = rg; r < 128; r += nrg) {
    const int64_t m = m0 + r;
    const float gm = g[m];
    const hv c = *(const hv*)(C + m * ld + n);
    const hv yv = *(const hv*)(Y + m * ld + n);
    hv ev = {};
    if (E) ev = *(const hv*)(E + m * ld + n);
    hv out;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const float dz = ((gm * wv[k]) * (float)c[k]) * omega;
      db[k] += dz;
      dw[k] += gm * (float)yv[k];
      da[k] += (gm * wv[k]) * (float)ev[k];
      out[k] = (_Float16)(dz * S);
    }
    *(hv*)(dZ + m * ld + n) = out;
  }
#pragma unroll
  for (int k = 0; k < V; ++k) {
    red[0][threadIdx.x * V + k] = db[k];
    red[1][threadIdx.x * V + k] = dw[k];
    red[2][threadIdx.x * V + k] = da[k];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < H; c += blockDim.x) {
    const int q = c / V, k = c % V;
    float a = 0.f, b = 0.f, d = 0.f;
    for (int gi = 0; gi < nrg; ++gi) {
      a += red[0][(gi * hq + q) * V + k];
      b += red[1][(gi * hq + q) * V + k];
      d += red[2][(gi * hq + q) * V + k];
    }
    db_part[(size_t)blockIdx.x * ld + c] = a;
    dwh_part[(size_t)blockIdx.x * ld + c] = b;
    if (E) da_part[(size_t)blockIdx.x * ld + c] = d;
  }
}

hipError_t head_bwd(const h16* C, const h16* Y, const float* g, const float* w_head, float omega,
                    int R, int H, const float* gscale, h16* dZ, float* db_part, float* dwh_part,
                    const h16* E, float* da_part, hipStream_t s) {
  // widths above 2048: launches over 1024-column windows (row stride H), each column's sums as in one
  const int win = H <= 2048 ? H : 1024;
  if (R % 128 || H < 4 || win % 4 || H % win || (E && !da_part)) return hipErrorInvalidValue;
  const bool v8 = win % 8 == 0 && 256 % (win / 8) == 0;
  if (!v8 && 256 % (win / 4)) return hipErrorInvalidValue;
  for (int nb = 0; nb < H; nb += win) {
    const h16* Ew = E ? E + nb : E;
    float* daw = da_part ? da_part + nb : da_part;
    if (v8)
      hipLaunchKernelGGL(head_bwd_kernel<8>, dim3(R / 128), dim3(256), 0, s, C + nb, Y + nb, g, w_head + nb, omega, R,
                         win, gscale, dZ + nb, db_part + nb, dwh_part + nb, Ew, daw, H);
    else
      hipLaunchKernelGGL(head_bwd_kernel<4>, dim3(R / 128), dim3(256), 0, s, C + nb, Y + nb, g, w_head + nb, omega, R,
                         win, gscale, dZ + nb, db_part + nb, dwh_part + nb, Ew, daw, H);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// ---------------------------------------------------------------------------------
// Deterministic column reduction of partial rows, two passes of the same kernel:
// pass 1 sums row chunks into tmp[64][ncols], pass 2 sums those 64 rows.  Up to kMaxColSegs
// reductions of one partial-row layout (same row stride and row count, e.g. db and the dW0
// columns of one NT_DX0 epilogue) share the two launches: segment z = blockIdx.z, with its own
// 64-row slice of tmp; every segment's summation order is the one-segment order.
__device__ __forceinline__ void col_reduce_block(const float* __restrict__ part, int64_t row_stride, int nrows,
                                                 int ncols, float* __restrict__ out, int64_t out_row_stride,
                                                 int out_stride, int accumulate) {
  __shared__ float red[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  const int chunk = blockIdx.y, nchunk = gridDim.y;
  const int r0 = (int)(((int64_t)chunk * nrows) / nchunk);
  const int r1 = (int)(((int64_t)(chunk + 1) * nrows) / nchunk);
  float s = 0.f;
  if (col < ncols) {
    // rows r0 + rg, r0 + rg + 4, ... summed in that order; 8 loads in flight ahead of the adds
    // (one dependent load per row made pass 1 latency-bound)
    int r = r0 + rg;
    for (; r + 28 < r1; r += 32) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(r + 4 * u) * row_stride + col];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; r < r1; r += 4) s += part[(int64_t)r * row_stride + col];
  }
  red[rg][threadIdx.x & 63] = s;
  __syncthreads();
  if (rg == 0 && col < ncols) {
    const float v = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    float* o = out + (int64_t)chunk * out_row_stride + (int64_t)col * out_stride;
    *o = accumulate ? (*o + v) : v;
  }
}

// pass: 0 = one pass (part -> out), 1 = row chunks -> tmp, 2 = tmp -> out
__global__ void col_reduce_kernel(ColSegs sg, int64_t row_stride, int nrows, int ncols, int pass, float* tmp,
                                  int accumulate) {
  const int z = blockIdx.z;
  float* tz = tmp + (int64_t)z * 64 * ncols;
  if (pass == 0)
    col_reduce_block(sg.src[z], row_stride, nrows, ncols, sg.out[z], 0, sg.out_stride[z], accumulate);
  else if (pass == 1)
    col_reduce_block(sg.src[z], row_stride, nrows, ncols, tz, ncols, 1, 0);
  else
    col_reduce_block(tz, ncols, 64, ncols, sg.out[z], 0, sg.out_stride[z], accumulate);
}

hipError_t col_reduce_multi(const ColSegs& sg, int64_t row_stride, int nrows, int ncols, int accumulate, float* tmp,
                            hipStream_t s) {
  if (sg.n < 1 || sg.n > kMaxColSegs) return hipErrorInvalidValue;
  const int cb = (ncols + 63) / 64;
  if (nrows <= 256) {
    hipLaunchKernelGGL(col_reduce_kernel, dim3(cb, 1, sg.n), dim3(256), 0, s, sg, row_stride, nrows, ncols, 0,
                       tmp, accumulate);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(col_reduce_kernel, dim3(cb, 64, sg.n), dim3(256), 0, s, sg, row_stride, nrows, ncols, 1, tmp,
                     0);
  hipLaunchKernelGGL(col_reduce_kernel, dim3(cb, 1, sg.n), dim3(256), 0, s, sg, row_stride, nrows, ncols, 2, tmp,
                     accumulate);
  return hipGetLastError();
}

hipError_t col_reduce(const float* part, int64_t row_stride, int nrows, int ncols, float* out,
                      int out_stride, int accumulate, float* tmp, hipStream_t s) {
  ColSegs sg = {};
  sg.n = 1;
  sg.src[0] = part;
  sg.out[0] = out;
  sg.out_stride[0] = out_stride;
  return col_reduce_multi(sg, row_stride, nrows, ncols, accumulate, tmp, s);
}

// out[0] (+)= sum(x[0..n))  -- single block, fixed order.
__global__ void sum_to_kernel(const float* __restrict__ x, int n, float* out, int accumulate) {
  __shared__ float scratch[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += x[i];
  s = block_sum(s, scratch);
  if (threadIdx.x == 0) out[0] = accumulate ? out[0] + s : s;
}

hipError_t sum_to(const float* x, int n, float* out, int accumulate, hipStream_t s) {
  hipLaunchKernelGGL(sum_to_kernel, dim3(1), dim3(1024), 0, s, x, n, out, accumulate);
  return hipGetLastError();
}

// two independent sum_to in one launch (block z: x_z -> out_z), each in sum_to's order; with
// flag_src, block 0 also adds (flag_src[0] != 0) to flag_dst[0] (the stall slot beside the sse)
__global__ void sum_to2_kernel(const float* __restrict__ x0, float* out0, const float* __restrict__ x1, float* out1,
                               int n, int accumulate, const int* __restrict__ flag_src, float* flag_dst) {
  __shared__ float scratch[16];
  const float* x = blockIdx.x ? x1 : x0;
  float* out = blockIdx.x ? out1 : out0;
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += x[i];
  s = block_sum(s, scratch);
  if (threadIdx.x == 0) {
    out[0] = accumulate ? out[0] + s : s;
    if (blockIdx.x == 0 && flag_src) {
      const float f = flag_src[0] != 0 ? 1.0f : 0.0f;
      flag_dst[0] = accumulate ? flag_dst[0] + f : f;
    }
  }
}

hipError_t sum_to2(const float* x0, float* out0, const float* x1, float* out1, int n, int accumulate, hipStream_t s,
                   const int* flag_src, float* flag_dst) {
  hipLaunchKernelGGL(sum_to2_kernel, dim3(2), dim3(1024), 0, s, x0, out0, x1, out1, n, accumulate, flag_src,
                     flag_dst);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------
// torch.optim.Adam step (run.py:116,186) over the flat fp32 parameter vector, following
// the CUDA reference's per-element rounding:
//   m = fma(1-b1, g-m, m)                      (lerp, small weight)
//   v = fma((1-b2)*g, g, v*b2)                 (mul_ + addcmul_)
//   d = sqrt(v) / sqrt(bc2) + eps              (correctly rounded sqrt/div)
//   p = p + ((-lr/bc1) * m) / d                (addcdiv_)
// bias corrections in fp64 from the device step counter.  A step the range guard rejects
// (guard_skip: an fp16 overflow, or a fused hand-off that timed out) leaves p, m, v untouched.
__global__ void adam_flat_kernel(float* __restrict__ p, const float* __restrict__ g,
                                 float* __restrict__ m, float* __restrict__ v, int64_t n,
                                 const OptState* __restrict__ st, const GuardState* __restrict__ guard,
                                 const float* __restrict__ sse) {
#pragma clang fp contract(off)
  if (guard_skip(guard, sse)) return;
  const double step = st->step + 1.0;
  const double bc1 = 1.0 - pow(st->beta1, step);
  const double bc2 = 1.0 - pow(st->beta2, step);
  const float neg_step_size = (float)((st->lr / bc1) * -1.0);
  const float bc2_sqrt = (float)sqrt(bc2);
  const float w1 = (float)(1.0 - st->beta1);
  const float b2 = (float)st->beta2;
  const float w2 = (float)(1.0 - st->beta2);
  const float eps = (float)st->eps;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i];
    float mi = m[i], vi = v[i];
    mi = __builtin_fmaf(w1, gi - mi, mi);
    vi = __builtin_fmaf(w2 * gi, gi, vi * b2);
    // sqrtf lowers to the correctly rounded sequence (hipcc's __fsqrt_rn is bare v_sqrt_f32)
    const float d = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = p[i] + (neg_step_size * mi) / d;
    m[i] = mi;
    v[i] = vi;
  }
}

hipError_t adam_flat(float* p, const float* g, float* m, float* v, int64_t n, const OptState* st,
                     hipStream_t s, const GuardState* guard, const float* sse) {
  hipLaunchKernelGGL(adam_flat_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0, s, p, g, m, v, n,
                     st, guard, sse);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------
// Range guard check (siren_apply_update, before Adam): guard->flag |= any non-finite value
// in the reduced gradient vector g[0..n).  One atomic per block that found one.  sse[1] (the
// reduced stall slot: non-zero when any micro-batch on any rank had a fused hand-off time out)
// marks the guard stalled, so every data-parallel rank skips the voided step, not only the one
// whose wait gave up.
__global__ void guard_check_kernel(const float* __restrict__ g, int64_t n, GuardState* guard,
                                   const float* __restrict__ sse) {
  __shared__ float scratch[4];
  float bad = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (!__builtin_isfinite(g[i])) bad = 1.f;
  bad = block_max(bad, scratch);
  if (threadIdx.x == 0 && bad > 0.f) atomicOr(&guard->flag, 1);
  if (threadIdx.x == 0 && blockIdx.x == 0 && sse && sse[1] != 0.f) atomicMax(&guard->stalls, 1);
}

hipError_t guard_check(const float* g, int64_t n, GuardState* guard, hipStream_t s, const float* sse) {
  hipError_t e = hipMemsetAsync(&guard->flag, 0, sizeof(int32_t), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(guard_check_kernel, dim3(grid_for(n, 256, 1024)), dim3(256), 0, s, g, n, guard, sse);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------
// ReduceLROnPlateau(mode='min', factor, patience, threshold=1e-4 rel, min_lr, eps=1e-8)
// .step(loss) (run.py:117,187) on device, after Adam used the current lr.  Also bumps the
// Adam step counter and records (loss, lr) history for the host to fetch lazily, at index
// last_epoch = scheduler steps of THIS run (a resumed run restores the Adam step from the
// checkpoint but, like run.py:106, starts a fresh scheduler).  A step the range guard
// rejects advances nothing: it lowers the guard's headroom instead, and the caller's next
// step recomputes the same gradients with the smaller backward scale.
__global__ void plateau_kernel(OptState* st, const float* sse, double n_total, float* loss_hist,
                               double* lr_hist, int64_t hist_cap, GuardState* guard) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  if (guard) {
    // a voided step (fused hand-off timeout): nothing advances, and the headroom is not to blame
    if (guard_stalled(guard)) return;
    if (guard_overflow(guard, sse)) {
      guard->headroom -= kHeadroomDrop;
      guard->clean = 0;
      guard->overflows += 1;
      return;
    }
    if (++guard->clean >= kHeadroomGrowAfter) {
      guard->clean = 0;
      if (guard->headroom < guard->headroom0) guard->headroom += 1;
    }
  }
  const float loss = (float)((double)sse[0] / n_total);
  const double cur = (double)loss;
  const int64_t k = (int64_t)st->last_epoch;  // index of this scheduler step in this run (0-based)
  st->step = st->step + 1.0;
  st->last_epoch += 1;
  if (cur < st->best * (1.0 - st->threshold)) {
    st->best = cur;
    st->num_bad = 0;
  } else {
    st->num_bad += 1;
  }
  if (st->num_bad > st->patience) {
    const double old_lr = st->lr;
    const double new_lr = fmax(old_lr * st->factor, st->min_lr);
    if (old_lr - new_lr > st->eps_lr) st->lr = new_lr;
    st->num_bad = 0;
  }
  if (k >= 0 && k < hist_cap) {
    loss_hist[k] = loss;
    lr_hist[k] = st->lr;
  }
}

hipError_t plateau_step(OptState* st, const float* sse, double n_total, float* loss_hist,
                        double* lr_hist, int64_t hist_cap, hipStream_t s, GuardState* guard) {
  hipLaunchKernelGGL(plateau_kernel, dim3(1), dim3(64), 0, s, st, sse, n_total, loss_hist, lr_hist,
                     hist_cap, guard);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------
// h16 shadows of a hidden weight W[o][k] (fp32 master): Wb = W, WTb = W^T, through a
// 64x64 LDS transpose so both stores are coalesced.
__global__ void cast_weight_kernel(const float* __restrict__ W, int H_out, int H_in,
                                   h16* __restrict__ Wb, h16* __restrict__ WTb) {
  __shared__ float tile[64][65];
  const int o0 = blockIdx.y * 64, k0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 256 threads: 64 x 4
  for (int r = ty; r < 64; r += 4) {
    const float w = W[(size_t)(o0 + r) * H_in + k0 + tx];
    tile[r][tx] = w;
    Wb[(size_t)(o0 + r) * H_in + k0 + tx] = (h16)w;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) WTb[(size_t)(k0 + r) * H_out + o0 + tx] = (h16)tile[tx][r];
}

hipError_t cast_weight(const float* W, int H_out, int H_in, h16* Wb, h16* WTb, hipStream_t s) {
  if (H_out % 64 || H_in % 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(cast_weight_kernel, dim3(H_in / 64, H_out / 64), dim3(256), 0, s, W, H_out, H_in,
                     Wb, WTb);
  return hipGetLastError();
}

// the shadows of every hidden layer (square H x H) in one launch: layer = blockIdx.z
__global__ void cast_weights_kernel(CastSet cs, int H) {
  const int l = blockIdx.z;
  __shared__ float tile[64][65];
  const float* __restrict__ W = cs.W[l];
  h16* __restrict__ Wb = cs.Wb[l];
  h16* __restrict__ WTb = cs.WTb[l];
  const int o0 = blockIdx.y * 64, k0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const float w = W[(size_t)(o0 + r) * H + k0 + tx];
    tile[r][tx] = w;
    Wb[(size_t)(o0 + r) * H + k0 + tx] = (h16)w;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) WTb[(size_t)(k0 + r) * H + o0 + tx] = (h16)tile[tx][r];
}

hipError_t cast_weights(const CastSet& cs, int H, hipStream_t s) {
  if (H % 64 || cs.n < 1 || cs.n > kMaxInner) return hipErrorInvalidValue;
  hipLaunchKernelGGL(cast_weights_kernel, dim3(H / 64, H / 64, cs.n), dim3(256), 0, s, cs, H);
  return hipGetLastError();
}

}  // namespace siren
