// Unfused fp32 layers for the module-level API outside the fused training step: a lone
// SineLayer (models.py:114-120, forward_with_intermediate), nn.Linear, Snake (models.py:235-241)
// and Tanh as SirenWithSnakeTanh.forward_with_activations (models.py:396-423) walks them.  The
// reference computes these in fp32 and so does this path (the fused SIREN step stores fp16).
//   linear:  pre = omega * (x W^T + b)            fp32 GEMM (kan_gemm) + bias/omega pass
//   act:     y = pre | sin(pre) | tanh(pre) | pre + sin^2(a pre) / a
//   act_bwd: gpre = gy * dy/dpre (+ gy * dy/da products for the Snake a column sums)
// Everything here is memory-bound elementwise work around the GEMMs; none of it is on the hot
// path (the engine never calls it).
#include <math.h>
#include "siren_common.h"
#include "siren_kernels.h"

namespace siren {

static inline int lay_grid(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}

// pre[r][o] = omega * (c[r][o] + b[o])  (in place on c: the torch addmm-then-scale rounding)
__global__ void bias_omega_kernel(float* __restrict__ c, const float* __restrict__ b, int64_t rows, int out,
                                  float omega) {
  const int64_t n = rows * out;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int o = (int)(e % out);
    const float z = b ? c[e] + b[o] : c[e];
    c[e] = omega * z;
  }
}

__global__ void act_kernel(int act, const float* __restrict__ x, int64_t rows, int cols, const float* __restrict__ a,
                           float* __restrict__ y) {
  const int64_t n = rows * cols;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const float v = x[e];
    float r = v;
    if (act == FP32_SIN) r = sinf(v);
    else if (act == FP32_TANH) r = tanhf(v);
    else if (act == FP32_SNAKE) {
      const float av = a[e % cols];
      const float s = sinf(v * av);
      r = v + (1.0f / av) * (s * s);
    }
    y[e] = r;
  }
}

// gpre = gy * dy/dpre;  Snake: da_prod[e] = gy * dy/da (column-summed by the caller)
__global__ void act_bwd_kernel(int act, const float* __restrict__ x, int64_t rows, int cols,
                               const float* __restrict__ a, const float* __restrict__ gy, float* __restrict__ gpre,
                               float* __restrict__ da_prod) {
  const int64_t n = rows * cols;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const float v = x[e], g = gy[e];
    float d = g;
    if (act == FP32_SIN) d = g * cosf(v);
    else if (act == FP32_TANH) {
      const float t = tanhf(v);
      d = g * (1.0f - t * t);
    } else if (act == FP32_SNAKE) {
      const float av = a[e % cols];
      float s, c;
      sincosf(v * av, &s, &c);
      d = g * (1.0f + 2.0f * s * c);
      if (da_prod) da_prod[e] = g * ((v * 2.0f * s * c - (s * s) / av) / av);
    }
    gpre[e] = d;
  }
}

// gz = gpre * omega (in place)
__global__ void scale_kernel(float* __restrict__ x, int64_t n, float s) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x)
    x[e] *= s;
}

hipError_t fp32_linear(const float* x, int64_t rows, int in, int out, const float* W, const float* b, float omega,
                       float* pre, hipStream_t s) {
  // pre[r][o] = sum_k x[r][k] W[o][k]
  hipError_t e = kan_gemm(x, in, 1, W, 1, in, (int)rows, out, in, 1, nullptr, pre, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(bias_omega_kernel, dim3(lay_grid(rows * out)), dim3(256), 0, s, pre, b, rows, out, omega);
  return hipGetLastError();
}

hipError_t fp32_act(int act, const float* x, int64_t rows, int cols, const float* a, float* y, hipStream_t s) {
  hipLaunchKernelGGL(act_kernel, dim3(lay_grid(rows * cols)), dim3(256), 0, s, act, x, rows, cols, a, y);
  return hipGetLastError();
}

hipError_t fp32_act_bwd(int act, const float* x, int64_t rows, int cols, const float* a, const float* gy,
                        float* gpre, float* da_prod, hipStream_t s) {
  hipLaunchKernelGGL(act_bwd_kernel, dim3(lay_grid(rows * cols)), dim3(256), 0, s, act, x, rows, cols, a, gy, gpre,
                     da_prod);
  return hipGetLastError();
}

// autograd of pre = omega (x W^T + b) given gpre: gz = omega gpre (in place), gW = gz^T x
// (split-K over rows into `slab`), gb = column sums of gz, gx = gz W
hipError_t fp32_linear_bwd(const float* x, int64_t rows, int in, int out, const float* W, float omega, float* gpre,
                           float* gx, float* gW, float* gb, float* slab, int splits, float* tmp, hipStream_t s) {
  hipLaunchKernelGGL(scale_kernel, dim3(lay_grid(rows * out)), dim3(256), 0, s, gpre, rows * out, omega);
  hipError_t e = hipGetLastError();
  // gW[o][k] = sum_r gz[r][o] x[r][k]
  if (e == hipSuccess) e = kan_gemm(gpre, 1, out, x, in, 1, out, in, rows, splits, slab, gW, s);
  if (e == hipSuccess && gb) e = col_reduce(gpre, out, (int)rows, out, gb, 1, 0, tmp, s);
  // gx[r][k] = sum_o gz[r][o] W[o][k]
  if (e == hipSuccess && gx) e = kan_gemm(gpre, out, 1, W, in, 1, (int)rows, in, out, 1, nullptr, gx, s);
  return e;
}

}  // namespace siren
