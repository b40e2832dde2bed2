// Does v_sin_f32 / v_cos_f32 reduce its argument exactly?  Compares sin(x) with sin(fract(x)) and
// cos(x) with cos(fract(x)) bit for bit (both in revolutions) over a sweep of |x| < 256 (the
// instructions' valid domain) -- if they agree, the epilogues' v_fract_f32 is redundant wherever
// the argument is known to lie inside the domain.  Measurement only.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/sin_fract_check.hip -o tools/micro/sin_fract_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

__global__ void check(uint64_t n, float lo, float hi, unsigned long long* bad, unsigned* first) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // x evenly spread over [lo, hi) plus every float near integers and half-integers via bit jitter
  const float t = (float)((double)i / (double)n);
  float x = lo + (hi - lo) * t;
  const unsigned jit = (unsigned)(i * 2654435761u) & 0xff;
  x = __uint_as_float(__float_as_uint(x) ^ (jit & 0x7));
  const float f = __builtin_amdgcn_fractf(x);
  const float s0 = __builtin_amdgcn_sinf(x), s1 = __builtin_amdgcn_sinf(f);
  const float c0 = __builtin_amdgcn_cosf(x), c1 = __builtin_amdgcn_cosf(f);
  if (__float_as_uint(s0) != __float_as_uint(s1) || __float_as_uint(c0) != __float_as_uint(c1)) {
    if (atomicAdd(bad, 1ull) == 0) *first = __float_as_uint(x);
  }
}

int main() {
  unsigned long long* bad;
  unsigned* first;
  hipMalloc(&bad, 8);
  hipMalloc(&first, 4);
  const float ranges[][2] = {{-1.f, 1.f}, {0.f, 1.f}, {-8.f, 8.f}, {-64.f, 64.f}, {-255.f, 255.f}};
  for (auto& r : ranges) {
    hipMemset(bad, 0, 8);
    hipMemset(first, 0, 4);
    const uint64_t n = 1ull << 28;
    hipLaunchKernelGGL(check, dim3((unsigned)(n / 256)), dim3(256), 0, 0, n, r[0], r[1], bad, first);
    unsigned long long hb = 0;
    unsigned hf = 0;
    hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost);
    float fx;
    memcpy(&fx, &hf, 4);
    printf("{\"range\": [%g, %g], \"samples\": %llu, \"mismatches\": %llu, \"first_x\": %.9g}\n", r[0], r[1],
           (unsigned long long)n, hb, hb ? fx : 0.f);
  }
  return 0;
}
