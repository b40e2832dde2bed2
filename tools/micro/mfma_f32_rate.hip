// Measurement only: issue rate of v_mfma_f32_16x16x4_f32 with operands from registers
// (NACC independent accumulators per wave), and the same with one ds_read_b128 per 4 MFMAs.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void rate_kernel(float* out, int iters, float seed) {
  f32x4 acc[NACC];
  for (int j = 0; j < NACC; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float a = seed + threadIdx.x, b = seed * 2.f;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
  }
  float s = 0.f;
  for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
__global__ __launch_bounds__(256) void rate_lds_kernel(float* out, int iters, float seed) {
  __shared__ __attribute__((aligned(16))) float t[64 * 68];
  for (int e = threadIdx.x; e < 64 * 68; e += 256) t[e] = seed + e;
  __syncthreads();
  f32x4 acc[NACC];
  for (int j = 0; j < NACC; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int lane = threadIdx.x & 63;
  const float* p = &t[(lane & 15) * 68 + 4 * (lane >> 4)];
  for (int i = 0; i < iters; ++i) {
    const float4 v = *reinterpret_cast<const float4*>(p + 16 * (i & 3));
#pragma unroll
    for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(v.x, v.y + j, acc[j], 0, 0, 0);
  }
  float s = 0.f;
  for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
static void run(const char* name, K kern, int nacc, int blocks, int iters, float* d) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, iters, 1.0f);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, iters, 1.0f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 16 * 16 * 4 * (double)nacc * iters * (blocks * 4);
  printf("%-10s nacc %d blocks %5d: %.3f ms  %.1f TFLOP/s\n", name, nacc, blocks, ms, flops / ms / 1e9);
}

int main() {
  float* d;
  hipMalloc(&d, 4096 * 256 * sizeof(float));
  for (int blocks : {256, 512, 1024, 2048}) {
    run("regs", rate_kernel<4>, 4, blocks, 4000, d);
    run("regs", rate_kernel<9>, 9, blocks, 2000, d);
    run("lds", rate_lds_kernel<4>, 4, blocks, 4000, d);
  }
  hipFree(d);
  return 0;
}
