// Measurement only: the two fp16 MFMA shapes of gfx950 in the forward GEMM's
// own geometry.  One block of 8 waves per CU (2 waves per SIMD, as the 256x256 ping-pong kernel),
// each wave computing a 128 x 64 output tile from LDS-resident random fp16 operands staged with the
// product's XOR swizzle, 64-deep K-steps repeated `iters` times:
//   A: v_mfma_f32_16x16x32_f16 -- 8 x 4 tiles, 2 k32 halves: 24 ds_read_b128 + 64 MFMA per K-step
//   B: v_mfma_f32_32x32x16_f16 -- 4 x 2 tiles, 4 k16 steps:  24 ds_read_b128 + 32 MFMA per K-step
// (the same LDS bytes and flops; B reads half the operand-register bytes per flop and twice the
// accumulator bytes).  Launches of either shape alternate over several rounds; the data are random
// (zero operands change the clock the chip holds, MI355X_MICROARCH.md DVFS item 1).
//   hipcc --offload-arch=gfx950 -O3 -o mfma_shape_rate mfma_shape_rate.hip && ./mfma_shape_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 h16;
typedef h16 h16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int ROWB = 128;  // one staged row: 64 fp16
__device__ __forceinline__ int swz(int r, int c) { return c ^ (r & 7); }

__device__ void stage(char* lds, const h16* src) {
  // 512 rows (256 X + 256 W) x 64 fp16 -> LDS with the source-side swizzle of the product kernel
  for (int e = threadIdx.x; e < 512 * 8; e += blockDim.x) {
    const int r = e >> 3, c = e & 7;
    *(uint4*)(lds + r * ROWB + (swz(r, c) << 4)) = *(const uint4*)(src + (size_t)r * 64 + c * 8);
  }
  __syncthreads();
}

__global__ __launch_bounds__(512, 2) void shape_a(const h16* src, float* out, int iters) {
  __shared__ __attribute__((aligned(16))) char lds[512 * ROWB];
  stage(lds, src + (size_t)(blockIdx.x & 7) * 512 * 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wm = wave >> 2, wn = wave & 3;
  const char* xs = lds + (wm * 128) * ROWB;
  const char* ws = lds + (256 + wn * 64) * ROWB;
  f32x4 acc[4][8];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int off = (lane & 15) * ROWB + (swz(lane & 15, (lane >> 4) + 4 * kk) << 4);
      h16x8 xf[8], wf[4];
#pragma unroll
      for (int j = 0; j < 8; ++j) xf[j] = *(const h16x8*)(xs + j * 16 * ROWB + off);
#pragma unroll
      for (int i = 0; i < 4; ++i) wf[i] = *(const h16x8*)(ws + i * 16 * ROWB + off);
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[i], xf[j], acc[i][j], 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(512, 2) void shape_b(const h16* src, float* out, int iters) {
  __shared__ __attribute__((aligned(16))) char lds[512 * ROWB];
  stage(lds, src + (size_t)(blockIdx.x & 7) * 512 * 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wm = wave >> 2, wn = wave & 3;
  const char* xs = lds + (wm * 128) * ROWB;
  const char* ws = lds + (256 + wn * 64) * ROWB;
  f32x16 acc[2][4];
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x16{};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k4 = 0; k4 < 4; ++k4) {
      const int off = (lane & 31) * ROWB + (swz(lane & 31, (lane >> 5) + 2 * k4) << 4);
      h16x8 xg[4], wg[2];
#pragma unroll
      for (int j = 0; j < 4; ++j) xg[j] = *(const h16x8*)(xs + j * 32 * ROWB + off);
#pragma unroll
      for (int i = 0; i < 2; ++i) wg[i] = *(const h16x8*)(ws + i * 32 * ROWB + off);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wg[i], xg[j], acc[i][j], 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 4; ++j)
      for (int r = 0; r < 16; ++r) s += acc[i][j][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4096, rounds = argc > 2 ? atoi(argv[2]) : 7, reps = 10;
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int blocks = cus;
  std::vector<h16> host((size_t)8 * 512 * 64);
  srand(1);
  for (auto& v : host) v = (h16)((rand() / (float)RAND_MAX - 0.5f) * 2.0f);
  h16* src;
  float* out;
  hipMalloc(&src, host.size() * sizeof(h16));
  hipMalloc(&out, (size_t)blocks * 512 * sizeof(float));
  hipMemcpy(src, host.data(), host.size() * sizeof(h16), hipMemcpyHostToDevice);
  const double flops = 2.0 * blocks * 256.0 * 256.0 * 64.0 * iters;  // per launch
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto time = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(512), 0, 0, src, out, iters);
    hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(512), 0, 0, src, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
  };
  // warm the clock up
  for (int w = 0; w < 3; ++w) time(shape_a);
  std::vector<float> ta, tb;
  for (int r = 0; r < rounds; ++r) {
    ta.push_back(time(shape_a));
    tb.push_back(time(shape_b));
  }
  auto med = [](std::vector<float> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  const float ma = med(ta), mb = med(tb);
  printf("{\"blocks\": %d, \"iters\": %d, \"rounds\": %d, \"ms_16x16x32\": %.4f, \"ms_32x32x16\": %.4f, "
         "\"tflops_16x16x32\": %.1f, \"tflops_32x32x16\": %.1f, \"ratio_16_over_32\": %.4f}\n",
         blocks, iters, rounds, ma, mb, flops / ma / 1e9, flops / mb / 1e9, mb / ma);
  return 0;
}
