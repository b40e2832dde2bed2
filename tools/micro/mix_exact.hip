// Measurement only: is v_fma_mix_f32 with a -0 addend bit-identical to v_cvt_f32_f16 + v_mul_f32?
// Every fp16 bit pattern h (both halves of a packed word) times a spread of fp32 values a.
//   hipcc --offload-arch=gfx950 -O3 -o mix_exact mix_exact.hip && ./mix_exact
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void k(const float* av, int na, unsigned* bad, unsigned* first) {
  const unsigned h = blockIdx.x * blockDim.x + threadIdx.x;  // 0 .. 65535
  if (h >= 65536) return;
  const unsigned w = h | (h << 16);
  const float nz = -0.0f;
  _Float16 hv;
  unsigned short hs = (unsigned short)h;
  __builtin_memcpy(&hv, &hs, 2);
  const float c = (float)hv;
  for (int i = 0; i < na; ++i) {
    const float a = av[i];
    float r0, r1;
    asm volatile("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[0,1,0]" : "=v"(r0) : "v"(a), "v"(w), "v"(nz));
    asm volatile("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "=v"(r1) : "v"(a), "v"(w), "v"(nz));
    const float ref = a * c;
    const unsigned rb = __float_as_uint(ref);
    if (ref != ref) continue;  // NaN products: payloads are not compared
    if (__float_as_uint(r0) != rb || __float_as_uint(r1) != rb) {
      if (atomicAdd(bad, 1u) == 0) {
        first[0] = h; first[1] = __float_as_uint(a); first[2] = rb; first[3] = __float_as_uint(r0);
        first[4] = __float_as_uint(r1);
      }
    }
  }
}

int main() {
  std::vector<float> a;
  const float base[] = {0.f, -0.f, 1.f, -1.f, 3.14159f, -2.5e-3f, 1e-20f, -1e-30f, 1e-38f, 1.5e-39f, -7e-45f, 65504.f, 1e30f, -3e38f};
  for (float x : base) a.push_back(x);
  for (int i = 0; i < 200; ++i) a.push_back(((i * 2654435761u) % 100000) * 1e-5f * ((i & 1) ? -1.f : 1.f) * (i % 7 == 0 ? 1e-6f : 1.f));
  float* da; unsigned *bad, *first;
  hipMalloc(&da, a.size() * 4); hipMalloc(&bad, 4); hipMalloc(&first, 20);
  hipMemcpy(da, a.data(), a.size() * 4, hipMemcpyHostToDevice);
  hipMemset(bad, 0, 4); hipMemset(first, 0, 20);
  hipLaunchKernelGGL(k, dim3(256), dim3(256), 0, 0, da, (int)a.size(), bad, first);
  unsigned hb, hf[5];
  hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
  hipMemcpy(hf, first, 20, hipMemcpyDeviceToHost);
  printf("{\"cases\": %zu, \"mismatches\": %u, \"first\": [%u, \"0x%08x\", \"0x%08x\", \"0x%08x\", \"0x%08x\"]}\n",
         a.size() * 65536, hb, hf[0], hf[1], hf[2], hf[3], hf[4]);
  return 0;
}
