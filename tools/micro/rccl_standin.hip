// Measurement only (tools/dp_overlap_bench.py): a CU-occupying stand-in for the RCCL ring
// all-reduce kernels that a data-parallel step runs on its communication stream, one launch per
// gradient bucket behind the backward's grad_ready events (engine.py SirenEngine.step).  A ring
// all-reduce of S bytes over G ranks moves 2 (G-1)/G S through each GPU and adds (G-1)/G S; RCCL
// does it with a few dozen persistent blocks (channels) for tens of microseconds per 4 MB bucket.
// The stand-in runs `blocks` blocks of 256 threads that reduce-copy the bucket (dst += src) `reps`
// times, so its CU footprint and duration can be dialled to that.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/micro/rccl_standin.hip -o tools/micro/librccl_standin.so
#include <hip/hip_runtime.h>

__global__ __launch_bounds__(256) void standin_kernel(float* __restrict__ dst, const float* __restrict__ src,
                                                      long n4, int reps) {
  float4* d = (float4*)dst;
  const float4* s = (const float4*)src;
  const long stride = (long)gridDim.x * blockDim.x;
  for (int r = 0; r < reps; ++r)
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
      const float4 a = s[i];
      float4 b = d[i];
      b.x += a.x * 0.0f;  // the bucket's values are unchanged: x + 0 (finite inputs)
      b.y += a.y * 0.0f;
      b.z += a.z * 0.0f;
      b.w += a.w * 0.0f;
      d[i] = b;
    }
}

extern "C" int rccl_standin(float* dst, const float* src, long n, int blocks, int reps, void* stream) {
  if (n % 4 || blocks < 1 || reps < 1) return 1;
  hipLaunchKernelGGL(standin_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, dst, src, n / 4, reps);
  return (int)hipGetLastError();
}
