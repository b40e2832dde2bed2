// Shared device types and helpers for the SIREN gfx950 kernels.
//
// Everything here is CDNA4-only (wave64, bf16 MFMA, LDS-DMA); no portability layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define LDS_AS __attribute__((address_space(3)))

namespace siren {

constexpr float kInv2Pi = 0.15915494309189535f;  // 1/(2*pi), rounded to fp32

// Bijective XCD-aware remap of a 1-D block id (cdna_hip_programming.md §5 "XCD swizzle
// must be bijective"): blocks b, b+8, b+16 ... are dealt to one XCD, so consecutive
// remapped ids share an L2.  Placement only changes speed, never results.
__device__ __forceinline__ int xcd_remap(int b, int nblk) {
  const int xcd = b & 7, local = b >> 3;
  const int q = nblk >> 3, r = nblk & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + local;
}

// LDS-DMA: each lane moves 16 B from its own global address into
// lds_base + 16*lane (lds_base is wave-uniform).
__device__ __forceinline__ void glds16(const void* gsrc, LDS_AS void* lds_base) {
  __builtin_amdgcn_global_load_lds(gsrc, lds_base, 16, 0, 0);
}

__device__ __forceinline__ LDS_AS void* lds_ptr(char* p) {
  return (LDS_AS void*)(p);
}

// LDS-DMA issued from inline asm: hipcc's waitcnt pass cannot see it, so it does NOT insert
// the conservative `s_waitcnt vmcnt(0)` before every later ds_read of the same __shared__
// array (it cannot prove the DMA targets another ring slot).  The caller orders the data
// with its own counted vmcnt + barrier (gemm_pipeline.h).  M0 is compiler-reserved, so it
// is saved and restored inside the one statement (cdna_hip_programming.md §5.7 item M0).
// `lds_byte` must be wave-uniform.
__device__ __forceinline__ void glds16_asm(const void* gsrc, unsigned lds_byte) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_byte))
      : "memory");
}

__device__ __forceinline__ unsigned lds_addr(const char* p) {
  return (unsigned)(uintptr_t)(const LDS_AS char*)(p);
}

__device__ __forceinline__ bf16x4 pack4(float a, float b, float c, float d) {
  bf16x4 r;
  r[0] = (bf16)a; r[1] = (bf16)b; r[2] = (bf16)c; r[3] = (bf16)d;
  return r;
}

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }

// Block-wide sum of one float per thread (blockDim.x multiple of 64, <= 1024).
// `scratch` must hold blockDim.x/64 floats.  Result valid in every thread.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scratch[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += scratch[i];  // fixed order: deterministic
  return s;
}

}  // namespace siren
