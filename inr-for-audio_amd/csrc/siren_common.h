// Shared device types and helpers for the SIREN gfx950 kernels.
//
// Everything here is CDNA4-only (wave64, h16 MFMA, LDS-DMA); no portability layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef _Float16 h16;
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define LDS_AS __attribute__((address_space(3)))

// LDS-DMA issue of the ping-pong K-loops' staging pieces (two halves 1 KiB apart in LDS; gemm_nt.hip,
// gemm_tn.hip): 1 = one statement per piece under one M0 value (glds16x2o_asm_s), 0 = one statement per
// DMA (glds16_asm_s / glds16_asm; measurement builds)
#ifndef SIREN_GLDS_PAIR
#define SIREN_GLDS_PAIR 1
#endif

namespace siren {

constexpr float kInv2Pi = 0.15915494309189535f;  // 1/(2*pi), rounded to fp32
constexpr float kInvPi = 0.31830988618379067f;   // 1/pi, rounded to fp32

// Snake y = z + sin^2(a z)/a (models.py:241) with dY/dz = 1 + sin(2az) and dY/da =
// (z sin(2az) - sin^2(az)/a)/a, from the double angle: sin^2(az) = (1 - cos 2az)/2, so one
// sin / cos pair of 2az (in revolutions) and 7 other VALU, where the single-angle form takes 11;
// ia = 1/a.  Error: away from small |az| the fp16 outputs and the fp32 argument bound it, as for the
// single angle.  For small |az|, 1 - cos 2az cancels (cos -> 1): t = sin^2(az)/a carries the
// absolute error of the hardware cos near 1 (~2^-24) over 2a, and E = (z s - t)/a that over a
// again -- ~1e-7 ABSOLUTE at a = 0.5 where E ~ z^2 is tiny (relative error then grows as z -> 0),
// where the single angle's t = s^2/a would keep E relatively exact.  That is about two fp16
// subnormal steps (2^-24 = 6e-8 is the fp16 output's own resolution near 0), so the double angle
// stays; tests/test_gpu_act.py::test_snake_small_az_error bounds it against fp64.
__device__ __forceinline__ void snake_epi(float z, float a, float ia, float& y, float& d, float& e) {
  const float x = __builtin_amdgcn_fractf((z * a) * kInvPi);  // 2 a z in revolutions
  const float s = __builtin_amdgcn_sinf(x), c = __builtin_amdgcn_cosf(x);
  const float t = __builtin_fmaf(-0.5f, c, 0.5f) * ia;  // sin^2(a z) / a
  y = z + t;
  d = 1.0f + s;
  e = __builtin_fmaf(z, s, -t) * ia;
}

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

// The same in the saddr form: wave-uniform 64-bit base in SGPRs plus a 32-bit per-lane byte
// offset, so that one VGPR of lane offset serves every piece whose lane pattern repeats.
__device__ __forceinline__ void glds16_asm_s(unsigned voff, const void* sbase, unsigned lds_byte) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(__builtin_amdgcn_readfirstlane(lds_byte))
      : "memory");
}

// Two LDS-DMAs of one staging piece in one statement (SIREN_GLDS_PAIR): the piece's second half lies
// 1 KiB further in LDS and `d` bytes further in the operand.  The instruction offset is added to the
// global AND the LDS address of an LDS-DMA, so both go out under one M0 value: the second takes
// offset:1024 with the lane offset voff1m = voff0 + d - 1024.  One M0 save / set / restore and one
// readfirstlane per piece instead of per DMA (round 6: forward -0.5%, dX -0.8%, bit-identical,
// profiles/r22/ab_glds_*.json).  An M0 stepped by s_add_u32 between the two DMAs instead clobbers SCC,
// which hipcc may hold live across the statement: the fused last layer's outputs changed (same A/B).
__device__ __forceinline__ void glds16x2o_asm_s(unsigned voff0, unsigned voff1m, const void* sbase, unsigned lds_byte) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %4\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %3\n\t"
      "global_load_lds_dwordx4 %2, %3 offset:1024\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff0), "v"(voff1m), "s"(sbase), "s"(lds_byte)
      : "memory");
}

// First SineLayer pre-activation z = t W0^T + b0 rounded as torch's CPU addmm (K=1: one fma;
// K=2: fma(t1, w1, t0*w0) + b) -- models.py:114-115 with is_first.
__device__ __forceinline__ float first_preact(int in_dim, float t0, float t1, float w0, float w1, float b) {
  return (in_dim == 1) ? __builtin_fmaf(t0, w0, b) : __builtin_fmaf(t1, w1, t0 * w0) + b;
}

// sin / cos of a (radians) for |a| < 2^17 via v_sin_f32 / v_cos_f32, which take revolutions:
//   r = fma(a, inv2pi_hi, -n) + a * inv2pi_lo,  n = rint(a * inv2pi_hi)
// fma forms a*inv2pi_hi - n with one rounding (|r| <= 1/2: error <= 2^-25 rev), the low part
// adds < 2e-4 rev with 2^-24 relative error, so r is within ~4e-8 rev (2.5e-7 rad) of a/(2pi)
// mod 1.  (OCML's sincosf with its large-argument reduction was 3x slower.)
__device__ __forceinline__ float rev_reduce(float a) {
  constexpr float kHi = 0x1.45f306p-3f;  // fp32(1/(2*pi))             0x3E22F983
  constexpr float kLo = 0x1.b93910p-28f; // fp32(1/(2*pi) - kHi) = 6.42e-9  0x31DC9C88
  const float n = __builtin_rintf(a * kHi);
  return __builtin_fmaf(a, kLo, __builtin_fmaf(a, kHi, -n));
}
__device__ __forceinline__ void sincos_rev(float a, float* s, float* c) {
  const float r = rev_reduce(a);
  *s = __builtin_amdgcn_sinf(r);
  *c = __builtin_amdgcn_cosf(r);
}

__device__ __forceinline__ unsigned lds_addr(const char* p) {
  return (unsigned)(uintptr_t)(const LDS_AS char*)(p);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
// a[r] * s + b[r], r = 0..3, as two v_pk_fma_f32 (one correctly rounded fma per element: bit for bit
// the four v_fma_f32 it replaces, at half their issue cost)
__device__ __forceinline__ void fma4_pk(f32x4 a, float s, float4 b, float (&x)[4]) {
  const f32x2 lo = __builtin_elementwise_fma(f32x2{a[0], a[1]}, f32x2{s, s}, f32x2{b.x, b.y});
  const f32x2 hi = __builtin_elementwise_fma(f32x2{a[2], a[3]}, f32x2{s, s}, f32x2{b.z, b.w});
  x[0] = lo.x; x[1] = lo.y; x[2] = hi.x; x[3] = hi.y;
}
// c[0..3] = the two halves
__device__ __forceinline__ void set4(float (&c)[4], f32x2 lo, f32x2 hi) {
  c[0] = lo.x; c[1] = lo.y; c[2] = hi.x; c[3] = hi.y;
}
// ((v0 w0 + v1 w1) + v2 w2) + v3 w3: the products as two v_pk_mul_f32, the sums in that order
__device__ __forceinline__ float dot4_pk(const float (&v)[4], float4 w) {
  const f32x2 lo = f32x2{v[0], v[1]} * f32x2{w.x, w.y};
  const f32x2 hi = f32x2{v[2], v[3]} * f32x2{w.z, w.w};
  return ((lo.x + lo.y) + hi.x) + hi.y;
}

__device__ __forceinline__ h16x4 pack4(float a, float b, float c, float d) {
  h16x4 r;
  r[0] = (h16)a; r[1] = (h16)b; r[2] = (h16)c; r[3] = (h16)d;
  return r;
}

__device__ __forceinline__ float bf2f(h16 x) { return (float)x; }

// 16x16 MFMA output layout -> 16-B row pieces.  A lane of 16-lane group g = lane>>4 holds 4
// consecutive columns 4g..4g+3 (one row, lane&15) of two adjacent 16-column subtiles, a and b.
// One v_permlane16_swap per dword (group 1 of a <-> group 0 of b, group 3 of a <-> group 2
// of b) leaves every lane 8 consecutive columns: subtile (g&1) (a: 0, b: 1), columns
// 8*(g>>1) .. +7 -- so a row's 32 columns go out as 4 dwordx4 instead of 8 dwordx2
// (cdna_hip_programming.md T21, 16x16 form).  The exchange is an involution: applied to a
// 16-B piece loaded from that position it restores the MFMA layout.
__device__ __forceinline__ uint4 swap16_pair(uint2 a, uint2 b) {
  const auto rx = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
  const auto ry = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
  return uint4{rx[0], ry[0], rx[1], ry[1]};
}
__device__ __forceinline__ void unswap16_pair(uint4 v, uint2& a, uint2& b) {
  const auto rx = __builtin_amdgcn_permlane16_swap(v.x, v.z, false, false);
  const auto ry = __builtin_amdgcn_permlane16_swap(v.y, v.w, false, false);
  a = uint2{rx[0], ry[0]};
  b = uint2{rx[1], ry[1]};
}
// column offset (in elements, from the pair's first column) of this lane's 8-column piece
__device__ __forceinline__ int swap16_col(int lane) { return ((lane >> 4) & 1) * 16 + 8 * (lane >> 5); }

__device__ __forceinline__ uint2 as_u2(h16x4 v) { return __builtin_bit_cast(uint2, v); }
__device__ __forceinline__ h16x4 as_h4(uint2 v) { return __builtin_bit_cast(h16x4, v); }

// fp32_first: an empty asm on a value that is stored as fp16 keeps its fp32 rounding.  Left alone,
// hipcc folds some (x * y) -> fp16 pairs into one v_fma_mixlo_f16, a single rounding, and which
// pairs it folds changes from build to build; the oracle and the fp32 column partials see the
// fp32 value.  Applied to the dX epilogues' (acc C) omega; a product by the power-of-two dZ scale
// is exact, so its fold changes nothing.
// a * (float)h + c, h = fp16 element R of a packed 4-element piece, in one v_fma_mix_f32: the
// instruction widens the fp16 operand exactly, so the result is the one of a v_cvt_f32_f16 and a
// v_fma_f32, with one VALU instead of two.  `volatile` keeps the statements in program order:
// left free, the scheduler hoists them in a cluster ahead of their consumers and spills.
template <int R>
__device__ __forceinline__ float fma_mix(float a, uint2 piece, float c) {
  static_assert(R >= 0 && R < 4, "element of a 4-element piece");
  const unsigned w = R < 2 ? piece.x : piece.y;
  float r;
  if constexpr (R & 1)
    asm volatile("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "=v"(r) : "v"(a), "v"(w), "v"(c));
  else
    asm volatile("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[0,1,0]" : "=v"(r) : "v"(a), "v"(w), "v"(c));
  return r;
}
// a * (float)h exactly (fma with a -0 addend: x + -0 = x for every x, signed zeros included)
template <int R>
__device__ __forceinline__ float mul_mix(float a, uint2 piece) { return fma_mix<R>(a, piece, -0.0f); }

// Sum over the 16 lanes of a DPP row (lanes with equal lane>>4): fixed rotation order, result
// in every lane of the row.
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x122, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xf, 0xf, false));
  return v;
}

// row16_sum of four values at once, one v_add_f32 with a DPP row_ror source per value and step
// (the same sums, bit for bit).  Written with the builtin, hipcc pairs the four chains' adds into
// v_pk_add_f32 and moves every DPP result into a register pair first: three instructions per add.
// The four chains are interleaved, so a chain's DPP read is three VALU after its last write (the
// gfx950 VALU-write -> DPP-read hazard needs two wait states); the leading s_nop covers the
// compiler's last write of an input.
__device__ __forceinline__ void row16_sum4(float (&v)[4]) {
  asm volatile(
      "s_nop 1\n\t"
      "v_add_f32_dpp %0, %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %1, %1, %1 row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %2, %2, %2 row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %3, %3, %3 row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %0, %0, %0 row_ror:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %1, %1, %1 row_ror:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %2, %2, %2 row_ror:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %3, %3, %3 row_ror:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %0, %0, %0 row_ror:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %1, %1, %1 row_ror:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %2, %2, %2 row_ror:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %3, %3, %3 row_ror:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %0, %0, %0 row_ror:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %1, %1, %1 row_ror:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %2, %2, %2 row_ror:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_add_f32_dpp %3, %3, %3 row_ror:1 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1"
      : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
}

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

// block_sum(a), block_sum(b) and block_max(c) in one pass: every value keeps its own reduction
// tree (the same results, bit for bit, as the three calls), with the three shuffle chains
// interleaved and one pair of barriers instead of three.  scratch: 3 * blockDim.x / 64 floats.
__device__ __forceinline__ void block_sum2_max(float& a, float& b, float& c, float* scratch) {
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
    c = fmaxf(c, __shfl_xor(c, o, 64));
  }
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    scratch[w] = a;
    scratch[nw + w] = b;
    scratch[2 * nw + w] = c;
  }
  __syncthreads();
  float s = 0.f, t = 0.f, m = 0.f;
  for (int i = 0; i < nw; ++i) {  // fixed order: deterministic
    s += scratch[i];
    t += scratch[nw + i];
    m = fmaxf(m, scratch[2 * nw + i]);
  }
  a = s;
  b = t;
  c = m;
}

// Block-wide max, same contract as block_sum.
__device__ __forceinline__ float block_max(float v, float* scratch) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scratch[w] = v;
  __syncthreads();
  float m = 0.f;
  for (int i = 0; i < nw; ++i) m = fmaxf(m, scratch[i]);
  return m;
}

}  // namespace siren
