// Shared K-loop of the SIREN MFMA GEMMs: an S-slot LDS ring filled by LDS-DMA with counted
// vmcnt waits (loads run S-1 K-steps ahead), one raw s_barrier per K-step, optional
// fragment prefetch across that barrier.
//
// Per K-step t (FP = false):
//     s_waitcnt vmcnt(G*(S-2))       -> this wave's loads of stage t have landed
//     s_waitcnt lgkmcnt(0); s_barrier -> every wave's have; every wave is done reading t-1
//     issue stage t+S-1 into slot (t-1) % S
//     read fragments of slot t % S -> MFMAs
// FP = true additionally reads stage t+1's fragments before stage t's MFMAs (one barrier
// per step still; the ring then runs S-2 steps ahead).
//
// LDS-DMA data is ordered for ds_read only by the issuing wave's vmcnt followed by a barrier
// (cdna_hip_programming.md §5 "Pipelining across barriers"); all LDS lives in ONE __shared__
// array so hipcc does not insert a vmcnt(0) before every ds_read (§5 item 4a).
#pragma once
#include "siren_common.h"

namespace siren {

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt immediate");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// NA x NB MFMA tiles per wave; KK = BK/32 k32 halves per K-step; G = LDS-DMA instructions per
// wave per stage.  stage(kt, slot) issues the loads of K-step kt; frags(slot, kk, A, B) fills
// the operand fragments of one k32 half.
template <int S, bool FP, int KK, int G, int NA, int NB, class StageFn, class FragFn>
__device__ __forceinline__ void mfma_pipeline(int nk, f32x4 (&acc)[NA][NB], StageFn&& stage,
                                              FragFn&& frags) {
  static_assert(S >= 2 && S <= 6, "ring depth");
  static_assert(!FP || S >= 3, "fragment prefetch needs >= 3 slots");
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) stage(s, s);

  auto mma = [&](bf16x8 (&A)[NA], bf16x8 (&B)[NB]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[i], B[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  if constexpr (!FP) {
    int slot = 0, fill = S - 1;  // slot of stage t, slot for stage t+S-1
    for (int t = 0; t < nk; ++t) {
      if (t + S - 2 < nk) wait_vmcnt<G * (S - 2)>();
      else wait_vmcnt<0>();
      wait_lgkm0();
      __builtin_amdgcn_s_barrier();
      if (t + S - 1 < nk) stage(t + S - 1, fill);
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        bf16x8 A[NA], B[NB];
        frags(slot, kk, A, B);
        mma(A, B);
      }
      slot = (slot + 1 == S) ? 0 : slot + 1;
      fill = (fill + 1 == S) ? 0 : fill + 1;
    }
  } else {
    static_assert(KK == 1, "fragment prefetch is built for BK = 32");
    // stage 0 landed -> first fragments
    if (S - 2 < nk) wait_vmcnt<G * (S - 2)>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    bf16x8 A0[NA], B0[NB], A1[NA], B1[NB];
    frags(0, 0, A0, B0);
    int slot = 0, fill = S - 1;
    for (int t = 0; t < nk; t += 2) {
      // ---- step t: fragments in (A0,B0); prefetch step t+1 into (A1,B1)
      {
        const int nslot = (slot + 1 == S) ? 0 : slot + 1;
        if (t + S - 2 < nk) wait_vmcnt<G * (S - 3)>();   // stage t+1 landed
        else wait_vmcnt<0>();
        wait_lgkm0();
        __builtin_amdgcn_s_barrier();
        if (t + S - 1 < nk) stage(t + S - 1, fill);
        if (t + 1 < nk) frags(nslot, 0, A1, B1);
        mma(A0, B0);
        slot = nslot;
        fill = (fill + 1 == S) ? 0 : fill + 1;
      }
      if (t + 1 >= nk) break;
      // ---- step t+1: fragments in (A1,B1); prefetch step t+2 into (A0,B0)
      {
        const int nslot = (slot + 1 == S) ? 0 : slot + 1;
        if (t + 1 + S - 2 < nk) wait_vmcnt<G * (S - 3)>();
        else wait_vmcnt<0>();
        wait_lgkm0();
        __builtin_amdgcn_s_barrier();
        if (t + S < nk) stage(t + S, fill);
        if (t + 2 < nk) frags(nslot, 0, A0, B0);
        mma(A1, B1);
        slot = nslot;
        fill = (fill + 1 == S) ? 0 : fill + 1;
      }
    }
  }
  // drain: no LDS-DMA may still target LDS when the epilogue reuses it
  wait_vmcnt<0>();
  wait_lgkm0();
  __builtin_amdgcn_s_barrier();
}

}  // namespace siren
