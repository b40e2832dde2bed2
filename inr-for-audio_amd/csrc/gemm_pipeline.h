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
#include <type_traits>
#include "siren_common.h"

namespace siren {

// f(integral_constant<int, I>) for I = B .. E-1, unrolled at compile time
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

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

  auto mma = [&](h16x8 (&A)[NA], h16x8 (&B)[NB]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[i], B[j], acc[i][j], 0, 0, 0);
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
        h16x8 A[NA], B[NB];
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
    h16x8 A0[NA], B0[NB], A1[NA], B1[NB];
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

__device__ __forceinline__ void lds_barrier() {
  wait_lgkm0();
  __builtin_amdgcn_s_barrier();
}

// Persistent S-slot ring for short-K GEMMs (K = hidden width): the block walks `ntiles`
// tiles and the ring runs straight across tile boundaries, S-1 stages ahead.
// vmcnt retires loads AND stores in issue order (MI355X_MICROARCH.md §vmcnt), so a stage
// issued after an epilogue's stores cannot be waited for without waiting for the stores too.
// The stages already in flight when an epilogue issues its stores are therefore waited for
// with SLACK more outstanding operations allowed (the stores drain under those K-steps); a
// wait for a stage issued after the stores is strict.  With S = 2 only one stage would be
// in flight, so the second stage of the next tile is issued early, into the slot the last
// K-step just read (one extra barrier per tile), before the epilogue.
//   stage(tile, kt, slot)  issues the LDS-DMA of K-step kt of the block's tile-th tile;
//   frags(slot, kk, A, B)  reads one k32 half of the operand fragments;
//   pre(tile)              issues the epilogue's own global loads (Cprev, ...) before the
//                          S = 2 early prefetch, so that waiting for them does not wait for it;
//   epi(tile)              consumes acc; the ring is NOT available to it (own LDS scratch;
//                          raw barriers only -- every wave calls epi the same number of times).
// SLACK = vector-memory instructions every wave's epilogue issues (a lower bound; 0 is always
// safe); G = vector-memory instructions per wave per stage.

// s_waitcnt vmcnt(G*y + (relaxed ? SLACK : 0)) for a wave-uniform y in [0, J]
template <int G, int SLACK, int J>
__device__ __forceinline__ void wait_stage(int y, bool relaxed) {
  if constexpr (J >= 0) {
    if (y == J) {
      if (relaxed) wait_vmcnt<G * J + SLACK>();
      else wait_vmcnt<G * J>();
      return;
    }
    wait_stage<G, SLACK, J - 1>(y, relaxed);
  } else {
    wait_vmcnt<0>();
  }
}

template <int S, int KK, int G, int NA, int NB, int SLACK, class StageFn, class FragFn, class PreFn,
          class EpiFn>
__device__ __forceinline__ void mfma_pipeline_tiles(int ntiles, int nk, f32x4 (&acc)[NA][NB],
                                                    StageFn&& stage, FragFn&& frags, PreFn&& pre,
                                                    EpiFn&& epi) {
  static_assert(S >= 2 && S <= 6, "ring depth");
  constexpr int YMAX = (S == 2) ? 1 : S - 2;  // younger stages in flight at a wait
  static_assert(SLACK >= 0 && G * YMAX + SLACK < 64, "vmcnt immediate");
  const int total = ntiles * nk;
  if (total <= 0) return;
  int it = 0, ik = 0;  // issue pointer (tile, K-step)
  int issued = 0;      // stages issued so far (global step index of the next one)
  int fill = 0;        // ring slot of the next stage
  auto issue = [&]() {
    stage(it, ik, fill);
    if (++ik == nk) { ik = 0; ++it; }
    ++issued;
    fill = (fill + 1 == S) ? 0 : fill + 1;
  };
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (issued < total) issue();
  int ct = 0, ck = 0, slot = 0;
  int relax = 0;  // K-steps left whose stage was issued before the last epilogue's stores
  for (int u = 0; u < total; ++u) {
    wait_stage<G, SLACK, YMAX>(issued - (u + 1), relax > 0);
    wait_lgkm0();
    __builtin_amdgcn_s_barrier();
    if (relax > 0) --relax;
    // stage u+S-1 goes into the slot K-step u-1 read (every wave is past the barrier)
    if (issued < total && issued < u + S) issue();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      h16x8 A[NA], B[NB];
      frags(slot, kk, A, B);
#pragma unroll
      for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[i], B[j], acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    if (++ck == nk) {
      pre(ct);
      if (S == 2 && issued == u + 2 && issued < total) {
        lds_barrier();  // every wave is done reading `slot` (== fill)
        issue();
      }
      relax = issued - (u + 1);  // stages in flight ahead of the stores
      epi(ct);
#pragma unroll
      for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      ck = 0;
      ++ct;
    }
    slot = (slot + 1 == S) ? 0 : slot + 1;
  }
  wait_vmcnt<0>();
  wait_lgkm0();
  __builtin_amdgcn_s_barrier();
}

// ---- Ping-pong K-loop of the 256x256 / 8-wave GEMMs ----------------------------------------
// (cdna_hip_programming.md §5, "The 256² 8-phase template": T2+T3+T4+T5.)  The 8 waves form two
// groups of 4 (grp = wave >> 2) that run ONE BARRIER APART: on every SIMD one wave issues its
// 16-MFMA cluster while its partner (the other group) issues LDS reads and LDS-DMA.  A K-tile
// (BK = 64) is 4 phases a, b, c, d; each phase is
//     MEM:  ds_read this phase's fragments; issue one staging piece (16 KiB = 2 LDS-DMA per
//           wave); [counted vmcnt]
//     s_barrier; setprio 1; 16 MFMA; lgkmcnt(0); setprio 0; s_barrier
// Group 1 executes one extra s_barrier first, so group 0's MFMA cluster runs between the same
// two barrier instances as group 1's MEM section and vice versa.
//
// Staging: 2 LDS slots (slot = K-tile & 1), each K-tile in 4 pieces pc 0..3.  Phase a of
// K-tile u issues pc 2 of u+1, b: pc 3 of u+1, c: pc 0 of u+2, d: pc 1 of u+2 (so the pieces
// of K-tile k go out at global phases 4k-6 .. 4k-3).  With the stagger, every wave's vmcnt in
// phase r precedes a barrier instance that every wave passes before its MEM section of phase
// r+1 (RAW), and a ds_read of phase q is retired (lgkmcnt(0)) before a barrier every wave
// passes before its MEM section of phase q+2 (WAR).  Hence the caller's contract:
//   last ds_read of pc 0 in phase <= a, pc 1 <= b, pc 2 <= c, pc 3 <= d   (WAR)
//   first ds_read of pc 0, pc 1 >= a (wait in d); pc 2 >= b (wait in a, or in b when first
//   read in c); pc 3 >= c (wait in b)                                      (RAW)
// Static schedule (tiles of an even number nk >= 2 of K-tiles, or one tile per block): every
// phase issues exactly one piece, so every wait is a compile-time vmcnt and the K-loop has no
// data-dependent branch.  The pieces a K-step issues belong to K-tiles u+1 and u+2, i.e. to the
// current tile or the next one, picked by `sel` between two operand bases the caller keeps.
// Past the block's last tile the issues re-read valid rows into LDS pieces that were already
// consumed and that nothing reads again; they are drained (vmcnt(0)) before the loop returns.
// WAITMASK bit PH = phase PH waits: vmcnt(8) keeps the pieces of phases r-3..r in flight, i.e.
// piece r-4 has landed.  A tile's epilogue (tile_end) issues >= E stores after the pieces then
// in flight; the waits of the next tile's first K-tile (whose awaited pieces are older than
// those stores) count them as in flight too: vmcnt(8 + E).
//   issue(sel, k, slot, phase_t<PC>)  LDS-DMA of piece PC of K-tile k of tile ti + sel into
//                                     LDS slot `slot`
//   read(phase_t<PH>, slot)           this wave's fragments for phase PH
//   mma(phase_t<PH>)                  its 16 MFMAs
//   set_tiles(ti)                     operand bases of tiles ti and ti + 1 (ti again at the
//                                     block's last tile)
//   tile_end(ti)                      epilogue with both groups aligned (equal barrier count)
//   more(ti)                          after tile_end(ti): does the block have a tile ti + 1?
//                                     (block-uniform; a static walk or the dynamic tile queue)
template <int PH>
using phase_t = std::integral_constant<int, PH>;

__device__ __forceinline__ void pp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");  // no LDS access moves across the barrier
  __builtin_amdgcn_sched_barrier(0);
}

template <int E, int WAITMASK, class IssueFn, class ReadFn, class MmaFn, class SetFn, class EndFn,
          class MoreFn>
__device__ __forceinline__ void pingpong_tiles(bool any, int nk, int grp, IssueFn&& issue,
                                                ReadFn&& read, MmaFn&& mma, SetFn&& set_tiles,
                                                EndFn&& tile_end, MoreFn&& more) {
  static_assert(E >= 0 && 8 + E < 64, "vmcnt immediate");
  if (!any || nk <= 0) return;
  set_tiles(0);
  issue(0, 0, 0, phase_t<0>{});
  issue(0, 0, 0, phase_t<1>{});
  issue(0, 0, 0, phase_t<2>{});
  issue(0, 0, 0, phase_t<3>{});
  issue(0, 1, 1, phase_t<0>{});
  issue(0, 1, 1, phase_t<1>{});
  wait_vmcnt<8>();  // this wave's share of K-tile 0's pieces 0, 1 has landed
  wait_lgkm0();
  pp_barrier();           // ... every wave's
  if (grp) pp_barrier();  // group 1 runs one barrier behind
  // one K-step (4 phases) of K-tile kt in LDS slot kt & 1; RELAXED: the tile's first K-step
  // after an epilogue whose E stores sit between the awaited pieces and the newest ones
  auto kstep = [&](int kt, auto relaxed) {
    constexpr bool RELAXED = decltype(relaxed)::value;
    const int slot = kt & 1;
    int ka = kt + 1, kb = kt + 2;
    const int sa = ka >= nk, sb = kb >= nk;
    ka -= sa ? nk : 0;
    kb -= sb ? nk : 0;
    auto phase = [&](auto ph) {
      constexpr int PH = decltype(ph)::value;
      read(ph, slot);
      if constexpr (PH < 2) issue(sa, ka, slot ^ 1, phase_t<PH + 2>{});
      else issue(sb, kb, slot, phase_t<PH - 2>{});
      if constexpr (((WAITMASK >> PH) & 1) != 0) wait_vmcnt<RELAXED ? 8 + E : 8>();
      pp_barrier();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      mma(ph);       // each MFMA waits (counted lgkmcnt) only for its fragments
      wait_lgkm0();  // every read of this slot has landed before the barrier that frees it
      __builtin_amdgcn_s_setprio(0);
      pp_barrier();
    };
    phase(phase_t<0>{});
    phase(phase_t<1>{});
    phase(phase_t<2>{});
    phase(phase_t<3>{});
  };
  for (int ti = 0;; ++ti) {
    if (ti == 0) kstep(0, std::false_type{});
    else kstep(0, std::true_type{});
    for (int kt = 1; kt < nk; ++kt) kstep(kt, std::false_type{});
    if (grp == 0) pp_barrier();  // meet group 1's last barrier: aligned
    tile_end(ti);
    const bool next = more(ti);
    if (!next) break;
    set_tiles(ti + 1);
    if (grp == 1) pp_barrier();  // group 1 one barrier behind again
  }
  wait_vmcnt<0>();
}

// Persistent two-segment variant of pingpong_tiles (the NT kernels' default, SIREN_NT_SEG2): a K-step
// is two segments of 32 MFMAs -- segment 0 = phases 0, 1 (reads pieces 0..2, issues piece 3 of K-tile
// kt + 1), segment 1 = phases 2, 3 (reads piece 3, issues pieces 0..2 of kt + 2) -- so 4 barriers per
// K-step instead of 8.  Each segment retires its own reads (lgkmcnt(0)) before its first barrier: the
// other group, one barrier behind, overwrites those pieces one barrier later (pingpong2_one_tile's
// rule).  Every wait is vmcnt(8) (8 + E in a tile's first K-step after an epilogue): the pieces
// issued in the two segments since the awaited ones.
// EARLY (SIREN_NT_EARLY, measurement): piece 3 of the next tile's K-tile 1 is issued at the tile end,
// before the epilogue's stores (slot 1 is free once both groups are aligned there), instead of in the
// next tile's first K-step; the prologue issues it for the first tile the same way.  The first wait
// that sits behind the stores then moves from K-step 1 segment 0 to K-step 1 segment 1 (segment 0 of
// K-step 1 waits with 8 + E after an epilogue, and K-step 0 segment 0 issues nothing).
template <int E, bool EARLY, class IssueFn, class ReadFn, class MmaFn, class SetFn, class EndFn, class MoreFn>
__device__ __forceinline__ void pingpong2_tiles(bool any, int nk, int grp, IssueFn&& issue, ReadFn&& read,
                                                MmaFn&& mma, SetFn&& set_tiles, EndFn&& tile_end, MoreFn&& more) {
  static_assert(E >= 0 && 8 + E < 64, "vmcnt immediate");
  if (!any || nk <= 0) return;
  set_tiles(0);
  issue(0, 0, 0, phase_t<0>{});
  issue(0, 0, 0, phase_t<1>{});
  issue(0, 0, 0, phase_t<2>{});
  issue(0, 0, 0, phase_t<3>{});
  issue(0, 1, 1, phase_t<0>{});
  issue(0, 1, 1, phase_t<1>{});
  issue(0, 1, 1, phase_t<2>{});
  if constexpr (EARLY) {
    issue(0, 1, 1, phase_t<3>{});
    wait_vmcnt<10>();  // K-tile 0's pieces 0..2 have landed (K0 p3, K1 p0..3 younger)
  } else {
    wait_vmcnt<8>();  // K-tile 0's pieces 0..2 (and the older ones) have landed
  }
  wait_lgkm0();
  pp_barrier();
  if (grp) pp_barrier();  // group 1 runs one barrier behind
  // RELAXED: both segments wait past an epilogue's E stores; RELAXED_A: segment 0 only (EARLY, K-step 1)
  auto kstep = [&](int kt, auto relaxed, auto relaxed_a, auto skip_a) {
    constexpr bool RELAXED = decltype(relaxed)::value, RELAXED_A = decltype(relaxed_a)::value;
    constexpr bool SKIP_A = decltype(skip_a)::value;  // EARLY, K-step 0: piece 3 of K-tile 1 is out already
    const int slot = kt & 1;
    int ka = kt + 1, kb = kt + 2;
    const int sa = ka >= nk, sb = kb >= nk;
    ka -= sa ? nk : 0;
    kb -= sb ? nk : 0;
    auto segment = [&](auto sg) {
      constexpr int SG = decltype(sg)::value;
      read(phase_t<2 * SG>{}, slot);
      read(phase_t<2 * SG + 1>{}, slot);
      if constexpr (SG == 0) {
        if constexpr (!SKIP_A) issue(sa, ka, slot ^ 1, phase_t<3>{});
      } else {
        issue(sb, kb, slot, phase_t<0>{});
        issue(sb, kb, slot, phase_t<1>{});
        issue(sb, kb, slot, phase_t<2>{});
      }
      constexpr bool R = RELAXED || (SG == 0 && RELAXED_A);
      wait_vmcnt<R ? 8 + E : 8>();
      wait_lgkm0();
      pp_barrier();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      mma(phase_t<2 * SG>{});
      mma(phase_t<2 * SG + 1>{});
      __builtin_amdgcn_s_setprio(0);
      pp_barrier();
    };
    segment(phase_t<0>{});
    segment(phase_t<1>{});
  };
  const std::false_type F{};
  const std::true_type T{};
  const std::integral_constant<bool, EARLY> EA{};
  for (int ti = 0;; ++ti) {
    if constexpr (!EARLY) {  // three inlined K-step bodies (more spill)
      if (ti == 0) kstep(0, F, F, F);
      else kstep(0, T, F, F);
      for (int kt = 1; kt < nk; ++kt) kstep(kt, F, F, F);
    } else {
      // one K-step body with wave-uniform flags (more inlined bodies spill)
      for (int kt = 0; kt < nk; ++kt) {
        const bool r = ti > 0 && kt == 0, ra = ti > 0 && kt == 1, sk = kt == 0;
        const int slot = kt & 1;
        int ka = kt + 1, kb = kt + 2;
        const int sa = ka >= nk, sb = kb >= nk;
        ka -= sa ? nk : 0;
        kb -= sb ? nk : 0;
        auto segment = [&](auto sg) {
          constexpr int SG = decltype(sg)::value;
          read(phase_t<2 * SG>{}, slot);
          read(phase_t<2 * SG + 1>{}, slot);
          if constexpr (SG == 0) {
            if (!sk) issue(sa, ka, slot ^ 1, phase_t<3>{});
          } else {
            issue(sb, kb, slot, phase_t<0>{});
            issue(sb, kb, slot, phase_t<1>{});
            issue(sb, kb, slot, phase_t<2>{});
          }
          if (r || (SG == 0 && ra)) wait_vmcnt<8 + E>();
          else wait_vmcnt<8>();
          wait_lgkm0();
          pp_barrier();
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_setprio(1);
          mma(phase_t<2 * SG>{});
          mma(phase_t<2 * SG + 1>{});
          __builtin_amdgcn_s_setprio(0);
          pp_barrier();
        };
        segment(phase_t<0>{});
        segment(phase_t<1>{});
      }
    }
    if (grp == 0) pp_barrier();  // meet group 1's last barrier: aligned
    if constexpr (EARLY) issue(1, nk > 1 ? 1 : 0, 1, phase_t<3>{});  // the next tile's K-tile 1, piece 3
    tile_end(ti);
    const bool next = more(ti);
    if (!next) break;
    set_tiles(ti + 1);
    if (grp == 1) pp_barrier();  // group 1 one barrier behind again
  }
  wait_vmcnt<0>();
}

// Two-segment variant (one tile per block, e.g. the split-K dW GEMM): a K-tile is two segments
// of 32 MFMAs instead of four phases of 16, halving the barriers.  Segment A reads pieces
// 0 .. NA-1 of K-tile u and issues pieces NA..3 of u+1 into the other slot; segment B reads
// pieces NA..3 of u and issues pieces 0 .. NA-1 of u+2 into this slot.  Each piece is 2 LDS-DMA
// per wave, so every wait is vmcnt(8) (the 4 pieces issued since the awaited ones).  A MEM
// section retires its own reads (lgkmcnt(0)) before its barrier: the other group overwrites
// those pieces one barrier later.  issue(k, slot, phase_t<PC>), read / mma(phase_t<SEG>).
template <int NA, class IssueFn, class ReadFn, class MmaFn>
__device__ __forceinline__ void pingpong2_one_tile(int nk, int grp, IssueFn&& issue, ReadFn&& read,
                                                   MmaFn&& mma) {
  static_assert(NA >= 1 && NA <= 3, "pieces per segment");
  if (nk <= 0) return;
  auto issue_range = [&](int k, int slot, auto lo, auto hi) {
    constexpr int LO = decltype(lo)::value, HI = decltype(hi)::value;
    if constexpr (LO < HI) {
      issue(k, slot, phase_t<LO>{});
      if constexpr (LO + 1 < HI) issue(k, slot, phase_t<LO + 1>{});
      if constexpr (LO + 2 < HI) issue(k, slot, phase_t<LO + 2>{});
    }
  };
  issue_range(0, 0, phase_t<0>{}, phase_t<NA>{});
  issue_range(0, 0, phase_t<NA>{}, phase_t<4>{});
  issue_range(1, 1, phase_t<0>{}, phase_t<NA>{});
  wait_vmcnt<8>();  // this wave's share of K-tile 0's A pieces has landed
  pp_barrier();
  if (grp) pp_barrier();  // group 1 runs one barrier behind
  for (int kt = 0; kt < nk; ++kt) {
    const int slot = kt & 1;
    auto segment = [&](auto sg) {
      constexpr int SG = decltype(sg)::value;
      read(sg, slot);
      if constexpr (SG == 0) issue_range(kt + 1, slot ^ 1, phase_t<NA>{}, phase_t<4>{});
      else issue_range(kt + 2, slot, phase_t<0>{}, phase_t<NA>{});
      wait_vmcnt<8>();
      wait_lgkm0();
      pp_barrier();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      mma(sg);
      __builtin_amdgcn_s_setprio(0);
      pp_barrier();
    };
    segment(phase_t<0>{});
    segment(phase_t<1>{});
  }
  if (grp == 0) pp_barrier();  // both groups end on the same barrier count
  wait_vmcnt<0>();
}

}  // namespace siren
