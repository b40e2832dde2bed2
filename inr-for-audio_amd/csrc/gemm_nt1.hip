// Forward SineLayer GEMM with the epilogue under the next tile's MFMAs (SIREN_OPT_NT_PIPE 5), and the
// same K loop with the epilogue at the tile's end (pipe 7).  MEASUREMENT OPTIONS, not the product:
// bit-identical to the ping-pong forward but slower (3.05 / 2.83 vs 2.30 ms per 2^20 x 1024^2
// launch): one wave per SIMD makes the K loop issue-bound.
//
//   Y = sin(omega (X W^T + b)),  C = cos(omega (X W^T + b))          -- models.py:114-115
//
// The ping-pong kernel (gemm_nt.hip) runs two wave groups per SIMD; both groups hold their
// accumulators until the tile's epilogue (sin/cos, pack, Y/C stores) is done, so the MFMA pipe is
// idle for that third of every tile.  Here each SIMD runs ONE wave, which keeps two accumulator
// sets (2 x 128 registers out of its 512): while the MFMAs of tile t accumulate into one set, the
// epilogue of tile t-1 reads the other, one 16-row x 32-column unit per K-tile, its VALU in the
// MFMA shadow and its two 16-B stores at the end of the K-tile.
//
// Geometry: 128 x 256 tiles (4 waves, each 128 rows x 64 columns = 8 x 4 v_mfma_f32_16x16x32_f16
// tiles, the same wave tile and epilogue layout as the ping-pong kernel), BK 64, a 3-stage LDS ring
// (3 x 48 KiB: K-tile kt + 3 reuses kt's stage, issued once every wave is past kt), one s_barrier per
// K-tile.  The K loop is unrolled (NK = K / 64 in {4, 8, 16}): the epilogue unit of each K-tile is
// then a compile-time register slice.  Accumulation order per output = K-tiles in order, k32 halves
// in order: bit-identical Y and C to the ping-pong kernel.
#include "gemm_pipeline.h"
#include "siren_common.h"
#include "siren_kernels.h"

namespace siren {
namespace {

constexpr int kBM = 128, kBN = 256, kBK = 64, kROWB = 2 * kBK;
constexpr int kSM = 8, kSN = 4;                      // MFMA tiles per wave: rows x columns
constexpr int kXB = kBM * kROWB, kWB = kBN * kROWB;  // 16 + 32 KiB staged per K-tile
constexpr int kSTAGE = kXB + kWB, kNST = 3;
constexpr int kBIAS = kNST * kSTAGE;
constexpr int kLDS = kBIAS + 4 * 1024;
constexpr int kPIECES = kSTAGE / 1024 / 4;  // LDS-DMA instructions per wave per K-tile (12)
constexpr int kUNITS = 16;                  // epilogue units per tile: 8 row blocks x 2 column pairs

__device__ __forceinline__ int swz(int r, int c) { return c ^ (r & 7); }

struct Acc {
  f32x4 v[kSN][kSM];
};

// An accumulator element read from its AGPR: with every epilogue read in this form both
// accumulator sets stay in the AGPR file (2 x 128 of its 256), the VGPRs keep the fragments.  The
// MFMA that last wrote the element ran a whole tile earlier (no hazard window to cover).
// Not volatile (a volatile asm statement is a scheduling boundary: the MFMAs could not be interleaved
// around it); the wave-uniform `token` (the K-tile's LDS stage, redefined every K-tile) keeps the
// optimizer from hoisting the read out of its K-tile.
__device__ __forceinline__ float agpr_read(float v, int token) {
  float r;
  asm("v_accvgpr_read_b32 %0, %1" : "=v"(r) : "a"(v), "s"(token));
  return r;
}

// DG: measurement-only variants (SIREN_DIAG builds, SIREN_OPT_NT_DIAG bits 10 / 11): 1 no epilogue,
// 2 epilogue arithmetic without its stores; the product instantiates DG = 0 only
// OVL: the epilogue of tile t - 1 under the MFMAs of tile t (pipe 5); false: at the tile's end
// (pipe 7: the same K loop, one accumulator set)
template <int NK, int DG, bool OVL>
__global__ __launch_bounds__(256, 1) void nt_fwd_one(NtParams p) {
  __shared__ __attribute__((aligned(16))) char smem[kLDS];
  static_assert(NK == 4 || NK == 8 || NK == 16, "units per K-tile");
  constexpr int UPK = kUNITS / NK;  // epilogue units per K-tile
  constexpr int S = (DG & 2) ? 0 : 2 * UPK;  // stores per K-tile (Y and C piece per unit)
  constexpr int K = NK * kBK;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int N = p.N;
  const int tn_shift = __builtin_ctz(N / kBN);  // N / 256 is 1, 2 or 4 (host-checked)
  const int ntiles = (p.M / kBM) << tn_shift;
  const int G = gridDim.x;
  const int bp = xcd_remap(blockIdx.x, G);  // consecutive tiles (one row band) on one XCD
  const int my = bp < ntiles ? (ntiles - bp + G - 1) / G : 0;
  float* bias_lds = (float*)(smem + kBIAS);
  for (int c = tid * 4; c < N; c += 256 * 4) *(float4*)(bias_lds + c) = *(const float4*)(p.bias + c);
  if (my == 0) return;
  const float xs = p.omega * kInv2Pi;

  auto tile_of = [&](int g, int& m0, int& n0) {
    const int tm = g >> tn_shift;
    m0 = tm * kBM;
    n0 = (g - (tm << tn_shift)) * kBN;
  };
  // LDS-DMA: piece i < 4 is X rows 8 (wave + 4 i) .. +7, piece i >= 4 W rows 8 (wave + 4 i - 16) .. +7;
  // each lane moves 16 B of row lane / 8, swizzled on the source side
  const unsigned lane_src = (unsigned)(((lane >> 3) * K + swz(lane >> 3, lane & 7) * 8) * 2);
  auto issue = [&](const h16* xb, const h16* wb, int kt, int stage) {
    const unsigned st = lds_addr(smem) + (unsigned)(stage * kSTAGE);
#pragma unroll
    for (int i = 0; i < kPIECES; ++i) {
      const int row = (i < 4) ? 8 * (wave + 4 * i) : 8 * (wave + 4 * i - 16);
      const uint64_t src = (uint64_t)(i < 4 ? xb : wb) + (uint64_t)row * (K * 2) + kt * kROWB;
      // (readfirstlane returns int: widen through unsigned, or an address with bit 31 set sign-extends)
      const uint64_t su = ((uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(src >> 32)) << 32) |
                          (uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)src);
      glds16_asm_s(lane_src, (const void*)su, st + (i < 4 ? 0u : (unsigned)kXB) + (unsigned)(row * kROWB));
    }
  };
  int koff[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) koff[kk] = (lane & 15) * kROWB + (swz(lane & 15, (lane >> 4) + 4 * kk) << 4);
  auto frags = [&](int stage, int kk, h16x8 (&A)[kSN], h16x8 (&B)[kSM]) {
    const char* xsb = smem + stage * kSTAGE;
    const char* wsb = xsb + kXB;
#pragma unroll
    for (int i = 0; i < kSN; ++i) A[i] = *(const h16x8*)(wsb + (wave * 64 + i * 16) * kROWB + koff[kk]);
#pragma unroll
    for (int j = 0; j < kSM; ++j) B[j] = *(const h16x8*)(xsb + (j * 16) * kROWB + koff[kk]);
  };
  auto mma = [&](Acc& acc, const h16x8 (&A)[kSN], const h16x8 (&B)[kSM], auto zero) {
#pragma unroll
    for (int j = 0; j < kSM; ++j)
#pragma unroll
      for (int i = 0; i < kSN; ++i) {
        if constexpr (decltype(zero)::value)
          acc.v[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[i], B[j], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        else
          acc.v[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[i], B[j], acc.v[i][j], 0, 0, 0);
      }
  };
  // ---- epilogue of one tile: unit u = (row block u >> 1, column pair u & 1), in two halves h (the
  // pair's two 16-column subtiles); acc.v[i][j][r] = out[m0 + 16 j + (lane & 15)][n0 + 64 wave + 16 i
  // + 4 (lane >> 4) + r] (the ping-pong kernel's layout and arithmetic, gemm_nt.hip NT_FWD)
  struct Epi {
    float4 bias[kSN];
    size_t base;  // element offset of this lane's 8-column piece in row m0 + (lane & 15)
  };
  auto epi_setup = [&](int g, Epi& e) {
    int m0, n0;
    tile_of(g, m0, n0);
    const int nq = n0 + wave * 64 + 4 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < kSN; ++i) {
      const float4 b = *(const float4*)(bias_lds + nq + i * 16);
      e.bias[i] = float4{b.x * xs, b.y * xs, b.z * xs, b.w * xs};
    }
    e.base = (size_t)(m0 + (lane & 15)) * N + n0 + wave * 64 + swap16_col(lane);
  };
  auto epi_half = [&](auto uc, auto hc, const Acc& acc, const Epi& e, int token, uint2& ys, uint2& cs) {
    constexpr int U = decltype(uc)::value, H = decltype(hc)::value;
    constexpr int J = U >> 1, I = 2 * (U & 1) + H;
    const float bb[4] = {e.bias[I].x, e.bias[I].y, e.bias[I].z, e.bias[I].w};
    float s[4], c[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float x = __builtin_amdgcn_fractf(__builtin_fmaf(agpr_read(acc.v[I][J][r], token), xs, bb[r]));
      s[r] = __builtin_amdgcn_sinf(x);
      c[r] = __builtin_amdgcn_cosf(x);
    }
    ys = as_u2(pack4(s[0], s[1], s[2], s[3]));
    cs = as_u2(pack4(c[0], c[1], c[2], c[3]));
  };
  auto epi_store = [&](auto uc, const Epi& e, const uint2 (&ys)[2], const uint2 (&cs)[2]) {
    constexpr int U = decltype(uc)::value, J = U >> 1, PP = U & 1;
    if constexpr ((DG & 2) != 0) {
      asm volatile("" ::"v"(ys[0]), "v"(ys[1]), "v"(cs[0]), "v"(cs[1]));
      return;
    }
    const size_t off = e.base + (size_t)(J * 16) * N + PP * 32;
    *(uint4*)(p.Y + off) = swap16_pair(ys[0], ys[1]);
    *(uint4*)(p.C + off) = swap16_pair(cs[0], cs[1]);
  };

  // ---- the walk: tile i of this block is g = bp + i G
  const h16 *x0 = p.X, *w0 = p.W, *x1 = p.X, *w1 = p.W;
  int g_cur = bp;
  auto bases = [&](int g, const h16*& xb, const h16*& wb) {
    int m0, n0;
    tile_of(g, m0, n0);
    xb = p.X + (size_t)m0 * K;
    wb = p.W + (size_t)n0 * K;
  };
  auto set_tile = [&](int i) {  // current tile i, the next one's bases (itself past the end)
    bases(g_cur, x0, w0);
    if (i + 1 < my) bases(g_cur + G, x1, w1);
    else { x1 = x0; w1 = w0; }
  };
  set_tile(0);
  int sb = 0;  // stage of the current K-tile
  issue(x0, w0, 0, 0);
  issue(x0, w0, 1, 1);
  issue(x0, w0, 2, 2);
  h16x8 A0[kSN], B0[kSM], A1[kSN], B1[kSM];
  wait_vmcnt<2 * kPIECES>();
  wait_lgkm0();  // and the bias vector's LDS stores
  __builtin_amdgcn_s_barrier();
  frags(0, 0, A0, B0);

  // scheduling: regions fenced at the barrier and the stores; inside a region 12 fragment reads
  // first, then each MFMA followed by its share of the epilogue VALU (the matrix pipe runs 16 cycles
  // per MFMA, the wave issues the VALU meanwhile)
  auto fence = [&]() { __builtin_amdgcn_sched_barrier(0); };
  auto interleave = [&]() {
    constexpr int VPM = (22 * UPK + 31) / 32;  // epilogue VALU per MFMA (22 per half-unit)
    __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);
    static_for<0, 32>([&](auto) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, VPM, 0);
    });
  };
  // one tile's K loop into `acc`; EPI: the epilogue of the previous tile (eacc, e) rides along.
  // prev_st: the previous tile issued epilogue stores too (the counted waits of K-tiles 0 and 1)
  auto run_tile = [&](Acc& acc, auto epi, const Acc& eacc, const Epi& e, bool prev_st) __attribute__((always_inline)) {
    constexpr bool EPI = decltype(epi)::value;
    static_for<0, NK>([&](auto kc) {
      constexpr int KT = decltype(kc)::value;
      uint2 ys[UPK][2], cs[UPK][2];
      // [A] this K-tile's second k32 half
      frags(sb, 1, A1, B1);
      // [B] first half's MFMAs; the first half of this K-tile's epilogue units
      mma(acc, A0, B0, std::integral_constant<bool, KT == 0>{});
      if constexpr (EPI) {
        static_for<0, UPK>([&](auto q) {
          constexpr int Q = decltype(q)::value;
          epi_half(std::integral_constant<int, KT * UPK + Q>{}, std::integral_constant<int, 0>{}, eacc, e, sb,
                   ys[Q][0], cs[Q][0]);
        });
      }
      interleave();
      fence();
      // [C] K-tile KT + 1 has landed (this wave's pieces: counted; every wave's: the barrier), and
      // every wave is past K-tile KT: its stage takes K-tile KT + 3
      constexpr int C2 = 12 + 2 * S, C1 = 12 + S;
      if constexpr (!EPI && !OVL && KT < 2) {
        // the previous tile's end-of-tile epilogue (2 kUNITS stores) sits after K-tiles 1 and 2's pieces
        if (prev_st) wait_vmcnt<12 + 2 * kUNITS>();
        else wait_vmcnt<12>();
      } else if constexpr (!EPI) {
        wait_vmcnt<12>();
      } else if constexpr (KT == 0) {
        if (prev_st) wait_vmcnt<C2>();
        else wait_vmcnt<12>();
      } else if constexpr (KT == 1) {
        if (prev_st) wait_vmcnt<C2>();
        else wait_vmcnt<C1>();
      } else {
        wait_vmcnt<C2>();
      }
      wait_lgkm0();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      fence();
      // [D] K-tile KT + 3 (of this tile or the next) into this K-tile's stage
      if constexpr (KT + 3 < NK) issue(x0, w0, KT + 3, sb);
      else issue(x1, w1, KT + 3 - NK, sb);
      fence();
      // [E] the next K-tile's first half
      const int sn = sb == kNST - 1 ? 0 : sb + 1;
      frags(sn, 0, A0, B0);
      // [F] second half's MFMAs; the second half of the epilogue units
      mma(acc, A1, B1, std::false_type{});
      if constexpr (EPI) {
        static_for<0, UPK>([&](auto q) {
          constexpr int Q = decltype(q)::value;
          epi_half(std::integral_constant<int, KT * UPK + Q>{}, std::integral_constant<int, 1>{}, eacc, e, sn,
                   ys[Q][1], cs[Q][1]);
        });
      }
      interleave();
      fence();
      if constexpr (EPI) {
        // [G] the units' stores
        static_for<0, UPK>([&](auto q) {
          constexpr int Q = decltype(q)::value;
          epi_store(std::integral_constant<int, KT * UPK + Q>{}, e, ys[Q], cs[Q]);
        });
      }
      fence();
      sb = sn;
    });
  };
  auto final_epi = [&](const Acc& acc, const Epi& e) __attribute__((always_inline)) {
    static_for<0, kUNITS>([&](auto u) {
      uint2 ys[2], cs[2];
      epi_half(u, std::integral_constant<int, 0>{}, acc, e, 0, ys[0], cs[0]);
      epi_half(u, std::integral_constant<int, 1>{}, acc, e, 0, ys[1], cs[1]);
      epi_store(u, e, ys, cs);
    });
  };

  // one loop body: the finished tile's accumulators are copied to the epilogue set (128 AGPR moves
  // per tile) while the MFMAs of the next one start from zero
  Acc a;
  Epi e;
  if constexpr (!OVL) {
    for (int i = 0; i < my; ++i) {
      run_tile(a, std::false_type{}, a, e, i > 0 && DG == 0);
      epi_setup(g_cur, e);
      if constexpr ((DG & 1) == 0) {
        final_epi(a, e);
      } else {  // keep every accumulator live (timing only)
        float t = 0.f;
#pragma unroll
        for (int ii = 0; ii < kSN; ++ii)
#pragma unroll
          for (int j = 0; j < kSM; ++j) t += a.v[ii][j][0] + a.v[ii][j][3];
        if (t == 1234.5f) p.Y[tid] = (h16)t;
      }
      if (i + 1 < my) {
        g_cur += G;
        set_tile(i + 1);
      }
    }
    wait_vmcnt<0>();
    return;
  }
  run_tile(a, std::false_type{}, a, e, false);
  for (int i = 1; i < my; ++i) {
    const Acc prev = a;
    epi_setup(g_cur, e);  // tile i - 1
    g_cur += G;
    set_tile(i);
    run_tile(a, std::integral_constant<bool, (DG & 1) == 0>{}, prev, e, i >= 2);
  }
  epi_setup(g_cur, e);
  if constexpr ((DG & 1) == 0) final_epi(a, e);
  else asm volatile("" ::"a"(a.v[0][0]));
  wait_vmcnt<0>();
}

}  // namespace

bool gemm_nt_one_ok(const NtParams& p) {
  const int nk = p.K / kBK;
  const int tn = p.N / kBN;
  return p.K % kBK == 0 && (nk == 4 || nk == 8 || nk == 16) && p.N % kBN == 0 && (tn == 1 || tn == 2 || tn == 4) &&
         p.M % kBM == 0 && p.M > 0;
}

template <int DG, bool OVL>
static void launch_one(const NtParams& p, int g, hipStream_t s) {
  switch (p.K / kBK) {
    case 4: hipLaunchKernelGGL((nt_fwd_one<4, DG, OVL>), dim3(g), dim3(256), 0, s, p); break;
    case 8: hipLaunchKernelGGL((nt_fwd_one<8, DG, OVL>), dim3(g), dim3(256), 0, s, p); break;
    default: hipLaunchKernelGGL((nt_fwd_one<16, DG, OVL>), dim3(g), dim3(256), 0, s, p); break;
  }
}

template <bool OVL>
static hipError_t launch_one_diag(const NtParams& p, int g, int diag, hipStream_t s) {
#ifdef SIREN_DIAG
  if (diag & 1024) launch_one<1, OVL>(p, g, s);
  else if (diag & 2048) launch_one<2, OVL>(p, g, s);
  else launch_one<0, OVL>(p, g, s);
#else
  if (diag) return hipErrorInvalidValue;
  launch_one<0, OVL>(p, g, s);
#endif
  return hipGetLastError();
}

hipError_t gemm_nt_one(const NtParams& p, int grid, int diag, bool overlap, hipStream_t s) {
  if (!gemm_nt_one_ok(p) || grid <= 0) return hipErrorInvalidValue;
  const int ntiles = (p.M / kBM) * (p.N / kBN);
  const int g = grid < ntiles ? grid : ntiles;
  return overlap ? launch_one_diag<true>(p, g, diag, s) : launch_one_diag<false>(p, g, diag, s);
}

}  // namespace siren
