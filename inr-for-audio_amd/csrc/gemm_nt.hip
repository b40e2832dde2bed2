// NT GEMM for the SIREN hidden layers on gfx950 h16 MFMA with fused epilogues.
//
//   acc[m][n] = sum_k X[m][k] * W[n][k]        (X: [M][K] h16, W: [N][K] h16, fp32 acc)
//
// Three epilogues (template MODE):
//   NT_FWD : a = omega*(acc + b[n]);  Y = sin a, C = cos a   (h16 out)     -- models.py:114-115
//            optional HEAD: per-row partial of sum_n Y[m][n]*w_head[n]      -- models.py:374-381
//   NT_DX  : dz = (acc * Cprev[m][n]) * omega_prev  (h16 out) + column partial sums (db)
//            = autograd of sin(omega*linear) for the layer below            -- models.py:114-115
//   NT_FWD_SNAKE : z = acc + b;  Y = z + sin^2(a z)/a, C = 1 + sin(2az) (dY/dz),
//            E = (z sin(2az) - sin^2(az)/a)/a (dY/da)                      -- models.py:235-241
//   NT_FWD_TANH  : z = acc + b;  Y = tanh z, C = 1 - Y^2                    -- models.py:366-372
//   NT_DX_SNAKE  : dz = acc * D (Cprev) + column partials of dz (db) and acc * E (da)
//   NT_DX0_SNAKE : same into a Linear + Snake first layer (Cprev = D0, omega 1) + da0 partials
//   NT_DX0 : same, into the fp32 first layer (Cprev = its cos from first_fwd): only the
//            column partial sums of dz and dz*t_j (db0, dW0) are written; dZ0 never
//            reaches HBM.
//
// Tiles: 256x256 with 8 waves (2x4, each 128x64 = 8x4 v_mfma_f32_16x16x32_f16 tiles),
// PERSISTENT: one block per CU walks its tiles and the double-buffered LDS ring runs across
// tile boundaries (gemm_pipeline.h mfma_pipeline_tiles): both first operand stages of tile
// i+1 are in flight before tile i's epilogue issues its stores, which then drain under
// tile i+1's first two K-steps.  A 128x128 / 4-wave config (2 blocks per CU, one tile per
// block) serves grids too small for 256x256.  Operands are staged HBM->LDS by LDS-DMA
// (global_load_lds_dwordx4 from inline asm), with an XOR swizzle on the SOURCE address so
// that the ds_read_b128 fragment reads are bank-conflict free (cdna_hip_programming.md
// §5.4 rule 21 / T2).
//
// MFMA operand roles are swapped (A := W rows, B := X rows) so each lane ends up holding 4
// consecutive output COLUMNS of one row (per-row bias loads as one float4); adjacent column
// subtiles are then exchanged across 16-lane groups (swap16_pair) so every epilogue store
// and Cprev load is a 16-B row piece.  The epilogue's store tail is issue-bound (measured:
// 64 scattered dwordx2 per lane cost 1.0 ms of a 2.8 ms forward GEMM), so halving the
// instruction count and keeping the stores behind two prefetched stages is what matters.
#include <mutex>

#include "gemm_pipeline.h"
#include "siren_common.h"
#include "siren_kernels.h"

#ifndef SIREN_XPOL
#define SIREN_XPOL 0  // cache policy of the X-operand LDS-DMA (glds16_asm_pol; measurement builds)
#endif
#ifndef SIREN_WPOL
#define SIREN_WPOL 0  // ... of the W operand
#endif
#ifndef SIREN_STPOL
#define SIREN_STPOL 0  // epilogue store cache policy (measurement builds; see st16)
#endif
#ifndef SIREN_FULLLINE
#define SIREN_FULLLINE 0  // forward epilogue stores as whole 128-B lines (measurement builds)
#endif

namespace siren {

// Source-side XOR swizzle of a staged [rows][BK] fp16 image (16-B chunks).  BK = 64 (128-B
// rows, 8 chunks): chunk ^ (row & 7).  BK = 32 (64-B rows, 4 chunks): chunk ^ H[(row>>2)&3]
// with H = {0,2,3,1}, which makes every 16-lane group of a ds_read_b128 fragment read hit
// 16 distinct 16-B bank slots.
template <int BK>
__device__ __forceinline__ int stage_swz(int r, int c) {
  if constexpr (BK == 64) return c ^ (r & 7);
  else return c ^ ((0x78 >> (2 * ((r >> 2) & 3))) & 3);  // H as 2-bit fields of 0x78
}

template <int BM_, int BN_, int WM_, int WN_, int BK_, int S_, bool PP_ = false, int PF_ = 0, int BPC_ = 1>
struct NtCfg {
  static constexpr int BM = BM_, BN = BN_, BK = BK_, S = S_;
  static constexpr int BPC = BPC_;  // persistent grid: blocks per CU (2: two independent tile
                                    // streams per CU, one's epilogue under the other's MFMAs)
  static constexpr bool PP = PP_;  // ping-pong K-loop (gemm_pipeline.h pingpong_tiles)
  // L2 prefetch of the X operand p.pf_dist K-steps ahead of the LDS-DMA: one 4-B touch per
  // 128-B line, PF instructions per wave per stage (BM*BK*2/128 lines over the block)
  static constexpr int PF = PF_;
  static constexpr int WM = WM_, WN = WN_, NWAVES = WM_ * WN_, THREADS = 64 * NWAVES;
  static constexpr int TM = BM / WM, TN = BN / WN;  // wave tile
  static constexpr int SM = TM / 16, SN = TN / 16;  // 16x16 MFMA tiles per wave
  static constexpr int ROWB = BK * 2;               // bytes per staged row
  static constexpr int RPI = 1024 / ROWB, SPR = ROWB / 16;  // rows / 16-B slots per DMA piece
  static constexpr int XBYTES = BM * ROWB, WBYTES = BN * ROWB;
  static constexpr int STAGE = XBYTES + WBYTES;
  static constexpr int RING = S * STAGE;
  // epilogue scratch behind the ring: HEAD row partials [WN][BM] or column sums [3][WM][BN],
  // then (NT_FWD) the whole bias and head weight vectors, staged once per block
  static constexpr int RED = 4 * (WN * BM > 4 * WM * BN ? WN * BM : 4 * WM * BN);
  static constexpr int MAXN = 1024;
  static constexpr int VEC = 4 * MAXN;  // one per-column fp32 vector
  static constexpr int XINSTR = XBYTES / 1024 / NWAVES;  // LDS-DMA instructions per wave per stage
  static constexpr int WINSTR = WBYTES / 1024 / NWAVES;
  static_assert(XBYTES % (1024 * NWAVES) == 0 && WBYTES % (1024 * NWAVES) == 0, "staging split");
  static_assert(SN % 2 == 0, "16-B row pieces pair adjacent column subtiles");
  static_assert(RING + RED + 3 * VEC + 256 <= 160 * 1024, "LDS");
};
using NtSmall = NtCfg<128, 128, 2, 2, 64, 2>;
// 256x256 variants (siren_set_option SIREN_OPT_NT_PIPE): BK 64 double buffer (one tile per
// block, or persistent), BK 32 rings of 4 / 3 slots (persistent)
using NtLarge = NtCfg<256, 256, 2, 4, 64, 2>;
using NtLargeR4 = NtCfg<256, 256, 2, 4, 32, 4>;
using NtLargeR3 = NtCfg<256, 256, 2, 4, 32, 3>;
// BK 64 double buffer, persistent, two wave groups in ping-pong (SIREN_OPT_NT_PIPE 4)
using NtLargePP = NtCfg<256, 256, 2, 4, 64, 2, true>;
// BK 64 double buffer, persistent, X prefetched into L2 ahead of the LDS-DMA (NT_PIPE 5)
using NtLargePF = NtCfg<256, 256, 2, 4, 64, 2, false, 1>;
// 128x256 tiles, 4 waves (1x4, 128x64 each), BK 32 3-slot ring, persistent with TWO blocks
// per CU (NT_PIPE 6) / BK 32 double buffer (NT_PIPE 7)
using NtMid3 = NtCfg<128, 256, 1, 4, 32, 3, false, 0, 2>;
using NtMid2 = NtCfg<128, 256, 1, 4, 32, 2, false, 0, 2>;

// LDS layout of one kernel instance: the ring, the epilogue reduction scratch, then only the
// per-column vectors its mode needs (bias for the forward modes, head weights with HEAD, Snake
// a), then the prefetch landing area -- so DX kernels and head-less forwards stay small enough
// for two blocks per CU where the config asks for it.
template <class Cfg, int MODE, bool HEAD>
struct NtLds {
  static constexpr int BIAS = Cfg::RING + Cfg::RED;
  static constexpr int HW = BIAS + (nt_is_fwd(MODE) ? Cfg::VEC : 0);
  static constexpr int A = HW + (HEAD ? Cfg::VEC : 0);
  static constexpr int PF = A + (MODE == NT_FWD_SNAKE ? Cfg::VEC : 0);
  static constexpr int QS = PF + (Cfg::PF ? 256 : 0);  // dynamic tile queue: 2 tile ids
  static constexpr int SIZE = QS + 16;
};

// Tile-queue counter set: 8 shard heads and the done counter 128 B apart, then 64 scratch words
// per shard
constexpr int kQueueHeads = 9 * 32, kQueueSet = kQueueHeads + 8 * 64;

// Dynamic tile queue (ping-pong K-loop).  A pull is one returning agent-scope atomic add on the
// block's shard head, issued at the start of a tile's epilogue and consumed after it: hipcc's
// own waitcnt then lets the epilogue's stores stay in flight (vmcnt retires in issue order).
// Wave 0 issues it with every lane active (lane 0 adds 1 to the head, lanes 1..63 add 0 to
// the shard's scratch words, so the head sees one add per pull and the returned VGPR is
// written in every lane).  The pull's VGPR lives only across the epilogue, not across the
// K-loop (no register to spare).  (An inline-asm pull whose VGPR hipcc does not know is in
// flight is unsafe: a register copy at a branch join reads it before it lands.)

constexpr bool nt_is_dx0(int m) { return m == NT_DX0 || m == NT_DX0_SNAKE; }

// store instructions every wave's epilogue issues (lower bound; see mfma_pipeline_tiles)
template <class Cfg, int MODE>
constexpr int epilogue_stores() {
  return (MODE == NT_FWD || MODE == NT_FWD_TANH) ? Cfg::SM * Cfg::SN
         : MODE == NT_FWD_SNAKE                 ? 3 * Cfg::SM * Cfg::SN / 2
         : (MODE == NT_DX || MODE == NT_DX_SNAKE) ? Cfg::SM * Cfg::SN / 2
                                                  : 0;
}

// QUEUE (ping-pong K-loop only): tiles from the dynamic queue p.tileq instead of the static walk
template <class Cfg, int MODE, bool HEAD, bool QUEUE = false>
__global__ __launch_bounds__(Cfg::THREADS, 2) void gemm_nt_kernel(NtParams p) {
  constexpr int BM = Cfg::BM, BN = Cfg::BN, BK = Cfg::BK, WN = Cfg::WN;
  constexpr int TM = Cfg::TM, TN = Cfg::TN, SM = Cfg::SM, SN = Cfg::SN;
  using Lay = NtLds<Cfg, MODE, HEAD>;
  __shared__ __attribute__((aligned(16))) char smem[Lay::SIZE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int K = p.K, N = p.N;
  const int tiles_n = N / BN;
  const int ntiles = (p.M / BM) * tiles_n;
  const bool tn_pow2 = (tiles_n & (tiles_n - 1)) == 0;  // N / BN is 1, 2, 4 or 8 at H <= 1024
  const int tn_shift = __builtin_ctz(tiles_n);
  // Block b takes tiles b', b'+G, ... with b' the XCD-grouped id: the G/8 blocks of one XCD
  // hold consecutive tile ids, i.e. they share X row-blocks in L2 at the same time.
  const int G = gridDim.x;
  const int bp = xcd_remap(blockIdx.x, G);
  // measurement-only ablation bits; the queue kernel is launched with none
  const int diag = (Cfg::PP && QUEUE) ? 0 : p.diag;
  const int my_tiles = (diag & 512) ? 0 : (ntiles - bp + G - 1) / G;  // diag bit 9: no tiles
  // Dynamic tile queue (ping-pong K-loop, NtParams::tileq).  With the static walk the four
  // blocks that share a row band of X drift apart over the launch and X is fetched ~1.6x from
  // HBM.  Instead the blocks of one shard (blockIdx % 8: one XCD under round-robin
  // dispatch -- speed only, any placement is correct) pull the tiles of their contiguous
  // eighth of the grid in order, so the blocks holding one row band are the ones that started
  // it at the same time.
  constexpr bool dyn = Cfg::PP && QUEUE;
  // Start stagger: blocks that run in lockstep hit their epilogues together and their
  // stores then arrive as one chip-wide burst; spreading the starts over a tile's duration
  // spreads the bursts.
  for (int i = (bp & 15) * p.stagger; i > 0; --i) __builtin_amdgcn_s_sleep(27);
  // global tile id g -> origin; the static walk's i-th tile of this block is g = bp + i * G
  auto tile_of = [&](int g, int& m0, int& n0) {
    const int tm = tn_pow2 ? (g >> tn_shift) : g / tiles_n;
    m0 = tm * BM;
    n0 = (g - tm * tiles_n) * BN;
  };

  // ---- LDS-DMA staging addresses -------------------------------------------------
  // One instruction moves 1 KiB = RPI rows x ROWB bytes.  Lane L lands at row L/SPR, 16-B
  // slot L%SPR, and carries the logical chunk stage_swz(row, slot) (source-side swizzle).
  constexpr int ROWB = Cfg::ROWB, RPI = Cfg::RPI, SPR = Cfg::SPR;
  size_t xrel[Cfg::XINSTR], wrel[Cfg::WINSTR];
#pragma unroll
  for (int j = 0; j < Cfg::XINSTR; ++j) {
    const int r = (wave * Cfg::XINSTR + j) * RPI + lane / SPR;
    xrel[j] = (size_t)r * K + stage_swz<BK>(r, lane % SPR) * 8;
  }
#pragma unroll
  for (int j = 0; j < Cfg::WINSTR; ++j) {
    const int r = (wave * Cfg::WINSTR + j) * RPI + lane / SPR;
    wrel[j] = (size_t)r * K + stage_swz<BK>(r, lane % SPR) * 8;
  }
  auto stage = [&](int ti, int kt, int slot) {
    int m0, n0;
    tile_of(bp + ti * G, m0, n0);
    const char* xs = smem + slot * Cfg::STAGE + wave * Cfg::XINSTR * 1024;
    const char* ws = smem + slot * Cfg::STAGE + Cfg::XBYTES + wave * Cfg::WINSTR * 1024;
    const h16* xk = p.X + (size_t)((diag & 1) ? (m0 & (4 * BM - 1)) : m0) * K + kt * BK;
    const h16* wk = p.W + (size_t)n0 * K + kt * BK;
#pragma unroll
    for (int j = 0; j < Cfg::XINSTR; ++j) glds16_asm(xk + xrel[j], lds_addr(xs + j * 1024));
#pragma unroll
    for (int j = 0; j < Cfg::WINSTR; ++j) glds16_asm(wk + wrel[j], lds_addr(ws + j * 1024));
    if constexpr (Cfg::PF > 0) {
      static_assert(Cfg::PF * Cfg::NWAVES * 32 * 128 == BM * ROWB, "one touch per 128-B X line");
      // K-step pf_dist ahead (always issued -- the counted waits assume PF ops per stage;
      // past the block's last tile it re-touches this stage)
      int pt = ti, pk = kt + p.pf_dist;
      while (pk >= p.K / BK) { pk -= p.K / BK; ++pt; }
      if (pt >= my_tiles) pt = ti, pk = kt;
      int pm0, pn0;
      tile_of(bp + pt * G, pm0, pn0);
#pragma unroll
      for (int j = 0; j < Cfg::PF; ++j) {
        const int r = (wave * Cfg::PF + j) * 32 + (lane & 31);
        gpf4_asm(p.X + (size_t)(pm0 + r) * K + pk * BK + (lane >> 5) * 32, lds_addr(smem + Lay::PF));
      }
    }
  };

  // ---- fragment read offsets --------------------------------------------------------
  // 16x16x32 operand: lane holds row (lane&15), k = 8*(lane>>4) .. +7 of a 32-deep half;
  // fragment rows start at multiples of 16, so the swizzle depends on the lane only.
  int koff[BK / 32];
#pragma unroll
  for (int kk = 0; kk < BK / 32; ++kk)
    koff[kk] = (lane & 15) * ROWB + (stage_swz<BK>(lane & 15, (lane >> 4) + 4 * kk) << 4);
  auto frags = [&](int slot, int kk, h16x8 (&A)[SN], h16x8 (&B)[SM]) {
    const char* xs = smem + slot * Cfg::STAGE;
    const char* ws = xs + Cfg::XBYTES;
#pragma unroll
    for (int i = 0; i < SN; ++i) A[i] = *(const h16x8*)(ws + (wn * TN + i * 16) * ROWB + koff[kk]);
#pragma unroll
    for (int j = 0; j < SM; ++j) B[j] = *(const h16x8*)(xs + (wm * TM + j * 16) * ROWB + koff[kk]);
  };

  f32x4 acc[SN][SM];
#pragma unroll
  for (int i = 0; i < SN; ++i)
#pragma unroll
    for (int j = 0; j < SM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- epilogue (per tile) ------------------------------------------------------------
  // acc[i][j][r] = out[m][n] with m = m0 + wm*TM + j*16 + (lane&15),
  //                              n = n0 + wn*TN + i*16 + 4*(lane>>4) + r.
  // Global traffic goes in 16-B row pieces: column subtiles (2p, 2p+1) are exchanged with
  // swap16_pair, this lane's piece starting at column ncol + 32p + swap16_col(lane).
  float* red = (float*)(smem + Cfg::RING);
  // 16-B epilogue store; SIREN_OPT_NT_DIAG bit 1 (measurement only) keeps the value live
  // and drops the store
  // SIREN_STPOL (measurement builds): cache policy of the epilogue's 16-B stores -- 0 plain,
  // 1 nt, 2 sc1 (write-through), 3 sc0 sc1.  The asm forms carry their own s_nop: hipcc's hazard
  // recognizer does not see that a VALU write of the data VGPRs must wait a cycle after a
  // 128-bit store (without it the outputs differed from the plain build's)
  auto st16 = [&](h16* dst, uint4 v) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    [[maybe_unused]] const u32x4 w = u32x4{v.x, v.y, v.z, v.w};
    if constexpr (SIREN_STPOL == 1) asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" ::"v"(dst), "v"(w) : "memory");
    else if constexpr (SIREN_STPOL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(dst), "v"(w) : "memory");
    else if constexpr (SIREN_STPOL == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(dst), "v"(w) : "memory");
    else *(uint4*)dst = v;
  };
  // NT_FWD: bias / head weights through LDS -- the epilogue then issues no global load
  // whose compiler-counted vmcnt wait would also cover the asm-issued stage prefetch.
  float* bias_lds = (float*)(smem + Lay::BIAS);
  float* hw_lds = (float*)(smem + Lay::HW);
  float* a_lds = (float*)(smem + Lay::A);  // Snake: a
  if constexpr (nt_is_fwd(MODE)) {
    for (int c = tid * 4; c < N; c += Cfg::THREADS * 4) {
      *(float4*)(bias_lds + c) = *(const float4*)(p.bias + c);
      if constexpr (HEAD) *(float4*)(hw_lds + c) = *(const float4*)(p.head_w + c);
      if constexpr (MODE == NT_FWD_SNAKE) *(float4*)(a_lds + c) = *(const float4*)(p.act_a + c);
    }
    // visible to other waves after the pipeline's first barrier
  }
  // dZ carries the backward storage scale S; the fp32 column partials leave unscaled
  const float inv_scale = (!nt_is_fwd(MODE) && p.gscale) ? p.gscale[1] : 1.0f;
  // NT_DX / NT_DX0 epilogue operands loaded by `pre` (before the next tile's early prefetch)
  constexpr int PRE_J = nt_is_fwd(MODE) ? 0 : (MODE == NT_DX ? SM : SM / 2);
  uint4 cp_in[PRE_J > 0 ? PRE_J : 1][SN / 2];
  float t_in[SM][2];
  // SIREN_FULLLINE (measurement builds): Cprev of row subtile j as two whole-line loads, rows
  // 0..7 (A) and 8..15 (B) of the subtile, each lane a 16-B piece; fl_pieces turns them into this
  // lane's two natural pieces (lanes l, l^8 trade one piece by DPP row_ror:8)
  constexpr bool FL_LOAD = SIREN_FULLLINE && SN == 4 && !nt_is_fwd(MODE);
  auto fl_load = [&](int mtop, int ncol, uint4 (&raw)[SN / 2]) {
    const size_t ra = (size_t)(mtop + (lane & 7)) * N + ncol + ((lane & 8) ? 32 : 0);
    raw[0] = *(const uint4*)(p.Cprev + ra);
    raw[1] = *(const uint4*)(p.Cprev + ra + (size_t)8 * N);
  };
  auto fl_pieces = [&](const uint4 (&raw)[SN / 2], int pp) {
    const bool hi = (lane & 8) != 0;
    const uint4 send = hi ? raw[0] : raw[1];
    uint4 recv;
    recv.x = __builtin_amdgcn_update_dpp(0, (int)send.x, 0x128, 0xf, 0xf, false);
    recv.y = __builtin_amdgcn_update_dpp(0, (int)send.y, 0x128, 0xf, 0xf, false);
    recv.z = __builtin_amdgcn_update_dpp(0, (int)send.z, 0x128, 0xf, 0xf, false);
    recv.w = __builtin_amdgcn_update_dpp(0, (int)send.w, 0x128, 0xf, 0xf, false);
    return pp == 0 ? (hi ? recv : raw[0]) : (hi ? raw[1] : recv);
  };
  auto pre = [&](int g) {
    int m0, n0;
    tile_of(g, m0, n0);
    const int npc = n0 + wn * TN + swap16_col(lane);
    const int mrow0 = m0 + wm * TM + (lane & 15);
    if constexpr (!nt_is_fwd(MODE)) {
#pragma unroll
      for (int j = 0; j < PRE_J; ++j) {
        if constexpr (FL_LOAD) {
          fl_load(m0 + wm * TM + j * 16, npc, cp_in[j]);
        } else {
#pragma unroll
          for (int pp = 0; pp < SN / 2; ++pp)
            cp_in[j][pp] = *(const uint4*)(p.Cprev + (size_t)(mrow0 + j * 16) * N + npc + pp * 32);
        }
      }
      if constexpr (nt_is_dx0(MODE)) {
#pragma unroll
        for (int j = 0; j < SM; ++j) {
          const size_t m = mrow0 + j * 16;
          t_in[j][0] = p.t[m * p.in_dim];
          t_in[j][1] = (p.in_dim > 1) ? p.t[m * p.in_dim + 1] : 0.f;
        }
      }
    }
  };
  auto epilogue = [&](int g) {
    int m0, n0;
    tile_of(g, m0, n0);
    const int tm = m0 / BM, tn = n0 / BN;
    const int npc = n0 + wn * TN + swap16_col(lane);      // swapped layout: this lane's piece
    const int mrow0 = m0 + wm * TM + (lane & 15);

    if constexpr (nt_is_fwd(MODE)) {
      const int nq = n0 + wn * TN + 4 * (lane >> 4);     // natural layout: this lane's columns
      const float xs = (MODE == NT_FWD) ? p.omega * kInv2Pi : 1.0f;
      float4 bias[SN], hw[SN];
#pragma unroll
      for (int i = 0; i < SN; ++i) {
        const float4 b = *(const float4*)(bias_lds + nq + i * 16);
        bias[i] = float4{b.x * xs, b.y * xs, b.z * xs, b.w * xs};
        if constexpr (HEAD) hw[i] = *(const float4*)(hw_lds + nq + i * 16);
      }
      float hp[SM];
#pragma unroll
      for (int j = 0; j < SM; ++j) hp[j] = 0.f;
#pragma unroll
      for (int j = 0; j < SM; ++j) {
        const size_t rowoff = (size_t)(mrow0 + j * 16) * N;
        uint4 yp[SN / 2], cpk[SN / 2], epk[SN / 2];
#pragma unroll
        for (int pp = 0; pp < SN / 2; ++pp) {
          uint2 ys[2], cs[2], es[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int i = 2 * pp + h;
            const float bb[4] = {bias[i].x, bias[i].y, bias[i].z, bias[i].w};
            float s[4], c[4], e[4];
            if constexpr (MODE == NT_FWD) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                // revolutions: sin(2*pi*x) with x = omega*(z + b)/(2*pi); fract keeps the
                // hardware sin/cos inside their reduced domain for any magnitude.
                const float x = __builtin_amdgcn_fractf(__builtin_fmaf(acc[i][j][r], xs, bb[r]));
                s[r] = __builtin_amdgcn_sinf(x);
                c[r] = __builtin_amdgcn_cosf(x);
              }
            } else if constexpr (MODE == NT_FWD_SNAKE) {
              const float4 a4 = *(const float4*)(a_lds + nq + i * 16);
              const float av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float z = acc[i][j][r] + bb[r];
                const float ia = 1.0f / av[r];
                const float x = __builtin_amdgcn_fractf((z * av[r]) * kInv2Pi);  // a z in revolutions
                const float sn = __builtin_amdgcn_sinf(x), cn = __builtin_amdgcn_cosf(x);
                const float s2 = sn * sn, sc2 = 2.0f * sn * cn;
                s[r] = z + s2 * ia;                    // models.py:241
                c[r] = 1.0f + sc2;                     // dY/dz
                e[r] = (z * sc2 - s2 * ia) * ia;       // dY/da
              }
            } else {  // NT_FWD_TANH
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float y = tanhf(acc[i][j][r] + bb[r]);
                s[r] = y;
                c[r] = 1.0f - y * y;
              }
            }
            ys[h] = as_u2(pack4(s[0], s[1], s[2], s[3]));
            cs[h] = as_u2(pack4(c[0], c[1], c[2], c[3]));
            if constexpr (MODE == NT_FWD_SNAKE) es[h] = as_u2(pack4(e[0], e[1], e[2], e[3]));
            if constexpr (HEAD)
              hp[j] += s[0] * hw[i].x + s[1] * hw[i].y + s[2] * hw[i].z + s[3] * hw[i].w;
          }
          yp[pp] = swap16_pair(ys[0], ys[1]);
          cpk[pp] = swap16_pair(cs[0], cs[1]);
          if constexpr (MODE == NT_FWD_SNAKE) epk[pp] = swap16_pair(es[0], es[1]);
        }
        if constexpr (SIREN_FULLLINE && SN == 4) {
          // lanes l and l^8 (rows r, r^8 of the subtile) trade one 16-B piece so that each store
          // instruction writes 8 whole 128-B row segments instead of 16 half ones:
          // A = rows 0..7 (low lanes their piece 0, high lanes the partner's piece 1), B = rows 8..15
          const bool hi = (lane & 8) != 0;
          const size_t ra = (size_t)(m0 + wm * TM + j * 16 + (lane & 7)) * N + npc + (hi ? 32 : 0);
          auto fl_store = [&](h16* dst, const uint4 (&pc)[SN / 2]) {
            const uint4 send = hi ? pc[0] : pc[1];
            uint4 recv;
            recv.x = __builtin_amdgcn_update_dpp(0, (int)send.x, 0x128, 0xf, 0xf, false);  // row_ror:8
            recv.y = __builtin_amdgcn_update_dpp(0, (int)send.y, 0x128, 0xf, 0xf, false);
            recv.z = __builtin_amdgcn_update_dpp(0, (int)send.z, 0x128, 0xf, 0xf, false);
            recv.w = __builtin_amdgcn_update_dpp(0, (int)send.w, 0x128, 0xf, 0xf, false);
            st16(dst + ra, hi ? recv : pc[0]);
            st16(dst + ra + (size_t)8 * N, hi ? pc[1] : recv);
          };
          fl_store(p.Y, yp);
          fl_store(p.C, cpk);
          if constexpr (MODE == NT_FWD_SNAKE) fl_store(p.E, epk);
        } else {
#pragma unroll
          for (int pp = 0; pp < SN / 2; ++pp) {
            st16(p.Y + rowoff + npc + pp * 32, yp[pp]);
            st16(p.C + rowoff + npc + pp * 32, cpk[pp]);
            if constexpr (MODE == NT_FWD_SNAKE) st16(p.E + rowoff + npc + pp * 32, epk[pp]);
          }
        }
      }
      if constexpr (HEAD) {
        // lanes l, l^16, l^32, l^48 hold the same row: fold them, then the WN column waves.
#pragma unroll
        for (int j = 0; j < SM; ++j) {
          hp[j] += __shfl_xor(hp[j], 16, 64);
          hp[j] += __shfl_xor(hp[j], 32, 64);
        }
        if (lane < 16) {
#pragma unroll
          for (int j = 0; j < SM; ++j) red[wn * BM + wm * TM + j * 16 + lane] = hp[j];
        }
        lds_barrier();
        if (tid < BM) {
          float s = 0.f;
#pragma unroll
          for (int w = 0; w < WN; ++w) s += red[w * BM + tid];
          p.head_part[(size_t)tn * p.M + m0 + tid] = s;
        }
      }
    } else {
      // column sums over this tile's BM rows (db / dW0 partials): per lane over its SM row
      // tiles, over the 16 row-lanes by DPP, then over the WM row waves through LDS.
      const int in_dim = nt_is_dx0(MODE) ? p.in_dim : 0;
      const int nred = (MODE == NT_DX_SNAKE) ? 2 : (MODE == NT_DX0_SNAKE ? 2 + in_dim : 1 + in_dim);
      // slots: 0 db; 1..in dW0 (NT_DX0*); 1 da (NT_DX_SNAKE); 3 da0 (NT_DX0_SNAKE, written as 1+in)
      float cs[4][SN][4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < SN; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) cs[q][i][r] = 0.f;

      const float om = p.omega;
#pragma unroll
      for (int j = 0; j < SM; ++j) {
        const int m = mrow0 + j * 16;
        const size_t rowoff = (size_t)m * N;
        float t0 = 0.f, t1 = 0.f;
        if constexpr (nt_is_dx0(MODE)) {
          t0 = t_in[j][0];
          t1 = t_in[j][1];
        }
        uint4 fl_raw[SN / 2];
        if constexpr (FL_LOAD) {
          if (j < PRE_J) {
            fl_raw[0] = cp_in[j < PRE_J ? j : 0][0];
            fl_raw[1] = cp_in[j < PRE_J ? j : 0][1];
          } else {
            fl_load(m0 + wm * TM + j * 16, npc, fl_raw);
          }
        }
#pragma unroll
        for (int pp = 0; pp < SN / 2; ++pp) {
          uint2 cpu[2];
          uint4 cpv;
          if constexpr (FL_LOAD) cpv = fl_pieces(fl_raw, pp);
          else cpv = (j < PRE_J) ? cp_in[j < PRE_J ? j : 0][pp] : *(const uint4*)(p.Cprev + rowoff + npc + pp * 32);
          unswap16_pair(cpv, cpu[0], cpu[1]);
          uint2 epu[2];
          if constexpr (MODE == NT_DX_SNAKE || MODE == NT_DX0_SNAKE)
            unswap16_pair(*(const uint4*)(p.Eprev + rowoff + npc + pp * 32), epu[0], epu[1]);
          uint2 dzp[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int i = 2 * pp + h;
            const h16x4 cp = as_h4(cpu[h]);
            float dz[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              dz[r] = (acc[i][j][r] * (float)cp[r]) * om;
              cs[0][i][r] += dz[r];
              if constexpr (nt_is_dx0(MODE)) {
                cs[1][i][r] += dz[r] * t0;
                cs[2][i][r] += dz[r] * t1;
              }
              if constexpr (MODE == NT_DX_SNAKE) cs[1][i][r] += acc[i][j][r] * (float)as_h4(epu[h])[r];
              if constexpr (MODE == NT_DX0_SNAKE) cs[3][i][r] += acc[i][j][r] * (float)as_h4(epu[h])[r];
            }
            dzp[h] = as_u2(pack4(dz[0], dz[1], dz[2], dz[3]));
          }
          if constexpr (MODE == NT_DX || MODE == NT_DX_SNAKE)
            st16(p.dZ + rowoff + npc + pp * 32, swap16_pair(dzp[0], dzp[1]));
        }
      }
      // partial layout: NT_DX [tm][N]; NT_DX0 [tm][1+in][N] with q=0 -> db0, q=1+j -> dW0[:, j];
      // NT_DX_SNAKE [tm][2][N] with q=0 -> db, q=1 -> da
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (q >= nred) break;
        // NT_DX0_SNAKE: da0 (slot 3) goes out as partial row 1 + in
        const bool da0 = (MODE == NT_DX0_SNAKE) && q == nred - 1;
#pragma unroll
        for (int i = 0; i < SN; ++i) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = row16_sum(da0 ? cs[3][i][r] : cs[q][i][r]);
          if ((lane & 15) == 0)
            *(float4*)(red + (q * Cfg::WM + wm) * BN + wn * TN + i * 16 + 4 * (lane >> 4)) =
                float4{v[0], v[1], v[2], v[3]};
        }
      }
      lds_barrier();
      if (tid < BN) {
        for (int q = 0; q < nred; ++q) {
          float s = 0.f;
#pragma unroll
          for (int w = 0; w < Cfg::WM; ++w) s += red[(q * Cfg::WM + w) * BN + tid];
          p.colsum_part[((size_t)tm * nred + q) * N + n0 + tid] = s * inv_scale;
        }
      }
    }
  };

  if constexpr (Cfg::PP) {
    static_assert(BM == 256 && BN == 256 && BK == 64 && Cfg::WM == 2 && WN == 4, "ping-pong geometry");
    const int nk = K / BK;
    // Staging pieces of a K-tile (16 KiB, 2 LDS-DMA per wave; 8 rows x 128 B per instruction):
    //   pc 0: W rows wn*64 + 0..31   (phase a)      pc 1: X rows wm*128 + 0..63   (phase a)
    //   pc 2: W rows wn*64 + 32..63  (phase b)      pc 3: X rows wm*128 + 64..127 (phases c)
    // Phases (m half, n half) of every wave's 128x64 tile: a (0,0), b (0,1), c (1,1), d (1,0).
    int psrc[4][2];
    unsigned pdst[4][2];
#pragma unroll
    for (int pc = 0; pc < 4; ++pc)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int pr0 = (2 * wave + j) * 8, hf = pc >> 1;
        const int lr0 = (pc & 1) ? (pr0 >> 6) * 128 + (pr0 & 63) + 64 * hf
                                 : (pr0 >> 5) * 64 + (pr0 & 31) + 32 * hf;
        const int lr = lr0 + (lane >> 3);
        psrc[pc][j] = lr * K + stage_swz<BK>(lr, lane & 7) * 8;
        pdst[pc][j] = ((pc & 1) ? 0u : (unsigned)Cfg::XBYTES) + (unsigned)(lr0 * ROWB);
      }
    // operand bases of the current tile (0) and the next one (1), set once per tile:
    // no division or 64-bit product in the per-phase scalar work
    const h16 *x0 = p.X, *x1 = p.X, *w0 = p.W, *w1 = p.W;
    // This block's current and next tile (global ids); the next one exists while g_next < g_lim.
    // Static walk: bp, bp + G, ...  Queue: shard s = blockIdx % 8 (one XCD under round-robin
    // dispatch -- speed only, any placement is correct) pulls tiles [s, s + 1) * ntiles / 8 in
    // order, so the blocks holding one row band of X are the ones that started it together.
    const int shard = blockIdx.x & 7;
    const int q_lo = (int)((long)shard * ntiles / 8);
    const int g_lim = dyn ? (int)((long)(shard + 1) * ntiles / 8) : (my_tiles > 0 ? ntiles : 0);
    int* const qhead = p.tileq + shard * 32;  // dereferenced only when dyn
    int* const qslot = (int*)(smem + Lay::QS);
    int g_cur = bp, g_next = bp + G;
    if (dyn) {
      if (tid == 0) {
        qslot[0] = q_lo + __hip_atomic_fetch_add(qhead, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        qslot[1] = q_lo + __hip_atomic_fetch_add(qhead, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      lds_barrier();
      g_cur = __builtin_amdgcn_readfirstlane(qslot[0]);
      g_next = __builtin_amdgcn_readfirstlane(qslot[1]);
      lds_barrier();  // read by every wave before wave 0 reuses the slot
    }
    auto more = [&](int) { return g_next < g_lim; };
    auto set_tiles = [&](int ti) {
      if (ti > 0) {
        g_cur = g_next;
        // queue: the pull tile_end(ti - 1) left in the slot
        g_next = dyn ? __builtin_amdgcn_readfirstlane(qslot[0]) : g_next + G;
      }
      auto bases = [&](int g, const h16*& xb, const h16*& wb) {
        int m0, n0;
        tile_of(g, m0, n0);
        const int xm0 = (diag & 1) ? (m0 & (4 * BM - 1)) : m0;
        xb = p.X + (size_t)xm0 * K;
        wb = p.W + (size_t)((diag & 4) ? 0 : n0) * K;  // diag bit 2: one W column tile (L2-resident W)
      };
      bases(g_cur, x0, w0);
      bases(g_next < g_lim ? g_next : g_cur, x1, w1);
    };
    auto issue = [&](int sel, int kt, int slot, auto pcc) {
      constexpr int PC = decltype(pcc)::value;
      const h16* src = ((PC & 1) ? (sel ? x1 : x0) : (sel ? w1 : w0)) + kt * BK;
      const char* dst = smem + slot * Cfg::STAGE;
#pragma unroll
      for (int j = 0; j < 2; ++j)
        glds16_asm_pol<(PC & 1) ? SIREN_XPOL : SIREN_WPOL>(src + psrc[PC][j], lds_addr(dst + pdst[PC][j]));
    };
    h16x8 xf[4][2], wf0[2][2], wf1[2][2];
    auto rd_w = [&](h16x8 (&wf)[2][2], const char* ws, int n_off) {
#pragma unroll
      for (int il = 0; il < 2; ++il)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          wf[il][kk] = *(const h16x8*)(ws + (wn * TN + n_off + il * 16) * ROWB + koff[kk]);
    };
    auto read = [&](auto ph, int slot) {
      constexpr int PH = decltype(ph)::value;
      const char* xs = smem + slot * Cfg::STAGE;
      const char* ws = xs + Cfg::XBYTES;
      if constexpr (PH == 0 || PH == 2) {
#pragma unroll
        for (int jl = 0; jl < 4; ++jl)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
            xf[jl][kk] = *(const h16x8*)(xs + (wm * TM + (PH == 2 ? 64 : 0) + jl * 16) * ROWB + koff[kk]);
      }
      if constexpr (PH == 0) rd_w(wf0, ws, 0);
      if constexpr (PH == 1) rd_w(wf1, ws, 32);
    };
    auto mma = [&](auto ph) {
      constexpr int PH = decltype(ph)::value;
      constexpr int MH = PH >> 1, NH = (PH == 1 || PH == 2) ? 1 : 0;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int il = 0; il < 2; ++il)
#pragma unroll
          for (int jl = 0; jl < 4; ++jl) {
            const h16x8 a = NH ? wf1[il][kk] : wf0[il][kk];
            acc[2 * NH + il][4 * MH + jl] =
                __builtin_amdgcn_mfma_f32_16x16x32_f16(a, xf[jl][kk], acc[2 * NH + il][4 * MH + jl], 0, 0, 0);
          }
    };
#ifdef SIREN_NT_STAMPS
    // diagnostic builds only (tools/nt_stamps.py): per tile {start, global tile id, end of the
    // MFMAs, end of the epilogue} on the chip-wide 100 MHz real-time counter
    unsigned long long st_prev = 0;
    auto rt_now = [] {
      unsigned long long t;
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
      return t;
    };
    if (p.stamps) st_prev = rt_now();
#endif
    auto tile_end = [&](int ti) {
      // both groups are aligned here
#ifdef SIREN_NT_STAMPS
      const unsigned long long st_m = p.stamps ? rt_now() : 0;
#endif
      pre(g_cur);
      int pend = 0;  // the tile after next
      if (dyn && wave == 0)
        pend = __hip_atomic_fetch_add(lane == 0 ? qhead : p.tileq + kQueueHeads + shard * 64 + lane, lane == 0 ? 1 : 0,
                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!(diag & 1024)) epilogue(g_cur);  // diag bit 10: no epilogue (timing only)
      if constexpr (dyn) {
        if (tid == 0) qslot[0] = q_lo + pend;
        lds_barrier();
      }
#ifdef SIREN_NT_STAMPS
      if (p.stamps) {
        const unsigned long long st_e = rt_now();
        unsigned long long cyc;
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(cyc)::"memory");
        if (tid == 0 && ti < 256) {
          unsigned long long* sp = p.stamps + ((size_t)blockIdx.x * 256 + ti) * 4;
          sp[0] = st_prev;
          sp[1] = cyc;  // shader-clock counter at st_e: the clock between two tiles
          sp[2] = st_m;
          sp[3] = st_e;
        }
        st_prev = st_e;
      }
#endif
#pragma unroll
      for (int i = 0; i < SN; ++i)
#pragma unroll
        for (int j = 0; j < SM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    };
    pingpong_tiles<epilogue_stores<Cfg, MODE>(), 0xB>(g_cur < g_lim, nk, wm, issue, read, mma, set_tiles,
                                                         tile_end, more);
    if (dyn && tid == 0) {
      // every pull of this block has returned (the loop ends with vmcnt(0)); the last block
      // to get here re-zeroes the queue for the next launch on this stream
      int* const done = p.tileq + 8 * 32;
      if (__hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1) {
        for (int q = 0; q < 8; ++q) __hip_atomic_store(p.tileq + q * 32, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  } else {
    mfma_pipeline_tiles<Cfg::S, BK / 32, Cfg::XINSTR + Cfg::WINSTR + Cfg::PF, SN, SM,
                        epilogue_stores<Cfg, MODE>(), Cfg::PF>(
        my_tiles, K / BK, acc, stage, frags, [&](int ti) { pre(bp + ti * G); },
        [&](int ti) { epilogue(bp + ti * G); }, p.stamps);
  }
}

static int g_num_cus = 0;
static int g_nt_grid_cap = 0;  // test hook: persistent grid size (0 = one block per CU)
void gemm_nt_set_grid_cap(int cap) { g_nt_grid_cap = cap; }
static int g_nt_stagger = 0;
void gemm_nt_set_stagger(int units) { g_nt_stagger = units; }
static int g_nt_diag = 0;
static int g_nt_pf_dist = 2;
void gemm_nt_set_pf_dist(int d) { g_nt_pf_dist = d; }
void gemm_nt_set_diag(int bits) { g_nt_diag = bits; }
static unsigned long long* g_nt_stamps = nullptr;
static int g_nt_queue = 1;  // 0 off, 1 forward modes, 2 every ping-pong mode
void gemm_nt_set_queue(int v) { g_nt_queue = v; }

// Tile-queue counters: one set per (device, stream), so launches that share a set are ordered
// by their stream.  A set is 8 shard heads and a done counter, 128 B apart, zero between
// launches (statically zero; each launch's last block re-zeroes it).
constexpr int kQueueSets = 16;
__device__ int g_ntq[kQueueSets][kQueueSet];
static int* nt_queue(hipStream_t s) {
  static std::mutex mu;  // host threads that launch concurrently get distinct sets
  std::lock_guard<std::mutex> lock(mu);
  static struct { int dev; hipStream_t s; } used[kQueueSets];
  static int nused = 0;
  static int* base[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!base[dev]) {
    void* b = nullptr;
    if (hipGetSymbolAddress(&b, HIP_SYMBOL(g_ntq)) != hipSuccess) return nullptr;
    base[dev] = (int*)b;
  }
  int k = 0;
  for (; k < nused; ++k)
    if (used[k].dev == dev && used[k].s == s) break;
  if (k == nused) {
    if (nused == kQueueSets) return nullptr;  // more streams than sets: static walk
    used[nused++] = {dev, s};
  }
  int per_dev = 0;  // index of this stream among the device's sets
  for (int j = 0; j < k; ++j) per_dev += used[j].dev == dev;
  return base[dev] + per_dev * kQueueSet;
}
#ifdef SIREN_NT_STAMPS
// diagnostic builds only: [grid][256 tiles][4] u64 device buffer, or null to stop recording
extern "C" void siren_debug_nt_stamps(void* buf) { g_nt_stamps = (unsigned long long*)buf; }
#endif

template <class Cfg, int MODE, bool HEAD>
static hipError_t launch_nt(const NtParams& p_in, hipStream_t s, bool persistent) {
  // the static ping-pong schedule assumes an even number (>= 2) of K-tiles per tile
  if (Cfg::PP && (p_in.K % (2 * Cfg::BK) != 0 || !persistent)) return hipErrorInvalidValue;
  NtParams p = p_in;
  p.stagger = persistent ? g_nt_stagger : 0;
  p.diag = g_nt_diag;
  p.pf_dist = g_nt_pf_dist;
  p.stamps = g_nt_stamps;
  const int ntiles = (p.M / Cfg::BM) * (p.N / Cfg::BN);
  if (g_num_cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        g_num_cus <= 0)
      g_num_cus = 256;
  }
  const int cap = g_nt_grid_cap > 0 ? g_nt_grid_cap : g_num_cus * Cfg::BPC;
  const int grid = persistent ? (ntiles < cap ? ntiles : cap) : ntiles;
  // the queue's shards are blockIdx % 8: every shard must have blocks
  // (measured: the forward gains 3-4%; dX is unchanged and dX0 loses 2%, its K-loop spills)
  const bool want = g_nt_queue == 2 || (g_nt_queue == 1 && nt_is_fwd(MODE));
  p.tileq = (Cfg::PP && want && !p.diag && grid % 8 == 0) ? nt_queue(s) : nullptr;
  if constexpr (Cfg::PP) {
    if (p.tileq) {
      hipLaunchKernelGGL((gemm_nt_kernel<Cfg, MODE, HEAD, true>), dim3(grid), dim3(Cfg::THREADS), 0, s, p);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((gemm_nt_kernel<Cfg, MODE, HEAD>), dim3(grid), dim3(Cfg::THREADS), 0, s, p);
  return hipGetLastError();
}

template <class Cfg>
static hipError_t dispatch_mode(int mode, bool head, const NtParams& p, hipStream_t s, bool persistent) {
  switch (mode) {
    case NT_FWD:
      return head ? launch_nt<Cfg, NT_FWD, true>(p, s, persistent)
                  : launch_nt<Cfg, NT_FWD, false>(p, s, persistent);
    case NT_DX: return launch_nt<Cfg, NT_DX, false>(p, s, persistent);
    case NT_DX0: return launch_nt<Cfg, NT_DX0, false>(p, s, persistent);
  }
  return hipErrorInvalidValue;
}

// first_linear=True: dX into the Linear + Snake first layer (default persistent K-loop / 128 tile)
template <class Cfg>
static hipError_t dispatch_dx0_snake(const NtParams& p, hipStream_t s, bool persistent) {
  return launch_nt<Cfg, NT_DX0_SNAKE, false>(p, s, persistent);
}

// Snake / Tanh layers: the default persistent K-loop (or the 128x128 tile)
template <class Cfg>
static hipError_t dispatch_act(int mode, bool head, const NtParams& p, hipStream_t s, bool persistent) {
  switch (mode) {
    case NT_FWD_SNAKE:
      return head ? launch_nt<Cfg, NT_FWD_SNAKE, true>(p, s, persistent)
                  : launch_nt<Cfg, NT_FWD_SNAKE, false>(p, s, persistent);
    case NT_FWD_TANH:
      return head ? launch_nt<Cfg, NT_FWD_TANH, true>(p, s, persistent)
                  : launch_nt<Cfg, NT_FWD_TANH, false>(p, s, persistent);
    case NT_DX_SNAKE: return launch_nt<Cfg, NT_DX_SNAKE, false>(p, s, persistent);
  }
  return hipErrorInvalidValue;
}

// tile override for A/B measurement: 0 = auto, 128 or 256; pipe (256x256): 0 = BK 64, one
// tile per block; 1 = BK 64 persistent (default); 2 = BK 32 4-slot ring persistent;
// 3 = BK 32 3-slot ring persistent; 4 = BK 64 persistent ping-pong (pingpong_tiles)
static int g_nt_tile = 0;
static int g_nt_pipe = -1;  // -1: automatic = ping-pong 4 for every mode (kernel_bench r06)
// Snake / Tanh / first-layer-Snake modes have two 256x256 variants: ping-pong (auto) and 1
static bool nt_pp() { return g_nt_pipe < 0 || g_nt_pipe == 4; }
void gemm_nt_set_tile(int tile) { g_nt_tile = tile; }
void gemm_nt_set_pipe(int v) { g_nt_pipe = v; }

int nt_choose_tile(int M, int N) {
  const bool large_ok = (M % 256 == 0) && (N % 256 == 0);
  if (g_nt_tile == 128 || !large_ok) return 128;
  if (g_nt_tile == 256) return 256;
  // the 256x256 tile (1 block/CU) needs >= 2 tiles per CU to keep 256 CUs busy
  return (long)(M / 256) * (N / 256) >= 512 ? 256 : 128;
}

hipError_t gemm_nt(int mode, bool head, const NtParams& p, hipStream_t s) {
  if (p.M % NtSmall::BM || p.N % NtSmall::BN || p.K % NtSmall::BK || p.M <= 0 || p.N > NtSmall::MAXN) return hipErrorInvalidValue;
  if (nt_is_dx0(mode) && (p.in_dim < 1 || p.in_dim > 2)) return hipErrorInvalidValue;
  if (mode == NT_DX0_SNAKE) {
    if (!p.Eprev) return hipErrorInvalidValue;
    if (p.tile == 256) {
      if (p.M % 256 || p.N % 256) return hipErrorInvalidValue;
      return nt_pp() ? dispatch_dx0_snake<NtLargePP>(p, s, true) : dispatch_dx0_snake<NtLarge>(p, s, true);
    }
    if (p.tile != 128) return hipErrorInvalidValue;
    return dispatch_dx0_snake<NtSmall>(p, s, false);
  }
  if (mode >= NT_FWD_SNAKE) {
    if ((mode == NT_FWD_SNAKE && (!p.act_a || !p.E)) || (mode == NT_DX_SNAKE && !p.Eprev))
      return hipErrorInvalidValue;
    if (p.tile == 256) {
      if (p.M % 256 || p.N % 256) return hipErrorInvalidValue;
      return nt_pp() ? dispatch_act<NtLargePP>(mode, head, p, s, true) : dispatch_act<NtLarge>(mode, head, p, s, true);
    }
    if (p.tile != 128) return hipErrorInvalidValue;
    return dispatch_act<NtSmall>(mode, head, p, s, false);
  }
  if (p.tile == 256) {
    if (p.M % 256 || p.N % 256) return hipErrorInvalidValue;
    const int pipe = g_nt_pipe >= 0 ? g_nt_pipe : 4;
    switch (pipe) {
      case 0: return dispatch_mode<NtLarge>(mode, head, p, s, false);
      case 2: return dispatch_mode<NtLargeR4>(mode, head, p, s, true);
      case 3: return dispatch_mode<NtLargeR3>(mode, head, p, s, true);
      case 4: return dispatch_mode<NtLargePP>(mode, head, p, s, true);
      case 5: return dispatch_mode<NtLargePF>(mode, head, p, s, true);
      case 6: return dispatch_mode<NtMid3>(mode, head, p, s, true);
      case 7: return dispatch_mode<NtMid2>(mode, head, p, s, true);
      default: return dispatch_mode<NtLarge>(mode, head, p, s, true);
    }
  }
  if (p.tile != 128) return hipErrorInvalidValue;
  return dispatch_mode<NtSmall>(mode, head, p, s, false);
}

}  // namespace siren
