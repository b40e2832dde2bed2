// NT GEMM for the SIREN hidden layers on gfx950 h16 MFMA with fused epilogues.
//
//   acc[m][n] = sum_k X[m][k] * W[n][k]        (X: [M][K] h16, W: [N][K] h16, fp32 acc)
//
// Epilogues (template MODE):
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
// tile boundaries; the default K-loop is the ping-pong of two wave groups one barrier apart
// (gemm_pipeline.h pingpong2_tiles: two 32-MFMA segments per K-step).  A 128x128 / 4-wave config
// (one tile per block) serves
// grids too small for 256x256.  Operands are staged HBM->LDS by LDS-DMA (global_load_lds_dwordx4
// from inline asm), with an XOR swizzle on the SOURCE address so that the ds_read_b128 fragment
// reads are bank-conflict free (cdna_hip_programming.md §5.4 rule 21 / T2).
//
// MFMA operand roles are swapped (A := W rows, B := X rows) so each lane ends up holding 4
// consecutive output COLUMNS of one row (per-row bias loads as one float4); adjacent column
// subtiles are then exchanged across 16-lane groups (swap16_pair) so every epilogue store
// and Cprev load is a 16-B row piece.  The epilogue's store tail is issue-bound (measured:
// 64 scattered dwordx2 per lane cost 1.0 ms of a 2.8 ms forward GEMM), so halving the
// instruction count and keeping the stores behind two prefetched stages is what matters.
//
// Measurement-only ablations (SIREN_OPT_NT_DIAG) exist only in builds with -DSIREN_DIAG
// (__graft_entry__.build_diagnostic); the product kernels carry none.
#include "gemm_pipeline.h"
#include "siren_common.h"
#include "siren_kernels.h"

// rows per Cprev/Eprev batch in the Snake dX epilogues (gemm_nt_kernel): NT_DX_SNAKE, NT_DX0_SNAKE
#ifndef SIREN_SNAKE_EB
#define SIREN_SNAKE_EB 2
#endif
#ifndef SIREN_SNAKE0_EB
#define SIREN_SNAKE0_EB 2
#endif

// ping-pong NT kernels: the two-segment K-step (gemm_pipeline.h pingpong2_tiles, 4 barriers per K-step;
// round 5: forward 2.269 -> 2.201 ms, fused last layer 2.401 -> 2.338, dX0 1.963 -> 1.924, dX 2.168 ->
// 2.156, bit-identical; profiles/r18/ab_seg2.json); 0 = the four-phase K-step (pingpong_tiles)
#ifndef SIREN_NT_SEG2
#define SIREN_NT_SEG2 1
#endif

#ifndef SIREN_NT_EARLY  // gemm_pipeline.h pingpong2_tiles EARLY for every mode (measurement; the fused
#define SIREN_NT_EARLY 0  // last layer and dX0 always take it: dX0 -0.7% cfg2, -5.3% cfg4, dX +0.1% / +2.2%,
#endif                    // profiles/r20/ab_early_dx.json)
// whole-line epilogue stores as non-temporal (global_store ... nt): cfg4 forward -6.0%, dX -1.3%, cfg2
// within 0.2% (profiles/r19/ab_full_lines.json u26); 0 = plain stores
#ifndef SIREN_NT_STNT
#define SIREN_NT_STNT 1
#endif
// lines_out: 0 = each lane's MFMA-layout 8-B halves straight into the line scratch; 1 = paired into 16-B row
// pieces by v_permlane16_swap first (round 5; measurement builds)
#ifndef SIREN_LINES_SWAP
#define SIREN_LINES_SWAP 0
#endif

#ifdef SIREN_DIAG
#define SIREN_DIAG_ON 1
#else
#define SIREN_DIAG_ON 0
#endif

namespace siren {

// Source-side XOR swizzle of a staged [rows][BK] fp16 image (16-B chunks).  BK = 64 (128-B
// rows, 8 chunks): chunk ^ (row & 7).
template <int BK>
__device__ __forceinline__ int stage_swz(int r, int c) {
  static_assert(BK == 64, "128-B staged rows");
  return c ^ (r & 7);
}

template <int BM_, int BN_, int WM_, int WN_, int BK_, int S_, bool PP_ = false>
struct NtCfg {
  static constexpr int BM = BM_, BN = BN_, BK = BK_, S = S_;
  static constexpr bool PP = PP_;  // ping-pong K-loop (gemm_pipeline.h pingpong2_tiles / pingpong_tiles)
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
// 256x256, BK 64 double buffer: one tile per block (SIREN_OPT_NT_PIPE 0) or persistent (1)
using NtLarge = NtCfg<256, 256, 2, 4, 64, 2>;
// the same, persistent, two wave groups in ping-pong (SIREN_OPT_NT_PIPE 4, the default)
using NtLargePP = NtCfg<256, 256, 2, 4, 64, 2, true>;

// LDS layout of one kernel instance: the ring, the epilogue reduction scratch, then only the
// per-column vectors its mode needs (bias for the forward modes, head weights with HEAD, Snake
// a), then the tile-queue slots.
// ACTL: the Snake / Tanh forward (ping-pong, no HEAD) with whole-line stores -- Tanh through the 16-KiB
// scratch, Snake (no 16 KiB left) in 8-row passes through 1 KiB per wave in the RED region.  gemm_nt
// takes it at K <= 512 only: at train()'s default width 256 Snake -19%, Tanh -16%; at 512 -3% / -6%;
// at 1024 +4.5% / +1.3% (profiles/r20/ab_act_lines.json, bit-identical).  The dX into a Snake layer
// (NT_DX_SNAKE) takes the same K <= 512 switch for whole-line dZ stores through the 16-KiB scratch
// (width 256 -1.2%, 512 -7.1%, bit-identical; profiles/r22/ab_dxsl_*.json)
template <class Cfg, int MODE, bool HEAD, bool ACTL = false>
struct NtLds {
  static constexpr int BIAS = Cfg::RING + Cfg::RED;
  static constexpr int HW = BIAS + (nt_is_fwd(MODE) ? Cfg::VEC : 0);
  static constexpr int A = HW + (HEAD ? Cfg::VEC : 0);
  static constexpr int IA = A + (nt_is_snake_fwd(MODE) ? Cfg::VEC : 0);   // Snake 1/a, divided once
  static constexpr int QS = IA + (nt_is_snake_fwd(MODE) ? Cfg::VEC : 0);  // dynamic tile queue: 2 tile ids
  // plain forward and dX, ping-pong config: a 2-KiB scratch per wave that turns the epilogue's 16-row x
  // 64-B store pieces into whole 128-B lines (the 128x128 config keeps two blocks per CU without it)
  // (the fused last layer walks statically: no queue slots, and its sine / Tanh kinds fit the scratch
  // in exactly 160 KiB)
  static constexpr int ST = QS + (nt_is_hb(MODE) ? 0 : 16);
  static constexpr bool LINES = Cfg::PP && (((MODE == NT_FWD || MODE == NT_DX) && !HEAD) ||
                                            MODE == NT_FWD_HB || MODE == NT_FWD_HB_TANH ||
                                            (ACTL && (MODE == NT_FWD_TANH || MODE == NT_DX_SNAKE) && !HEAD));
  // the Snake forward without HEAD: 8-row passes through 1 KiB per wave at Cfg::RING (RED, which only
  // HEAD and the backward modes use)
  static constexpr bool HALF = Cfg::PP && ACTL && MODE == NT_FWD_SNAKE && !HEAD;
  static_assert(!HALF || Cfg::RED >= Cfg::NWAVES * 1024, "half-line scratch");
  static constexpr int DM = ST;  // HALF: 64 lanes x 32 B of write-only slots
  static constexpr int SIZE = ST + (LINES ? Cfg::NWAVES * 2048 : 0) + (HALF ? 64 * 32 : 0);
  static_assert(SIZE <= 160 * 1024, "LDS");
};

// Tile-queue counter set (caller-owned, SIREN_TILEQ_INTS ints): 8 shard heads 128 B apart, then
// 64 scratch words per shard.  The launcher zeroes it on the stream right before every queue
// launch, so no state carries from one launch to the next.
constexpr int kQueueHeads = 8 * 32, kQueueSet = kQueueHeads + 8 * 64;
static_assert(kQueueSet == kTileqInts, "siren_hip.h SIREN_TILEQ_INTS");

// Dynamic tile queue (ping-pong K-loop).  A pull is one returning agent-scope atomic add on the
// block's shard head, issued at the start of a tile's epilogue and consumed after it: hipcc's
// own waitcnt then lets the epilogue's stores stay in flight (vmcnt retires in issue order).
// Wave 0 issues it with every lane active (lane 0 adds 1 to the head, lanes 1..63 add 0 to
// the shard's scratch words, so the head sees one add per pull and the returned VGPR is
// written in every lane).  The pull's VGPR lives only across the epilogue, not across the
// K-loop (no register to spare).  The pull is a compiler-visible atomic, never inline asm: an
// asm pull's VGPR is not known to hipcc to be in flight, so a register copy at a branch join can
// read it before it lands -- a stale tile id that never reaches the shard's limit keeps the
// block walking forever (the round-2 hang).  Every pulled id is range-checked and a
// block walks at most its shard's tile count, so no id can keep a block walking.

constexpr bool nt_is_dx0(int m) { return m == NT_DX0 || m == NT_DX0_SNAKE; }

// tanh for the fp16-stored Tanh epilogues (NT_FWD_TANH, NT_FWD_HB_TANH), branch-free on the hardware
// exp2 / rcp: sign(x) (1 - e) / (1 + e) with e = exp(-2|x|) (a few fp32 ulp), and the odd Taylor
// polynomial below |x| < 1/16 where 1 - e would cancel.  Its x^7 term is below fp32 resolution
// there (2e-9 relative), so it stops at x^5: max relative error 8.7e-8, the fp32 rounding floor,
// with fp16 outputs equal to the degree-7 form's on 200 k points of [0, 1/16].  ocml's tanhf
// is branchy and its temporaries made the fused Tanh head spill 184 B per lane; the outputs are
// stored in fp16 (2^-11), where the two agree to within the parity tests' fp16 bounds.
__device__ __forceinline__ float tanh_epi(float x) {
  const float ax = __builtin_fabsf(x);
  const float e = __builtin_amdgcn_exp2f(ax * -2.8853900817779268f);  // exp(-2|x|) = 2^(-2|x| / ln 2)
  const float big = (1.0f - e) * __builtin_amdgcn_rcpf(1.0f + e);
  const float x2 = ax * ax;
  const float small = ax * (1.0f + x2 * (-0.33333333f + x2 * 0.13333334f));
  return __builtin_copysignf(ax < 0.0625f ? small : big, x);
}

// NT_FWD_HB: head_part word not yet published by its column tile's block (launch_nt fills it)
constexpr unsigned kHeadPending = 0xFFFFFFFFu;
// polls before a hand-off wait gives up: a poll (an agent-scope load and s_sleep 1) takes 0.16 us
// (measured, tools/handoff_timeout.py: 5.4 s at 2^25 polls, profiles/r22/handoff_timeout.json), so
// 2^23 polls are ~1.3 s, against a partner that normally publishes within one tile period (~40 us).
// A wait that gives up is counted in the range guard's stall word (NtParams::stall ->
// GuardState::stalls), which voids the step: the update kernels skip it and the engine raises
// (include/siren_hip.h siren_guard); every other wait of the step then stops within kStallCheck polls
constexpr int kHeadSpinLimit = 1 << 23;
// a waiting thread re-reads the stall word every kStallCheck polls (power of two)
constexpr int kStallCheck = 256;

// store instructions every wave's epilogue issues (lower bound; see mfma_pipeline_tiles)
template <class Cfg, int MODE>
constexpr int epilogue_stores() {
  return (MODE == NT_FWD || MODE == NT_FWD_TANH) ? Cfg::SM * Cfg::SN
         : MODE == NT_FWD_SNAKE                 ? 3 * Cfg::SM * Cfg::SN / 2
         : (MODE == NT_DX || MODE == NT_DX_SNAKE || nt_is_hb(MODE)) ? Cfg::SM * Cfg::SN / 2
                                                  : 0;
}

// QUEUE (ping-pong K-loop only): tiles from the dynamic queue p.tileq instead of the static walk
template <class Cfg, int MODE, bool HEAD, bool QUEUE = false, bool ACTL = false>
__global__ __launch_bounds__(Cfg::THREADS, 2) void gemm_nt_kernel(NtParams p) {
  constexpr int BM = Cfg::BM, BN = Cfg::BN, BK = Cfg::BK, WN = Cfg::WN;
  constexpr int TM = Cfg::TM, TN = Cfg::TN, SM = Cfg::SM, SN = Cfg::SN;
  using Lay = NtLds<Cfg, MODE, HEAD, ACTL>;
  __shared__ __attribute__((aligned(16))) char smem[Lay::SIZE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  // N: this launch's columns (a window of at most MAXN of a wider layer: gemm_nt); LD: the row stride
  // of every [M][*] operand and output (the layer's full width; the host offsets the pointers)
  const int K = p.K, N = p.N, LD = p.ld;
  const int tiles_n = N / BN;
  const int ntiles = (p.M / BM) * tiles_n;
  const bool tn_pow2 = (tiles_n & (tiles_n - 1)) == 0;  // N / BN is 1, 2, 4 or 8 at H <= 1024
  const int tn_shift = __builtin_ctz(tiles_n);
  // Block b takes tiles b', b'+G, ... with b' the XCD-grouped id: the G/8 blocks of one XCD
  // hold consecutive tile ids, i.e. they share X row-blocks in L2 at the same time.
  const int G = gridDim.x;
  const int bp = xcd_remap(blockIdx.x, G);
  // measurement-only ablation bits (SIREN_DIAG builds; the queue kernel is launched with none):
  // 1 X from the first 4 row bands (L2-resident X), 4 W from column tile 0, 8 X from the first 256
  // row bands (128 MB: beyond L2, inside the Infinity Cache), 512 no tiles, 1024 no epilogue
  const int diag = (SIREN_DIAG_ON && !(Cfg::PP && QUEUE)) ? p.diag : 0;
  const int my_tiles = (diag & 512) ? 0 : (ntiles - bp + G - 1) / G;
  // Dynamic tile queue (ping-pong K-loop, NtParams::tileq).  With the static walk the four
  // blocks that share a row band of X drift apart over the launch and X is fetched ~1.6x from
  // HBM.  Instead the blocks of one shard (blockIdx % 8: one XCD under round-robin
  // dispatch -- speed only, any placement is correct) pull the tiles of their contiguous
  // eighth of the grid in order, so the blocks holding one row band are the ones that started
  // it at the same time.
  constexpr bool dyn = Cfg::PP && QUEUE;
  static_assert(!(dyn && nt_is_hb(MODE)), "the fused last layer walks statically (no queue slots in LDS)");
  // global tile id g -> origin; the static walk's i-th tile of this block is g = bp + i * G
  auto tile_of = [&](int g, int& m0, int& n0) {
    const int tm = tn_pow2 ? (g >> tn_shift) : g / tiles_n;
    m0 = tm * BM;
    n0 = (g - tm * tiles_n) * BN;
  };
  auto xrow = [&](int m0) { return (diag & 1) ? (m0 & (4 * BM - 1)) : (diag & 8) ? (m0 & (256 * BM - 1)) : m0; };

  // ---- LDS-DMA staging addresses (non-ping-pong K-loops) ------------------------------
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
    const h16* xk = p.X + (size_t)xrow(m0) * K + kt * BK;
    const h16* wk = p.W + (size_t)n0 * K + kt * BK;
#pragma unroll
    for (int j = 0; j < Cfg::XINSTR; ++j) glds16_asm(xk + xrel[j], lds_addr(xs + j * 1024));
#pragma unroll
    for (int j = 0; j < Cfg::WINSTR; ++j) glds16_asm(wk + wrel[j], lds_addr(ws + j * 1024));
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
  auto st16 = [&](h16* dst, uint4 v) { *(uint4*)dst = v; };
  // the whole-line stores (plain forward, dX): non-temporal (SIREN_NT_STNT)
  auto stl = [&](h16* dst, uint4 v) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    if constexpr (SIREN_NT_STNT != 0) __builtin_nontemporal_store(__builtin_bit_cast(u32x4, v), (u32x4*)dst);
    else *(uint4*)dst = v;
  };
  // Whole 128-B lines per store (Lay::LINES): the wave's 16-row x 64-column fp16 piece of one
  // output (lane: row lane & 15, 16-B chunks 4 pp + swap16_col(lane) / 8) goes through its 2-KiB LDS
  // scratch, 16-B chunks XOR-swizzled by row (conflict-free both ways), and each store writes rows
  // 8q .. 8q+7 as 8 lanes x 16 B per row.  Same bytes and store count as 16 rows x 64 B, but no
  // half-line writes.  Same-wave LDS accesses complete in order, so the reads see this
  // wave's writes and the next output's writes follow the reads.  row = the piece's first row and
  // col = the wave's first column, both wave-uniform: each store is then a wave-uniform 64-bit base in
  // SGPRs plus a 32-bit lane offset that is the same for every piece (the saddr form), where per-lane
  // 64-bit addresses cost 10 64-bit VALU per row piece (v_mad_i64_i32, v_lshl_add_u64; gfx950 listing)
  // v[i]: this lane's 4 columns of column subtile i in the MFMA layout (row lane & 15, columns 16 i + 4 g ..
  // + 3, g = lane >> 4), packed fp16: 8 B at byte 32 i + 8 g of the row's line.  Each goes into the scratch as
  // one 8-B half of its swizzled 16-B chunk 2 i + (g >> 1) (SIREN_LINES_SWAP 1: first paired into 16-B row
  // pieces across 16-lane groups by v_permlane16_swap, as round 5 did -- 4 VALU per row piece more)
  // lines_out in two halves (the non-HALF path): lines_get exchanges one row piece through the wave's
  // scratch into this lane's two 16-B line chunks, lines_put stores them.  The plain forward runs them
  // a row apart, so a row's LDS round trip completes under the next row's sin / cos
  auto lines_get = [&](const uint2 (&v)[Cfg::SN], uint4 (&line)[2]) {
    static_assert(Cfg::SN == 4, "a wave's row piece is one 128-B line");
    const int pr = lane & 15, pc = swap16_col(lane) >> 3;
    const int g = lane >> 4;
    const int qr = lane >> 3, qc = lane & 7;
    char* sc = smem + Lay::ST + wave * 2048;
    if constexpr (SIREN_LINES_SWAP != 0) {
#pragma unroll
      for (int pp = 0; pp < Cfg::SN / 2; ++pp) {
        const int c = pp * 4 + pc;
        *(uint4*)(sc + pr * 128 + ((c ^ (pr & 7)) << 4)) = swap16_pair(v[2 * pp], v[2 * pp + 1]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < Cfg::SN; ++i) {
        const int c = 2 * i + (g >> 1);
        *(uint2*)(sc + pr * 128 + ((c ^ (pr & 7)) << 4) + ((g & 1) << 3)) = v[i];
      }
    }
    __builtin_amdgcn_wave_barrier();  // cross-lane exchange: the reads stay after every lane's writes
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int r = qr + 8 * q;
      line[q] = *(const uint4*)(sc + r * 128 + ((qc ^ (r & 7)) << 4));
    }
    __builtin_amdgcn_wave_barrier();  // ... and the next output's writes after these reads
  };
  auto lines_put = [&](h16* out, int row, int col, const uint4 (&line)[2]) {
    const int qr = lane >> 3, qc = lane & 7;
    const char* ub = (const char*)(out + (size_t)row * LD + col);
    unsigned lo = (unsigned)((qr * LD + qc * 8) * 2);
    asm("" : "+v"(lo));  // kept 32-bit at the stores (a hoisted 64-bit zext defeats the saddr form)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      unsigned lq = lo;
      asm("" : "+v"(lq));  // one opaque copy per store: no store's address is derived from another's
      stl((h16*)(ub + (size_t)(16 * q) * LD + lq), line[q]);
    }
  };
  auto lines_out = [&](h16* out, int row, int col, const uint2 (&v)[Cfg::SN]) {
    static_assert(Cfg::SN == 4, "a wave's row piece is one 128-B line");
    const int pr = lane & 15, pc = swap16_col(lane) >> 3;  // this lane's piece: row, 16-B chunk
    const int g = lane >> 4;                                // MFMA layout: 16-lane group
    const int qr = lane >> 3, qc = lane & 7;                // line layout: row (+ 8 q), chunk
    uint4 vs[SIREN_LINES_SWAP ? Cfg::SN / 2 : 1];
    if constexpr (SIREN_LINES_SWAP != 0) {
#pragma unroll
      for (int pp = 0; pp < Cfg::SN / 2; ++pp) vs[pp] = swap16_pair(v[2 * pp], v[2 * pp + 1]);
    }
    const char* ub = (const char*)(out + (size_t)row * LD + col);
    unsigned lo = (unsigned)((qr * LD + qc * 8) * 2);
    asm("" : "+v"(lo));  // kept 32-bit at the stores (a hoisted 64-bit zext defeats the saddr form)
    if constexpr (Lay::HALF) {
      // rows 8h .. 8h+7 per pass.  No lane may skip a pass's write: the compiler treats the scratch
      // per lane, and a write under a divergent branch was moved past the other lanes' reads (wrong
      // rows, gfx950 listing; a DPP exchange that avoids it spilled).  So every lane writes both its
      // chunks in both passes, those of the other pass's rows to slots nobody reads (Lay::DM,
      // shared by the block's waves: garbage by design).
      char* sh = smem + Cfg::RING + wave * 1024;
      char* dm = smem + Lay::DM + lane * 32;
      const int r8 = pr & 7;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bool mine = (pr >> 3) == h;
        if constexpr (SIREN_LINES_SWAP != 0) {
#pragma unroll
          for (int pp = 0; pp < Cfg::SN / 2; ++pp) {
            const int c = pp * 4 + pc;
            *(uint4*)(mine ? sh + r8 * 128 + ((c ^ r8) << 4) : dm + pp * 16) = vs[pp];
          }
        } else {
#pragma unroll
          for (int i = 0; i < Cfg::SN; ++i) {
            const int c = 2 * i + (g >> 1);
            *(uint2*)(mine ? sh + r8 * 128 + ((c ^ r8) << 4) + ((g & 1) << 3) : dm + i * 8) = v[i];
          }
        }
        // the exchange is across lanes: no LDS access moves over these (LDS is in order within a
        // wave, so they cost no wait; the ordering no longer rests on how the select is written)
        __builtin_amdgcn_wave_barrier();
        const uint4 line = *(const uint4*)(sh + qr * 128 + ((qc ^ qr) << 4));
        __builtin_amdgcn_wave_barrier();
        unsigned lh = lo;
        asm("" : "+v"(lh));  // one opaque copy per store: no store's address is derived from another's
        stl((h16*)(ub + (size_t)(16 * h) * LD + lh), line);
      }
      return;
    }
    uint4 line[2];
    lines_get(v, line);
    lines_put(out, row, col, line);
  };
  // NT_FWD: bias / head weights through LDS -- the epilogue then issues no global load
  // whose compiler-counted vmcnt wait would also cover the asm-issued stage prefetch.
  float* bias_lds = (float*)(smem + Lay::BIAS);
  float* hw_lds = (float*)(smem + Lay::HW);
  float* a_lds = (float*)(smem + Lay::A);    // Snake: a
  float* ia_lds = (float*)(smem + Lay::IA);  // Snake: 1/a (the same IEEE quotient the epilogue used per element)
  if constexpr (nt_is_fwd(MODE)) {
    // the sine modes' bias in revolutions, b * omega / (2 pi), once per block (the same fp32 product the
    // epilogues formed per tile); 1 for Snake / Tanh
    const float xb = (MODE == NT_FWD || MODE == NT_FWD_HB) ? p.omega * kInv2Pi : 1.0f;
    for (int c = tid * 4; c < N; c += Cfg::THREADS * 4) {
      const float4 b4 = *(const float4*)(p.bias + c);
      *(float4*)(bias_lds + c) = float4{b4.x * xb, b4.y * xb, b4.z * xb, b4.w * xb};
      if constexpr (HEAD) *(float4*)(hw_lds + c) = *(const float4*)(p.head_w + c);
      if constexpr (nt_is_snake_fwd(MODE)) {
        const float4 a4 = *(const float4*)(p.act_a + c);
        *(float4*)(a_lds + c) = a4;
        *(float4*)(ia_lds + c) = float4{1.0f / a4.x, 1.0f / a4.y, 1.0f / a4.z, 1.0f / a4.w};
      }
    }
    // visible to other waves after the pipeline's first barrier
  }
  // dZ carries the backward storage scale S; the fp32 column partials leave unscaled
  const float inv_scale = (!nt_is_fwd(MODE) && p.gscale) ? p.gscale[1] : 1.0f;
  // the fused last layer's S, 1/S and head bias, loaded once here: loaded in the epilogue, each
  // tile's phase 2 waited at vmcnt(0) for them, i.e. for the next tile's stages issued before it
  float hb_scale[2] = {1.0f, 1.0f}, hb_bias = 0.0f;
  if constexpr (nt_is_hb(MODE)) {
    hb_scale[0] = p.gscale[0];
    hb_scale[1] = p.gscale[1];
    hb_bias = p.b_head[0];
    // in VGPRs (3 of the 20 free): as SGPRs they pushed 12 more SGPR spills into VGPR lanes
    asm volatile("" : "+v"(hb_scale[0]), "+v"(hb_scale[1]), "+v"(hb_bias));
  }
  // NT_DX / NT_DX0 epilogue operands loaded by `pre` (before the next tile's early prefetch).  The
  // rest are loaded by the epilogue in one batch once earlier pieces are consumed (their
  // accumulators free the registers), so a batch waits once, not once per piece behind the
  // in-order vmcnt (which also covers the next tile's stages and this tile's stores).  NT_DX and
  // NT_DX0 preload every row (NT_DX0 has room for it since its products use v_fma_mix and its
  // row sums v_add_f32_dpp: 229 VGPRs, against 235 with half the rows before).  The Snake modes
  // (Cprev AND Eprev per piece) go in batches of EB rows with both column pairs of a row
  // together: `pre` loads pair 0 of the first batch, and each batch loads the next one before
  // its own dZ stores.
  constexpr bool HAS_E = (MODE == NT_DX_SNAKE || MODE == NT_DX0_SNAKE);
  constexpr int PRE_J = (nt_is_fwd(MODE) || HAS_E) ? 0 : SM;
  // Snake modes: EB = 2 rows per batch, two batches in flight (gfx950 listing: 238 / 247 VGPRs
  // for NT_DX_SNAKE / NT_DX0_SNAKE, no spills; 4 rows spill 164-196 B): dX Snake 2.559 -> 2.530 ms
  // against 4-row batches loaded at use (profiles/r16c/ab_snake_dx_pipelined.json)
  constexpr int EB0 = (MODE == NT_DX0_SNAKE) ? SIREN_SNAKE0_EB : SIREN_SNAKE_EB;
  constexpr int EB = EB0 < SM ? EB0 : SM;
  static_assert(SM % EB == 0, "Snake epilogue batches");
  // Row-piece accesses of the epilogues: a wave-uniform row base (SGPRs) plus a 32-bit lane byte offset kept
  // 32-bit at the access by an opaque copy, so that hipcc emits the saddr form (one SGPR pair, one VGPR)
  // instead of per-lane 64-bit address arithmetic (v_mad_i64_i32, v_lshl_add_u64: lines_out)
  auto at_lane = [](const void* ub, unsigned lo) -> char* {
    asm("" : "+v"(lo));
    return (char*)ub + lo;
  };
  // this lane's 16-B piece of a row piece (row lane & 15, columns swap16_col(lane) ..): byte offset in [*][LD] fp16
  const unsigned lane_piece = (unsigned)(((lane & 15) * LD + swap16_col(lane)) * 2);
  auto rowp = [&](const h16* base, int row_u, int col_u) { return (const char*)(base + (size_t)row_u * LD + col_u); };
  uint4 cp_in[PRE_J > 0 ? PRE_J : 1][SN / 2];
  uint4 ce_in[HAS_E ? EB : 1][2];
  float t_in[SM][2];
  auto pre = [&](int g) {
    int m0, n0;
    tile_of(g, m0, n0);
    const int mrowu = m0 + wm * TM, ncu = n0 + wn * TN;  // the wave's first row and column (wave-uniform)
    if constexpr (!nt_is_fwd(MODE)) {
#pragma unroll
      for (int j = 0; j < PRE_J; ++j)
#pragma unroll
        for (int pp = 0; pp < SN / 2; ++pp)
          cp_in[j][pp] = *(const uint4*)at_lane(rowp(p.Cprev, mrowu + j * 16, ncu), lane_piece + pp * 64);
      if constexpr (HAS_E) {
#pragma unroll
        for (int j = 0; j < EB; ++j) {
          ce_in[j][0] = *(const uint4*)at_lane(rowp(p.Cprev, mrowu + j * 16, ncu), lane_piece);
          ce_in[j][1] = *(const uint4*)at_lane(rowp(p.Eprev, mrowu + j * 16, ncu), lane_piece);
        }
      }
      if constexpr (nt_is_dx0(MODE)) {
#pragma unroll
        for (int j = 0; j < SM; ++j) {
          const float* tb = p.t + (size_t)(mrowu + j * 16) * p.in_dim;
          const unsigned lt = (unsigned)((lane & 15) * p.in_dim * 4);
          t_in[j][0] = *(const float*)at_lane(tb, lt);
          t_in[j][1] = (p.in_dim > 1) ? *(const float*)at_lane(tb, lt + 4) : 0.f;
        }
      }
    }
  };
  auto epilogue = [&](int g) {
    int m0, n0;
    tile_of(g, m0, n0);
    const int tm = m0 / BM, tn = n0 / BN;
    const int npc = n0 + wn * TN + swap16_col(lane);      // swapped layout: this lane's piece
    const int mrowu = m0 + wm * TM;                       // the wave's first row (wave-uniform)
    const int mrow0 = mrowu + (lane & 15);

    if constexpr (nt_is_hb(MODE)) {
      // The last hidden layer fused with the head, the loss gradient and the head backward, for
      // the three last-layer kinds (models.py:114-115, 235-241, 366-372).
      // ---- phase 1: the layer's outputs for the head partial of the band's rows over this column
      // tile, summed exactly as NT_FWD(_SNAKE/_TANH) + HEAD sums them.  Sine / Tanh: Y and C (= cos,
      // or 1 - Y^2) rounded to fp16 as the unfused forward stores them, packed IN PLACE of their
      // accumulators (4 fp32 -> 4 + 4 fp16: the same 4 VGPRs, so nothing more is live across the
      // hand-off than the accumulators).  Snake has three fp16 outputs (Y, D, E): Y and D go in
      // place of the accumulators, E to the layer's E buffer, read back during phase 2.
      constexpr bool SNK = MODE == NT_FWD_HB_SNAKE, TNH = MODE == NT_FWD_HB_TANH;
      const int nq = n0 + wn * TN + 4 * (lane >> 4);
      const float xs = (MODE == NT_FWD_HB) ? p.omega * kInv2Pi : 1.0f;
      float4 bias[SN], hw[SN];  // (bias_lds holds b * xs)
#pragma unroll
      for (int i = 0; i < SN; ++i) {
        bias[i] = *(const float4*)(bias_lds + nq + i * 16);
        hw[i] = *(const float4*)(hw_lds + nq + i * 16);
      }
      float hp[SM];
      uint2 epair[2];  // Snake: fp16 E of one row piece's two column subtiles
#pragma unroll
      for (int j = 0; j < SM; ++j) {
        hp[j] = 0.f;
#pragma unroll
        for (int q = 0; q < SN / 2; ++q) {
          const int pp = (Cfg::PP && j >= SM / 2) ? SN / 2 - 1 - q : q;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int i = 2 * pp + h;
            const float bb[4] = {bias[i].x, bias[i].y, bias[i].z, bias[i].w};
            float sv[4];
            if constexpr (SNK) {
              const float4 a4 = *(const float4*)(a_lds + nq + i * 16);
              const float4 ia4 = *(const float4*)(ia_lds + nq + i * 16);
              const float av[4] = {a4.x, a4.y, a4.z, a4.w}, iav[4] = {ia4.x, ia4.y, ia4.z, ia4.w};
              float cv[4], ev[4];
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                snake_epi(acc[i][j][r] + bb[r], av[r], iav[r], sv[r], cv[r], ev[r]);
              }
              // Y and D packed in place of the accumulators; E goes to HBM (p.E, the layer's E
              // buffer) in 16-B row pieces once both subtiles of the pair have it, and phase 3 reads
              // it back (held in registers, 64 more VGPRs across the hand-off spilled 400 B per lane)
              const uint2 yv = as_u2(pack4(sv[0], sv[1], sv[2], sv[3])), cw = as_u2(pack4(cv[0], cv[1], cv[2], cv[3]));
              acc[i][j] = __builtin_bit_cast(f32x4, uint4{yv.x, yv.y, cw.x, cw.y});
              epair[h] = as_u2(pack4(ev[0], ev[1], ev[2], ev[3]));
              asm volatile("" : "+v"(acc[i][j]));
            } else {
              float cv[4], xa[4];
              if constexpr (!TNH) fma4_pk(acc[i][j], xs, bias[i], xa);  // as the plain forward
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                if constexpr (TNH) {
                  const float y = tanh_epi(acc[i][j][r] + bb[r]);
                  sv[r] = y;
                  cv[r] = 1.0f - y * y;
                } else {
                  const float x = __builtin_amdgcn_fractf(xa[r]);
                  sv[r] = __builtin_amdgcn_sinf(x);
                  cv[r] = __builtin_amdgcn_cosf(x);
                }
              }
              const uint2 yv = as_u2(pack4(sv[0], sv[1], sv[2], sv[3])), cw = as_u2(pack4(cv[0], cv[1], cv[2], cv[3]));
              acc[i][j] = __builtin_bit_cast(f32x4, uint4{yv.x, yv.y, cw.x, cw.y});
              // opaque: the packing happens here (left to itself the compiler sinks the cos past the
              // hand-off into phase 2, keeping the fp32 arguments live across it: 372 B of spills)
              asm volatile("" : "+v"(acc[i][j]));
            }
            hp[j] += dot4_pk(sv, hw[i]);
          }
          if constexpr (SNK)
            st16((h16*)at_lane(rowp(p.E, mrowu + j * 16, n0 + wn * TN), lane_piece + pp * 64), swap16_pair(epair[0], epair[1]));
        }
      }
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
      // ---- the band hand-off: publish this column tile's partial of each row, take the other
      // column tiles' partials as their blocks publish them (the band's tiles_n tiles run in
      // lockstep on tiles_n consecutive blocks of one XCD; DESIGN §4 "fused head backward"), then
      // head_loss for the band's rows.  The partial itself is the flag: head_part is filled with
      // kHeadPending before the launch and a published value is never that pattern (NaN is
      // stored canonical), so no fence orders it -- one agent-scope atomic word each way.
      // g_lds sits past the column-partial scratch of phase 2 (3 partial rows with Snake)
      float* g_lds = red + (SNK ? 3 * Cfg::WM * BN : WN * BM);
      float e2 = 0.f, gv = 0.f;
      if (tid < BM) {
        float own = 0.f;
#pragma unroll
        for (int w = 0; w < WN; ++w) own += red[w * BM + tid];
        const int m = m0 + tid;
        unsigned* hpu = (unsigned*)p.head_part;
        // SIREN_OPT_HB_FAULT bit 0 (SIREN_DIAG builds): column tile 1 never publishes (test hook)
        if (!(SIREN_DIAG_ON && (p.hb_fault & 1) && tn == 1))
          __hip_atomic_store(hpu + (size_t)tn * p.M + m, own == own ? __float_as_uint(own) : 0x7fc00000u,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // the row's target, loaded before the partners are polled: its latency runs under the polls (loaded
        // after them, the block waited one more memory round trip per tile)
        // (unconditional, the row clamped into [0, n_valid), and retired unconditionally below: a load or a use
        // under `m < n_valid` left the register's reuse in phase 2 behind a vmcnt(0), i.e. behind the dZ_L stores)
        // (the empty asm keeps hipcc from hoisting the now always-valid load above `tid < BM`, into the waves
        // that never consume it)
        asm volatile("" ::: "memory");
        const float tgt = p.target[min(m, p.n_valid > 0 ? p.n_valid - 1 : 0)];
        float o = 0.f;  // head_loss_kernel's order: partials j = 0, 1, ..., then the bias
        for (int jt = 0; jt < tiles_n; ++jt) {
          float v = own;
          if (jt != tn) {
            unsigned u;
            int polls = 0;
            while ((u = __hip_atomic_load(hpu + (size_t)jt * p.M + m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) ==
                   kHeadPending) {
              // bounded: a partner kept off the chip (CUs held by another process) voids the step
              // instead of hanging the launch -- the band's partial becomes NaN and the wait is
              // counted in the guard's stall word, which makes the update skip the step and the
              // engine raise (a NaN alone would pass guard_skip and reach the weights)
              if (++polls > p.spin_limit) {
                u = 0x7fc00000u;
                if (p.stall) __hip_atomic_fetch_add(p.stall, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
              }
              // fail fast: once any wait of this step (this launch or an earlier micro-batch's) has given
              // up, the step is void already -- every other wait stops within kStallCheck polls instead
              // of spending its own whole limit (the stall word is sticky until the host clears it)
              if ((polls & (kStallCheck - 1)) == 0 && p.stall &&
                  __hip_atomic_load(p.stall, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
                u = 0x7fc00000u;
                break;
              }
              __builtin_amdgcn_s_sleep(1);
            }
            v = __uint_as_float(u);
          }
          o += v;
        }
        o += hb_bias;
        const float a = p.head_omega * o;
        const float ov = p.head_omega > 0.f ? sinf(a) : o;
        asm volatile("" ::"v"(tgt));  // consumed here on every path (the use below is under m < n_valid)
        if (m < p.n_valid) {
          const float err = ov - tgt;
          if (p.loss_mode == 1) {
            e2 = fabsf(err);
            gv = (err > 0.f ? 1.0f : (err < 0.f ? -1.0f : 0.f)) * p.gfac;
          } else {
            e2 = err * err;
            gv = err * p.gfac;
          }
          if (p.head_omega > 0.f) gv = (gv * cosf(a)) * p.head_omega;
        }
        g_lds[tid] = gv;
        if (tn == 0) {
          p.out[m] = ov;
          p.g[m] = gv;
        }
      }
      // the band's loss and bias-gradient partials (head_loss_kernel's 256-row blocks and sums;
      // threads >= BM add zeros); the block sums' barriers also publish g_lds.  max|g| of the band
      // (head_loss_kernel's gmax partial): the next launch's backward scale for a Snake last layer
      float se = e2, gs = gv, gx = fabsf(gv);
      block_sum2_max(se, gs, gx, g_lds + BM);
      if (tn == 0 && tid == 0) {
        p.sse_part[tm] = se;
        p.gsum_part[tm] = gs;
        if (p.gmax_part) p.gmax_part[tm] = gx;
      }
      // ---- phase 2: head_bwd_kernel on the registers: dz = ((g w) C) omega stored x S (omega 1 for
      // Snake / Tanh: C is their derivative), column partials of dz (db_L) and of g Y (dw_head) over
      // the tile's rows
      constexpr int NQ = 2;  // db_L, dw_head here; a Snake's da_L in phase 3
      // g x S per row: S is a power of two, so ((g S) w) C = ((g w) C) S exactly and the stored dz x S
      // needs no multiply of its own; the column partials sum dz S, g S Y (and g S w E) and leave
      // multiplied by 1/S -- power-of-two scalings commute with every rounding, so dZ_L and the
      // partials are bit for bit those of the unscaled order (head_bwd_kernel's ((g w) C) omega)
      const float om = (MODE == NT_FWD_HB) ? p.omega : 1.0f, S = hb_scale[0], invS = hb_scale[1];
      float gm[SM];
#pragma unroll
      for (int j = 0; j < SM; ++j) gm[j] = g_lds[wm * TM + j * 16 + (lane & 15)] * S;
      // rows outermost, both column pairs of a row piece back to back: each 128-B row segment of
      // dZ_L is then written whole by two consecutive stores (column pairs outermost wrote each
      // line's halves a pass apart: the HBM writes came to 2.63 GB for the 2.15 GB of dZ_L, PMC)
      float cs[SN / 2][NQ][2][4];  // [column pair][db_L, dw_head][subtile h][column r]
#pragma unroll
      for (int pp = 0; pp < SN / 2; ++pp)
#pragma unroll
        for (int q = 0; q < NQ; ++q)
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int r = 0; r < 4; ++r) cs[pp][q][h][r] = 0.f;
      // Snake: row j's E pieces are loaded as phase 2 reaches row j, ahead of its dZ_L stores (the
      // registers of row j's accumulators free up as it goes); phase 3 reads them from registers
      uint4 eall[SNK ? SM : 1][SNK ? SN / 2 : 1];
      uint4 ldz[2];  // row j-1's dZ_L line chunks
#pragma unroll
      for (int j = 0; j < SM; ++j) {
        if constexpr (SNK) {
#pragma unroll
          for (int pp = 0; pp < SN / 2; ++pp)
            eall[j][pp] = *(const uint4*)at_lane(rowp(p.E, mrowu + j * 16, n0 + wn * TN), lane_piece + pp * 64);
        }
        uint2 dzq[SN];  // whole-line stores (Lay::LINES): this row piece's MFMA-layout halves
#pragma unroll
        for (int pp = 0; pp < SN / 2; ++pp) {
          uint2 dzp[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int i = 2 * pp + h;
            // the sine kind keeps phase 1's head weights in registers (same 239 VGPRs); the Snake / Tanh
            // kinds re-read them from LDS per row (in registers they reach 255-256 VGPRs and spill)
            const float4 w4 = (MODE == NT_FWD_HB) ? hw[i] : *(const float4*)(hw_lds + nq + i * 16);
            const uint4 pk = __builtin_bit_cast(uint4, acc[i][j]);
            const uint2 yh = uint2{pk.x, pk.y}, ch = uint2{pk.z, pk.w};
            // head_bwd_kernel's dz, ((g w) C) omega (bit-identical), times S (gm carries it; omega
            // is exactly 1 for a Snake / Tanh layer).  The fp32 x fp32 products and the db_L sums go
            // in pairs (v_pk_mul_f32 / v_pk_add_f32: per element the same rounding as the scalar
            // instruction); the products by an fp16 operand stay v_fma_mix_f32 (no packed form)
            const f32x2 gw01 = f32x2{gm[j], gm[j]} * f32x2{w4.x, w4.y};
            const f32x2 gw23 = f32x2{gm[j], gm[j]} * f32x2{w4.z, w4.w};
            f32x2 d01 = f32x2{mul_mix<0>(gw01.x, ch), mul_mix<1>(gw01.y, ch)};
            f32x2 d23 = f32x2{mul_mix<2>(gw23.x, ch), mul_mix<3>(gw23.y, ch)};
            if constexpr (MODE == NT_FWD_HB) {
              d01 *= f32x2{om, om};
              d23 *= f32x2{om, om};
              asm volatile("" : "+v"(d01), "+v"(d23));  // rounded to fp32 before the fp16 store (fp32_first)
            }
            const f32x2 c01 = f32x2{cs[pp][0][h][0], cs[pp][0][h][1]} + d01;
            const f32x2 c23 = f32x2{cs[pp][0][h][2], cs[pp][0][h][3]} + d23;
            cs[pp][0][h][0] = c01.x; cs[pp][0][h][1] = c01.y; cs[pp][0][h][2] = c23.x; cs[pp][0][h][3] = c23.y;
            static_for<0, 4>([&](auto rc) {
              constexpr int r = decltype(rc)::value;
              cs[pp][1][h][r] = fma_mix<r>(gm[j], yh, cs[pp][1][h][r]);
            });
            dzp[h] = as_u2(pack4(d01.x, d01.y, d23.x, d23.y));
          }
          if constexpr (Lay::LINES) {
            dzq[2 * pp] = dzp[0];
            dzq[2 * pp + 1] = dzp[1];
          }
          else st16((h16*)at_lane(rowp(p.dZ, mrowu + j * 16, n0 + wn * TN), lane_piece + pp * 64), swap16_pair(dzp[0], dzp[1]));
        }
        if constexpr (Lay::LINES) {
          // a row apart, as the forward: row j-1's dZ_L stores after row j's arithmetic
          if (j > 0) lines_put(p.dZ, mrowu + (j - 1) * 16, n0 + wn * TN, ldz);
          lines_get(dzq, ldz);
          if (j == SM - 1) lines_put(p.dZ, mrowu + j * 16, n0 + wn * TN, ldz);
        }
      }
#pragma unroll
      for (int pp = 0; pp < SN / 2; ++pp)
#pragma unroll
        for (int q = 0; q < NQ; ++q)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = cs[pp][q][h][r];
            row16_sum4(v);
            if ((lane & 15) == 0)
              *(float4*)(red + (q * Cfg::WM + wm) * BN + wn * TN + (2 * pp + h) * 16 + 4 * (lane >> 4)) =
                  float4{v[0], v[1], v[2], v[3]};
          }
      if constexpr (SNK) {
        // ---- phase 3 (Snake): da_L partials, sum over the tile's rows of (g w) E, with E read back
        // from where phase 1 stored it (L2: written a hand-off earlier) during phase 2
#pragma unroll
        for (int pp = 0; pp < SN / 2; ++pp) {
          uint4 eq[SM];
#pragma unroll
          for (int j = 0; j < SM; ++j) eq[j] = eall[j][pp];
          float da[2][4];
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int r = 0; r < 4; ++r) da[h][r] = 0.f;
#pragma unroll
          for (int j = 0; j < SM; ++j) {
            uint2 eu[2];
            unswap16_pair(eq[j], eu[0], eu[1]);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const float4 w4 = *(const float4*)(hw_lds + nq + (2 * pp + h) * 16);
              const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
              static_for<0, 4>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                da[h][r] = fma_mix<r>(gm[j] * wv[r], eu[h], da[h][r]);
              });
            }
          }
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = da[h][r];
            row16_sum4(v);
            if ((lane & 15) == 0)
              *(float4*)(red + (2 * Cfg::WM + wm) * BN + wn * TN + (2 * pp + h) * 16 + 4 * (lane >> 4)) =
                  float4{v[0], v[1], v[2], v[3]};
          }
        }
      }
      lds_barrier();
      if (tid < BN) {
        constexpr int NP = SNK ? 3 : 2;  // partial rows: db_L, dw_head (, da_L)
#pragma unroll
        for (int q = 0; q < NP; ++q) {
          float sum = 0.f;
#pragma unroll
          for (int w = 0; w < Cfg::WM; ++w) sum += red[(q * Cfg::WM + w) * BN + tid];
          p.colsum_part[((size_t)tm * NP + q) * LD + n0 + tid] = sum * invS;  // sums of x S: exact
        }
      }
    } else if constexpr (nt_is_fwd(MODE)) {
      const int nq = n0 + wn * TN + 4 * (lane >> 4);     // natural layout: this lane's columns
      const float xs = (MODE == NT_FWD) ? p.omega * kInv2Pi : 1.0f;
      float4 bias[SN], hw[SN];  // (bias_lds holds b * xs)
#pragma unroll
      for (int i = 0; i < SN; ++i) {
        bias[i] = *(const float4*)(bias_lds + nq + i * 16);
        if constexpr (HEAD) hw[i] = *(const float4*)(hw_lds + nq + i * 16);
      }
      float hp[SM];
#pragma unroll
      for (int j = 0; j < SM; ++j) hp[j] = 0.f;
      uint4 ly[2], lc[2];  // NT_FWD: row j-1's Y / C line chunks, stored after row j's arithmetic
#pragma unroll
      for (int j = 0; j < SM; ++j) {
        const size_t rowoff = (size_t)(mrow0 + j * 16) * LD;
        uint4 yp[SN / 2], cpk[SN / 2], epk[SN / 2];  // 16-B row pieces (the per-lane stores)
        uint2 yh[SN], chh[SN], eh[SN];                // MFMA-layout halves (lines_out)
#pragma unroll
        for (int q = 0; q < SN / 2; ++q) {
          // ping-pong tiles: the lower row half takes its column pairs in reverse, the order of
          // the K-loop's serpentine phases (a: pair 0 / rows 0-3, b: 1 / 0-3, c: 1 / 4-7, d: 0 /
          // 4-7) -- the head partial sums keep that summation order
          const int pp = (Cfg::PP && j >= SM / 2) ? SN / 2 - 1 - q : q;
          uint2 ys[2], cs[2], es[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int i = 2 * pp + h;
            const float bb[4] = {bias[i].x, bias[i].y, bias[i].z, bias[i].w};
            float s[4], c[4], e[4];
            if constexpr (MODE == NT_FWD) {
              // revolutions: sin(2*pi*x) with x = omega*(z + b)/(2*pi) (packed fmas); fract keeps
              // the hardware sin/cos inside their reduced domain for any magnitude.
              float xa[4];
              fma4_pk(acc[i][j], xs, bias[i], xa);
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float x = __builtin_amdgcn_fractf(xa[r]);
                s[r] = __builtin_amdgcn_sinf(x);
                c[r] = __builtin_amdgcn_cosf(x);
              }
            } else if constexpr (MODE == NT_FWD_SNAKE) {
              const float4 a4 = *(const float4*)(a_lds + nq + i * 16);
              const float4 ia4 = *(const float4*)(ia_lds + nq + i * 16);
              const float av[4] = {a4.x, a4.y, a4.z, a4.w}, iav[4] = {ia4.x, ia4.y, ia4.z, ia4.w};
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                snake_epi(acc[i][j][r] + bb[r], av[r], iav[r], s[r], c[r], e[r]);
              }
            } else {  // NT_FWD_TANH
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float y = tanh_epi(acc[i][j][r] + bb[r]);
                s[r] = y;
                c[r] = 1.0f - y * y;
              }
            }
            ys[h] = yh[i] = as_u2(pack4(s[0], s[1], s[2], s[3]));
            cs[h] = chh[i] = as_u2(pack4(c[0], c[1], c[2], c[3]));
            if constexpr (MODE == NT_FWD_SNAKE) es[h] = eh[i] = as_u2(pack4(e[0], e[1], e[2], e[3]));
            if constexpr (HEAD) hp[j] += dot4_pk(s, hw[i]);
          }
          if constexpr (!(Lay::LINES || Lay::HALF)) {
            yp[pp] = swap16_pair(ys[0], ys[1]);
            cpk[pp] = swap16_pair(cs[0], cs[1]);
            if constexpr (MODE == NT_FWD_SNAKE) epk[pp] = swap16_pair(es[0], es[1]);
          }
        }
        if (SIREN_DIAG_ON && (diag & 2048)) {  // diag bit 11: the epilogue without its stores (timing only)
          unsigned keep = 0;
#pragma unroll
          for (int i = 0; i < SN; ++i) keep ^= yh[i].x ^ yh[i].y ^ chh[i].x ^ chh[i].y;
          asm volatile("" ::"v"(keep));
          continue;
        }
        if constexpr (Lay::LINES && MODE == NT_FWD && !HEAD) {
          // a row apart: row j-1's stores after row j's arithmetic, row j's exchange now
          if (j > 0) {
            lines_put(p.Y, mrowu + (j - 1) * 16, n0 + wn * TN, ly);
            lines_put(p.C, mrowu + (j - 1) * 16, n0 + wn * TN, lc);
          }
          lines_get(yh, ly);
          lines_get(chh, lc);
          if (j == SM - 1) {
            lines_put(p.Y, mrowu + j * 16, n0 + wn * TN, ly);
            lines_put(p.C, mrowu + j * 16, n0 + wn * TN, lc);
          }
          continue;
        }
        if constexpr (Lay::LINES || Lay::HALF) {
          // whole-line stores (lines_out): forward -4.6%, cfg4 -6.5% (static walk,
          // profiles/r19/ab_full_lines.json)
          lines_out(p.Y, mrowu + j * 16, n0 + wn * TN, yh);
          lines_out(p.C, mrowu + j * 16, n0 + wn * TN, chh);
          if constexpr (MODE == NT_FWD_SNAKE) lines_out(p.E, mrowu + j * 16, n0 + wn * TN, eh);
          continue;
        }
#pragma unroll
        for (int pp = 0; pp < SN / 2; ++pp) {
          // (per-lane addresses here: the head forward has no registers for at_lane's copies -- Snake spilled)
          st16(p.Y + rowoff + npc + pp * 32, yp[pp]);
          st16(p.C + rowoff + npc + pp * 32, cpk[pp]);
          if constexpr (MODE == NT_FWD_SNAKE) st16(p.E + rowoff + npc + pp * 32, epk[pp]);
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
      // partial layout: NT_DX [tm][N]; NT_DX0 [tm][1+in][N] with q=0 -> db0, q=1+j -> dW0[:, j];
      // NT_DX_SNAKE [tm][2][N] with q=0 -> db, q=1 -> da.  flush(i): column subtile i's partials
      // over this wave's rows (DPP across the 16 row lanes) into the LDS scratch
      auto flush = [&](auto ic) {
        constexpr int i = decltype(ic)::value;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (q >= nred) break;
          // NT_DX0_SNAKE: da0 (slot 3) goes out as partial row 1 + in
          const bool da0 = (MODE == NT_DX0_SNAKE) && q == nred - 1;
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = da0 ? cs[3][i][r] : cs[q][i][r];
          row16_sum4(v);
          if ((lane & 15) == 0)
            *(float4*)(red + (q * Cfg::WM + wm) * BN + wn * TN + i * 16 + 4 * (lane >> 4)) =
                float4{v[0], v[1], v[2], v[3]};
        }
      };
      // the 16-B piece (row subtile j, column pair pp) from its Cprev (and Eprev) piece.  Each column
      // partial sums its rows in order 0 .. SM-1 whatever order the pieces go in
      // NT_DX_SNAKE with whole-line stores (Lay::LINES): a row piece's MFMA-layout halves (the Snake batches
      // below take both column pairs of a row back to back, pair 1 last)
      uint2 dzrow[SN];
      auto piece = [&](auto jc, auto ppc, const uint4& cpv, const uint4& epv) {
        constexpr int j = decltype(jc)::value, pp = decltype(ppc)::value;
        const size_t rowoff = (size_t)(mrow0 + j * 16) * LD;
        float t0 = 0.f, t1 = 0.f;
        if constexpr (nt_is_dx0(MODE)) {
          t0 = t_in[j][0];
          t1 = t_in[j][1];
        }
        uint2 cpu[2];
        unswap16_pair(cpv, cpu[0], cpu[1]);
        uint2 epu[2];
        if constexpr (HAS_E) unswap16_pair(epv, epu[0], epu[1]);
        uint2 dzp[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int i = 2 * pp + h;
          // (acc C) omega, paired as in the NT_DX / NT_DX0 loop below
          f32x2 d01 = f32x2{mul_mix<0>(acc[i][j][0], cpu[h]), mul_mix<1>(acc[i][j][1], cpu[h])} * f32x2{om, om};
          f32x2 d23 = f32x2{mul_mix<2>(acc[i][j][2], cpu[h]), mul_mix<3>(acc[i][j][3], cpu[h])} * f32x2{om, om};
          asm volatile("" : "+v"(d01), "+v"(d23));  // rounded to fp32 before the fp16 store (fp32_first)
          set4(cs[0][i], f32x2{cs[0][i][0], cs[0][i][1]} + d01, f32x2{cs[0][i][2], cs[0][i][3]} + d23);
          if constexpr (nt_is_dx0(MODE)) {
            set4(cs[1][i], __builtin_elementwise_fma(d01, f32x2{t0, t0}, f32x2{cs[1][i][0], cs[1][i][1]}),
                 __builtin_elementwise_fma(d23, f32x2{t0, t0}, f32x2{cs[1][i][2], cs[1][i][3]}));
            set4(cs[2][i], __builtin_elementwise_fma(d01, f32x2{t1, t1}, f32x2{cs[2][i][0], cs[2][i][1]}),
                 __builtin_elementwise_fma(d23, f32x2{t1, t1}, f32x2{cs[2][i][2], cs[2][i][3]}));
          }
          static_for<0, 4>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            if constexpr (MODE == NT_DX_SNAKE) cs[1][i][r] = fma_mix<r>(acc[i][j][r], epu[h], cs[1][i][r]);
            if constexpr (MODE == NT_DX0_SNAKE) cs[3][i][r] = fma_mix<r>(acc[i][j][r], epu[h], cs[3][i][r]);
          });
          dzp[h] = as_u2(pack4(d01.x, d01.y, d23.x, d23.y));
        }
        if constexpr (MODE == NT_DX_SNAKE && Lay::LINES) {
          dzrow[2 * pp] = dzp[0];
          dzrow[2 * pp + 1] = dzp[1];
          if constexpr (pp == SN / 2 - 1) lines_out(p.dZ, mrowu + j * 16, n0 + wn * TN, dzrow);
        } else if constexpr (MODE == NT_DX || MODE == NT_DX_SNAKE) {
          st16((h16*)at_lane(rowp(p.dZ, mrowu + j * 16, n0 + wn * TN), lane_piece + pp * 64), swap16_pair(dzp[0], dzp[1]));
        }
      };
      if constexpr (HAS_E) {
        // batches of EB rows, both column pairs of a row back to back: the two 64-B halves of each
        // row's 128-B Cprev / Eprev / dZ segments are read and written together (pair 0 of the
        // first EB rows comes from `pre`)
        static_assert(SN == 4, "two column pairs");
        // software-pipelined: batch bq+1 is loaded before batch bq's dZ stores go out, so waiting
        // for a batch never waits for earlier stores (vmcnt retires in issue order)
        uint4 cq[2][EB][2], eq[2][EB][2];  // [buffer][row][column pair]
        auto load_batch = [&](auto bqc) {
          constexpr int bq = decltype(bqc)::value, bf = bq & 1;
#pragma unroll
          for (int jj = 0; jj < EB; ++jj)
#pragma unroll
            for (int pp = 0; pp < 2; ++pp) {
              if (bq == 0 && pp == 0) {
                cq[bf][jj][pp] = ce_in[jj][0];
                eq[bf][jj][pp] = ce_in[jj][1];
              } else {
                const int ru = mrowu + (bq * EB + jj) * 16;
                cq[bf][jj][pp] = *(const uint4*)at_lane(rowp(p.Cprev, ru, n0 + wn * TN), lane_piece + pp * 64);
                eq[bf][jj][pp] = *(const uint4*)at_lane(rowp(p.Eprev, ru, n0 + wn * TN), lane_piece + pp * 64);
              }
            }
        };
        load_batch(std::integral_constant<int, 0>{});
        static_for<0, SM / EB>([&](auto bqc) {
          constexpr int bq = decltype(bqc)::value, bf = bq & 1;
          if constexpr (bq + 1 < SM / EB) load_batch(std::integral_constant<int, bq + 1>{});
          static_for<0, EB>([&](auto jc) {
            constexpr int jj = decltype(jc)::value;
            piece(std::integral_constant<int, bq * EB + jj>{}, std::integral_constant<int, 0>{}, cq[bf][jj][0], eq[bf][jj][0]);
            piece(std::integral_constant<int, bq * EB + jj>{}, std::integral_constant<int, 1>{}, cq[bf][jj][1], eq[bf][jj][1]);
          });
        });
        static_for<0, SN>([&](auto ic) { flush(ic); });
      } else {
        // NT_DX / NT_DX0: rows in order, both column pairs of a row together (rows >= PRE_J loaded
        // at use), then the column partials.  The same arithmetic as `piece`, kept as a plain loop:
        // written through the lambda, NT_DX0 takes 252-256 VGPRs instead of 239-244 (gfx950 listing)
        uint4 ldz[2];  // NT_DX: row j-1's dZ line chunks
#pragma unroll
        for (int j = 0; j < SM; ++j) {
          const size_t rowoff = (size_t)(mrow0 + j * 16) * LD;
          float t0 = 0.f, t1 = 0.f;
          if constexpr (nt_is_dx0(MODE)) {
            t0 = t_in[j][0];
            t1 = t_in[j][1];
          }
          uint2 dzq[SN];  // NT_DX with whole-line stores: this row piece's MFMA-layout halves
#pragma unroll
          for (int pp = 0; pp < SN / 2; ++pp) {
            uint2 cpu[2];
            const uint4 cpv =
                (j < PRE_J) ? cp_in[j < PRE_J ? j : 0][pp]
                            : *(const uint4*)at_lane(rowp(p.Cprev, mrowu + j * 16, n0 + wn * TN), lane_piece + pp * 64);
            unswap16_pair(cpv, cpu[0], cpu[1]);
            uint2 dzp[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int i = 2 * pp + h;
              // (acc C) omega: the fp16 product in v_fma_mix_f32, the rest in pairs (v_pk_mul_f32,
              // v_pk_add_f32, v_pk_fma_f32: per element the rounding of the scalar instruction)
              f32x2 d01 = f32x2{mul_mix<0>(acc[i][j][0], cpu[h]), mul_mix<1>(acc[i][j][1], cpu[h])} * f32x2{om, om};
              f32x2 d23 = f32x2{mul_mix<2>(acc[i][j][2], cpu[h]), mul_mix<3>(acc[i][j][3], cpu[h])} * f32x2{om, om};
              asm volatile("" : "+v"(d01), "+v"(d23));  // rounded to fp32 before the fp16 store (fp32_first)
              set4(cs[0][i], f32x2{cs[0][i][0], cs[0][i][1]} + d01, f32x2{cs[0][i][2], cs[0][i][3]} + d23);
              if constexpr (nt_is_dx0(MODE)) {
                set4(cs[1][i], __builtin_elementwise_fma(d01, f32x2{t0, t0}, f32x2{cs[1][i][0], cs[1][i][1]}),
                     __builtin_elementwise_fma(d23, f32x2{t0, t0}, f32x2{cs[1][i][2], cs[1][i][3]}));
                set4(cs[2][i], __builtin_elementwise_fma(d01, f32x2{t1, t1}, f32x2{cs[2][i][0], cs[2][i][1]}),
                     __builtin_elementwise_fma(d23, f32x2{t1, t1}, f32x2{cs[2][i][2], cs[2][i][3]}));
              }
              dzp[h] = as_u2(pack4(d01.x, d01.y, d23.x, d23.y));
            }
            if constexpr (Lay::LINES && MODE == NT_DX) {
              dzq[2 * pp] = dzp[0];
              dzq[2 * pp + 1] = dzp[1];
            }
            else if constexpr (MODE == NT_DX)
              st16((h16*)at_lane(rowp(p.dZ, mrowu + j * 16, n0 + wn * TN), lane_piece + pp * 64), swap16_pair(dzp[0], dzp[1]));
          }
          if constexpr (Lay::LINES && MODE == NT_DX) {
            // a row apart, as the forward: row j-1's stores after row j's arithmetic
            if (j > 0) lines_put(p.dZ, mrowu + (j - 1) * 16, n0 + wn * TN, ldz);
            lines_get(dzq, ldz);
            if (j == SM - 1) lines_put(p.dZ, mrowu + j * 16, n0 + wn * TN, ldz);
          }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (q >= nred) break;
#pragma unroll
          for (int i = 0; i < SN; ++i) {
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = cs[q][i][r];
            row16_sum4(v);
            if ((lane & 15) == 0)
              *(float4*)(red + (q * Cfg::WM + wm) * BN + wn * TN + i * 16 + 4 * (lane >> 4)) =
                  float4{v[0], v[1], v[2], v[3]};
          }
        }
      }
      lds_barrier();
      if (tid < BN) {
        for (int q = 0; q < nred; ++q) {
          float s = 0.f;
#pragma unroll
          for (int w = 0; w < Cfg::WM; ++w) s += red[(q * Cfg::WM + w) * BN + tid];
          p.colsum_part[((size_t)tm * nred + q) * LD + n0 + tid] = s * inv_scale;
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
    // Every piece starts at a row multiple of 8 (lr0), so the source swizzle depends on the lane
    // only: the per-lane part of the source offset is one VGPR (lane_src, bytes) for all pieces,
    // the row part (urow, bytes) is wave-uniform and goes into the SGPR base of the saddr form
    // of the LDS-DMA (measured: forward 2.278 -> 2.220 ms, 221-229 instead of 234-242 VGPRs).
    int urow[4][2];
    unsigned pdst[4][2];
    const unsigned lane_src = (unsigned)(((lane >> 3) * K + stage_swz<BK>(lane >> 3, lane & 7) * 8) * 2);
#pragma unroll
    for (int pc = 0; pc < 4; ++pc)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int pr0 = (2 * wave + j) * 8, hf = pc >> 1;
        const int lr0 = (pc & 1) ? (pr0 >> 6) * 128 + (pr0 & 63) + 64 * hf
                                 : (pr0 >> 5) * 64 + (pr0 & 31) + 32 * hf;
        urow[pc][j] = lr0 * K * 2;
        pdst[pc][j] = ((pc & 1) ? 0u : (unsigned)Cfg::XBYTES) + (unsigned)(lr0 * ROWB);
      }
    // operand bases of the current tile (0) and the next one (1), set once per tile:
    // no division or 64-bit product in the per-phase scalar work
    const h16 *x0 = p.X, *x1 = p.X, *w0 = p.W, *w1 = p.W;
    // This block's current and next tile (global ids); the next one exists while it lies in
    // [g_lo, g_lim).  Static walk: bp, bp + G, ...  Queue: shard s = blockIdx % 8 (one XCD under
    // round-robin dispatch -- speed only, any placement is correct) pulls tiles
    // [s, s + 1) * ntiles / 8 in order, so the blocks holding one row band of X are the ones that
    // started it together.
    const int shard = blockIdx.x & 7;
    const int q_lo = (int)((long)shard * ntiles / 8);
    const int g_lo = dyn ? q_lo : 0;
    const int g_lim = dyn ? (int)((long)(shard + 1) * ntiles / 8) : (my_tiles > 0 ? ntiles : 0);
    auto in_range = [&](int g) { return (unsigned)(g - g_lo) < (unsigned)(g_lim - g_lo); };
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
    // a block walks at most its shard's tile count, whatever ids it pulls
    auto more = [&](int ti) { return in_range(g_next) && ti + 1 < g_lim - g_lo; };
    auto set_tiles = [&](int ti) {
      if (ti > 0) {
        g_cur = g_next;
        // queue: the pull tile_end(ti - 1) left in the slot
        g_next = dyn ? __builtin_amdgcn_readfirstlane(qslot[0]) : g_next + G;
      }
      auto bases = [&](int g, const h16*& xb, const h16*& wb) {
        int m0, n0;
        tile_of(g, m0, n0);
        xb = p.X + (size_t)xrow(m0) * K;
        wb = p.W + (size_t)((diag & 4) ? 0 : n0) * K;  // diag bit 2: one W column tile (L2-resident W)
      };
      bases(g_cur, x0, w0);
      bases(in_range(g_next) ? g_next : g_cur, x1, w1);
    };
    // the piece's second 8 rows: 8 rows further in the operand, 1 KiB further in LDS
    // (urow[PC][1] = urow[PC][0] + 8 rows, pdst[PC][1] = pdst[PC][0] + 1 KiB: glds16x2o_asm_s's offset:1024)
    const unsigned lane_src8 = lane_src + (unsigned)(16 * K) - 1024u;
    auto issue = [&](int sel, int kt, int slot, auto pcc) {
      constexpr int PC = decltype(pcc)::value;
      const h16* src = ((PC & 1) ? (sel ? x1 : x0) : (sel ? w1 : w0)) + kt * BK;
      const char* dst = smem + slot * Cfg::STAGE;
      if constexpr (SIREN_GLDS_PAIR != 0) {
        glds16x2o_asm_s(lane_src, lane_src8, (const char*)src + urow[PC][0], lds_addr(dst + pdst[PC][0]));
      } else {
#pragma unroll
        for (int j = 0; j < 2; ++j)
          glds16_asm_s(lane_src, (const char*)src + urow[PC][j], lds_addr(dst + pdst[PC][j]));
      }
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
    // issue order: serpentine over (X fragment jl, W fragment il), reversed for the second k32
    // half, so every two consecutive MFMAs share an operand (each accumulator still takes kk 0
    // then 1: bit-identical).  Measured against A-shared runs (il outer): forward -1.4 to -2.3%,
    // dX -0.6 to -1.6%, dX0 -0.8 to -1.0%, three boxes (tools/variants.py ord / ord2)
    auto mma = [&](auto ph) {
      constexpr int PH = decltype(ph)::value;
      constexpr int MH = PH >> 1, NH = (PH == 1 || PH == 2) ? 1 : 0;
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int kk = t >> 3, u = t & 7, jq = u >> 1;
        const int jl = kk ? 3 - jq : jq;
        const int il = ((t >> 1) & 1) ? 1 - (u & 1) : (u & 1);
        const h16x8 a = NH ? wf1[il][kk] : wf0[il][kk];
        acc[2 * NH + il][4 * MH + jl] =
            __builtin_amdgcn_mfma_f32_16x16x32_f16(a, xf[jl][kk], acc[2 * NH + il][4 * MH + jl], 0, 0, 0);
      }
    };
    auto tile_end = [&](int) {
      // both groups are aligned here
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
#pragma unroll
      for (int i = 0; i < SN; ++i)
#pragma unroll
        for (int j = 0; j < SM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    };
    if constexpr (SIREN_NT_SEG2 != 0)
      // EARLY (the next tile's K-tile 1 piece 3 before the epilogue's stores): the fused last layer
      // gains 2.3% (cfg2) / 0.8% (cfg4), the plain forward loses 2.3% at cfg2 (profiles/r20/ab_early.json)
      pingpong2_tiles<epilogue_stores<Cfg, MODE>(), SIREN_NT_EARLY != 0 || nt_is_hb(MODE) || MODE == NT_DX0>(
          in_range(g_cur), nk, wm, issue, read, mma, set_tiles, tile_end, more);
    else
      pingpong_tiles<epilogue_stores<Cfg, MODE>(), 0xB>(in_range(g_cur), nk, wm, issue, read, mma, set_tiles,
                                                         tile_end, more);
  } else {
    mfma_pipeline_tiles<Cfg::S, BK / 32, Cfg::XINSTR + Cfg::WINSTR, SN, SM, epilogue_stores<Cfg, MODE>()>(
        my_tiles, K / BK, acc, stage, frags, [&](int ti) { pre(bp + ti * G); },
        [&](int ti) { epilogue(bp + ti * G); });
  }
}

static int g_num_cus[64] = {};
static int g_nt_grid_cap = 0;  // test hook: persistent grid size (0 = one block per CU)
void gemm_nt_set_grid_cap(int cap) { g_nt_grid_cap = cap; }
static int g_nt_diag = 0;
bool gemm_nt_set_diag(int bits) {
  if (!SIREN_DIAG_ON && bits) return false;  // product builds carry no ablation
  g_nt_diag = bits;
  return true;
}
static int g_nt_queue = 1;  // 0 off, 1 forward modes, 2 every ping-pong mode
void gemm_nt_set_queue(int v) { g_nt_queue = v; }
static int g_hb_fault = 0;  // SIREN_OPT_HB_FAULT (SIREN_DIAG builds)
bool gemm_nt_set_hb_fault(int v) {
  if (!SIREN_DIAG_ON && v) return false;  // product builds carry no fault injection
  g_hb_fault = v;
  return true;
}

// CU count of the stream's device (queried once per device)
static int stream_cus(hipStream_t s) {
  int dev = 0;
  if (hipStreamGetDevice(s, &dev) != hipSuccess && hipGetDevice(&dev) != hipSuccess) dev = 0;
  if (dev < 0 || dev >= 64) return 256;
  if (g_num_cus[dev] <= 0) {
    int n = 0;
    g_num_cus[dev] = (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
                         ? n : 256;
  }
  return g_num_cus[dev];
}

// NT_FWD_HB co-residency: blocks per CU for the fused kernel x CUs >= grid (queried once per device)
static int g_hb_per_cu[3][64] = {};
static bool hb_coresident(int mode, int grid, hipStream_t s);

template <class Cfg, int MODE, bool HEAD, bool ACTL = false>
static hipError_t launch_nt(const NtParams& p_in, hipStream_t s, bool persistent) {
  // the static ping-pong schedule assumes an even number (>= 2) of K-tiles per tile
  if (Cfg::PP && (p_in.K % (2 * Cfg::BK) != 0 || !persistent)) return hipErrorInvalidValue;
  NtParams p = p_in;
  p.diag = g_nt_diag;
  const int ntiles = (p.M / Cfg::BM) * (p.N / Cfg::BN);
  const int cap = g_nt_grid_cap > 0 ? g_nt_grid_cap : stream_cus(s);
  const int grid = persistent ? (ntiles < cap ? ntiles : cap) : ntiles;
  // the queue's shards are blockIdx % 8: every shard must have blocks
  // (measured: the forward gains 3-4%; dX is unchanged and dX0 loses 2%, its K-loop spills)
  const bool want = g_nt_queue == 2 || (g_nt_queue == 1 && nt_is_fwd(MODE));
  if constexpr (nt_is_hb(MODE)) {
    // the static walk g = bp + i G with G a multiple of tiles_n: the tiles_n column tiles of a row
    // band are tile i of tiles_n consecutive blocks (one XCD under the xcd_remap order), which wait
    // for each other's head partials.  Blocks are dispatched in order, so a waiting block's
    // partners are resident or next in line (at most tiles_n - 1 blocks per XCD wait on blocks
    // not yet dispatched while every fully resident band group runs on).
    // Co-residency: every block of the grid must be resident at once on an idle device (the
    // launcher checks the occupancy; the caller falls back to the unfused launches when it fails),
    // and the wait itself is bounded (kHeadSpinLimit), so CUs taken by other work can slow the
    // hand-off or fail the step loudly, never hang it.  G is rounded down to a multiple of
    // 8 * tiles_n when the grid allows it, so that the G/8 blocks xcd_remap deals to each XCD hold
    // whole band groups: a band's tiles then share one L2.
    static_assert(Cfg::PP, "fused head: ping-pong persistent walk");
    const int tiles_n = p.N / Cfg::BN;
    if (p.diag || tiles_n > 4 || p.M % Cfg::BM) return hipErrorInvalidValue;
    int g = grid;
    if (g >= 8 * tiles_n) g -= g % (8 * tiles_n);
    else g -= g % tiles_n;
    if (g < tiles_n) g = tiles_n;
    if (!hb_coresident(MODE, g, s)) return hipErrorCooperativeLaunchTooLarge;
    p.hb_fault = g_hb_fault & 0xff;
    p.spin_limit = (g_hb_fault >> 8) > 0 ? (g_hb_fault >> 8) : kHeadSpinLimit;
    const hipError_t e = hipMemsetAsync(p.head_part, 0xFF, (size_t)tiles_n * p.M * sizeof(float), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((gemm_nt_kernel<Cfg, MODE, HEAD>), dim3(g), dim3(Cfg::THREADS), 0, s, p);
    return hipGetLastError();
  }
  if constexpr (Cfg::PP && !nt_is_hb(MODE)) {
    if (p.tileq && want && !p.diag && grid % 8 == 0) {
      // the counter set starts every launch at zero, ordered on the launch's own stream
      // (graph capture records the memset as a node before the kernel)
      const hipError_t e = hipMemsetAsync(p.tileq, 0, kQueueSet * sizeof(int), s);
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL((gemm_nt_kernel<Cfg, MODE, HEAD, true, ACTL>), dim3(grid), dim3(Cfg::THREADS), 0, s, p);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((gemm_nt_kernel<Cfg, MODE, HEAD, false, ACTL>), dim3(grid), dim3(Cfg::THREADS), 0, s, p);
  return hipGetLastError();
}

static bool hb_coresident(int mode, int grid, hipStream_t s) {
  int dev = 0;
  if (hipStreamGetDevice(s, &dev) != hipSuccess && hipGetDevice(&dev) != hipSuccess) dev = 0;
  if (dev < 0 || dev >= 64 || !nt_is_hb(mode)) return false;
  int& per_cu = g_hb_per_cu[mode - NT_FWD_HB][dev];
  if (per_cu == 0) {
    const void* fn = mode == NT_FWD_HB         ? reinterpret_cast<const void*>(&gemm_nt_kernel<NtLargePP, NT_FWD_HB, true>)
                     : mode == NT_FWD_HB_SNAKE ? reinterpret_cast<const void*>(&gemm_nt_kernel<NtLargePP, NT_FWD_HB_SNAKE, true>)
                                               : reinterpret_cast<const void*>(&gemm_nt_kernel<NtLargePP, NT_FWD_HB_TANH, true>);
    int n = 0;
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, NtLargePP::THREADS, 0);
    per_cu = (e == hipSuccess && n > 0) ? n : -1;
  }
  return per_cu > 0 && (long)per_cu * stream_cus(s) >= grid;
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
      if (head) return launch_nt<Cfg, NT_FWD_SNAKE, true>(p, s, persistent);
      return (Cfg::PP && p.K <= 512) ? launch_nt<Cfg, NT_FWD_SNAKE, false, true>(p, s, persistent)
                                     : launch_nt<Cfg, NT_FWD_SNAKE, false>(p, s, persistent);
    case NT_FWD_TANH:
      if (head) return launch_nt<Cfg, NT_FWD_TANH, true>(p, s, persistent);
      return (Cfg::PP && p.K <= 512) ? launch_nt<Cfg, NT_FWD_TANH, false, true>(p, s, persistent)
                                     : launch_nt<Cfg, NT_FWD_TANH, false>(p, s, persistent);
    case NT_DX_SNAKE:
      return (Cfg::PP && p.K <= 512) ? launch_nt<Cfg, NT_DX_SNAKE, false, true>(p, s, persistent)
                                     : launch_nt<Cfg, NT_DX_SNAKE, false>(p, s, persistent);
  }
  return hipErrorInvalidValue;
}

// tile override for A/B measurement: 0 = auto, 128 or 256; pipe (256x256): 0 = BK 64, one
// tile per block; 1 = BK 64 persistent; 4 = BK 64 persistent ping-pong (pingpong2_tiles)
static int g_nt_tile = 0;
static int g_nt_pipe = -1;  // -1: automatic = ping-pong 4 for every mode (kernel_bench r06)
static bool nt_pp() { return g_nt_pipe < 0 || (g_nt_pipe >= 4 && g_nt_pipe <= 7); }
void gemm_nt_set_tile(int tile) { g_nt_tile = tile; }
void gemm_nt_set_pipe(int v) { g_nt_pipe = v; }

int nt_choose_tile(int M, int N) {
  const bool large_ok = (M % 256 == 0) && (N % 256 == 0);
  if (g_nt_tile == 128 || !large_ok) return 128;
  if (g_nt_tile == 256) return 256;
  // the 256x256 tile (1 block/CU) needs >= 2 tiles per CU to keep 256 CUs busy
  return (long)(M / 256) * (N / 256) >= 512 ? 256 : 128;
}

bool gemm_nt_head_fusable(int M, int N, hipStream_t s, int mode) {
  if (!(nt_choose_tile(M, N) == 256 && nt_pp() && M % 256 == 0 && N % 256 == 0 && N / 256 <= 4 && N % 128 == 0))
    return false;
  // the grid launch_nt will use must be co-resident (one block per CU on an idle device)
  const int ntiles = (M / 256) * (N / 256), cap = g_nt_grid_cap > 0 ? g_nt_grid_cap : stream_cus(s);
  return hb_coresident(mode, ntiles < cap ? ntiles : cap, s);
}

static hipError_t gemm_nt_window(int mode, bool head, const NtParams& p, hipStream_t s) {
  if (p.M % NtSmall::BM || p.N % NtSmall::BN || p.K % NtSmall::BK || p.M <= 0 || p.N > NtSmall::MAXN) return hipErrorInvalidValue;
  if (nt_is_hb(mode)) {
    if (!head || p.tile != 256 || !gemm_nt_head_fusable(p.M, p.N, s, mode)) return hipErrorInvalidValue;
    if (!p.head_w || !p.head_part || !p.gscale || !p.dZ || !p.colsum_part || !p.b_head || !p.out || !p.g ||
        !p.sse_part || !p.gsum_part || (p.n_valid > 0 && !p.target) || (mode == NT_FWD_HB_SNAKE && (!p.act_a || !p.E)))
      return hipErrorInvalidValue;
    if (mode == NT_FWD_HB_SNAKE) return launch_nt<NtLargePP, NT_FWD_HB_SNAKE, true>(p, s, true);
    if (mode == NT_FWD_HB_TANH) return launch_nt<NtLargePP, NT_FWD_HB_TANH, true>(p, s, true);
    return launch_nt<NtLargePP, NT_FWD_HB, true>(p, s, true);
  }
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
  if (mode >= NT_FWD_SNAKE && mode <= NT_DX_SNAKE) {
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
    // pipe 5: the forward with its epilogue under the next tile's MFMAs (gemm_nt1.hip)
    if ((pipe == 5 || pipe == 7) && mode == NT_FWD && !head && p.ld == p.N && gemm_nt_one_ok(p))
      return gemm_nt_one(p, g_nt_grid_cap > 0 ? g_nt_grid_cap : stream_cus(s), g_nt_diag, pipe == 5, s);
    // pipe 6: the forward with one wave per SIMD on 256x256 tiles (gemm_nt2.hip)
    if (pipe == 6 && mode == NT_FWD && !head && p.ld == p.N && gemm_nt_big_ok(p))
      return gemm_nt_big(p, g_nt_grid_cap > 0 ? g_nt_grid_cap : stream_cus(s), g_nt_diag, s);
    switch (pipe) {
      case 0: return dispatch_mode<NtLarge>(mode, head, p, s, false);
      case 4:
      case 5:  // (pipes 5-7 cover the plain forward only; every other mode takes the ping-pong)
      case 6:
      case 7: return dispatch_mode<NtLargePP>(mode, head, p, s, true);
      default: return dispatch_mode<NtLarge>(mode, head, p, s, true);
    }
  }
  if (p.tile != 128) return hipErrorInvalidValue;
  return dispatch_mode<NtSmall>(mode, head, p, s, false);
}

// A layer wider than the epilogue's per-column LDS vectors (MAXN = 1024 columns) runs as launches over
// column windows of MAXN: each window is the same GEMM on rows nb .. nb + MAXN of W with its slice
// of every per-column vector, its column slice of every [M][N] operand (row stride p.N, NtParams::ld)
// and its tiles' head partials.  Every output element and column partial is computed exactly as in
// one launch over all N (a column's arithmetic never involves another column), so the windowed
// result is the one-launch result.  The fused last layer (one band's column tiles hand off their
// head partials) is not windowed: gemm_nt_head_fusable is false above 4 column tiles.
hipError_t gemm_nt(int mode, bool head, const NtParams& p, hipStream_t s) {
  constexpr int WIN = NtSmall::MAXN;
  static_assert(NtSmall::MAXN == NtLargePP::MAXN && NtSmall::MAXN == NtLarge::MAXN, "one window width");
  NtParams q = p;
  q.ld = p.N;
  if (p.N <= WIN || nt_is_hb(mode)) return gemm_nt_window(mode, head, q, s);
  if (p.N % WIN || p.tile <= 0 || p.tile > 256) return hipErrorInvalidValue;
  for (int nb = 0; nb < p.N; nb += WIN) {
    q.N = WIN;
    q.W = p.W + (size_t)nb * p.K;
    auto col = [&](auto* v) { return v ? v + nb : v; };
    q.bias = col(p.bias);
    q.act_a = col(p.act_a);
    q.head_w = col(p.head_w);
    q.Y = col(p.Y);
    q.C = col(p.C);
    q.E = col(p.E);
    q.Cprev = col(p.Cprev);
    q.Eprev = col(p.Eprev);
    q.dZ = col(p.dZ);
    q.colsum_part = col(p.colsum_part);
    q.head_part = p.head_part ? p.head_part + (size_t)(nb / p.tile) * p.M : nullptr;
    const hipError_t e = gemm_nt_window(mode, head, q, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace siren
