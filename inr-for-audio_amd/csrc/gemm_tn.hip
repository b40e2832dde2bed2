// TN GEMM for the SIREN weight gradient on gfx950 h16 MFMA, split-K over coordinates.
//
//   dW[o][k] = sum_n dZ[n][o] * Y[n][k]          (autograd addmm backward, models.py:114-115)
//
// The reduction index n is the SLOW index of both operands, so both tiles are staged
// row-major ([n][col], coalesced LDS-DMA) and the MFMA fragments are gathered with the
// gfx950 hardware transpose read ds_read_b64_tr_b16 (cdna_hip_programming.md T10).
// Roles: MFMA A := Y (i = k), B := dZ (j = o), so each lane's 4 accumulator registers are 4
// consecutive k of one o row -> the reduce kernel writes float4 rows of dW.
//
// Each block owns one BI x BJ tile of dW^T and a contiguous slice of the coordinates; the
// fp32 partial tile goes to a slab in MFMA-native order (1 KiB contiguous per store
// instruction).  dw_reduce sums the slices in a fixed order (deterministic).
// Tiles: 128x128 / 4 waves (small grids) or 256x256 / 8 waves (half the LDS-fill bytes per
// flop); the choice is made once per call by tn_choose_tile and passed to both kernels.
#include "gemm_pipeline.h"
#include "siren_common.h"
#include "siren_kernels.h"

namespace siren {

template <int BI_, int BJ_, int WM_, int WN_, int BK_ = 64, int S_ = 2, int PP_ = 0>
struct TnCfg {
  static constexpr int BI = BI_, BJ = BJ_, BK = BK_, S = S_;
  static constexpr int PP = PP_;  // ping-pong K-loop: 1 pingpong_tiles, 2 pingpong2_one_tile
  static constexpr int WM = WM_, WN = WN_, NWAVES = WM_ * WN_, THREADS = 64 * NWAVES;
  static constexpr int TI = BI / WM, TJ = BJ / WN, SI = TI / 16, SJ = TJ / 16;
  static constexpr int YROW = BI * 2, ZROW = BJ * 2;       // bytes per staged row
  static constexpr int YBYTES = BK * YROW, ZBYTES = BK * ZROW;
  static constexpr int STAGE = YBYTES + ZBYTES, LDS = S * STAGE;
  static constexpr int YINSTR = YBYTES / 1024 / NWAVES, ZINSTR = ZBYTES / 1024 / NWAVES;
  static constexpr int TILE_FLOATS = BI * BJ;
  static_assert(YBYTES % (1024 * NWAVES) == 0 && ZBYTES % (1024 * NWAVES) == 0, "staging split");
  static_assert(LDS <= 160 * 1024, "LDS");
};
using TnSmall = TnCfg<128, 128, 2, 2>;
using TnLarge = TnCfg<256, 256, 2, 4>;          // slab geometry of every 256x256 variant
using TnL0 = TnCfg<256, 256, 2, 4, 64, 2>;      // BK 64, double buffer
using TnL1 = TnCfg<256, 256, 2, 4, 32, 4>;      // BK 32, 4-slot ring
using TnL2 = TnCfg<256, 256, 2, 4, 32, 5>;      // BK 32, 5-slot ring
using TnLPP = TnCfg<256, 256, 2, 4, 64, 2, 1>;  // BK 64, two wave groups in ping-pong
using TnLPP2 = TnCfg<256, 256, 2, 4, 64, 2, 2>;  // the same, two 32-MFMA segments per K-tile

// Chunk swizzle of a staged [64][cols] image: physical 16-B chunk = c ^ f(r).  With
// h(r) = (r&3) | ((r>>3)&1)<<2 and f = 2h, the 8 rows a 32-lane half touches in one
// transposed read occupy 8 distinct 32-B bank slots (conflict-free) for any row length
// that is a multiple of 256 B.
__device__ __forceinline__ int tn_swz(int r) { return ((r & 3) | (((r >> 3) & 1) << 2)) << 1; }

// One 16x16x32 operand fragment = two ds_read_b64_tr_b16: rows 8g+0..3 then 8g+4..7 of the
// [n][col] image (the second block sits 4 rows further down).
typedef short s16x8 __attribute__((ext_vector_type(8)));
template <int ROW>
__device__ __forceinline__ h16x8 tr_frag(const char* p) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(p));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(p + 4 * ROW));
  const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(h16x8, v);
}

template <class Cfg>
__global__ __launch_bounds__(Cfg::THREADS, 2) void gemm_tn_kernel(TnParams p) {
  constexpr int BK = Cfg::BK, SI = Cfg::SI, SJ = Cfg::SJ, TI = Cfg::TI, TJ = Cfg::TJ;
  constexpr int YROW = Cfg::YROW, ZROW = Cfg::ZROW;
  __shared__ __attribute__((aligned(16))) char smem[Cfg::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / Cfg::WN, wn = wave % Cfg::WN;  // wm -> k (i), wn -> o (j)
  const int tiles_i = p.Hin / Cfg::BI, tiles_j = p.Hout / Cfg::BJ;
  const int ntile = tiles_i * tiles_j;
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int slice = g / ntile, tile = g - slice * ntile;
  const int ti = tile / tiles_j, tj = tile - ti * tiles_j;
  const int k0 = ti * Cfg::BI, o0 = tj * Cfg::BJ;

  const int nks = p.R / BK;
  const int ks_begin = (int)(((int64_t)slice * nks) / p.splits);
  const int ks_end = (int)(((int64_t)(slice + 1) * nks) / p.splits);

  // staging: one instruction writes 1 KiB = 1024/ROW rows; lane L -> row L/(ROW/16),
  // 16-B slot L%(ROW/16), carrying logical chunk slot ^ f(row).
  size_t yoff[Cfg::YINSTR], zoff[Cfg::ZINSTR];
#pragma unroll
  for (int j = 0; j < Cfg::YINSTR; ++j) {
    constexpr int RPI = 1024 / YROW, SPR = YROW / 16;
    const int r = (wave * Cfg::YINSTR + j) * RPI + lane / SPR;
    yoff[j] = (size_t)r * p.Hin + k0 + (((lane % SPR) ^ tn_swz(r)) * 8);
  }
#pragma unroll
  for (int j = 0; j < Cfg::ZINSTR; ++j) {
    constexpr int RPI = 1024 / ZROW, SPR = ZROW / 16;
    const int r = (wave * Cfg::ZINSTR + j) * RPI + lane / SPR;
    zoff[j] = (size_t)r * p.Hout + o0 + (((lane % SPR) ^ tn_swz(r)) * 8);
  }
  auto stage = [&](int kt, int buf) {
    const int ks = ks_begin + kt;
    char* ys = smem + buf * Cfg::STAGE + wave * Cfg::YINSTR * 1024;
    char* zs = smem + buf * Cfg::STAGE + Cfg::YBYTES + wave * Cfg::ZINSTR * 1024;
    const h16* yb = p.Y + (size_t)ks * BK * p.Hin;
    const h16* zb = p.dZ + (size_t)ks * BK * p.Hout;
#pragma unroll
    for (int j = 0; j < Cfg::YINSTR; ++j) glds16_asm(yb + yoff[j], lds_addr(ys + j * 1024));
#pragma unroll
    for (int j = 0; j < Cfg::ZINSTR; ++j) glds16_asm(zb + zoff[j], lds_addr(zs + j * 1024));
  };

  // transposed-read addresses: group g = lane>>4, lane-in-group 4q+p supplies row q (+4 for
  // the second read) of the 4-row block starting at 8g (+32 for the second k32 half),
  // columns col0 + 4p .. +3.  Row r = 32kk + 8g + 4h + q, so tn_swz(r) is the same for every
  // (kk, h): the swizzle only permutes 16-B column chunks per lane.
  const int grp = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int fl = tn_swz(8 * grp + q);
  int colA[SI], colB[SJ];
#pragma unroll
  for (int s = 0; s < SI; ++s)
    colA[s] = (8 * grp + q) * YROW + ((pp & 1) << 3) + (((2 * (wm * SI + s) + (pp >> 1)) ^ fl) << 4);
#pragma unroll
  for (int s = 0; s < SJ; ++s)
    colB[s] = (8 * grp + q) * ZROW + ((pp & 1) << 3) + (((2 * (wn * SJ + s) + (pp >> 1)) ^ fl) << 4);

  f32x4 acc[SI][SJ];
#pragma unroll
  for (int i = 0; i < SI; ++i)
#pragma unroll
    for (int j = 0; j < SJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto frags = [&](int slot, int kk, h16x8 (&A)[SI], h16x8 (&B)[SJ]) {
    const char* ys = smem + slot * Cfg::STAGE;
    const char* zs = ys + Cfg::YBYTES;
#pragma unroll
    for (int s = 0; s < SI; ++s) A[s] = tr_frag<YROW>(ys + kk * 32 * YROW + colA[s]);
#pragma unroll
    for (int s = 0; s < SJ; ++s) B[s] = tr_frag<ZROW>(zs + kk * 32 * ZROW + colB[s]);
  };
  if constexpr (Cfg::PP) {
    static_assert(Cfg::BI == 256 && Cfg::BJ == 256 && BK == 64 && Cfg::WM == 2 && Cfg::WN == 4,
                  "ping-pong geometry");
    // Staging pieces of a K-tile (64 coordinates; 16 KiB = 2 LDS-DMA per wave, 2 rows of 512 B
    // per instruction): pc 0 = dZ rows 0..31, pc 1 = Y rows 0..31, pc 2 = dZ rows 32..63,
    // pc 3 = Y rows 32..63.  Phases (k32 half, i half): a (0,0), b (0,1), c (1,1), d (1,0), so
    // pc 0 is read in a, pc 1 in a-b, pc 2 in c, pc 3 in c-d (pingpong_tiles contract).
    int yo[2][2], zo[2][2];
    unsigned po[2][2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r0 = 32 * kk + 4 * wave + 2 * j, r = r0 + (lane >> 5);
        const int ch = ((lane & 31) ^ tn_swz(r)) * 8;
        yo[kk][j] = r * p.Hin + k0 + ch;
        zo[kk][j] = r * p.Hout + o0 + ch;
        po[kk][j] = (unsigned)(r0 * YROW);
      }
    const int nkl = ks_end - ks_begin;
    // one tile per block: pieces addressed past it (sel = 1, or past the slice's last K-step)
    // re-read a valid K-step into LDS pieces already consumed (pingpong_tiles contract)
    auto issue = [&](int sel, int kt, int slot, auto pcc) {
      constexpr int PC = decltype(pcc)::value, KK = PC >> 1;
      const int ks = ks_begin + min(sel ? 0 : kt, nkl - 1);
      const char* dst = smem + slot * Cfg::STAGE;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if constexpr ((PC & 1) != 0)
          glds16_asm(p.Y + (size_t)ks * BK * p.Hin + yo[KK][j], lds_addr(dst + po[KK][j]));
        else
          glds16_asm(p.dZ + (size_t)ks * BK * p.Hout + zo[KK][j], lds_addr(dst + Cfg::YBYTES + po[KK][j]));
      }
    };
    if constexpr (Cfg::PP == 2) {
      // segment A = k32 half 0 (pieces 0, 1), B = half 1 (pieces 2, 3); all 8 i-subtiles each
      h16x8 a8[8], b4[4];
      // SIREN_GLDS_PAIR (siren_common.h): a piece's two DMAs (rows r and r + 2, 1 KiB apart in LDS) from one
      // wave-uniform base in SGPRs and 32-bit lane byte offsets, one statement per piece
      unsigned yb0[2], yb1[2], zb0[2], zb1[2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        yb0[kk] = (unsigned)yo[kk][0] * 2u;
        yb1[kk] = (unsigned)yo[kk][1] * 2u - 1024u;  // glds16x2o_asm_s's offset:1024
        zb0[kk] = (unsigned)zo[kk][0] * 2u;
        zb1[kk] = (unsigned)zo[kk][1] * 2u - 1024u;
      }
      auto issue2 = [&](int kt, int slot, auto pcc) {
        constexpr int PC = decltype(pcc)::value, KK = PC >> 1;
        const int ks = ks_begin + min(kt, nkl - 1);  // past the slice: a consumed piece re-read
        const char* dst = smem + slot * Cfg::STAGE;
        if constexpr (SIREN_GLDS_PAIR != 0) {
          static_assert(2 * Cfg::YROW == 1024 && 2 * Cfg::ZROW == 1024, "a piece's halves are 1 KiB apart");
          const bool y = (PC & 1) != 0;
          const void* base = y ? (const void*)(p.Y + (size_t)ks * BK * p.Hin) : (const void*)(p.dZ + (size_t)ks * BK * p.Hout);
          const unsigned lds = lds_addr(dst + (y ? 0 : Cfg::YBYTES) + po[KK][0]);
          glds16x2o_asm_s(y ? yb0[KK] : zb0[KK], y ? yb1[KK] : zb1[KK], base, lds);
        } else {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            if constexpr ((PC & 1) != 0)
              glds16_asm(p.Y + (size_t)ks * BK * p.Hin + yo[KK][j], lds_addr(dst + po[KK][j]));
            else
              glds16_asm(p.dZ + (size_t)ks * BK * p.Hout + zo[KK][j], lds_addr(dst + Cfg::YBYTES + po[KK][j]));
          }
        }
      };
      auto read2 = [&](auto sg, int slot) {
        constexpr int KK = decltype(sg)::value;
        const char* ys = smem + slot * Cfg::STAGE;
        const char* zs = ys + Cfg::YBYTES;
#pragma unroll
        for (int il = 0; il < 8; ++il) a8[il] = tr_frag<YROW>(ys + KK * 32 * YROW + colA[il]);
#pragma unroll
        for (int j = 0; j < 4; ++j) b4[j] = tr_frag<ZROW>(zs + KK * 32 * ZROW + colB[j]);
      };
      // serpentine over (il, j): every two consecutive MFMAs share an operand (independent
      // accumulators: bit-identical); measured -1.0% against il-major rows (tools/variants.py tnserp)
      auto mma2 = [&](auto sg) {
#pragma unroll
        for (int t = 0; t < 32; ++t) {
          const int il = t >> 2, jq = t & 3, j = (il & 1) ? 3 - jq : jq;
          acc[il][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8[il], b4[j], acc[il][j], 0, 0, 0);
        }
      };
      pingpong2_one_tile<2>(nkl, wm, issue2, read2, mma2);
    } else {
    h16x8 af[4], bf[4];
    auto read = [&](auto ph, int slot) {
      constexpr int PH = decltype(ph)::value, KK = PH >> 1, IH = (PH == 1 || PH == 2) ? 1 : 0;
      const char* ys = smem + slot * Cfg::STAGE;
      const char* zs = ys + Cfg::YBYTES;
#pragma unroll
      for (int il = 0; il < 4; ++il) af[il] = tr_frag<YROW>(ys + KK * 32 * YROW + colA[4 * IH + il]);
      if constexpr (PH == 0 || PH == 2) {
#pragma unroll
        for (int j = 0; j < 4; ++j) bf[j] = tr_frag<ZROW>(zs + KK * 32 * ZROW + colB[j]);
      }
    };
    auto mma = [&](auto ph) {
      constexpr int PH = decltype(ph)::value, IH = (PH == 1 || PH == 2) ? 1 : 0;
#pragma unroll
      for (int il = 0; il < 4; ++il)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[4 * IH + il][j] =
              __builtin_amdgcn_mfma_f32_16x16x32_f16(af[il], bf[j], acc[4 * IH + il][j], 0, 0, 0);
    };
    pingpong_tiles<0, 0xA>(true, nkl, wm, issue, read, mma, [](int) {}, [](int) {},
                               [](int) { return false; });
    }
  } else {
    mfma_pipeline<Cfg::S, false, BK / 32, Cfg::YINSTR + Cfg::ZINSTR>(ks_end - ks_begin, acc, stage, frags);
  }

  // native-order slab store: [slice][tile][wave][i*SJ+j][lane] float4
  float4* dst = (float4*)(p.slab + ((size_t)slice * ntile + tile) * Cfg::TILE_FLOATS) +
                (size_t)wave * SI * SJ * 64 + lane;
#pragma unroll
  for (int i = 0; i < SI; ++i)
#pragma unroll
    for (int j = 0; j < SJ; ++j)
      dst[(i * SJ + j) * 64] = float4{acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
}

static int g_tn_tile = 0;
static int g_tn_pipe = -1;  // -1: automatic = 4, two-segment ping-pong (fastest, kernel_bench r06)
void gemm_tn_set_tile(int tile) { g_tn_tile = tile; }
void gemm_tn_set_pipe(int v) { g_tn_pipe = v; }

int tn_choose_tile(int R, int Hin, int Hout) {
  const bool large_ok = (Hin % 256 == 0) && (Hout % 256 == 0);
  if (g_tn_tile == 128 || !large_ok) return 128;
  if (g_tn_tile == 256) return 256;
  // 256x256 tiles when slices of >= 8 K-steps still give >= 512 blocks
  const long blocks = (long)(R / 64 / 8) * (Hin / 256) * (Hout / 256);
  return blocks >= 512 ? 256 : 128;
}

template <class Cfg>
static hipError_t launch_tn(const TnParams& p, hipStream_t s) {
  const int grid = (p.Hin / Cfg::BI) * (p.Hout / Cfg::BJ) * p.splits;
  hipLaunchKernelGGL(gemm_tn_kernel<Cfg>, dim3(grid), dim3(Cfg::THREADS), 0, s, p);
  return hipGetLastError();
}

hipError_t gemm_tn_dw(const TnParams& p, hipStream_t s) {
  if (p.Hin % 128 || p.Hout % 128 || p.R % 64 || p.R <= 0 || p.splits < 1) return hipErrorInvalidValue;
  if (p.tile == 256) {
    if (p.Hin % 256 || p.Hout % 256) return hipErrorInvalidValue;
    switch (g_tn_pipe >= 0 ? g_tn_pipe : 4) {
      case 0: return launch_tn<TnL0>(p, s);
      case 1: return (p.R % 32) ? hipErrorInvalidValue : launch_tn<TnL1>(p, s);
      case 2: return launch_tn<TnL2>(p, s);
      case 3: return launch_tn<TnLPP>(p, s);
      case 4: return launch_tn<TnLPP2>(p, s);
    }
    return hipErrorInvalidValue;
  }
  if (p.tile != 128) return hipErrorInvalidValue;
  return launch_tn<TnSmall>(p, s);
}

// Slab decode (mirrors gemm_tn_kernel): float4 index q within a tile:
//   lane = q & 63, ij = (q>>6) % (SI*SJ) (i = ij / SJ, j = ij % SJ), wave = (q>>6) / (SI*SJ)
//   k = ti*BI + wm*TI + i*16 + 4*(lane>>4) + {0..3},  o = tj*BJ + wn*TJ + j*16 + (lane&15)
template <class Cfg>
__global__ void dw_reduce_kernel(const float4* __restrict__ slab, int splits, int Hin, int Hout,
                                 float* __restrict__ grad, int accumulate,
                                 const float* __restrict__ gscale) {
  constexpr int SUB = Cfg::SI * Cfg::SJ;
  const float inv = gscale ? gscale[1] : 1.0f;  // undo the dZ storage scale (exact: 2^-k)
  const int tiles_j = Hout / Cfg::BJ;
  const int ntile = (Hin / Cfg::BI) * tiles_j;
  constexpr int TQ = Cfg::TILE_FLOATS / 4;
  const int64_t total = (int64_t)ntile * TQ;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total;
       q += (int64_t)gridDim.x * blockDim.x) {
    // fixed split order s = 0, 1, ..., splits - 1; the loads go out U at a time, the last chunk's too (a
    // dependent load per split made the reduce latency-bound: 52 us for 128 splits of a 512^2 slab; 8 in
    // flight and a one-at-a-time tail left width 256's 256 splits at 18 us per layer, 3.5 TB/s)
    constexpr int U = 16;
    float4 w[U];
    const int n1 = splits < U ? splits : U;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (u < n1) w[u] = slab[q + (int64_t)u * total];
    float4 v = w[0];
#pragma unroll
    for (int u = 1; u < U; ++u)
      if (u < n1) { v.x += w[u].x; v.y += w[u].y; v.z += w[u].z; v.w += w[u].w; }
    for (int s = n1; s < splits; s += U) {
      const int n = splits - s < U ? splits - s : U;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (u < n) w[u] = slab[q + (int64_t)(s + u) * total];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (u < n) { v.x += w[u].x; v.y += w[u].y; v.z += w[u].z; v.w += w[u].w; }
    }
    v.x *= inv; v.y *= inv; v.z *= inv; v.w *= inv;
    const int tile = (int)(q / TQ);
    const int within = (int)(q - (int64_t)tile * TQ);
    const int lane = within & 63, blk = within >> 6;
    const int ij = blk % SUB, wave = blk / SUB;
    const int i = ij / Cfg::SJ, j = ij % Cfg::SJ;
    const int wm = wave / Cfg::WN, wn = wave % Cfg::WN;
    const int ti = tile / tiles_j, tj = tile - ti * tiles_j;
    const int k = ti * Cfg::BI + wm * Cfg::TI + i * 16 + 4 * (lane >> 4);
    const int o = tj * Cfg::BJ + wn * Cfg::TJ + j * 16 + (lane & 15);
    float4* out = (float4*)(grad + (size_t)o * Hin + k);
    if (accumulate) {
      float4 a = *out;
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
      *out = a;
    } else {
      *out = v;
    }
  }
}

hipError_t dw_reduce(const float* slab, int splits, int Hin, int Hout, int tile, float* grad,
                     int accumulate, const float* gscale, hipStream_t s) {
  // one wave per block, so that a small slab (H = 256: 16 384 float4 columns) still spreads over every CU
  const int64_t total = (int64_t)Hin * Hout / 4;
  int grid = (int)((total + 63) / 64);
  if (grid > 8192) grid = 8192;
  if (tile == 256) {
    hipLaunchKernelGGL(dw_reduce_kernel<TnLarge>, dim3(grid), dim3(64), 0, s, (const float4*)slab, splits,
                       Hin, Hout, grad, accumulate, gscale);
  } else if (tile == 128) {
    hipLaunchKernelGGL(dw_reduce_kernel<TnSmall>, dim3(grid), dim3(64), 0, s, (const float4*)slab, splits,
                       Hin, Hout, grad, accumulate, gscale);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace siren
