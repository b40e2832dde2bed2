// Forward SineLayer GEMM, one wave per SIMD on 256x256 tiles (SIREN_OPT_NT_PIPE 6).  MEASUREMENT
// OPTION, not the product: bit-identical to the ping-pong forward, 2.76 vs 2.30 ms (the K loop alone
// 2.06 vs 1.59: issue-bound with one wave per SIMD, and the 64-B rows split every 128-B line across
// two K-tiles).  The reasoning it was built on:
//
//   Y = sin(omega (X W^T + b)),  C = cos(omega (X W^T + b))          -- models.py:114-115
//
// Why: one wave's vector issue is the binding budget of these GEMMs -- an
// MFMA 16x16x32 holds the SIMD's issue for 8 of its 16 cycles, an LDS-DMA piece costs ~60 issue
// cycles, and the ping-pong kernel's two waves per SIMD pay that issue twice over, plus 8 barriers
// per K-tile.  Here ONE wave per SIMD holds a 128x128 accumulator tile in the AGPR file (256 of
// its 512 registers), so a 256x256 tile needs only 4 waves: per 64 MFMAs a wave issues 8 LDS-DMA
// pieces and 16 fragment reads (pipe 5's 128x256 tile needed 12 pieces), with one barrier per
// K-tile.  BK 32 (64-B staged rows), a 4-stage ring (128 KiB): K-tile kt + 4 is issued into kt's
// stage as soon as every wave is past kt (its fragments were read during kt - 1), three K-tiles
// ahead of use.  The epilogue runs at the tile's end as in the ping-pong kernel (same arithmetic,
// same lane layout), so Y and C are bit-identical to it.
#include "gemm_pipeline.h"
#include "siren_common.h"
#include "siren_kernels.h"

namespace siren {
namespace {

constexpr int kBM = 256, kBN = 256, kBK = 32, kROWB = 2 * kBK;  // 64-B staged rows
constexpr int kSM = 8, kSN = 8;                                  // wave tile 128 x 128
constexpr int kXB = kBM * kROWB, kWB = kBN * kROWB;              // 16 + 16 KiB per K-tile
constexpr int kSTAGE = kXB + kWB, kNST = 4;
constexpr int kBIAS = kNST * kSTAGE;
constexpr int kLDS = kBIAS + 4 * 1024;
constexpr int kPIECES = kSTAGE / 1024 / 4;  // LDS-DMA instructions (16 rows x 64 B) per wave per K-tile

// 64-B rows hold 4 16-B chunks: chunk c of row r sits in slot c ^ ((r >> 2) & 3), so the 16 rows a
// ds_read_b128 quarter-wave reads (one chunk each) cover all 64 banks once
__device__ __forceinline__ int swz64(int r, int c) { return c ^ ((r >> 2) & 3); }

struct Acc {
  f32x4 v[kSN][kSM];
};
struct Frag {
  h16x8 a[kSN], b[kSM];
};

template <int DG>
__global__ __launch_bounds__(256, 1) void nt_fwd_big(NtParams p) {
  __shared__ __attribute__((aligned(16))) char smem[kLDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int K = p.K, N = p.N;
  const int nk = K / kBK;  // a multiple of 4 (host-checked): K-tile kt of every tile uses stage kt & 3
  const int tn_shift = __builtin_ctz(N / kBN);
  const int ntiles = (p.M / kBM) << tn_shift;
  const int G = gridDim.x;
  const int bp = xcd_remap(blockIdx.x, G);
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
  // LDS-DMA piece i of this wave: i < 4 X rows 16 (wave + 4 i) .. +15, i >= 4 W rows 16 (wave + 4 (i - 4));
  // lane moves 16 B of row lane / 4, chunk swizzled on the source side
  const unsigned lane_src = (unsigned)(((lane >> 2) * K + swz64(lane >> 2, lane & 3) * 8) * 2);
  auto issue = [&](const h16* xb, const h16* wb, int kt, int stage) {
    const unsigned st = lds_addr(smem) + (unsigned)(stage * kSTAGE);
#pragma unroll
    for (int i = 0; i < kPIECES; ++i) {
      const int row = 16 * (wave + 4 * (i & 3));
      const uint64_t src = (uint64_t)(i < 4 ? xb : wb) + (uint64_t)row * (K * 2) + (uint64_t)kt * kROWB;
      // (readfirstlane returns int: widen through unsigned, or an address with bit 31 set sign-extends)
      const uint64_t su = ((uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(src >> 32)) << 32) |
                          (uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)src);
      glds16_asm_s(lane_src, (const void*)su, st + (i < 4 ? 0u : (unsigned)kXB) + (unsigned)(row * kROWB));
    }
  };
  const int koff = (lane & 15) * kROWB + (swz64(lane & 15, lane >> 4) << 4);
  auto frags = [&](int stage, Frag& f) {
    const char* xsb = smem + stage * kSTAGE;
    const char* wsb = xsb + kXB;
#pragma unroll
    for (int i = 0; i < kSN; ++i) f.a[i] = *(const h16x8*)(wsb + (wn * 128 + i * 16) * kROWB + koff);
#pragma unroll
    for (int j = 0; j < kSM; ++j) f.b[j] = *(const h16x8*)(xsb + (wm * 128 + j * 16) * kROWB + koff);
  };
  // serpentine over (j, i) so consecutive MFMAs share an operand; every accumulator takes its
  // K-tiles in order (bit-identical)
  auto mma = [&](Acc& acc, const Frag& f, auto zero) {
#pragma unroll
    for (int j = 0; j < kSM; ++j)
#pragma unroll
      for (int ii = 0; ii < kSN; ++ii) {
        const int i = (j & 1) ? kSN - 1 - ii : ii;
        if constexpr (decltype(zero)::value)
          acc.v[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f.a[i], f.b[j], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        else
          acc.v[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f.a[i], f.b[j], acc.v[i][j], 0, 0, 0);
      }
  };
  // ---- epilogue: acc.v[i][j][r] = out[m0 + 128 wm + 16 j + (lane & 15)][n0 + 128 wn + 16 i + 4 (lane >> 4) + r],
  // the ping-pong kernel's NT_FWD arithmetic and 16-B row pieces (gemm_nt.hip)
  auto epilogue = [&](int g, const Acc& acc) {
    int m0, n0;
    tile_of(g, m0, n0);
    const int nq = n0 + wn * 128 + 4 * (lane >> 4);
    const size_t base = (size_t)(m0 + wm * 128 + (lane & 15)) * N + n0 + wn * 128 + swap16_col(lane);
#pragma unroll
    for (int j = 0; j < kSM; ++j) {
#pragma unroll
      for (int pp = 0; pp < kSN / 2; ++pp) {
        uint2 ys[2], cs[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int i = 2 * pp + h;
          const float4 b4 = *(const float4*)(bias_lds + nq + i * 16);
          const float bb[4] = {b4.x * xs, b4.y * xs, b4.z * xs, b4.w * xs};
          float s[4], c[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float x = __builtin_amdgcn_fractf(__builtin_fmaf(acc.v[i][j][r], xs, bb[r]));
            s[r] = __builtin_amdgcn_sinf(x);
            c[r] = __builtin_amdgcn_cosf(x);
          }
          ys[h] = as_u2(pack4(s[0], s[1], s[2], s[3]));
          cs[h] = as_u2(pack4(c[0], c[1], c[2], c[3]));
        }
        if constexpr ((DG & 2) == 0) {
          const size_t off = base + (size_t)(j * 16) * N + pp * 32;
          *(uint4*)(p.Y + off) = swap16_pair(ys[0], ys[1]);
          *(uint4*)(p.C + off) = swap16_pair(cs[0], cs[1]);
        } else {
          asm volatile("" ::"v"(ys[0]), "v"(ys[1]), "v"(cs[0]), "v"(cs[1]));
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // one row block at a time (no hoisted accumulator reads)
    }
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
  auto set_tile = [&](int i) {
    bases(g_cur, x0, w0);
    if (i + 1 < my) bases(g_cur + G, x1, w1);
    else { x1 = x0; w1 = w0; }  // past the end: re-read this tile's rows (never consumed)
  };
  set_tile(0);
#pragma unroll
  for (int s = 0; s < kNST; ++s) issue(x0, w0, s, s);
  wait_vmcnt<3 * kPIECES>();
  wait_lgkm0();  // and the bias vector's LDS stores
  __builtin_amdgcn_s_barrier();
  Frag f0, f1;
  frags(0, f0);

  // one K-tile: K-tile kt + 1 has landed (counted for this wave, the barrier for every wave), every
  // wave is past kt - 1 ... and read kt's fragments during kt - 1, so kt's stage takes kt + 4; then
  // kt's MFMAs with kt + 1's fragment reads under them.  WAIT: younger vector-memory ops allowed at the
  // wait -- 2 K-tiles of pieces, or 63 right after an epilogue (its 64 stores sit in between: the
  // first of them, issued a whole epilogue earlier, and the older pieces must be done)
  auto ktile = [&](Acc& acc, auto st, auto zero, const Frag& fc, Frag& fn, int kt, bool after_epi) {
    constexpr int ST = decltype(st)::value;
    if (after_epi) wait_vmcnt<63>();
    else wait_vmcnt<2 * kPIECES>();
    wait_lgkm0();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 4 < nk) issue(x0, w0, kt + 4, ST);
    else issue(x1, w1, kt + 4 - nk, ST);
    __builtin_amdgcn_sched_barrier(0);
    frags((ST + 1) & 3, fn);
    mma(acc, fc, zero);
    // the fragment reads first, then the MFMAs with the reads' waits between them
    __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 64, 0);
    __builtin_amdgcn_sched_barrier(0);
  };
  Acc acc;
  for (int i = 0; i < my; ++i) {
    const bool ae = i > 0 && DG == 0;  // (the measurement variants store nothing)
    // K-tiles 0..3 (stages 0..3; the first three wait past the previous epilogue's stores)
    ktile(acc, std::integral_constant<int, 0>{}, std::true_type{}, f0, f1, 0, ae);
    ktile(acc, std::integral_constant<int, 1>{}, std::false_type{}, f1, f0, 1, ae);
    ktile(acc, std::integral_constant<int, 2>{}, std::false_type{}, f0, f1, 2, ae);
    ktile(acc, std::integral_constant<int, 3>{}, std::false_type{}, f1, f0, 3, false);
    for (int kt = 4; kt < nk; kt += 4) {
      ktile(acc, std::integral_constant<int, 0>{}, std::false_type{}, f0, f1, kt, false);
      ktile(acc, std::integral_constant<int, 1>{}, std::false_type{}, f1, f0, kt + 1, false);
      ktile(acc, std::integral_constant<int, 2>{}, std::false_type{}, f0, f1, kt + 2, false);
      ktile(acc, std::integral_constant<int, 3>{}, std::false_type{}, f1, f0, kt + 3, false);
    }
    if constexpr ((DG & 1) == 0) {
      epilogue(g_cur, acc);
    } else {  // keep every accumulator live (timing only)
      float t = 0.f;
#pragma unroll
      for (int ii = 0; ii < kSN; ++ii)
#pragma unroll
        for (int j = 0; j < kSM; ++j) t += acc.v[ii][j][0] + acc.v[ii][j][3];
      if (t == 1234.5f) p.Y[tid] = (h16)t;
    }
    if (i + 1 < my) {
      g_cur += G;
      set_tile(i + 1);
    }
  }
  wait_vmcnt<0>();
}

}  // namespace

bool gemm_nt_big_ok(const NtParams& p) {
  const int tn = p.N / kBN;
  return p.K % (4 * kBK) == 0 && p.K >= 4 * kBK && p.N % kBN == 0 && (tn == 1 || tn == 2 || tn == 4) &&
         p.M % kBM == 0 && p.M > 0;
}

hipError_t gemm_nt_big(const NtParams& p, int grid, int diag, hipStream_t s) {
  if (!gemm_nt_big_ok(p) || grid <= 0) return hipErrorInvalidValue;
  const int ntiles = (p.M / kBM) * (p.N / kBN);
  const int g = grid < ntiles ? grid : ntiles;
#ifdef SIREN_DIAG
  if (diag & 1024) hipLaunchKernelGGL(nt_fwd_big<1>, dim3(g), dim3(256), 0, s, p);
  else if (diag & 2048) hipLaunchKernelGGL(nt_fwd_big<2>, dim3(g), dim3(256), 0, s, p);
  else hipLaunchKernelGGL(nt_fwd_big<0>, dim3(g), dim3(256), 0, s, p);
#else
  if (diag) return hipErrorInvalidValue;
  hipLaunchKernelGGL(nt_fwd_big<0>, dim3(g), dim3(256), 0, s, p);
#endif
  return hipGetLastError();
}

}  // namespace siren
