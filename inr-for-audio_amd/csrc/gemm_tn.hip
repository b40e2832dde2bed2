// TN GEMM for the SIREN weight gradient on gfx950 bf16 MFMA, split-K over coordinates.
//
//   dW[o][k] = sum_n dZ[n][o] * Y[n][k]          (autograd addmm backward, models.py:114-115)
//
// The reduction index n is the SLOW index of both operands, so both tiles are staged
// row-major ([n][col], coalesced LDS-DMA) and the MFMA fragments are gathered with the
// gfx950 hardware transpose read ds_read_b64_tr_b16 (cdna_hip_programming.md T10).
// Roles: MFMA A := Y (i = k), B := dZ (j = o), so each lane's 4 accumulator registers are 4
// consecutive k of one o row -> the reduce kernel writes float4 rows of dW.
//
// Each block owns one 128x128 tile of dW and a contiguous slice of the coordinates; the
// fp32 partial tile goes to a slab in MFMA-native order (1 KiB contiguous per store
// instruction).  dw_reduce sums the slices in a fixed order (deterministic).
#include "siren_common.h"
#include "siren_kernels.h"

namespace siren {
namespace tn {
constexpr int BI = 128, BJ = 128, BK = 64, THREADS = 256;
constexpr int ROW_BYTES = 256;                 // 128 bf16 columns
constexpr int OPND_BYTES = BK * ROW_BYTES;     // 16 KiB
constexpr int STAGE_BYTES = 2 * OPND_BYTES;
constexpr int LDS_BYTES = 2 * STAGE_BYTES;     // 64 KiB
constexpr int TILE_FLOATS = BI * BJ;
}  // namespace tn

// Chunk swizzle of the [64][128] image: physical 16-B chunk = c ^ f(r).  With
// h(r) = (r&3) | ((r>>3)&1)<<2 and f = 2h, the 8 rows a 32-lane half touches in one
// transposed read occupy 8 distinct 32-B bank slots (conflict-free).
__device__ __forceinline__ int tn_swz(int r) { return ((r & 3) | (((r >> 3) & 1) << 2)) << 1; }

// One 16x16x32 operand fragment = two ds_read_b64_tr_b16: rows 8g+0..3 then 8g+4..7 of the
// [n][col] image (the second block sits 4 rows = 4*256 B further down).
typedef short s16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ bf16x8 tr_frag(const char* p) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(p));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(p + 4 * 256));
  const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

__global__ __launch_bounds__(256, 2) void gemm_tn_kernel(TnParams p) {
  using namespace tn;
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;  // wm -> k (i), wn -> o (j)
  const int tiles_i = p.Hin / BI, tiles_j = p.Hout / BJ;
  const int ntile = tiles_i * tiles_j;
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int slice = g / ntile, tile = g - slice * ntile;
  const int ti = tile / tiles_j, tj = tile - ti * tiles_j;
  const int k0 = ti * BI, o0 = tj * BJ;

  const int nks = p.R / BK;
  const int ks_begin = (int)(((int64_t)slice * nks) / p.splits);
  const int ks_end = (int)(((int64_t)(slice + 1) * nks) / p.splits);

  // staging: instruction j of wave w writes rows r = 16w + 4j + (lane>>4), slot lane&15
  const int srow_base = wave * 16 + (lane >> 4);
  auto src_off = [&](int j, int ld, int col0) -> size_t {
    const int r = srow_base + 4 * j;
    const int c = (lane & 15) ^ tn_swz(r);
    return (size_t)r * ld + col0 + c * 8;
  };
  size_t yoff[4], zoff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    yoff[j] = src_off(j, p.Hin, k0);
    zoff[j] = src_off(j, p.Hout, o0);
  }
  auto stage = [&](int ks, int buf) {
    char* ys = smem + buf * STAGE_BYTES + wave * 16 * ROW_BYTES;
    char* zs = ys + OPND_BYTES;
    const bf16* yb = p.Y + (size_t)ks * BK * p.Hin;
    const bf16* zb = p.dZ + (size_t)ks * BK * p.Hout;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      glds16(yb + yoff[j], lds_ptr(ys + j * 1024));
      glds16(zb + zoff[j], lds_ptr(zs + j * 1024));
    }
  };

  // transposed-read addresses: group g = lane>>4, lane-in-group 4q+p supplies row q
  // (+4 for the second read) of the 4-row block starting at 8g (+32 for kk=1), columns
  // col0 + 4p .. +3.
  // Row r = 32kk + 8grp + 4h + q, so tn_swz(r) = 2*(q | (grp&1)<<2) is the same for every
  // (kk, h): the swizzle only permutes the 16-B column chunks per lane.
  const int grp = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int fl = tn_swz(8 * grp + q);
  const int rbase = (8 * grp + q) * ROW_BYTES + ((pp & 1) << 3);
  int colA[4], colB[4];  // byte offset of logical chunk (8w + 2sub + (pp>>1)) after swizzle
#pragma unroll
  for (int sub = 0; sub < 4; ++sub) {
    colA[sub] = rbase + (((8 * wm + 2 * sub + (pp >> 1)) ^ fl) << 4);
    colB[sub] = rbase + (((8 * wn + 2 * sub + (pp >> 1)) ^ fl) << 4);
  }

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (ks_begin < ks_end) {
    stage(ks_begin, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int ks = ks_begin; ks < ks_end; ++ks) {
      const int cur = (ks - ks_begin) & 1;
      if (ks + 1 < ks_end) stage(ks + 1, cur ^ 1);
      const char* ys = smem + cur * STAGE_BYTES;
      const char* zs = ys + OPND_BYTES;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[4], bfz[4];
        const int kofs = kk * 32 * ROW_BYTES;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          af[s] = tr_frag(ys + kofs + colA[s]);
          bfz[s] = tr_frag(zs + kofs + colB[s]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfz[j], acc[i][j], 0, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }

  // native-order slab store: [slice][tile][wave][i*4+j][lane] float4
  float4* dst = (float4*)(p.slab + ((size_t)slice * ntile + tile) * TILE_FLOATS) + (size_t)wave * 16 * 64 + lane;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      dst[(i * 4 + j) * 64] = float4{acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
}

hipError_t gemm_tn_dw(const TnParams& p, hipStream_t s) {
  if (p.Hin % tn::BI || p.Hout % tn::BJ || p.R % tn::BK || p.R <= 0 || p.splits < 1)
    return hipErrorInvalidValue;
  const int grid = (p.Hin / tn::BI) * (p.Hout / tn::BJ) * p.splits;
  hipLaunchKernelGGL(gemm_tn_kernel, dim3(grid), dim3(tn::THREADS), 0, s, p);
  return hipGetLastError();
}

// Slab decode (must mirror gemm_tn_kernel): float4 index q within a tile:
//   lane = q & 63, ij = (q>>6) & 15 (i = ij>>2, j = ij&3), wave = q >> 10 (wm = wave>>1, wn = wave&1)
//   k = ti*128 + wm*64 + i*16 + 4*(lane>>4) + {0..3},  o = tj*128 + wn*64 + j*16 + (lane&15)
__global__ void dw_reduce_kernel(const float4* __restrict__ slab, int splits, int Hin, int Hout,
                                 float* __restrict__ grad, int accumulate) {
  const int tiles_j = Hout / tn::BJ;
  const int ntile = (Hin / tn::BI) * tiles_j;
  const int64_t total = (int64_t)ntile * (tn::TILE_FLOATS / 4);
  const int64_t stride = total;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total;
       q += (int64_t)gridDim.x * blockDim.x) {
    float4 v = slab[q];
    for (int s = 1; s < splits; ++s) {
      const float4 w = slab[q + s * stride];
      v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
    }
    const int tile = (int)(q >> 12);
    const int within = (int)(q & 4095);
    const int lane = within & 63, ij = (within >> 6) & 15, wave = within >> 10;
    const int ti = tile / tiles_j, tj = tile - ti * tiles_j;
    const int k = ti * 128 + (wave >> 1) * 64 + (ij >> 2) * 16 + 4 * (lane >> 4);
    const int o = tj * 128 + (wave & 1) * 64 + (ij & 3) * 16 + (lane & 15);
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

hipError_t dw_reduce(const float* slab, int splits, int Hin, int Hout, float* grad, int accumulate,
                     hipStream_t s) {
  const int64_t total = (int64_t)(Hin / tn::BI) * (Hout / tn::BJ) * (tn::TILE_FLOATS / 4);
  int grid = (int)((total + 255) / 256);
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(dw_reduce_kernel, dim3(grid), dim3(256), 0, s, (const float4*)slab, splits, Hin,
                     Hout, grad, accumulate);
  return hipGetLastError();
}

}  // namespace siren
