// NT GEMM for the SIREN hidden layers on gfx950 bf16 MFMA with fused epilogues.
//
//   acc[m][n] = sum_k X[m][k] * W[n][k]        (X: [M][K] bf16, W: [N][K] bf16, fp32 acc)
//
// Three epilogues (template MODE):
//   NT_FWD : a = omega*(acc + b[n]);  Y = sin a, C = cos a   (bf16 out)     -- models.py:114-115
//            optional HEAD: per-row partial of sum_n Y[m][n]*w_head[n]      -- models.py:374-381
//   NT_DX  : dz = (acc * Cprev[m][n]) * omega_prev  (bf16 out) + column partial sums (db)
//            = autograd of sin(omega*linear) for the layer below            -- models.py:114-115
//   NT_DX0 : same as NT_DX but the layer below is the fp32 first layer: its cos is
//            recomputed exactly in fp32 from (t, W0, b0) and only the column partial sums
//            of dz*t_j (dW0) and dz (db0) are written; dZ0 never reaches HBM.
//
// Tile 128x128x64, 256 threads = 4 waves in a 2(M) x 2(N) grid, each wave 64x64 as 4x4
// v_mfma_f32_16x16x32_bf16 tiles.  Operands are staged HBM->LDS by LDS-DMA
// (global_load_lds_dwordx4), double-buffered (64 KiB, 2 blocks/CU), with an XOR swizzle
// applied on the SOURCE address so that the ds_read_b128 fragment reads are bank-conflict
// free (cdna_hip_programming.md §5.4 rule 21 / T2).
//
// MFMA operand roles are swapped (A := W rows, B := X rows) so each lane ends up holding 4
// consecutive output COLUMNS of one row: 8-byte contiguous bf16 stores, and per-row bias
// loads as one float4.
#include "siren_common.h"
#include "siren_kernels.h"

namespace siren {
namespace nt {
constexpr int BM = 128, BN = 128, BK = 64, THREADS = 256;
constexpr int OPND_BYTES = BM * BK * 2;       // 16 KiB: one 128x64 bf16 tile
constexpr int STAGE_BYTES = 2 * OPND_BYTES;   // X tile + W tile
constexpr int LDS_BYTES = 2 * STAGE_BYTES;    // double buffer = 64 KiB
constexpr int RED_STRIDE = BN + 4;            // padded fp32 row for the epilogue reductions
}  // namespace nt

template <int MODE, bool HEAD>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(NtParams p) {
  using namespace nt;
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int K = p.K, N = p.N;
  const int tiles_n = N / BN;
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = g / tiles_n, tn = g - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- LDS-DMA staging addresses -------------------------------------------------
  // Each wave moves rows [32*wave, 32*wave+32) of both tiles in 4 instructions of 8 rows.
  // Lane L of an instruction lands at LDS row r = L>>3, 16-B slot s = L&7 and must carry
  // the logical 16-B chunk c = s ^ (r & 7) of that row (source-side swizzle).
  const int srow = lane >> 3;
  const int schunk = (lane & 7) ^ srow;
  const bf16* xg = p.X + (size_t)(m0 + wave * 32 + srow) * K + schunk * 8;
  const bf16* wg = p.W + (size_t)(n0 + wave * 32 + srow) * K + schunk * 8;
  const size_t row8 = (size_t)8 * K;

  auto stage = [&](int kt, int buf) {
    char* xs = smem + buf * STAGE_BYTES + wave * 32 * 128;
    char* ws = xs + OPND_BYTES;
    const bf16* xk = xg + kt * BK;
    const bf16* wk = wg + kt * BK;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      glds16(xk + j * row8, lds_ptr(xs + j * 1024));
      glds16(wk + j * row8, lds_ptr(ws + j * 1024));
    }
  };

  // ---- fragment read offsets --------------------------------------------------------
  // 16x16x32 operand: lane holds row (lane&15), k = 8*(lane>>4) .. +7 of a 32-deep half.
  // Physical slot of logical chunk c in row r is c ^ (r&7); r&7 == lane&7 here.
  const int frow = lane & 15;
  int koff[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
    koff[kk] = frow * 128 + ((((lane >> 4) + 4 * kk) ^ (lane & 7)) << 4);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    const char* xs = smem + cur * STAGE_BYTES;
    const char* ws = xs + OPND_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[4], bfm[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = *(const bf16x8*)(ws + (wn * 64 + i * 16) * 128 + koff[kk]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bfm[j] = *(const bf16x8*)(xs + (wm * 64 + j * 16) * 128 + koff[kk]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfm[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue ------------------------------------------------------------------
  // acc[i][j][r] = out[m][n] with m = m0 + wm*64 + j*16 + (lane&15),
  //                              n = n0 + wn*64 + i*16 + 4*(lane>>4) + r.
  const int nq = n0 + wn * 64 + 4 * (lane >> 4);
  const int mrow0 = m0 + wm * 64 + (lane & 15);
  float* red = (float*)smem;  // reuse LDS (all waves passed the final barrier)

  if constexpr (MODE == NT_FWD) {
    const float xs = p.omega * kInv2Pi;
    float4 bias[4], hw[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bias[i] = *(const float4*)(p.bias + nq + i * 16);
      if constexpr (HEAD) hw[i] = *(const float4*)(p.head_w + nq + i * 16);
    }
    float hp[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const size_t rowoff = (size_t)(mrow0 + j * 16) * N;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float bb[4] = {bias[i].x, bias[i].y, bias[i].z, bias[i].w};
        float s[4], c[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // revolutions: sin(2*pi*x) with x = omega*(z + b)/(2*pi); fract keeps the
          // hardware sin/cos inside their reduced domain for any magnitude.
          const float x = __builtin_amdgcn_fractf((acc[i][j][r] + bb[r]) * xs);
          s[r] = __builtin_amdgcn_sinf(x);
          c[r] = __builtin_amdgcn_cosf(x);
        }
        *(bf16x4*)(p.Y + rowoff + nq + i * 16) = pack4(s[0], s[1], s[2], s[3]);
        *(bf16x4*)(p.C + rowoff + nq + i * 16) = pack4(c[0], c[1], c[2], c[3]);
        if constexpr (HEAD)
          hp[j] += s[0] * hw[i].x + s[1] * hw[i].y + s[2] * hw[i].z + s[3] * hw[i].w;
      }
    }
    if constexpr (HEAD) {
      // lanes l, l^16, l^32, l^48 hold the same row: fold them, then the two wn waves.
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        hp[j] += __shfl_xor(hp[j], 16, 64);
        hp[j] += __shfl_xor(hp[j], 32, 64);
      }
      if (lane < 16) {
#pragma unroll
        for (int j = 0; j < 4; ++j) red[wn * BM + wm * 64 + j * 16 + lane] = hp[j];
      }
      __syncthreads();
      if (tid < BM) p.head_part[(size_t)tn * p.M + m0 + tid] = red[tid] + red[BM + tid];
    }
  } else {
    // column sums over this block's 128 rows (db / dW0 partials)
    float cs[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[i][r] = 0.f;

    if constexpr (MODE == NT_DX) {
      const float om = p.omega;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const size_t rowoff = (size_t)(mrow0 + j * 16) * N;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bf16x4 cp = *(const bf16x4*)(p.Cprev + rowoff + nq + i * 16);
          float dz[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            dz[r] = (acc[i][j][r] * (float)cp[r]) * om;
            cs[i][r] += dz[r];
          }
          *(bf16x4*)(p.dZ + rowoff + nq + i * 16) = pack4(dz[0], dz[1], dz[2], dz[3]);
        }
      }
      // LDS transpose-reduce: red[32 row-lanes][128 cols]
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *(float4*)(red + (wm * 16 + (lane & 15)) * RED_STRIDE + wn * 64 + i * 16 + 4 * (lane >> 4)) =
            float4{cs[i][0], cs[i][1], cs[i][2], cs[i][3]};
      __syncthreads();
      if (tid < BN) {
        float s = 0.f;
#pragma unroll 8
        for (int r = 0; r < 32; ++r) s += red[r * RED_STRIDE + tid];
        p.colsum_part[(size_t)tm * N + n0 + tid] = s;
      }
    } else {  // NT_DX0: first layer, in_dim in {1, 2}
      const float om0 = p.omega;
      const int in_dim = p.in_dim;
      float w0[4][4][2], b0[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = nq + i * 16 + r;
          b0[i][r] = p.b0[n];
          w0[i][r][0] = p.W0[n * in_dim];
          w0[i][r][1] = (in_dim > 1) ? p.W0[n * in_dim + 1] : 0.f;
        }
      float cw[4][4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) cw[i][r][0] = cw[i][r][1] = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = mrow0 + j * 16;
        const float t0 = p.t[(size_t)m * in_dim];
        const float t1 = (in_dim > 1) ? p.t[(size_t)m * in_dim + 1] : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            // exact fp32 restatement of the first-layer pre-activation (see first_fwd)
            float z;
            if (in_dim == 1) z = __builtin_fmaf(t0, w0[i][r][0], b0[i][r]);
            else z = __builtin_fmaf(t1, w0[i][r][1], t0 * w0[i][r][0]) + b0[i][r];
            const float a = om0 * z;
            const float dz = (acc[i][j][r] * cosf(a)) * om0;
            cs[i][r] += dz;
            cw[i][r][0] += dz * t0;
            cw[i][r][1] += dz * t1;
          }
      }
      // three reductions through LDS: db0, dW0[:,0], dW0[:,1]
      const int nred = 1 + in_dim;
      for (int q = 0; q < nred; ++q) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (q == 0) ? cs[i][r] : cw[i][r][q - 1];
          *(float4*)(red + (wm * 16 + (lane & 15)) * RED_STRIDE + wn * 64 + i * 16 + 4 * (lane >> 4)) =
              float4{v[0], v[1], v[2], v[3]};
        }
        __syncthreads();
        if (tid < BN) {
          float s = 0.f;
#pragma unroll 8
          for (int r = 0; r < 32; ++r) s += red[r * RED_STRIDE + tid];
          // partial layout [tm][q][N]: q=0 -> db0, q=1+j -> dW0[:, j]
          p.colsum_part[((size_t)tm * nred + q) * N + n0 + tid] = s;
        }
        __syncthreads();
      }
    }
  }
}

template <int MODE, bool HEAD>
static hipError_t launch_nt(const NtParams& p, hipStream_t s) {
  const int grid = (p.M / nt::BM) * (p.N / nt::BN);
  hipLaunchKernelGGL((gemm_nt_kernel<MODE, HEAD>), dim3(grid), dim3(nt::THREADS), 0, s, p);
  return hipGetLastError();
}

hipError_t gemm_nt(int mode, bool head, const NtParams& p, hipStream_t s) {
  if (p.M % nt::BM || p.N % nt::BN || p.K % nt::BK || p.M <= 0) return hipErrorInvalidValue;
  switch (mode) {
    case NT_FWD: return head ? launch_nt<NT_FWD, true>(p, s) : launch_nt<NT_FWD, false>(p, s);
    case NT_DX: return launch_nt<NT_DX, false>(p, s);
    case NT_DX0:
      if (p.in_dim < 1 || p.in_dim > 2) return hipErrorInvalidValue;
      return launch_nt<NT_DX0, false>(p, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace siren
