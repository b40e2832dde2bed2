"""Measurement-only variants of the product kernels, kept OUT of the product source: each variant is
a set of textual patches applied to a temporary copy of inr-for-audio_amd/csrc, compiled to
inr-for-audio_amd/libsiren_<name>.so (never loaded by the package; tools/ab_bench.py times it
beside the product library in one process and checks bit-identity).

    python tools/variants.py st_nt fl        # build
    python tools/ab_bench.py --libs base=inr-for-audio_amd/libsiren_hip.so,fl=inr-for-audio_amd/libsiren_fl.so
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "inr-for-audio_amd", "csrc")
sys.path.insert(0, os.path.join(ROOT, "inr-for-audio_amd"))
from buildinfo import SOURCES  # noqa: E402  (the product library's source list)

_ST16 = "  auto st16 = [&](h16* dst, uint4 v) { *(uint4*)dst = v; };"


def _st16_asm(pol: str) -> str:
    # the asm store carries its own s_nop: a VALU write of the data VGPRs must wait a cycle after a
    # 128-bit store, which hipcc's hazard recognizer does not see inside inline asm
    return ("  auto st16 = [&](h16* dst, uint4 v) {\n"
            "    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));\n"
            "    const u32x4 w = u32x4{v.x, v.y, v.z, v.w};\n"
            f"    asm volatile(\"global_store_dwordx4 %0, %1, off {pol}\\n\\ts_nop 1\" ::\"v\"(dst), \"v\"(w) : \"memory\");\n"
            "  };")


_FL_OLD = """#pragma unroll
        for (int pp = 0; pp < SN / 2; ++pp) {
          st16(p.Y + rowoff + npc + pp * 32, yp[pp]);
          st16(p.C + rowoff + npc + pp * 32, cpk[pp]);
          if constexpr (MODE == NT_FWD_SNAKE) st16(p.E + rowoff + npc + pp * 32, epk[pp]);
        }"""
# whole 128-B lines: lanes l and l^8 (rows r, r^8 of the subtile) trade one 16-B piece by DPP
# row_ror:8, so each store instruction writes 8 whole row segments instead of 16 half ones
_FL_NEW = """if constexpr (SN == 4 && MODE == NT_FWD) {
          const bool hi = (lane & 8) != 0;
          const size_t ra = (size_t)(m0 + wm * TM + j * 16 + (lane & 7)) * N + npc + (hi ? 32 : 0);
          auto fl_store = [&](h16* dst, const uint4 (&pc)[SN / 2]) {
            const uint4 send = hi ? pc[0] : pc[1];
            uint4 recv;
            recv.x = __builtin_amdgcn_update_dpp(0, (int)send.x, 0x128, 0xf, 0xf, false);
            recv.y = __builtin_amdgcn_update_dpp(0, (int)send.y, 0x128, 0xf, 0xf, false);
            recv.z = __builtin_amdgcn_update_dpp(0, (int)send.z, 0x128, 0xf, 0xf, false);
            recv.w = __builtin_amdgcn_update_dpp(0, (int)send.w, 0x128, 0xf, 0xf, false);
            st16(dst + ra, hi ? recv : pc[0]);
            st16(dst + ra + (size_t)8 * N, hi ? pc[1] : recv);
          };
          fl_store(p.Y, yp);
          fl_store(p.C, cpk);
        } else {
#pragma unroll
          for (int pp = 0; pp < SN / 2; ++pp) {
            st16(p.Y + rowoff + npc + pp * 32, yp[pp]);
            st16(p.C + rowoff + npc + pp * 32, cpk[pp]);
            if constexpr (MODE == NT_FWD_SNAKE) st16(p.E + rowoff + npc + pp * 32, epk[pp]);
          }
        }"""

# forward epilogue stores through buffer descriptors of the wave's 128-row band (base in SGPRs,
# one 32-bit lane offset, the row subtile in soffset) instead of 64-bit per-lane addresses
_BST_OLD1 = """      float hp[SM];
#pragma unroll
      for (int j = 0; j < SM; ++j) hp[j] = 0.f;"""
_BST_NEW1 = """      float hp[SM];
#pragma unroll
      for (int j = 0; j < SM; ++j) hp[j] = 0.f;
      const size_t obase = (size_t)(m0 + wm * TM) * N + n0;
      const auto rsy = __builtin_amdgcn_make_buffer_rsrc(p.Y + obase, (short)0, TM * N * 2, 0x00020000);
      const auto rsc = __builtin_amdgcn_make_buffer_rsrc(p.C + obase, (short)0, TM * N * 2, 0x00020000);
      const int qv = ((lane & 15) * N + wn * TN + swap16_col(lane)) * 2;
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));"""
_BST_OLD2 = """          st16(p.Y + rowoff + npc + pp * 32, yp[pp]);
          st16(p.C + rowoff + npc + pp * 32, cpk[pp]);"""
_BST_NEW2 = """          if constexpr (MODE == NT_FWD) {
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{yp[pp].x, yp[pp].y, yp[pp].z, yp[pp].w}, rsy, qv + pp * 64,
                                                   j * 16 * N * 2, 0);
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{cpk[pp].x, cpk[pp].y, cpk[pp].z, cpk[pp].w}, rsc,
                                                   qv + pp * 64, j * 16 * N * 2, 0);
          } else {
            st16(p.Y + rowoff + npc + pp * 32, yp[pp]);
            st16(p.C + rowoff + npc + pp * 32, cpk[pp]);
          }"""

# the forward epilogue's pre-activation as packed fp32 FMAs (v_pk_fma_f32: two per instruction)
_PK_OLD = """#pragma unroll
              for (int r = 0; r < 4; ++r) {
                // revolutions: sin(2*pi*x) with x = omega*(z + b)/(2*pi); fract keeps the
                // hardware sin/cos inside their reduced domain for any magnitude.
                const float x = __builtin_amdgcn_fractf(__builtin_fmaf(acc[i][j][r], xs, bb[r]));
                s[r] = __builtin_amdgcn_sinf(x);
                c[r] = __builtin_amdgcn_cosf(x);
              }"""
_PK_NEW = """typedef float f32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
              for (int r = 0; r < 4; r += 2) {
                const f32x2 z2 = __builtin_elementwise_fma(f32x2{acc[i][j][r], acc[i][j][r + 1]}, f32x2{xs, xs},
                                                           f32x2{bb[r], bb[r + 1]});
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                  const float x = __builtin_amdgcn_fractf(z2[q]);
                  s[r + q] = __builtin_amdgcn_sinf(x);
                  c[r + q] = __builtin_amdgcn_cosf(x);
                }
              }"""

# fused head (NT_FWD_HB) cost split: no hand-off (each block uses its own partial for all column
# tiles: WRONG g, timing only)
_HB_WAIT_OLD = """            while ((u = __hip_atomic_load(hpu + (size_t)jt * p.M + m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) ==
                   kHeadPending) {"""
_HB_WAIT_NEW = """            u = __float_as_uint(own) + jt;
            while (polls == 12345) {"""
# no hand-off at all: the partials are neither published nor awaited (WRONG g, timing and write
# attribution only: head_part receives no stores)
_HB_PUB_OLD = """        __hip_atomic_store(hpu + (size_t)tn * p.M + m, own == own ? __float_as_uint(own) : 0x7fc00000u,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);"""
_HB_PUB_NEW = """        if (own == 12345.0f) hpu[(size_t)tn * p.M + m] = __float_as_uint(own);"""

# phase 2 without its dZ stores (the column partials still computed): WRONG dZ, timing only
_HB_ST_OLD = """          st16(p.dZ + (size_t)(mrow0 + j * 16) * N + npc + pp * 32, swap16_pair(dzp[0], dzp[1]));"""
_HB_ST_NEW = """          if (gm[j] == 12345.0f) st16(p.dZ + (size_t)(mrow0 + j * 16) * N + npc + pp * 32, swap16_pair(dzp[0], dzp[1]));"""
# no phase 2 at all (only phase 1 and the hand-off): timing only
_HB_PH2_OLD = """      for (int pp = 0; pp < SN / 2; ++pp) {
        float cs[NQ][2][4];  // [db_L, dw_head, da_L][subtile h][column r]"""
_HB_PH2_NEW = """      for (int pp = 0; pp < (p.n_valid == -7 ? SN / 2 : 0); ++pp) {
        float cs[NQ][2][4];  // [db_L, dw_head, da_L][subtile h][column r]"""

# forward stores folded onto the first 512 rows of Y / C (1 MB each: L2-resident, no HBM write-back):
# WRONG outputs, timing only -- prices the forward's 4.3 GB of output writes against HBM
_L2ST_OLD = """          st16(p.Y + rowoff + npc + pp * 32, yp[pp]);
          st16(p.C + rowoff + npc + pp * 32, cpk[pp]);"""
_L2ST_NEW = """          st16(p.Y + (rowoff & (size_t)(512 * N - 1)) + npc + pp * 32, yp[pp]);
          st16(p.C + (rowoff & (size_t)(512 * N - 1)) + npc + pp * 32, cpk[pp]);"""

# forward epilogue computes everything but issues no stores (a never-true guard keeps the values):
# WRONG outputs, timing only -- the epilogue's VALU alone against its stores
_NOST_NEW = """          if (yp[pp].x == 0x12345u && cpk[pp].y == 0x6789u) {
            st16(p.Y + rowoff + npc + pp * 32, yp[pp]);
            st16(p.C + rowoff + npc + pp * 32, cpk[pp]);
          }"""

# whole 128-B line dZ stores in the NT_DX epilogue (both 16-B pieces of a row subtile computed
# first, then traded as in "fl")
_DXFL_OLD1 = """#pragma unroll
        for (int pp = 0; pp < SN / 2; ++pp) {
          uint2 cpu[2];"""
_DXFL_NEW1 = """        uint4 dzq[SN / 2];
#pragma unroll
        for (int pp = 0; pp < SN / 2; ++pp) {
          uint2 cpu[2];"""
_DXFL_OLD2 = """          if constexpr (MODE == NT_DX || MODE == NT_DX_SNAKE)
            st16(p.dZ + rowoff + npc + pp * 32, swap16_pair(dzp[0], dzp[1]));
        }"""
_DXFL_NEW2 = """          if constexpr (MODE == NT_DX || MODE == NT_DX_SNAKE) dzq[pp] = swap16_pair(dzp[0], dzp[1]);
        }
        if constexpr (MODE == NT_DX && SN == 4) {
          const bool hi = (lane & 8) != 0;
          const size_t ra = (size_t)(m0 + wm * TM + j * 16 + (lane & 7)) * N + npc + (hi ? 32 : 0);
          const uint4 send = hi ? dzq[0] : dzq[1];
          uint4 recv;
          recv.x = __builtin_amdgcn_update_dpp(0, (int)send.x, 0x128, 0xf, 0xf, false);
          recv.y = __builtin_amdgcn_update_dpp(0, (int)send.y, 0x128, 0xf, 0xf, false);
          recv.z = __builtin_amdgcn_update_dpp(0, (int)send.z, 0x128, 0xf, 0xf, false);
          recv.w = __builtin_amdgcn_update_dpp(0, (int)send.w, 0x128, 0xf, 0xf, false);
          st16(p.dZ + ra, hi ? recv : dzq[0]);
          st16(p.dZ + ra + (size_t)8 * N, hi ? dzq[1] : recv);
        } else if constexpr (MODE == NT_DX || MODE == NT_DX_SNAKE) {
#pragma unroll
          for (int pp = 0; pp < SN / 2; ++pp) st16(p.dZ + rowoff + npc + pp * 32, dzq[pp]);
        }"""

# dW GEMM operands from 8 K-steps of the slice only (L2-resident Y and dZ): WRONG dW, timing only --
# prices the dW K-loop's operand latency
_DWL2_OLD = """        const int ks = ks_begin + min(kt, nkl - 1);  // past the slice: a consumed piece re-read"""
_DWL2_NEW = """        const int ks = ks_begin + (min(kt, nkl - 1) & 7);"""

# MFMA issue order inside a ping-pong phase: column subtile (X fragment) outer, so consecutive MFMAs
# share their B operand instead of their A operand (every accumulator keeps its k order:
# bit-identical) -- operand toggling between consecutive MFMAs, timing only
_ORD_OLD = """#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int il = 0; il < 2; ++il)
#pragma unroll
          for (int jl = 0; jl < 4; ++jl) {
            const h16x8 a = NH ? wf1[il][kk] : wf0[il][kk];"""
_ORD_NEW = """#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int jl = 0; jl < 4; ++jl)
#pragma unroll
          for (int il = 0; il < 2; ++il) {
            const h16x8 a = NH ? wf1[il][kk] : wf0[il][kk];"""
_TNORD_OLD = """#pragma unroll
        for (int il = 0; il < 8; ++il)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[il][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8[il], b4[j], acc[il][j], 0, 0, 0);"""
_TNORD_NEW = """#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int il = 0; il < 8; ++il)
            acc[il][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8[il], b4[j], acc[il][j], 0, 0, 0);"""

# the same, serpentine: every consecutive pair of MFMAs shares one operand, across the column
# subtiles and across the two k32 halves (per-accumulator k order unchanged: bit-identical)
_ORD2_NEW = """#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int kk = t >> 3, u = t & 7, jq = u >> 1;
        const int jl = kk ? 3 - jq : jq;
        const int il = ((t >> 1) & 1) ? 1 - (u & 1) : (u & 1);
            const h16x8 a = NH ? wf1[il][kk] : wf0[il][kk];"""

# dW two-segment MFMA order, serpentine over (il, j): consecutive MFMAs share an operand across
# the il boundaries too (bit-identical) -- timing only
_TNSERP_NEW = """#pragma unroll
        for (int t = 0; t < 32; ++t) {
          const int il = t >> 2, jq = t & 3, j = (il & 1) ? 3 - jq : jq;
          acc[il][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8[il], b4[j], acc[il][j], 0, 0, 0);
        }"""

# ping-pong K-loops without the s_setprio around each MFMA cluster (the barriers alone order the
# two wave groups; bit-identical) -- timing only
_PRIO_OLD1 = """      __builtin_amdgcn_s_setprio(1);
      mma(ph);       // each MFMA waits (counted lgkmcnt) only for its fragments
      wait_lgkm0();  // every read of this slot has landed before the barrier that frees it
      __builtin_amdgcn_s_setprio(0);"""
_PRIO_NEW1 = """      mma(ph);
      wait_lgkm0();"""
_PRIO_OLD2 = """      __builtin_amdgcn_s_setprio(1);
      mma(sg);
      __builtin_amdgcn_s_setprio(0);"""
_PRIO_NEW2 = """      mma(sg);"""

# Snake fused last layer: E (dY/da) parked in the dZ_L buffer across the hand-off instead of 64
# VGPRs (the product's 400 B of spills): phase 1 stores each row piece's E where its dZ_L piece
# will go, phase 2 loads it back right before overwriting it with dZ_L (the lines stay in L2, so
# HBM sees the final dZ_L only if they are not evicted in between).  Outputs bit-identical.
_HBS_EZ_OLD1 = """            hp[j] += sv[0] * hw[i].x + sv[1] * hw[i].y + sv[2] * hw[i].z + sv[3] * hw[i].w;
          }
        }
      }"""
_HBS_EZ_NEW1 = """            hp[j] += sv[0] * hw[i].x + sv[1] * hw[i].y + sv[2] * hw[i].z + sv[3] * hw[i].w;
          }
          if constexpr (SNK)
            st16(p.dZ + (size_t)(mrow0 + j * 16) * N + npc + pp * 32,
                 swap16_pair(e16[SNK ? 2 * pp : 0][SNK ? j : 0], e16[SNK ? 2 * pp + 1 : 0][SNK ? j : 0]));
        }
      }"""
_HBS_EZ_OLD2 = """          uint2 dzp[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int i = 2 * pp + h;
            const float4 w4 = *(const float4*)(hw_lds + nq + i * 16);"""
_HBS_EZ_NEW2 = """          uint2 dzp[2];
          uint2 eu[2];
          if constexpr (SNK) unswap16_pair(*(const uint4*)(p.dZ + (size_t)(mrow0 + j * 16) * N + npc + pp * 32), eu[0], eu[1]);
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int i = 2 * pp + h;
            const float4 w4 = *(const float4*)(hw_lds + nq + i * 16);"""
_HBS_EZ_OLD3 = """              const h16x4 eh = as_h4(e16[SNK ? i : 0][SNK ? j : 0]);"""
_HBS_EZ_NEW3 = """              const h16x4 eh = as_h4(eu[h]);"""

# fused last layer, phase 2 rows outermost: both 16-B halves of a dZ_L row segment stored back to back
_HB_JO_OLD = '#pragma unroll\n      for (int pp = 0; pp < SN / 2; ++pp) {\n        float cs[NQ][2][4];  // [db_L, dw_head][subtile h][column r]\n#pragma unroll\n        for (int q = 0; q < NQ; ++q)\n#pragma unroll\n          for (int h = 0; h < 2; ++h)\n#pragma unroll\n            for (int r = 0; r < 4; ++r) cs[q][h][r] = 0.f;\n#pragma unroll\n        for (int j = 0; j < SM; ++j) {\n          uint2 dzp[2];\n#pragma unroll\n          for (int h = 0; h < 2; ++h) {\n            const int i = 2 * pp + h;\n            const float4 w4 = *(const float4*)(hw_lds + nq + i * 16);\n            const float wv[4] = {w4.x, w4.y, w4.z, w4.w};\n            float cf[4], yf[4];\n            const uint4 pk = __builtin_bit_cast(uint4, acc[i][j]);\n            const h16x4 yh = as_h4(uint2{pk.x, pk.y}), ch = as_h4(uint2{pk.z, pk.w});\n#pragma unroll\n            for (int r = 0; r < 4; ++r) {\n              yf[r] = (float)yh[r];\n              cf[r] = (float)ch[r];\n            }\n            float d[4];\n#pragma unroll\n            for (int r = 0; r < 4; ++r) {\n              const float dz = ((gm[j] * wv[r]) * cf[r]) * om;\n              cs[0][h][r] += dz;\n              cs[1][h][r] += gm[j] * yf[r];\n              d[r] = dz * S;\n            }\n            dzp[h] = as_u2(pack4(d[0], d[1], d[2], d[3]));\n          }\n          st16(p.dZ + (size_t)(mrow0 + j * 16) * N + npc + pp * 32, swap16_pair(dzp[0], dzp[1]));\n        }\n#pragma unroll\n        for (int q = 0; q < NQ; ++q)\n#pragma unroll\n          for (int h = 0; h < 2; ++h) {\n            float v[4];\n#pragma unroll\n            for (int r = 0; r < 4; ++r) v[r] = row16_sum(cs[q][h][r]);\n            if ((lane & 15) == 0)\n              *(float4*)(red + (q * Cfg::WM + wm) * BN + wn * TN + (2 * pp + h) * 16 + 4 * (lane >> 4)) =\n                  float4{v[0], v[1], v[2], v[3]};\n          }\n      }\n'
_HB_JO_NEW = "      // rows outermost, both column pairs of a row piece back to back: each 128-B row segment of\n      // dZ_L is then written whole by two consecutive stores (column pairs outermost wrote each\n      // line's halves a pass apart: the HBM writes came to 2.63 GB for the 2.15 GB of dZ_L, PMC)\n      float cs[SN / 2][NQ][2][4];  // [column pair][db_L, dw_head][subtile h][column r]\n#pragma unroll\n      for (int pp = 0; pp < SN / 2; ++pp)\n#pragma unroll\n        for (int q = 0; q < NQ; ++q)\n#pragma unroll\n          for (int h = 0; h < 2; ++h)\n#pragma unroll\n            for (int r = 0; r < 4; ++r) cs[pp][q][h][r] = 0.f;\n#pragma unroll\n      for (int j = 0; j < SM; ++j) {\n#pragma unroll\n        for (int pp = 0; pp < SN / 2; ++pp) {\n          uint2 dzp[2];\n#pragma unroll\n          for (int h = 0; h < 2; ++h) {\n            const int i = 2 * pp + h;\n            const float4 w4 = *(const float4*)(hw_lds + nq + i * 16);\n            const float wv[4] = {w4.x, w4.y, w4.z, w4.w};\n            float cf[4], yf[4];\n            const uint4 pk = __builtin_bit_cast(uint4, acc[i][j]);\n            const h16x4 yh = as_h4(uint2{pk.x, pk.y}), ch = as_h4(uint2{pk.z, pk.w});\n#pragma unroll\n            for (int r = 0; r < 4; ++r) {\n              yf[r] = (float)yh[r];\n              cf[r] = (float)ch[r];\n            }\n            float d[4];\n#pragma unroll\n            for (int r = 0; r < 4; ++r) {\n              const float dz = ((gm[j] * wv[r]) * cf[r]) * om;\n              cs[pp][0][h][r] += dz;\n              cs[pp][1][h][r] += gm[j] * yf[r];\n              d[r] = dz * S;\n            }\n            dzp[h] = as_u2(pack4(d[0], d[1], d[2], d[3]));\n          }\n          st16(p.dZ + (size_t)(mrow0 + j * 16) * N + npc + pp * 32, swap16_pair(dzp[0], dzp[1]));\n        }\n      }\n#pragma unroll\n      for (int pp = 0; pp < SN / 2; ++pp)\n#pragma unroll\n        for (int q = 0; q < NQ; ++q)\n#pragma unroll\n          for (int h = 0; h < 2; ++h) {\n            float v[4];\n#pragma unroll\n            for (int r = 0; r < 4; ++r) v[r] = row16_sum(cs[pp][q][h][r]);\n            if ((lane & 15) == 0)\n              *(float4*)(red + (q * Cfg::WM + wm) * BN + wn * TN + (2 * pp + h) * 16 + 4 * (lane >> 4)) =\n                  float4{v[0], v[1], v[2], v[3]};\n          }\n"

VARIANTS = {
    "noprio": {"gemm_pipeline.h": [(_PRIO_OLD1, _PRIO_NEW1), (_PRIO_OLD2, _PRIO_NEW2)]},
    "tnserp": {"gemm_tn.hip": [(_TNORD_OLD, _TNSERP_NEW)]},
    "ord2": {"gemm_nt.hip": [(_ORD_OLD, _ORD2_NEW)]},
    "ord": {"gemm_nt.hip": [(_ORD_OLD, _ORD_NEW)], "gemm_tn.hip": [(_TNORD_OLD, _TNORD_NEW)]},
    "dw_l2": {"gemm_tn.hip": [(_DWL2_OLD, _DWL2_NEW)]},
    "dxfl": {"gemm_nt.hip": [(_DXFL_OLD1, _DXFL_NEW1), (_DXFL_OLD2, _DXFL_NEW2)]},
    "fl_dxfl": {"gemm_nt.hip": [(_FL_OLD, _FL_NEW), (_DXFL_OLD1, _DXFL_NEW1), (_DXFL_OLD2, _DXFL_NEW2)]},
    "st_none": {"gemm_nt.hip": [(_L2ST_OLD, _NOST_NEW)]},
    "fl_nt": {"gemm_nt.hip": [(_ST16, _st16_asm("nt")), (_FL_OLD, _FL_NEW)]},  # whole-line non-temporal
    "st_l2": {"gemm_nt.hip": [(_L2ST_OLD, _L2ST_NEW)]},
    "hb_nowait": {"gemm_nt.hip": [(_HB_WAIT_OLD, _HB_WAIT_NEW)]},
    "hb_jouter": {"gemm_nt.hip": [(_HB_JO_OLD, _HB_JO_NEW)]},
    "hbs_ez": {"gemm_nt.hip": [(_HBS_EZ_OLD1, _HBS_EZ_NEW1), (_HBS_EZ_OLD2, _HBS_EZ_NEW2), (_HBS_EZ_OLD3, _HBS_EZ_NEW3)]},
    "hb_nopub": {"gemm_nt.hip": [(_HB_WAIT_OLD, _HB_WAIT_NEW), (_HB_PUB_OLD, _HB_PUB_NEW)]},
    "hb_nopub_nostore": {"gemm_nt.hip": [(_HB_WAIT_OLD, _HB_WAIT_NEW), (_HB_PUB_OLD, _HB_PUB_NEW),
                                         (_HB_ST_OLD, _HB_ST_NEW)]},
    "hb_nostore": {"gemm_nt.hip": [(_HB_ST_OLD, _HB_ST_NEW)]},
    "hb_noph2": {"gemm_nt.hip": [(_HB_PH2_OLD, _HB_PH2_NEW)]},
    "pkfma": {"gemm_nt.hip": [(_PK_OLD, _PK_NEW)]},
    "bst": {"gemm_nt.hip": [(_BST_OLD1, _BST_NEW1), (_BST_OLD2, _BST_NEW2)]},
    "st_sc1": {"gemm_nt.hip": [(_ST16, _st16_asm("sc1"))]},          # write-through epilogue stores
    "st_nt": {"gemm_nt.hip": [(_ST16, _st16_asm("nt"))]},            # non-temporal epilogue stores
    "st_sc0sc1": {"gemm_nt.hip": [(_ST16, _st16_asm("sc0 sc1"))]},
    "fl": {"gemm_nt.hip": [(_FL_OLD, _FL_NEW)]},                     # whole-line forward stores
}


# Snake dX epilogue: Cprev / Eprev read non-temporally (streamed past L2), so that the two 2 GB
# epilogue streams do not evict the K-loop's X / W tiles (NT_DX_SNAKE fetched 2.4x its operands)
_DXS_NT_HELPER_OLD = "  auto st16 = [&](h16* dst, uint4 v) { *(uint4*)dst = v; };"
_DXS_NT_HELPER_NEW = (_DXS_NT_HELPER_OLD + """
  auto ldnt = [](const h16* src) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_nontemporal_load((const u32x4*)src);
    return uint4{v.x, v.y, v.z, v.w};
  };""")
_DXS_NT_OLD1 = """          ce_in[j][0] = *(const uint4*)(p.Cprev + off);
          ce_in[j][1] = *(const uint4*)(p.Eprev + off);"""
_DXS_NT_NEW1 = """          ce_in[j][0] = ldnt(p.Cprev + off);
          ce_in[j][1] = ldnt(p.Eprev + off);"""
_DXS_NT_OLD2 = """                cq[jj] = *(const uint4*)(p.Cprev + off);
                eq[jj] = *(const uint4*)(p.Eprev + off);"""
_DXS_NT_NEW2 = """                cq[jj] = ldnt(p.Cprev + off);
                eq[jj] = ldnt(p.Eprev + off);"""
VARIANTS["dxs_nt"] = {"gemm_nt.hip": [(_DXS_NT_HELPER_OLD, _DXS_NT_HELPER_NEW), (_DXS_NT_OLD1, _DXS_NT_NEW1),
                                      (_DXS_NT_OLD2, _DXS_NT_NEW2)]}

# the fused last layer with the plain 16-row x 64-B dZ_L stores (before the whole-line scratch)
VARIANTS["hbplain"] = {"gemm_nt.hip": [("""                                            MODE == NT_FWD_HB || MODE == NT_FWD_HB_TANH);""",
                                        """                                            false);""")]}


# the EARLY tile-boundary schedule (gemm_pipeline.h pingpong2_tiles) for dX and dX0 too
VARIANTS["early_dx"] = {"gemm_nt.hip": [("SIREN_NT_EARLY != 0 || nt_is_hb(MODE)>(",
                                         "SIREN_NT_EARLY != 0 || nt_is_hb(MODE) || MODE == NT_DX || MODE == NT_DX0>(")]}

# the Snake / Tanh forward with 16-row store pieces at every K (the product takes whole lines at K <= 512)
VARIANTS["actplain"] = {"gemm_nt.hip": [("(Cfg::PP && p.K <= 512)", "(Cfg::PP && p.K <= 0)")]}

# the first layer's Y0 / C0 stores non-temporal
VARIANTS["ffnt"] = {"elementwise.hip": [
    ("    *(h16x8*)(Y0 + m * ld + n) = yv;\n    if constexpr (STORE_C) *(h16x8*)(C0 + m * ld + n) = cv;",
     "    __builtin_nontemporal_store(yv, (h16x8*)(Y0 + m * ld + n));\n"
     "    if constexpr (STORE_C) __builtin_nontemporal_store(cv, (h16x8*)(C0 + m * ld + n));")]}


# LDS-DMA issue one statement per DMA (siren_common.h SIREN_GLDS_PAIR 0: the round-5 issue path; the
# product issues a staging piece's two DMAs under one M0 value)
VARIANTS["glds0"] = {}
# plain (write-back) whole-line epilogue stores instead of non-temporal ones (gemm_nt.hip SIREN_NT_STNT)
VARIANTS["stnt0"] = {}
# the whole-line epilogue stores with `sc1` (inline asm, saddr form): gfx950 drops an sc1-stored line from
# the XCD's L2 instead of keeping it (MI355X_MICROARCH.md store table) -- do 8 MB of Y / C per tile round
# stop evicting W and X?  (asm stores are invisible to hipcc's vmcnt counting: its waits only get stricter;
# the s_nop covers the store-data VGPR write hazard hipcc cannot see inside asm, as _st16_asm's)
_STSC1 = ('      stl((h16*)(ub + (size_t)(16 * q) * LD + lq), line[q]);',
          '      { typedef unsigned u32x4 __attribute__((ext_vector_type(4)));\n'
          '        asm volatile("global_store_dwordx4 %0, %1, %2 sc1\\n\\ts_nop 1" :: "v"(lq), "v"(__builtin_bit_cast(u32x4, line[q])),\n'
          '                     "s"(ub + (size_t)(16 * q) * LD) : "memory"); }')
VARIANTS["stsc1"] = {"gemm_nt.hip": [_STSC1]}
# PROBE (wrong outputs, timing only): group 0 (waves 0-3) issues every LDS-DMA and stores nothing, group 1
# (waves 4-7) stores its own lines twice (its rows and group 0's: the same bytes) and never waits on vmcnt
# in the K-loop -- the forward's K-loop waits then no longer sit behind the epilogue's stores in any
# wave's in-order vmcnt.  Prices that coupling (10.8 k cycles per tile) before an LDS
# hand-off of group 0's outputs is built.  Non-EARLY K-loop only (the plain forward).
VARIANTS["dmag0"] = {"gemm_nt.hip": [
    ("""    int urow[4][2];
    unsigned pdst[4][2];""",
     """    int urow[4][2], urowp[4][2];
    unsigned pdst[4][2], pdstp[4][2];"""),
    ("""        urow[pc][j] = lr0 * K * 2;
        pdst[pc][j] = ((pc & 1) ? 0u : (unsigned)Cfg::XBYTES) + (unsigned)(lr0 * ROWB);
      }""",
     """        urow[pc][j] = lr0 * K * 2;
        pdst[pc][j] = ((pc & 1) ? 0u : (unsigned)Cfg::XBYTES) + (unsigned)(lr0 * ROWB);
        const int qr0 = (2 * (wave + 4) + j) * 8;
        const int lq0 = (pc & 1) ? (qr0 >> 6) * 128 + (qr0 & 63) + 64 * hf : (qr0 >> 5) * 64 + (qr0 & 31) + 32 * hf;
        urowp[pc][j] = lq0 * K * 2;
        pdstp[pc][j] = ((pc & 1) ? 0u : (unsigned)Cfg::XBYTES) + (unsigned)(lq0 * ROWB);
      }"""),
    ("""        glds16x2o_asm_s(lane_src, lane_src8, (const char*)src + urow[PC][0], lds_addr(dst + pdst[PC][0]));
      } else {""",
     """        if (wm == 0) {
          glds16x2o_asm_s(lane_src, lane_src8, (const char*)src + urow[PC][0], lds_addr(dst + pdst[PC][0]));
          glds16x2o_asm_s(lane_src, lane_src8, (const char*)src + urowp[PC][0], lds_addr(dst + pdstp[PC][0]));
        }
      } else {"""),
    ("""      stl((h16*)(ub + (size_t)(16 * q) * LD + lq), line[q]);
    }
  };""",
     """      if (wm == 1) {
        stl((h16*)(ub + (size_t)(16 * q) * LD + lq), line[q]);
        stl((h16*)(ub - (size_t)256 * LD + (size_t)(16 * q) * LD + lq), line[q]);
      }
    }
  };"""),
  ],
  "gemm_pipeline.h": [
    ("""    if constexpr (EARLY) {
    issue(0, 1, 1, phase_t<3>{});
    wait_vmcnt<10>();  // K-tile 0's pieces 0..2 have landed (K0 p3, K1 p0..3 younger)
  } else {
    wait_vmcnt<8>();  // K-tile 0's pieces 0..2 (and the older ones) have landed
  }""".replace("    if constexpr (EARLY) {", "  if constexpr (EARLY) {"),
     """  if constexpr (EARLY) {
    issue(0, 1, 1, phase_t<3>{});
    wait_vmcnt<10>();  // K-tile 0's pieces 0..2 have landed (K0 p3, K1 p0..3 younger)
  } else {
    if (grp == 0) wait_vmcnt<16>();
  }"""),
    ("""      constexpr bool R = RELAXED || (SG == 0 && RELAXED_A);
      wait_vmcnt<R ? 8 + E : 8>();""",
     """      if (grp == 0) wait_vmcnt<16>();"""),
  ]}
# its store half alone (both groups issue their DMAs and wait as in the product): group 1 stores its lines
# twice, group 0 none (wrong outputs, timing only) -- dmag0 minus this = the DMA / store decoupling
VARIANTS["st1x2"] = {"gemm_nt.hip": [VARIANTS["dmag0"]["gemm_nt.hip"][3]]}
VARIANTS["lswap"] = {}
# every ping-pong NT kernel with the EARLY tile boundary (the product takes it for the fused last layer and
# dX0 only): round 5 measured the plain forward +2.3% at cfg2 and -2.3% at cfg4 -- a K-dependent choice?
VARIANTS["early"] = {}
DEFINES = {"glds0": ("SIREN_GLDS_PAIR=0",), "stnt0": ("SIREN_NT_STNT=0",), "lswap": ("SIREN_LINES_SWAP=1",),
           "early": ("SIREN_NT_EARLY=1",)}

# whole-line dZ stores in the dX into a Snake layer at K <= 512 (round 5's parked patch; adopted in the
# product in round 6, so this patch only applies to a round-5 tree: kept as the record of the A/B)
VARIANTS["dxsl"] = {"gemm_nt.hip": [
    ("(ACTL && MODE == NT_FWD_TANH && !HEAD));", "(ACTL && (MODE == NT_FWD_TANH || MODE == NT_DX_SNAKE) && !HEAD));"),
    ("""      auto piece = [&](auto jc, auto ppc, const uint4& cpv, const uint4& epv) {""",
     """      uint4 dzrow[SN / 2];  // NT_DX_SNAKE with whole-line stores (Lay::LINES): a row piece's two 16-B pieces
      auto piece = [&](auto jc, auto ppc, const uint4& cpv, const uint4& epv) {"""),
    ("""        if constexpr (MODE == NT_DX || MODE == NT_DX_SNAKE)
          st16(p.dZ + rowoff + npc + pp * 32, swap16_pair(dzp[0], dzp[1]));
      };""",
     """        if constexpr (MODE == NT_DX_SNAKE && Lay::LINES) {
          dzrow[pp] = swap16_pair(dzp[0], dzp[1]);
          if constexpr (pp == SN / 2 - 1) lines_out(p.dZ, mrow0 + j * 16, n0 + wn * TN, dzrow);
        } else if constexpr (MODE == NT_DX || MODE == NT_DX_SNAKE) {
          st16(p.dZ + rowoff + npc + pp * 32, swap16_pair(dzp[0], dzp[1]));
        }
      };"""),
    ("""    case NT_DX_SNAKE: return launch_nt<Cfg, NT_DX_SNAKE, false>(p, s, persistent);""",
     """    case NT_DX_SNAKE:
      return (Cfg::PP && p.K <= 512) ? launch_nt<Cfg, NT_DX_SNAKE, false, true>(p, s, persistent)
                                     : launch_nt<Cfg, NT_DX_SNAKE, false>(p, s, persistent);"""),
]}


def build(name: str, extra_defines=()) -> str:
    extra_defines = (*DEFINES.get(name, ()), *extra_defines)
    patches = VARIANTS[name]
    out = os.path.join(ROOT, "inr-for-audio_amd", f"libsiren_{name}.so")
    with tempfile.TemporaryDirectory() as tmp:
        for f in os.listdir(CSRC):
            shutil.copy(os.path.join(CSRC, f), tmp)
        for f, reps in patches.items():
            p = os.path.join(tmp, f)
            s = open(p).read()
            for old, new in reps:
                if old not in s:
                    raise SystemExit(f"variant {name}: patch target not found in {f}")
                s = s.replace(old, new)
            open(p, "w").write(s)
        capi = os.path.join(tmp, "capi.hip")
        s = open(capi).read().replace('"../../include/siren_hip.h"', f'"{ROOT}/include/siren_hip.h"')
        open(capi, "w").write(s)
        cmd = [os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"), "--offload-arch=gfx950", "-O3", "-std=c++17",
               "-fPIC", "-shared", "-ffp-contract=off", *[f"-D{d}" for d in extra_defines],
               *[os.path.join(tmp, f) for f in SOURCES], "-o", out]
        subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
    return out


if __name__ == "__main__":
    for nm in sys.argv[1:]:
        print(build(nm))
