// Measurement only: variants of the head backward stream (elementwise.hip head_bwd_kernel) at
// the cfg2 shape (2^20 rows x 1024): reads C, Y (fp16) and g, writes dZ (fp16) and per-block
// column partials of db and dw_head.  Variants: rows per block, row unroll, non-temporal
// loads of the read-once C / Y.  Prints ms per launch and the HBM rate of the 6 GB stream.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro/head_bwd_bench.hip -o /tmp/hbb && /tmp/hbb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef _Float16 h16;
typedef _Float16 hv8 __attribute__((ext_vector_type(8)));

template <int ROWS, int UNROLL, bool NT>
__global__ __launch_bounds__(256) void hb_kernel(const h16* __restrict__ C, const h16* __restrict__ Y,
                                                 const float* __restrict__ g, const float* __restrict__ w,
                                                 float omega, float S, int H, h16* __restrict__ dZ,
                                                 float* __restrict__ db_part, float* __restrict__ dw_part) {
  constexpr int V = 8;
  __shared__ float red[2][256 * V];
  const int hq = H / V;
  const int cq = threadIdx.x % hq, rg = threadIdx.x / hq, nrg = blockDim.x / hq;
  const int n = cq * V;
  float wv[V], db[V], dw[V];
#pragma unroll
  for (int k = 0; k < V; ++k) {
    wv[k] = w[n + k];
    db[k] = dw[k] = 0.f;
  }
  const long m0 = (long)blockIdx.x * ROWS;
#pragma unroll UNROLL
  for (int r = rg; r < ROWS; r += nrg) {
    const long m = m0 + r;
    const float gm = g[m];
    hv8 c, yv;
    if constexpr (NT) {
      c = __builtin_nontemporal_load((const hv8*)(C + m * H + n));
      yv = __builtin_nontemporal_load((const hv8*)(Y + m * H + n));
    } else {
      c = *(const hv8*)(C + m * H + n);
      yv = *(const hv8*)(Y + m * H + n);
    }
    hv8 out;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const float dz = ((gm * wv[k]) * (float)c[k]) * omega;
      db[k] += dz;
      dw[k] += gm * (float)yv[k];
      out[k] = (h16)(dz * S);
    }
    *(hv8*)(dZ + m * H + n) = out;
  }
#pragma unroll
  for (int k = 0; k < V; ++k) {
    red[0][threadIdx.x * V + k] = db[k];
    red[1][threadIdx.x * V + k] = dw[k];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < H; c += blockDim.x) {
    const int q = c / V, k = c % V;
    float a = 0.f, b = 0.f;
    for (int gi = 0; gi < nrg; ++gi) {
      a += red[0][(gi * hq + q) * V + k];
      b += red[1][(gi * hq + q) * V + k];
    }
    db_part[(size_t)blockIdx.x * H + c] = a;
    dw_part[(size_t)blockIdx.x * H + c] = b;
  }
}

int main() {
  const int R = 1 << 20, H = 1024;
  h16 *C, *Y, *dZ;
  float *g, *w, *dbp, *dwp;
  hipMalloc(&C, (size_t)R * H * 2);
  hipMalloc(&Y, (size_t)R * H * 2);
  hipMalloc(&dZ, (size_t)R * H * 2);
  hipMalloc(&g, R * 4);
  hipMalloc(&w, H * 4);
  hipMalloc(&dbp, (size_t)(R / 128) * H * 4);
  hipMalloc(&dwp, (size_t)(R / 128) * H * 4);
  hipMemset(C, 0x11, (size_t)R * H * 2);
  hipMemset(Y, 0x22, (size_t)R * H * 2);
  hipMemset(g, 0, R * 4);
  hipMemset(w, 0, H * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  struct V { const char* name; void (*fn)(const h16*, const h16*, const float*, const float*, h16*, float*, float*); };
#define VAR(ROWS, UN, NT)                                                                                       \
  V{#ROWS "_u" #UN "_nt" #NT, [](const h16* c, const h16* y, const float* gg, const float* ww, h16* dz, float* a, \
                                float* b) {                                                                    \
      hipLaunchKernelGGL((hb_kernel<ROWS, UN, NT>), dim3((1 << 20) / ROWS), dim3(256), 0, 0, c, y, gg, ww, 30.f,  \
                         1.f, 1024, dz, a, b);                                                                 \
    }}
  std::vector<V> vs = {VAR(128, 4, false), VAR(128, 8, false), VAR(128, 4, true), VAR(256, 4, false),
                       VAR(256, 8, false), VAR(256, 8, true), VAR(512, 8, false), VAR(512, 8, true)};
  const int reps = 10;
  for (int round = 0; round < 3; ++round)
    for (auto& v : vs) {
      v.fn(C, Y, g, w, dZ, dbp, dwp);
      hipEventRecord(e0);
      for (int i = 0; i < reps; ++i) v.fn(C, Y, g, w, dZ, dbp, dwp);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      ms /= reps;
      if (round == 2) printf("%-16s %.4f ms  %.2f TB/s\n", v.name, ms, 6.0 * R * H / (ms * 1e-3) / 1e12);
    }
  return 0;
}
