// Internal host-side launchers for the SIREN gfx950 kernels (not the public C-ABI;
// that lives in include/siren_hip.h and capi.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace siren {

typedef _Float16 h16;  // activation / weight-shadow / gradient storage (fp16)

// NT_FWD_SNAKE / NT_FWD_TANH: Linear + Snake / Tanh forward epilogues; NT_DX_SNAKE: dX into
// a Snake layer (derivative D and d/da E of the layer below), SURVEY §8 f3
// NT_DX0_SNAKE: dX into a Linear + Snake first layer (first_linear=True): dz = acc * D0, partials
// of db0, dW0 (x t_j) and da0 = sum acc * E0
// NT_FWD_HB: the last hidden SineLayer fused with the head, the loss gradient and the head backward
// (training only): writes dZ_L x S instead of Y_L / C_L (see gemm_nt.hip)
// NT_FWD_HB_SNAKE / NT_FWD_HB_TANH: the same for a Linear + Snake / Linear + Tanh last layer
// (run.py:30's default train() stack ends in Snake layers)
enum NtMode { NT_FWD = 0, NT_DX = 1, NT_DX0 = 2, NT_FWD_SNAKE = 3, NT_FWD_TANH = 4, NT_DX_SNAKE = 5,
              NT_DX0_SNAKE = 6, NT_FWD_HB = 7, NT_FWD_HB_SNAKE = 8, NT_FWD_HB_TANH = 9 };
constexpr bool nt_is_hb(int m) { return m == NT_FWD_HB || m == NT_FWD_HB_SNAKE || m == NT_FWD_HB_TANH; }
constexpr bool nt_is_fwd(int m) { return m == NT_FWD || m == NT_FWD_SNAKE || m == NT_FWD_TANH || nt_is_hb(m); }
// forward modes that evaluate a Snake (they stage a and 1/a in LDS)
constexpr bool nt_is_snake_fwd(int m) { return m == NT_FWD_SNAKE || m == NT_FWD_HB_SNAKE; }

struct NtParams {
  const h16* X;  // [M][K]
  const h16* W;  // [N][K]
  int M, N, K;
  int ld;         // row stride of the [M][*] operands and outputs: gemm_nt sets it (= N; column
                  // windows of a layer wider than 1024 keep the layer's width)
  int tile;       // 128 or 256 (nt_choose_tile): partials are per tile-row / tile-column
  float omega;  // FWD: this layer's omega; DX: omega of the layer below; DX0: omega_0
  // NT_FWD
  const float* bias;    // [N]
  h16* Y;              // [M][N]
  h16* C;              // [M][N]  sine: cos; Snake: dY/dz = 1 + sin(2az); Tanh: 1 - y^2
  h16* E;              // [M][N]  Snake only: dY/da = (z sin(2az) - sin^2(az)/a) / a
  const float* act_a;  // [N]     Snake only: a (per output column)
  const float* head_w;  // [N]          (HEAD only)
  float* head_part;     // [N/128][M]   (HEAD only)
  // NT_DX / NT_DX0
  const h16* Cprev;    // [M][N]  cos of the layer below (NT_DX); D of a Snake / 1-y^2 of a Tanh
  const h16* Eprev;    // [M][N]  NT_DX_SNAKE: E of the Snake layer below
  h16* dZ;             // [M][N]  (NT_DX)
  float* colsum_part;   // NT_DX: [M/128][N];  NT_DX0: [M/128][1+in][N];  NT_DX_SNAKE: [M/128][2][N];
                        // NT_DX0_SNAKE: [M/128][2+in][N] (db0, dW0[:, j], da0)
  // NT_DX0 (Cprev = cos of the first layer)
  const float* t;       // [M][in]
  int in_dim;
  const float* gscale;  // NT_DX / NT_DX0: {S, 1/S} -- column partials are multiplied by 1/S
                        // (null = unscaled)
  int diag;             // SIREN_OPT_NT_DIAG ablation bits (SIREN_DIAG measurement builds only)
  // ping-pong K-loop only: caller-owned tile-queue counter set of kTileqInts ints (null = the
  // static walk b, b + G, ...); gemm_nt zeroes it on the stream before each queue launch
  int* tileq;
  // NT_FWD_HB* (with head_w / head_part; gscale = {S, 1/S} set beforehand by grad_scale_bound, or
  // for a Snake last layer by grad_scale from the previous launch's max|g|; dZ = dZ_L x S;
  // colsum_part [M/256][2][N] = partials of db_L and dw_head, Snake [M/256][3][N] + da_L):
  // head_loss's inputs and outputs for the band's rows
  const float* target;  // [M]
  const float* b_head;  // [1]
  float* out;           // [M]
  float* g;             // [M] dLoss/d(head linear output)
  float* sse_part;      // [M/256]
  float* gsum_part;     // [M/256]
  int n_valid, loss_mode;
  float gfac, head_omega;
  float* gmax_part;     // [M/256] max|g| per band (NT_FWD_HB*; null = not written)
  // NT_FWD_HB*: a hand-off wait that gives up (spin_limit polls) adds 1 here (GuardState::stalls;
  // null = only the NaN partial); hb_fault: SIREN_OPT_HB_FAULT injection (SIREN_DIAG builds only)
  int* stall;
  int spin_limit, hb_fault;
};
constexpr int kTileqInts = 768;  // == SIREN_TILEQ_INTS (include/siren_hip.h)

int nt_choose_tile(int M, int N);
hipError_t gemm_nt(int mode, bool head, const NtParams& p, hipStream_t s);
// the forward (NT_FWD, no head) with its epilogue under the next tile's MFMAs: one wave per SIMD,
// 128x256 tiles, K / 64 in {4, 8, 16}, N / 256 in {1, 2, 4} (gemm_nt1.hip; SIREN_OPT_NT_PIPE 5)
bool gemm_nt_one_ok(const NtParams& p);
hipError_t gemm_nt_one(const NtParams& p, int grid, int diag, bool overlap, hipStream_t s);  // pipe 5 / 7
// the forward (NT_FWD, no head) with one wave per SIMD on 256x256 tiles, BK 32, 4-stage ring:
// K % 128 == 0, N / 256 in {1, 2, 4} (gemm_nt2.hip; SIREN_OPT_NT_PIPE 6)
bool gemm_nt_big_ok(const NtParams& p);
hipError_t gemm_nt_big(const NtParams& p, int grid, int diag, hipStream_t s);
// NT_FWD_HB is available for this shape under the current tile / K-loop settings
// also false when the fused launch's grid could not be co-resident (occupancy x CUs < grid)
bool gemm_nt_head_fusable(int M, int N, hipStream_t s, int mode = NT_FWD_HB);
void gemm_nt_set_tile(int tile);  // 0 = auto, 128, 256 (A/B measurement)
void gemm_tn_set_tile(int tile);
void gemm_nt_set_pipe(int v);     // 256x256 K-loop: 4 ping-pong (default), 1 persistent, 0 one tile per block
void gemm_tn_set_pipe(int v);     // 256x256 K-loop variant (TnL0..TnL2)
void gemm_nt_set_grid_cap(int cap);  // persistent grid size override (0 = #CUs)
bool gemm_nt_set_diag(int bits);     // SIREN_OPT_NT_DIAG (false: not a SIREN_DIAG build)
void gemm_nt_set_queue(int on);       // SIREN_OPT_NT_QUEUE: dynamic tile queue (ping-pong K-loop)
bool gemm_nt_set_hb_fault(int v);     // SIREN_OPT_HB_FAULT (false: not a SIREN_DIAG build)
struct TnParams {
  const h16* Y;   // [R][Hin]   layer input (A role: dW column index k)
  const h16* dZ;  // [R][Hout]  layer pre-activation gradient (B role: dW row index o)
  int R, Hin, Hout;
  int splits;
  int tile;        // 128 or 256 (tn_choose_tile); dw_reduce must be given the same value
  float* slab;     // [splits][Hout*Hin] fp32 in MFMA-native order (see dw_reduce)
};

int tn_choose_tile(int R, int Hin, int Hout);
hipError_t gemm_tn_dw(const TnParams& p, hipStream_t s);
// grad[o][k] (+)= sum_s slab[s]  (grad row-major [Hout][Hin])
// (scaled by gscale[1] = 1/S when gscale is non-null: dZ carries the backward scale S)
hipError_t dw_reduce(const float* slab, int splits, int Hin, int Hout, int tile, float* grad,
                     int accumulate, const float* gscale, hipStream_t s);

// elementwise / reduction kernels (elementwise.hip)
hipError_t coords_fill(float* t, int64_t rows, int64_t offset, int64_t n_total, hipStream_t s);
hipError_t coords_fill_grid(float* xy, int64_t rows, int64_t offset, int64_t height, int width, hipStream_t s);

// fp16 backward range guard (include/siren_hip.h siren_guard)
struct GuardState {
  int32_t flag, headroom, clean, overflows, headroom0;
  int32_t stalls;  // fused last layer: timed-out hand-off waits (sticky; the host clears it)
};
constexpr int kHeadroomDefault = 6;      // grad_scale target exponent without a guard
constexpr int kHeadroomDrop = 4;         // per rejected step (S / 16)
constexpr int kHeadroomMin = -14;        // below this a non-finite gradient is passed through
constexpr int kHeadroomGrowAfter = 1000; // clean steps before headroom grows back by one
// true when the step's gradients hold a non-finite value, the loss is finite (so it is the
// fp16 dZ storage that overflowed, not a diverged fit) and the headroom can still drop
__device__ __forceinline__ bool guard_overflow(const GuardState* g, const float* sse) {
  return g && g->flag && __builtin_isfinite(sse[0]) && g->headroom > kHeadroomMin;
}
// a fused last layer's hand-off timed out: the step's loss and gradients are void
__device__ __forceinline__ bool guard_stalled(const GuardState* g) { return g && g->stalls != 0; }
// the update is skipped (Adam leaves p, m, v untouched; the scheduler does not step)
__device__ __forceinline__ bool guard_skip(const GuardState* g, const float* sse) {
  return guard_stalled(g) || guard_overflow(g, sse);
}
// sse (nullable): the reduced [sse, stall slot] pair of siren_grads (a non-zero stall slot marks the guard stalled)
hipError_t guard_check(const float* g, int64_t n, GuardState* guard, hipStream_t s, const float* sse = nullptr);
// a0 / E0 non-null: Linear + Snake first layer (first_linear=True); C0 null: Y0 only
hipError_t first_fwd(const float* t, int in_dim, const float* W0, const float* b0, float omega0,
                     int R, int H, h16* Y0, h16* C0, hipStream_t s, const float* a0 = nullptr,
                     h16* E0 = nullptr);
hipError_t head_loss(const float* head_part, int nparts, int R, const float* b_head, const float* y,
                     int n_valid, float gfac, float* out, float* g, float* sse_part,
                     float* gsum_part, float* gmax_part, hipStream_t s, float head_omega = 0.f,
                     int loss_mode = 0);
hipError_t gmax_partials(const float* g, int R, float* gmax_part, hipStream_t s);
hipError_t head_sine_chain(const float* head_part, int nparts, int R, const float* b_head, float omega, float* g,
                           hipStream_t s);
// S before the forward (NT_FWD_HB): from a loss-independent bound of max|g| -- ymax_part holds
// (n_valid+255)/256 max|target| partials; act_bound = |dY/dz| bound of the last layer
hipError_t grad_scale_bound(const float* ymax_part, int nparts, const float* w_head, const float* b_head, int H,
                            float gfac, float head_omega, int loss_mode, float act_bound, float* gscale,
                            hipStream_t s, const GuardState* guard = nullptr);
// gscale[0] = S (dZ storage scale), gscale[1] = 1/S; from (R+255)/256 max|g| partials
hipError_t grad_scale(const float* gmax_part, int nparts, const float* w_head, int H, float omega,
                      float* gscale, hipStream_t s, const GuardState* guard = nullptr);
// E != null (Snake last layer): da_part[R/128][H] = partial sums of g*w_head*E
hipError_t head_bwd(const h16* C, const h16* Y, const float* g, const float* w_head, float omega,
                    int R, int H, const float* gscale, h16* dZ, float* db_part, float* dwh_part,
                    const h16* E, float* da_part, hipStream_t s);
// out[c*out_stride] (+)= sum_r part[r*row_stride + c]; tmp holds >= 64*ncols floats
hipError_t col_reduce(const float* part, int64_t row_stride, int nrows, int ncols, float* out,
                      int out_stride, int accumulate, float* tmp, hipStream_t s);
// up to kMaxColSegs col_reduce of one partial-row layout in one launch pair (results identical to
// one col_reduce per segment); tmp holds >= n*64*ncols floats
constexpr int kMaxColSegs = 4;
struct ColSegs {
  const float* src[kMaxColSegs];
  float* out[kMaxColSegs];
  int out_stride[kMaxColSegs];
  int n;
};
hipError_t col_reduce_multi(const ColSegs& sg, int64_t row_stride, int nrows, int ncols, int accumulate, float* tmp,
                            hipStream_t s);

// unfused fp32 layers (layer_fp32.hip): lone SineLayer / Linear / Snake / Tanh modules
enum Fp32Act { FP32_IDENTITY = 0, FP32_SIN = 1, FP32_TANH = 2, FP32_SNAKE = 3 };  // == siren_fp32_act
hipError_t fp32_linear(const float* x, int64_t rows, int in, int out, const float* W, const float* b, float omega,
                       float* pre, hipStream_t s);
hipError_t fp32_act(int act, const float* x, int64_t rows, int cols, const float* a, float* y, hipStream_t s);
hipError_t fp32_act_bwd(int act, const float* x, int64_t rows, int cols, const float* a, const float* gy,
                        float* gpre, float* da_prod, hipStream_t s);
hipError_t fp32_linear_bwd(const float* x, int64_t rows, int in, int out, const float* W, float omega, float* gpre,
                           float* gx, float* gW, float* gb, float* slab, int splits, float* tmp, hipStream_t s);

// KAN (kan.hip): fp32, grid_size 5, spline_order 3 (9 A-columns per input)
// fused layer kernels (the bases are recomputed in LDS; A and dA never reach HBM)
hipError_t kan_fwd_fused(const float* X, const float* grid, const float* W, int64_t N, int in, int out, float* Y,
                         hipStream_t s);
int64_t kan_dw_slab_floats(int in, int out, int splits);
// split-K over the rows: at most max_splits slabs of out x 9 in floats
hipError_t kan_dw_fused(const float* X, const float* grid, const float* G, int64_t N, int in, int out,
                        int64_t max_splits, float* slab, float* dW, hipStream_t s);
hipError_t kan_dx_fused(const float* X, const float* grid, const float* Gout, const float* WT, int64_t N, int in,
                        int out, float* Gin, hipStream_t s);
// dW and Gin of a layer with out <= 64 in one pass (bases and G rows read once)
hipError_t kan_bwd_fused(const float* X, const float* grid, const float* G, const float* WT, int64_t N, int in, int out,
                         int64_t max_splits, float* slab, float* dW, float* Gin, hipStream_t s);
// the last layer (out = 1, in <= 64): wave-per-row forward (inference)
hipError_t kan_head_fwd(const float* X, const float* grid, const float* W, int64_t N, int in, float* Y, hipStream_t s);
// the last layer's forward + MSE gradient + backward in one pass (out = 1, in <= 64); *nparts
// squared-error partials
hipError_t kan_head_train(const float* X, const float* grid, const float* W, const float* y, int64_t N, int in,
                          int64_t n_valid, float gfac, int64_t slots, int64_t max_parts, float* out, float* g,
                          float* sse_part, float* slab, float* dW, float* Gin, int* nparts, hipStream_t s);
// W = [base_w | spline_w * scaler] as [out][9 in], and (WT != null) its transpose [9 in][out]
hipError_t kan_combine(const float* base_w, const float* spline_w, const float* scaler, int out, int in, float* W,
                       float* WT, hipStream_t s);
hipError_t kan_param_grads(const float* dW, const float* spline_w, const float* scaler, int out, int in,
                           int accumulate, float* g_base, float* g_spline, float* g_scaler, hipStream_t s);
hipError_t kan_gemm(const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk, int64_t sbn, int M,
                    int N, int64_t K, int splits, float* C, float* out, hipStream_t s);

struct OptState {      // device-resident optimizer + ReduceLROnPlateau state (run.py:116-117)
  double lr;           // current learning rate (param_groups[0]['lr'])
  double best;         // plateau: best loss so far (init +inf)
  double step;         // Adam step count (torch keeps it as a float tensor)
  int32_t num_bad;     // plateau: num_bad_epochs
  int32_t last_epoch;  // number of scheduler.step() calls
  double min_lr, factor, threshold, eps_lr;
  int32_t patience, pad0;
  double beta1, beta2, eps;
};

hipError_t adam_flat(float* p, const float* g, float* m, float* v, int64_t n, const OptState* st,
                     hipStream_t s, const GuardState* guard = nullptr, const float* sse = nullptr);
hipError_t plateau_step(OptState* st, const float* sse, double n_total, float* loss_hist,
                        double* lr_hist, int64_t hist_cap, hipStream_t s, GuardState* guard = nullptr);
hipError_t cast_weight(const float* W, int H_out, int H_in, h16* Wb, h16* WTb, hipStream_t s);
// cast_weight of n square H x H layers in one launch
constexpr int kMaxInner = 16;  // == SIREN_MAX_INNER
struct CastSet {
  const float* W[kMaxInner];
  h16* Wb[kMaxInner];
  h16* WTb[kMaxInner];
  int n;
};
hipError_t cast_weights(const CastSet& cs, int H, hipStream_t s);
hipError_t sum_to(const float* x, int n, float* out, int accumulate, hipStream_t s);
// sum_to(x0 -> out0) and sum_to(x1 -> out1) in one launch; flag_src non-null: also
// flag_dst[0] (+)= (flag_src[0] != 0)
hipError_t sum_to2(const float* x0, float* out0, const float* x1, float* out1, int n, int accumulate, hipStream_t s,
                   const int* flag_src = nullptr, float* flag_dst = nullptr);

}  // namespace siren
