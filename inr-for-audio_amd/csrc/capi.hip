// C-ABI of libsiren_hip.so (include/siren_hip.h): argument validation, the fused
// training-step launch sequence, and thin wrappers over the individual kernels.
#include <string.h>
#include <vector>
#include "../../include/siren_hip.h"
#include "siren_kernels.h"

using namespace siren;

static_assert(sizeof(siren_opt_state) == sizeof(OptState), "opt state layout");
static_assert(sizeof(siren_guard) == sizeof(GuardState), "guard layout");
static_assert(SIREN_TILEQ_INTS == kTileqInts, "tile-queue set size");
static_assert(SIREN_MAX_INNER == siren::kMaxInner, "max hidden layers");
static_assert((int)SIREN_FP32_SNAKE == (int)siren::FP32_SNAKE && (int)SIREN_FP32_SIN == (int)siren::FP32_SIN &&
                  (int)SIREN_FP32_TANH == (int)siren::FP32_TANH, "fp32 act codes");

namespace {

inline hipStream_t S(void* s) { return (hipStream_t)s; }
inline const h16* B(const uint16_t* p) { return (const h16*)p; }
inline h16* B(uint16_t* p) { return (h16*)p; }

#define SIREN_TRY(expr)                        \
  do {                                         \
    const hipError_t _e = (expr);              \
    if (_e != hipSuccess) return (int)_e;      \
  } while (0)

// ---- optional per-launch HIP-event profiling (bench.py uses it inside its timed region) ----
struct ProfState {
  bool on = false;
  bool open = false;            // a record was begun by prof_begin
  uint32_t mask = 0xffffffffu;  // kinds bracketed (siren_profile_mask)
  std::vector<hipEvent_t> ev;   // 2 per record
  std::vector<int> kind;
  std::vector<int> nl;          // launches inside each record
  int used = 0;
};
ProfState g_prof;

inline void prof_begin(int kind, hipStream_t s) {
  g_prof.open = false;
  if (!g_prof.on || g_prof.used >= (int)g_prof.kind.size() || !((g_prof.mask >> kind) & 1u)) return;
  (void)hipEventRecord(g_prof.ev[2 * g_prof.used], s);
  g_prof.kind[g_prof.used] = kind;
  g_prof.open = true;
}
inline void prof_end(hipStream_t s, int launches = 1) {
  if (!g_prof.open) return;
  (void)hipEventRecord(g_prof.ev[2 * g_prof.used + 1], s);
  g_prof.nl[g_prof.used] = launches;
  g_prof.used++;
  g_prof.open = false;
}

#define SIREN_PROF(kind, s, expr)            \
  do {                                       \
    prof_begin((kind), (s));                 \
    const hipError_t _pe = (expr);           \
    prof_end((s));                           \
    if (_pe != hipSuccess) return _pe;       \
  } while (0)

// 128, 256, 512, 1024 (one launch per GEMM), then multiples of 1024 up to SIREN_MAX_HIDDEN (column
// windows of 1024: gemm_nt, first_fwd, head_bwd)
bool hidden_ok(int h) {
  return (h >= 128 && h % 128 == 0 && h <= 1024 && 256 % (h / 4) == 0) || (h > 1024 && h % 1024 == 0 && h <= SIREN_MAX_HIDDEN);
}

int check_net(const siren_net* n) {
  if (!n) return SIREN_ERR_NULL;
  if (n->in_dim < 1 || n->in_dim > 2) return SIREN_ERR_CONFIG;
  if (!hidden_ok(n->hidden)) return SIREN_ERR_SHAPE;
  if (n->n_inner < 1 || n->n_inner > SIREN_MAX_INNER) return SIREN_ERR_CONFIG;
  if (!n->W0 || !n->b0 || !n->w_head || !n->b_head) return SIREN_ERR_NULL;
  for (int i = 0; i < n->n_inner; ++i) {
    if (!n->b[i] || !n->Wh[i] || !n->WTh[i]) return SIREN_ERR_NULL;
    if (n->act[i] < SIREN_ACT_SINE || n->act[i] > SIREN_ACT_TANH) return SIREN_ERR_CONFIG;
    if (n->act[i] == SIREN_ACT_SNAKE && !n->a[i]) return SIREN_ERR_NULL;
  }
  if (n->first_snake && !n->a0) return SIREN_ERR_NULL;
  if (!(n->head_omega >= 0.f)) return SIREN_ERR_CONFIG;
  return SIREN_OK;
}

// forward mode of an inner layer kind; omega its epilogue / derivative factor
int fwd_mode(int act) { return act == SIREN_ACT_SNAKE ? NT_FWD_SNAKE : (act == SIREN_ACT_TANH ? NT_FWD_TANH : NT_FWD); }
float act_omega(const siren_net* n, int i) { return n->act[i] == SIREN_ACT_SINE ? n->omega : 1.0f; }
// bound of |dY/dz| of inner layer i (grad_scale headroom): omega, 2 (Snake), 1 (Tanh)
float act_bound(const siren_net* n, int i) {
  return n->act[i] == SIREN_ACT_SINE ? n->omega : (n->act[i] == SIREN_ACT_SNAKE ? 2.0f : 1.0f);
}

int check_batch(const siren_net* n, const siren_batch* b, bool train) {
  if (!b) return SIREN_ERR_NULL;
  if (b->rows <= 0 || b->rows % SIREN_ROW_TILE || b->n_valid < 0 || b->n_valid > b->rows)
    return SIREN_ERR_SHAPE;
  if (!b->coords || !b->out || !b->head_part || !b->g || !b->sse_part || !b->gsum_part)
    return SIREN_ERR_NULL;
  for (int i = 0; i <= n->n_inner; ++i)
    if (!b->Y[i] || !b->C[i]) return SIREN_ERR_NULL;
  for (int i = 0; i < n->n_inner; ++i)
    if (n->act[i] == SIREN_ACT_SNAKE && !b->E[i + 1]) return SIREN_ERR_NULL;
  if (n->first_snake && !b->E[0]) return SIREN_ERR_NULL;
  if (train) {
    if (!b->target || !b->dZ[0] || !b->dZ[1] || !b->col_part || !b->col_part2 || !b->red_tmp ||
        !b->slab || !b->gmax_part || !b->gscale)
      return SIREN_ERR_NULL;
    if (b->splits < 1 || b->n_total <= 0) return SIREN_ERR_CONFIG;
  }
  if (b->loss_mode < 0 || b->loss_mode > 1) return SIREN_ERR_CONFIG;
  return SIREN_OK;
}

// record batch->grad_ready[k] (if set) on the stream
inline hipError_t mark_ready(const siren_batch* b, int k, hipStream_t s) {
  return b->grad_ready[k] ? hipEventRecord((hipEvent_t)b->grad_ready[k], s) : hipSuccess;
}

// one segment of a multi-segment column reduction (capi's sets never exceed kMaxColSegs)
inline void seg_add(ColSegs& sg, const float* src, float* out, int out_stride = 1) {
  if (sg.n < kMaxColSegs) {
    sg.src[sg.n] = src;
    sg.out[sg.n] = out;
    sg.out_stride[sg.n] = out_stride;
  }
  ++sg.n;  // a set past kMaxColSegs is rejected by col_reduce_multi
}

// the fused last-layer mode of a last inner layer kind
int hb_mode(int act) {
  return act == SIREN_ACT_SNAKE ? NT_FWD_HB_SNAKE : (act == SIREN_ACT_TANH ? NT_FWD_HB_TANH : NT_FWD_HB);
}
// SIREN_OPT_HEAD_FUSE: siren_train_step runs the last layer as NT_FWD_HB* when it can.  A Snake last
// layer needs a backward scale before its forward that no bound gives tightly (|Y| is not bounded
// by 1): it fuses only when the caller says gmax_part holds a previous launch's max|g| partials
// (siren_batch.head_scale_prev); the range guard catches a step whose |g| outgrew that scale.
int g_head_fuse = 1;
bool head_fused(const siren_net* n, const siren_batch* b, hipStream_t s) {
  const int act = n->act[n->n_inner - 1];
  if (!g_head_fuse || (act == SIREN_ACT_SNAKE && !b->head_scale_prev)) return false;
  // the hand-off's timeout is only made loud through the guard's stall word: without a guard a
  // timed-out band would reach Adam as a NaN gradient, so a guard-less batch runs unfused
  if (!b->guard) return false;
  return gemm_nt_head_fusable(b->rows, n->hidden, s, hb_mode(act));
}

// forward through all layers + head partials; returns hip status.  hb: the last layer is the
// fused NT_FWD_HB (training; gfac = the loss gradient factor, b->gscale already set)
hipError_t run_forward(const siren_net* n, siren_batch* b, hipStream_t s, bool hb = false, float gfac = 0.f) {
  const int R = b->rows, H = n->hidden, L = n->n_inner;
  SIREN_PROF(SIREN_PROF_FIRST_FWD, s, first_fwd(b->coords, n->in_dim, n->W0, n->b0, n->omega0, R, H, B(b->Y[0]),
                                                B(b->C[0]), s, n->first_snake ? n->a0 : nullptr,
                                                n->first_snake ? B(b->E[0]) : nullptr));
  // the run of plain forward layers is ONE profiling record (back-to-back launches: one event
  // pair per run instead of per launch, so the per-launch dispatch latency inside the bracket
  // is paid once; bench.py divides by the launch count)
  int run = 0;
  auto close_run = [&]() {
    if (run > 0) prof_end(s, run);
    run = 0;
  };
  for (int i = 0; i < L; ++i) {
    NtParams p = {};
    p.X = B(b->Y[i]);
    p.W = B(n->Wh[i]);
    p.M = R; p.N = H; p.K = H;
    p.tile = nt_choose_tile(R, H);
    p.omega = n->omega;
    p.bias = n->b[i];
    p.Y = B(b->Y[i + 1]);
    p.C = B(b->C[i + 1]);
    p.E = B(b->E[i + 1]);
    p.act_a = n->a[i];
    const bool head = (i == L - 1);
    p.head_w = n->w_head;
    p.head_part = b->head_part;
    p.tileq = b->tileq;
    if (head && hb) {
      p.target = b->target; p.b_head = n->b_head; p.out = b->out; p.g = b->g;
      p.sse_part = b->sse_part; p.gsum_part = b->gsum_part;
      p.n_valid = b->n_valid; p.loss_mode = b->loss_mode; p.gfac = gfac; p.head_omega = n->head_omega;
      p.gscale = b->gscale; p.dZ = B(b->dZ[0]); p.colsum_part = b->col_part;
      p.gmax_part = b->gmax_part;  // this launch's max|g|: the next one's scale (Snake last layer)
      p.stall = b->guard ? &((GuardState*)b->guard)->stalls : nullptr;  // a timed-out hand-off voids the step
      close_run();
      SIREN_PROF(SIREN_PROF_HEAD_FWD, s, gemm_nt(hb_mode(n->act[i]), true, p, s));
      continue;
    }
    if (run == 0) prof_begin(SIREN_PROF_INNER_FWD, s);
    const hipError_t e = gemm_nt(fwd_mode(n->act[i]), head, p, s);
    if (e != hipSuccess) {
      close_run();
      return e;
    }
    if (g_prof.open) ++run;
  }
  close_run();
  return hipSuccess;
}

}  // namespace

extern "C" {

int siren_abi_version(void) { return SIREN_ABI_VERSION; }

// __graft_entry__._compile passes the hash of the sources and defines; the marker prefix lets the
// build step read it from the file without loading the library
#ifndef SIREN_BUILD_ID
#define SIREN_BUILD_ID "unknown"
#endif
static const char kBuildId[] = "SIREN_BUILD_ID=" SIREN_BUILD_ID;
const char* siren_build_id(void) { return kBuildId + 15; }

int64_t siren_struct_size(int32_t which) {
  switch (which) {
    case 0: return sizeof(siren_net);
    case 1: return sizeof(siren_grads);
    case 2: return sizeof(siren_batch);
    case 3: return sizeof(siren_opt_state);
    case 4: return sizeof(siren_kan_net);
    case 5: return sizeof(siren_kan_grads);
    case 6: return sizeof(siren_kan_batch);
    case 7: return sizeof(siren_guard);
  }
  return -1;
}

const char* siren_status_string(int status) {
  switch (status) {
    case SIREN_OK: return "ok";
    case SIREN_ERR_SHAPE: return "unsupported or inconsistent shape";
    case SIREN_ERR_NULL: return "required device pointer is NULL";
    case SIREN_ERR_CONFIG: return "unsupported configuration";
  }
  return hipGetErrorString((hipError_t)status);
}

int32_t siren_nt_tile(int32_t rows, int32_t hidden) { return nt_choose_tile(rows, hidden); }
int32_t siren_dw_tile(int32_t rows, int32_t hidden) { return tn_choose_tile(rows, hidden, hidden); }

int32_t siren_default_splits(int32_t rows, int32_t hidden) {
  // 256 tiles: one round of one block per CU (GEMM + fixed-order slab reduce measured best:
  // 2^20 x 1024 at 16 splits 1.731 ms vs 32 1.752; 220 160 x 512 at 64 splits 0.132 vs 128
  // 0.152, tools/kernel_bench.py --dw-splits); 128 tiles: ~1024 blocks-worth.  No slice
  // thinner than 8 K-steps.
  const int tile = tn_choose_tile(rows, hidden, hidden);
  const int ntile = (hidden / tile) * (hidden / tile);
  int splits = (tile == 256 ? 256 : 1024) / (ntile > 0 ? ntile : 1);
  const int nks = rows / 64;
  const int max_splits = nks / 8 > 0 ? nks / 8 : 1;
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  return splits;
}

int64_t siren_slab_floats(int32_t hidden, int32_t splits) {
  return (int64_t)splits * hidden * hidden;
}

int siren_forward(const siren_net* net, siren_batch* batch, void* stream) {
  int st = check_net(net);
  if (st) return st;
  if ((st = check_batch(net, batch, false))) return st;
  hipStream_t s = S(stream);
  SIREN_TRY(run_forward(net, batch, s));
  // out = sum of head partials + bias (g/sse unused at inference: n_valid = 0 path)
  SIREN_TRY(head_loss(batch->head_part, net->hidden / nt_choose_tile(batch->rows, net->hidden),
                      batch->rows, net->b_head, batch->out,
                      0, 0.f, batch->out, batch->g, batch->sse_part, batch->gsum_part, nullptr, s,
                      net->head_omega));
  return SIREN_OK;
}

static int check_grads(const siren_net* net, const siren_grads* gr) {
  if (!gr || !gr->W0 || !gr->b0 || !gr->w_head || !gr->b_head) return SIREN_ERR_NULL;
  for (int i = 0; i < net->n_inner; ++i) {
    if (!gr->W[i] || !gr->b[i]) return SIREN_ERR_NULL;
    if (net->act[i] == SIREN_ACT_SNAKE && !gr->a[i]) return SIREN_ERR_NULL;
  }
  if (net->first_snake && !gr->a0) return SIREN_ERR_NULL;
  return SIREN_OK;
}

// autograd of models.py:388-394 given dLoss/dout in batch->g (rows >= n_valid are zero).  hb: the
// forward's NT_FWD_HB already wrote dZ_L and the [R/256][2][H] partials of db_L and dw_head
static int run_backward(const siren_net* net, const siren_grads* gr, siren_batch* b, hipStream_t s,
                        bool hb = false) {
  const int R = b->rows, H = net->hidden, L = net->n_inner, in = net->in_dim;
  const int ntile = nt_choose_tile(R, H), tntile = tn_choose_tile(R, H, H);
  const int prow = R / ntile;  // partial rows written by the NT_DX / NT_DX0 epilogues
  if (hb) {
    // [R/256][2][H] partials of db_L, dw_head; a Snake last layer [R/256][3][H] with da_L
    const bool snake_last = net->act[L - 1] == SIREN_ACT_SNAKE;
    ColSegs sg = {};
    seg_add(sg, b->col_part + H, gr->w_head);
    seg_add(sg, b->col_part, gr->b[L - 1]);
    if (snake_last) seg_add(sg, b->col_part + 2 * H, gr->a[L - 1]);
    SIREN_PROF(SIREN_PROF_REDUCE, s, col_reduce_multi(sg, (snake_last ? 3 : 2) * H, prow, H, 1, b->red_tmp, s));
  } else {
    const bool snake_last = net->act[L - 1] == SIREN_ACT_SNAKE;
    float* da_last = b->col_part + (int64_t)(R / 128) * H;  // second H-wide slab of col_part
    SIREN_PROF(SIREN_PROF_HEAD, s, grad_scale(b->gmax_part, (R + 255) / 256, net->w_head, H,
                                              act_bound(net, L - 1), b->gscale, s,
                                              (const GuardState*)b->guard));
    SIREN_PROF(SIREN_PROF_HEAD, s, head_bwd(B(b->C[L]), B(b->Y[L]), b->g, net->w_head, act_omega(net, L - 1),
                                            R, H, b->gscale, B(b->dZ[0]), b->col_part, b->col_part2,
                                            snake_last ? B(b->E[L]) : nullptr, snake_last ? da_last : nullptr, s));
    ColSegs sg = {};
    seg_add(sg, b->col_part2, gr->w_head);
    seg_add(sg, b->col_part, gr->b[L - 1]);
    if (snake_last) seg_add(sg, da_last, gr->a[L - 1]);
    SIREN_PROF(SIREN_PROF_REDUCE, s, col_reduce_multi(sg, H, R / 128, H, 1, b->red_tmp, s));
  }
  SIREN_TRY(mark_ready(b, L + 1, s));  // head: w_head, b_head (and sse, summed before the backward)

  int cur = 0;
  for (int i = L - 1; i >= 0; --i) {
    TnParams tp = {};
    tp.Y = B(b->Y[i]);
    tp.dZ = B(b->dZ[cur]);
    tp.R = R; tp.Hin = H; tp.Hout = H;
    tp.splits = b->splits;
    tp.tile = tntile;
    tp.slab = b->slab;
    SIREN_PROF(SIREN_PROF_BWD_DW, s, gemm_tn_dw(tp, s));
    SIREN_PROF(SIREN_PROF_REDUCE, s, dw_reduce(b->slab, b->splits, H, H, tntile, gr->W[i], 1,
                                                       b->gscale, s));
    SIREN_TRY(mark_ready(b, i, s));  // W_i now; b_i and a_i were reduced one stage earlier

    NtParams p = {};
    p.X = B(b->dZ[cur]);
    p.W = B(net->WTh[i]);
    p.M = R; p.N = H; p.K = H;
    p.tile = ntile;
    p.colsum_part = b->col_part;
    p.gscale = b->gscale;
    p.tileq = b->tileq;  // used only with SIREN_OPT_NT_QUEUE 2
    if (i > 0) {
      const bool snake = net->act[i - 1] == SIREN_ACT_SNAKE;
      p.omega = act_omega(net, i - 1);
      p.Cprev = B(b->C[i]);
      p.Eprev = B(b->E[i]);
      p.dZ = B(b->dZ[cur ^ 1]);
      SIREN_PROF(SIREN_PROF_BWD_DX, s, gemm_nt(snake ? NT_DX_SNAKE : NT_DX, false, p, s));
      const int64_t rs = (int64_t)(snake ? 2 : 1) * H;
      ColSegs sg = {};
      seg_add(sg, b->col_part, gr->b[i - 1]);
      if (snake) seg_add(sg, b->col_part + H, gr->a[i - 1]);
      SIREN_PROF(SIREN_PROF_REDUCE, s, col_reduce_multi(sg, rs, prow, H, 1, b->red_tmp, s));
      cur ^= 1;
    } else {
      const bool fs = net->first_snake != 0;
      p.omega = fs ? 1.0f : net->omega0;
      p.Cprev = B(b->C[0]);
      p.Eprev = B(b->E[0]);
      p.t = b->coords;
      p.in_dim = in;
      SIREN_PROF(SIREN_PROF_BWD_DX0, s, gemm_nt(fs ? NT_DX0_SNAKE : NT_DX0, false, p, s));
      const int64_t rs = (int64_t)(fs ? 2 + in : 1 + in) * H;
      // db0, the in columns of dW0 (stride in) and a0: one launch pair
      ColSegs sg = {};
      if (fs) seg_add(sg, b->col_part + (int64_t)(1 + in) * H, gr->a0);
      seg_add(sg, b->col_part, gr->b0);
      for (int j = 0; j < in; ++j) seg_add(sg, b->col_part + (int64_t)(1 + j) * H, gr->W0 + j, in);
      SIREN_PROF(SIREN_PROF_REDUCE, s, col_reduce_multi(sg, rs, prow, H, 1, b->red_tmp, s));
      SIREN_TRY(mark_ready(b, L, s));
    }
  }
  return SIREN_OK;
}

int siren_train_step(const siren_net* net, const siren_grads* gr, siren_batch* b, void* stream) {
  int st = check_net(net);
  if (st) return st;
  if ((st = check_batch(net, b, true))) return st;
  if ((st = check_grads(net, gr))) return st;
  if (!gr->sse) return SIREN_ERR_NULL;
  hipStream_t s = S(stream);
  const int R = b->rows, H = net->hidden;

  if (b->zero_grads && gr->flat) SIREN_TRY(hipMemsetAsync(gr->flat, 0, gr->flat_len * sizeof(float), s));

  // mean backward: MSELoss 2 err / N, L1Loss sign(err) / N
  const float gfac = (float)((b->loss_mode == 1 ? 1.0 : 2.0) / b->n_total);
  const bool hb = head_fused(net, b, s);
  if (hb) {
    // the fused head needs the backward scale S before the forward.  Sine / Tanh last layer
    // (|Y_L| <= 1): from the bound of max|g| (elementwise.hip grad_scale_bound) instead of the
    // step's max|g|.  Snake: from the previous launch's max|g| partials in gmax_part (grad_scale,
    // the unfused path's own scale rule on last step's g)
    const int L = net->n_inner, nv = b->n_valid, nyp = (nv + 255) / 256;
    if (net->act[L - 1] == SIREN_ACT_SNAKE) {
      SIREN_PROF(SIREN_PROF_HEAD, s, grad_scale(b->gmax_part, (R + 255) / 256, net->w_head, H, act_bound(net, L - 1),
                                                b->gscale, s, (const GuardState*)b->guard));
    } else {
      if (nv > 0) SIREN_PROF(SIREN_PROF_HEAD, s, gmax_partials(b->target, nv, b->gmax_part, s));
      SIREN_PROF(SIREN_PROF_HEAD, s, grad_scale_bound(b->gmax_part, nyp, net->w_head, net->b_head, H, gfac,
                                                      net->head_omega, b->loss_mode, act_bound(net, L - 1),
                                                      b->gscale, s, (const GuardState*)b->guard));
    }
  }
  // ---- forward (models.py:388-394) + MSE / L1 (run.py:161-169) ----
  SIREN_TRY(run_forward(net, b, s, hb, gfac));
  if (!hb)
    SIREN_PROF(SIREN_PROF_HEAD, s, head_loss(b->head_part, H / nt_choose_tile(R, H), R, net->b_head,
                                             b->target, b->n_valid, gfac, b->out, b->g, b->sse_part,
                                             b->gsum_part, b->gmax_part, s, net->head_omega, b->loss_mode));
  const int nsum = (R + 255) / 256;
  // sse[1]: the fused hand-off's stall flag rides the gradient all-reduce with the sse (siren_grads.sse)
  const int* stall = (hb && b->guard) ? &((const GuardState*)b->guard)->stalls : nullptr;
  SIREN_PROF(SIREN_PROF_REDUCE, s, sum_to2(b->sse_part, gr->sse, b->gsum_part, gr->b_head, nsum, 1, s, stall,
                                           gr->sse + 1));
  // ---- backward (autograd of run.py:185) ----
  return run_backward(net, gr, b, s, hb);
}

int siren_backward(const siren_net* net, const siren_grads* gr, siren_batch* b, void* stream) {
  int st = check_net(net);
  if (st) return st;
  if ((st = check_batch(net, b, true))) return st;
  if ((st = check_grads(net, gr))) return st;
  hipStream_t s = S(stream);
  if (b->zero_grads && gr->flat) SIREN_TRY(hipMemsetAsync(gr->flat, 0, gr->flat_len * sizeof(float), s));
  // last_linear=False: chain dLoss/dout through the final sin (head_part is the forward's)
  if (net->head_omega > 0.f)
    SIREN_TRY(head_sine_chain(b->head_part, net->hidden / nt_choose_tile(b->rows, net->hidden), b->rows,
                              net->b_head, net->head_omega, b->g, s));
  // bias of the head: sum of g; max |g| partials for the backward storage scale
  SIREN_TRY(sum_to(b->g, b->rows, gr->b_head, 1, s));
  SIREN_TRY(gmax_partials(b->g, b->rows, b->gmax_part, s));
  return run_backward(net, gr, b, s);
}

int siren_apply_update(const siren_net* net, float* params, const float* grads_flat, float* exp_avg,
                       float* exp_avg_sq, int64_t n_params, float* const* W_fp32, uint16_t* const* Wh,
                       uint16_t* const* WTh, siren_opt_state* state, const float* sse, double n_total,
                       float* loss_hist, double* lr_hist, int64_t hist_cap, siren_guard* guard,
                       void* stream) {
  int st = check_net(net);
  if (st) return st;
  if (!params || !grads_flat || !exp_avg || !exp_avg_sq || !state || !sse || !W_fp32 || !Wh || !WTh)
    return SIREN_ERR_NULL;
  hipStream_t s = S(stream);
  // the fp16 shadows of every hidden layer, refreshed by one launch after Adam
  CastSet cs = {};
  cs.n = net->n_inner;
  for (int i = 0; i < net->n_inner; ++i) {
    if (!W_fp32[i] || !Wh[i] || !WTh[i]) return SIREN_ERR_NULL;
    cs.W[i] = W_fp32[i];
    cs.Wb[i] = B(Wh[i]);
    cs.WTb[i] = B(WTh[i]);
  }
  GuardState* gd = (GuardState*)guard;
  if (gd) SIREN_PROF(SIREN_PROF_UPDATE, s, guard_check(grads_flat, n_params, gd, s, sse));
  SIREN_PROF(SIREN_PROF_UPDATE, s, adam_flat(params, grads_flat, exp_avg, exp_avg_sq, n_params,
                                             (const OptState*)state, s, gd, sse));
  SIREN_PROF(SIREN_PROF_UPDATE, s, cast_weights(cs, net->hidden, s));
  SIREN_PROF(SIREN_PROF_UPDATE, s, plateau_step((OptState*)state, sse, n_total, loss_hist, lr_hist, hist_cap, s,
                                                gd));
  return SIREN_OK;
}

// ---- individual kernels ----------------------------------------------------------------

int siren_coords_fill(float* t, int64_t rows, int64_t offset, int64_t n_total, void* stream) {
  if (!t) return SIREN_ERR_NULL;
  if (rows < 0 || offset < 0 || n_total < 1) return SIREN_ERR_SHAPE;
  return (int)coords_fill(t, rows, offset, n_total, S(stream));
}

int siren_coords_fill_grid(float* xy, int64_t rows, int64_t offset, int64_t height, int32_t width,
                           void* stream) {
  if (!xy) return SIREN_ERR_NULL;
  if (rows < 0 || offset < 0 || height < 1 || width < 1) return SIREN_ERR_SHAPE;
  return (int)coords_fill_grid(xy, rows, offset, height, width, S(stream));
}

int siren_first_fwd(const float* t, int32_t in_dim, const float* W0, const float* b0, float omega0,
                    int32_t rows, int32_t hidden, uint16_t* Y0, uint16_t* C0, void* stream) {
  if (!t || !W0 || !b0 || !Y0 || !C0) return SIREN_ERR_NULL;
  if (in_dim < 1 || in_dim > 2) return SIREN_ERR_CONFIG;
  if (rows < 0 || hidden < 8 || hidden % 8 || (hidden <= 2048 ? 256 % (hidden / 8) != 0 : (hidden % 1024 || hidden > SIREN_MAX_HIDDEN)))
    return SIREN_ERR_SHAPE;
  return (int)first_fwd(t, in_dim, W0, b0, omega0, rows, hidden, B(Y0), B(C0), S(stream));
}

int siren_inner_fwd(const uint16_t* X, const uint16_t* Wh, const float* b, float omega, int32_t rows,
                    int32_t hidden, uint16_t* Y, uint16_t* C, const float* head_w, float* head_part,
                    int32_t* tileq, void* stream) {
  if (!X || !Wh || !b || !Y || !C) return SIREN_ERR_NULL;
  if (!hidden_ok(hidden) || rows <= 0 || rows % SIREN_ROW_TILE) return SIREN_ERR_SHAPE;
  if (head_w && !head_part) return SIREN_ERR_NULL;
  NtParams p = {};
  p.X = B(X); p.W = B(Wh); p.M = rows; p.N = hidden; p.K = hidden;
  p.tile = nt_choose_tile(rows, hidden);
  p.omega = omega; p.bias = b; p.Y = B(Y); p.C = B(C);
  p.head_w = head_w; p.head_part = head_part; p.tileq = tileq;
  return (int)gemm_nt(NT_FWD, head_w != nullptr, p, S(stream));
}

int siren_head_loss(const float* head_part, int32_t nparts, int32_t rows, const float* b_head,
                    const float* y, int32_t n_valid, double n_total, float* out, float* g,
                    float* sse_part, float* gsum_part, float* gmax_part, void* stream) {
  if (!head_part || !b_head || !out || !g || !sse_part || !gsum_part) return SIREN_ERR_NULL;
  if (n_valid > 0 && !y) return SIREN_ERR_NULL;
  if (rows <= 0 || nparts < 1 || n_valid > rows || n_total <= 0) return SIREN_ERR_SHAPE;
  return (int)head_loss(head_part, nparts, rows, b_head, y, n_valid, (float)(2.0 / n_total), out, g,
                        sse_part, gsum_part, gmax_part, S(stream));
}

int siren_grad_scale(const float* gmax_part, int32_t nparts, const float* w_head, int32_t hidden,
                     float omega, float* gscale, void* stream) {
  if (!gmax_part || !w_head || !gscale) return SIREN_ERR_NULL;
  if (nparts < 1 || hidden < 1) return SIREN_ERR_SHAPE;
  return (int)grad_scale(gmax_part, nparts, w_head, hidden, omega, gscale, S(stream));
}

int siren_head_bwd(const uint16_t* C, const uint16_t* Y, const float* g, const float* w_head,
                   float omega, int32_t rows, int32_t hidden, const float* gscale, uint16_t* dZ,
                   float* db_part, float* dwh_part, const uint16_t* E, float* da_part, void* stream) {
  if (!C || !Y || !g || !w_head || !dZ || !db_part || !dwh_part) return SIREN_ERR_NULL;
  if (E && !da_part) return SIREN_ERR_NULL;
  if (!hidden_ok(hidden) || rows <= 0 || rows % SIREN_ROW_TILE) return SIREN_ERR_SHAPE;
  return (int)head_bwd(B(C), B(Y), g, w_head, omega, rows, hidden, gscale, B(dZ), db_part, dwh_part,
                       B(E), da_part, S(stream));
}

int siren_head_fused_fwd(const uint16_t* X, const uint16_t* Wh, const float* b, float omega, int32_t rows,
                         int32_t hidden, const float* w_head, const float* b_head, float head_omega, const float* y,
                         int32_t n_valid, double n_total, int32_t loss_mode, const float* gscale, float* head_part,
                         float* out, float* g, float* sse_part, float* gsum_part, uint16_t* dZ, float* part,
                         void* stream) {
  if (!X || !Wh || !b || !w_head || !b_head || !gscale || !head_part || !out || !g || !sse_part || !gsum_part ||
      !dZ || !part || (n_valid > 0 && !y))
    return SIREN_ERR_NULL;
  if (!hidden_ok(hidden) || rows <= 0 || rows % 256 || n_valid < 0 || n_valid > rows || !(n_total > 0))
    return SIREN_ERR_SHAPE;
  if (loss_mode < 0 || loss_mode > 1 || !(head_omega >= 0.f)) return SIREN_ERR_CONFIG;
  if (!gemm_nt_head_fusable(rows, hidden, S(stream))) return SIREN_ERR_CONFIG;
  NtParams p = {};
  p.X = B(X); p.W = B(Wh); p.M = rows; p.N = hidden; p.K = hidden;
  p.tile = nt_choose_tile(rows, hidden);
  p.omega = omega; p.bias = b; p.head_w = w_head; p.head_part = head_part;
  p.target = y; p.b_head = b_head; p.out = out; p.g = g; p.sse_part = sse_part; p.gsum_part = gsum_part;
  p.n_valid = n_valid; p.loss_mode = loss_mode; p.gfac = (float)((loss_mode == 1 ? 1.0 : 2.0) / n_total);
  p.head_omega = head_omega; p.gscale = gscale; p.dZ = B(dZ); p.colsum_part = part;
  return (int)gemm_nt(NT_FWD_HB, true, p, S(stream));
}

int siren_head_fused_fwd_act(const uint16_t* X, const uint16_t* Wh, const float* b, int32_t act, float omega,
                             const float* a, int32_t rows, int32_t hidden, const float* w_head, const float* b_head,
                             float head_omega, const float* y, int32_t n_valid, double n_total, int32_t loss_mode,
                             const float* gscale, float* head_part, float* out, float* g, float* sse_part,
                             float* gsum_part, float* gmax_part, uint16_t* dZ, float* part, uint16_t* E,
                             void* stream) {
  if (!X || !Wh || !b || !w_head || !b_head || !gscale || !head_part || !out || !g || !sse_part || !gsum_part ||
      !dZ || !part || (n_valid > 0 && !y) || (act == SIREN_ACT_SNAKE && (!a || !E)))
    return SIREN_ERR_NULL;
  if (!hidden_ok(hidden) || rows <= 0 || rows % 256 || n_valid < 0 || n_valid > rows || !(n_total > 0))
    return SIREN_ERR_SHAPE;
  if (act < SIREN_ACT_SINE || act > SIREN_ACT_TANH || loss_mode < 0 || loss_mode > 1 || !(head_omega >= 0.f))
    return SIREN_ERR_CONFIG;
  if (!gemm_nt_head_fusable(rows, hidden, S(stream), hb_mode(act))) return SIREN_ERR_CONFIG;
  NtParams p = {};
  p.X = B(X); p.W = B(Wh); p.M = rows; p.N = hidden; p.K = hidden;
  p.tile = nt_choose_tile(rows, hidden);
  p.omega = omega; p.bias = b; p.act_a = a; p.head_w = w_head; p.head_part = head_part;
  p.target = y; p.b_head = b_head; p.out = out; p.g = g; p.sse_part = sse_part; p.gsum_part = gsum_part;
  p.gmax_part = gmax_part;
  p.n_valid = n_valid; p.loss_mode = loss_mode; p.gfac = (float)((loss_mode == 1 ? 1.0 : 2.0) / n_total);
  p.head_omega = head_omega; p.gscale = gscale; p.dZ = B(dZ); p.colsum_part = part; p.E = B(E);
  return (int)gemm_nt(hb_mode(act), true, p, S(stream));
}

int siren_grad_scale_bound(const float* y, int32_t n_valid, float* ymax_part, const float* w_head,
                           const float* b_head, int32_t hidden, double n_total, float head_omega, int32_t loss_mode,
                           float act_bound, float* gscale, void* stream) {
  if (!w_head || !b_head || !gscale || (n_valid > 0 && (!y || !ymax_part))) return SIREN_ERR_NULL;
  if (n_valid < 0 || hidden < 1 || !(n_total > 0)) return SIREN_ERR_SHAPE;
  if (loss_mode < 0 || loss_mode > 1) return SIREN_ERR_CONFIG;
  hipStream_t s = S(stream);
  if (n_valid > 0) SIREN_TRY(gmax_partials(y, n_valid, ymax_part, s));
  return (int)grad_scale_bound(ymax_part, (n_valid + 255) / 256, w_head, b_head, hidden,
                               (float)((loss_mode == 1 ? 1.0 : 2.0) / n_total), head_omega, loss_mode, act_bound,
                               gscale, s);
}

int siren_inner_fwd_act(const uint16_t* X, const uint16_t* Wh, const float* b, int32_t act,
                        float omega, const float* a, int32_t rows, int32_t hidden, uint16_t* Y,
                        uint16_t* C, uint16_t* E, const float* head_w, float* head_part,
                        int32_t* tileq, void* stream) {
  if (!X || !Wh || !b || !Y || !C) return SIREN_ERR_NULL;
  if (act < SIREN_ACT_SINE || act > SIREN_ACT_TANH) return SIREN_ERR_CONFIG;
  if (act == SIREN_ACT_SNAKE && (!a || !E)) return SIREN_ERR_NULL;
  if (!hidden_ok(hidden) || rows <= 0 || rows % SIREN_ROW_TILE) return SIREN_ERR_SHAPE;
  if (head_w && !head_part) return SIREN_ERR_NULL;
  NtParams p = {};
  p.X = B(X); p.W = B(Wh); p.M = rows; p.N = hidden; p.K = hidden;
  p.tile = nt_choose_tile(rows, hidden);
  p.omega = omega; p.bias = b; p.Y = B(Y); p.C = B(C); p.E = B(E); p.act_a = a;
  p.head_w = head_w; p.head_part = head_part; p.tileq = tileq;
  return (int)gemm_nt(fwd_mode(act), head_w != nullptr, p, S(stream));
}

int siren_inner_bwd_dx_act(const uint16_t* dZ, const uint16_t* WTh, const uint16_t* Cprev,
                           const uint16_t* Eprev, int32_t act_prev, float omega_prev, int32_t rows,
                           int32_t hidden, const float* gscale, uint16_t* dZprev, float* part,
                           void* stream) {
  if (!dZ || !WTh || !Cprev || !dZprev || !part) return SIREN_ERR_NULL;
  if (act_prev < SIREN_ACT_SINE || act_prev > SIREN_ACT_TANH) return SIREN_ERR_CONFIG;
  if (act_prev == SIREN_ACT_SNAKE && !Eprev) return SIREN_ERR_NULL;
  if (!hidden_ok(hidden) || rows <= 0 || rows % SIREN_ROW_TILE) return SIREN_ERR_SHAPE;
  NtParams p = {};
  p.X = B(dZ); p.W = B(WTh); p.M = rows; p.N = hidden; p.K = hidden;
  p.tile = nt_choose_tile(rows, hidden);
  p.omega = act_prev == SIREN_ACT_SINE ? omega_prev : 1.0f;
  p.Cprev = B(Cprev); p.Eprev = B(Eprev); p.dZ = B(dZprev); p.colsum_part = part;
  p.gscale = gscale;
  return (int)gemm_nt(act_prev == SIREN_ACT_SNAKE ? NT_DX_SNAKE : NT_DX, false, p, S(stream));
}

int siren_inner_bwd_dx(const uint16_t* dZ, const uint16_t* WTh, const uint16_t* Cprev, float omega_prev,
                       int32_t rows, int32_t hidden, const float* gscale, uint16_t* dZprev,
                       float* db_part, void* stream) {
  if (!dZ || !WTh || !Cprev || !dZprev || !db_part) return SIREN_ERR_NULL;
  if (!hidden_ok(hidden) || rows <= 0 || rows % SIREN_ROW_TILE) return SIREN_ERR_SHAPE;
  NtParams p = {};
  p.X = B(dZ); p.W = B(WTh); p.M = rows; p.N = hidden; p.K = hidden;
  p.tile = nt_choose_tile(rows, hidden);
  p.omega = omega_prev; p.Cprev = B(Cprev); p.dZ = B(dZprev); p.colsum_part = db_part;
  p.gscale = gscale;
  return (int)gemm_nt(NT_DX, false, p, S(stream));
}

int siren_first_bwd_dx(const uint16_t* dZ1, const uint16_t* WTh1, const uint16_t* C0, const float* t,
                       int32_t in_dim, float omega0, int32_t rows, int32_t hidden, const float* gscale,
                       float* part, void* stream) {
  if (!dZ1 || !WTh1 || !C0 || !t || !part) return SIREN_ERR_NULL;
  if (in_dim < 1 || in_dim > 2) return SIREN_ERR_CONFIG;
  if (!hidden_ok(hidden) || rows <= 0 || rows % SIREN_ROW_TILE) return SIREN_ERR_SHAPE;
  NtParams p = {};
  p.X = B(dZ1); p.W = B(WTh1); p.M = rows; p.N = hidden; p.K = hidden;
  p.tile = nt_choose_tile(rows, hidden);
  p.omega = omega0; p.Cprev = B(C0); p.t = t; p.in_dim = in_dim; p.colsum_part = part;
  p.gscale = gscale;
  return (int)gemm_nt(NT_DX0, false, p, S(stream));
}

int siren_inner_bwd_dw(const uint16_t* Y, const uint16_t* dZ, int32_t rows, int32_t hidden,
                       int32_t splits, int32_t tile, float* slab, void* stream) {
  if (!Y || !dZ || !slab) return SIREN_ERR_NULL;
  if (!hidden_ok(hidden) || rows <= 0 || rows % 64 || splits < 1) return SIREN_ERR_SHAPE;
  if (tile != 0 && tile != 128 && tile != 256) return SIREN_ERR_CONFIG;
  TnParams p = {};
  p.Y = B(Y); p.dZ = B(dZ); p.R = rows; p.Hin = hidden; p.Hout = hidden; p.splits = splits;
  p.tile = tile ? tile : tn_choose_tile(rows, hidden, hidden);
  p.slab = slab;
  return (int)gemm_tn_dw(p, S(stream));
}

int siren_dw_reduce(const float* slab, int32_t splits, int32_t hidden, int32_t tile, float* grad,
                    int32_t accumulate, const float* gscale, void* stream) {
  if (!slab || !grad) return SIREN_ERR_NULL;
  if (!hidden_ok(hidden) || splits < 1) return SIREN_ERR_SHAPE;
  if (tile != 128 && tile != 256) return SIREN_ERR_CONFIG;
  return (int)dw_reduce(slab, splits, hidden, hidden, tile, grad, accumulate, gscale, S(stream));
}

int siren_col_reduce(const float* part, int64_t row_stride, int32_t nrows, int32_t ncols, float* out,
                     int32_t out_stride, int32_t accumulate, float* tmp, void* stream) {
  if (!part || !out || (nrows > 256 && !tmp)) return SIREN_ERR_NULL;
  if (nrows < 1 || ncols < 1 || out_stride < 1) return SIREN_ERR_SHAPE;
  return (int)col_reduce(part, row_stride, nrows, ncols, out, out_stride, accumulate, tmp, S(stream));
}

int siren_adam_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                    const siren_opt_state* state, void* stream) {
  if (!params || !grads || !exp_avg || !exp_avg_sq || !state) return SIREN_ERR_NULL;
  if (n < 0) return SIREN_ERR_SHAPE;
  return (int)adam_flat(params, grads, exp_avg, exp_avg_sq, n, (const OptState*)state, S(stream));
}

int siren_plateau_step(siren_opt_state* state, const float* sse, double n_total, float* loss_hist,
                       double* lr_hist, int64_t hist_cap, void* stream) {
  if (!state || !sse) return SIREN_ERR_NULL;
  if (hist_cap > 0 && (!loss_hist || !lr_hist)) return SIREN_ERR_NULL;
  return (int)plateau_step((OptState*)state, sse, n_total, loss_hist, lr_hist, hist_cap, S(stream));
}

int siren_cast_weight(const float* W, int32_t h_out, int32_t h_in, uint16_t* Wh, uint16_t* WTh,
                      void* stream) {
  if (!W || !Wh || !WTh) return SIREN_ERR_NULL;
  if (h_out % 64 || h_in % 64) return SIREN_ERR_SHAPE;
  return (int)cast_weight(W, h_out, h_in, B(Wh), B(WTh), S(stream));
}

int siren_fp32_linear(const float* x, int64_t rows, int32_t in, int32_t out, const float* W, const float* b,
                      float omega, float* pre, void* stream) {
  if (!x || !W || !pre) return SIREN_ERR_NULL;
  if (rows < 1 || rows > INT32_MAX || in < 1 || out < 1) return SIREN_ERR_SHAPE;
  return (int)fp32_linear(x, rows, in, out, W, b, omega, pre, S(stream));
}

static bool fp32_act_ok(int32_t act) { return act >= SIREN_FP32_IDENTITY && act <= SIREN_FP32_SNAKE; }

int siren_fp32_act(int32_t act, const float* x, int64_t rows, int32_t cols, const float* a, float* y, void* stream) {
  if (!fp32_act_ok(act)) return SIREN_ERR_CONFIG;
  if (!x || !y || (act == SIREN_FP32_SNAKE && !a)) return SIREN_ERR_NULL;
  if (rows < 0 || cols < 1) return SIREN_ERR_SHAPE;
  return (int)fp32_act(act, x, rows, cols, a, y, S(stream));
}

int siren_fp32_act_bwd(int32_t act, const float* x, int64_t rows, int32_t cols, const float* a, const float* gy,
                       float* gx, float* da, float* da_prod, float* tmp, void* stream) {
  if (!fp32_act_ok(act)) return SIREN_ERR_CONFIG;
  if (!x || !gy || !gx) return SIREN_ERR_NULL;
  if (act == SIREN_FP32_SNAKE && (!a || (da && (!da_prod || !tmp)))) return SIREN_ERR_NULL;
  if (rows < 1 || rows > INT32_MAX || cols < 1) return SIREN_ERR_SHAPE;
  hipStream_t s = S(stream);
  const bool want_da = act == SIREN_FP32_SNAKE && da;
  SIREN_TRY(fp32_act_bwd(act, x, rows, cols, a, gy, gx, want_da ? da_prod : nullptr, s));
  if (want_da) SIREN_TRY(col_reduce(da_prod, cols, (int)rows, cols, da, 1, 0, tmp, s));
  return SIREN_OK;
}

int siren_fp32_linear_bwd(const float* x, int64_t rows, int32_t in, int32_t out, const float* W, float omega,
                          float* gpre, float* gx, float* gW, float* gb, float* slab, int32_t splits, float* tmp,
                          void* stream) {
  if (!x || !W || !gpre || !gW || (splits > 1 && !slab) || (gb && !tmp)) return SIREN_ERR_NULL;
  if (rows < 1 || rows > INT32_MAX || in < 1 || out < 1 || splits < 1) return SIREN_ERR_SHAPE;
  return (int)fp32_linear_bwd(x, rows, in, out, W, omega, gpre, gx, gW, gb, slab, splits, tmp, S(stream));
}

int siren_set_option(int32_t option, int32_t value) {
  switch (option) {
    case SIREN_OPT_NT_TILE:
    case SIREN_OPT_TN_TILE:
      if (value != 0 && value != 128 && value != 256) return SIREN_ERR_CONFIG;
      if (option == SIREN_OPT_NT_TILE) gemm_nt_set_tile(value);
      else gemm_tn_set_tile(value);
      return SIREN_OK;
    case SIREN_OPT_NT_PIPE:
      if (value != -1 && value != 0 && value != 1 && (value < 4 || value > 7)) return SIREN_ERR_CONFIG;
      gemm_nt_set_pipe(value);
      return SIREN_OK;
    case SIREN_OPT_TN_PIPE:
      if (value < -1 || value > 4) return SIREN_ERR_CONFIG;
      gemm_tn_set_pipe(value);
      return SIREN_OK;
    case SIREN_OPT_NT_GRID:
      if (value < 0) return SIREN_ERR_CONFIG;
      gemm_nt_set_grid_cap(value);
      return SIREN_OK;
    case SIREN_OPT_NT_DIAG:
      if (value < 0 || (value & ~(1 | 4 | 8 | 512 | 1024 | 2048))) return SIREN_ERR_CONFIG;
      return gemm_nt_set_diag(value) ? SIREN_OK : SIREN_ERR_CONFIG;
    case SIREN_OPT_NT_QUEUE:
      if (value < 0 || value > 2) return SIREN_ERR_CONFIG;
      gemm_nt_set_queue(value);
      return SIREN_OK;
    case SIREN_OPT_HEAD_FUSE:
      if (value < 0 || value > 1) return SIREN_ERR_CONFIG;
      g_head_fuse = value;
      return SIREN_OK;
    case SIREN_OPT_HB_FAULT:
      return (value >= 0 && gemm_nt_set_hb_fault(value)) ? SIREN_OK : SIREN_ERR_CONFIG;
  }
  return SIREN_ERR_CONFIG;
}

// ---- profiling API ---------------------------------------------------------------------
int siren_profile_enable(int32_t max_records) {
  for (hipEvent_t e : g_prof.ev) (void)hipEventDestroy(e);
  g_prof.ev.clear();
  g_prof.kind.clear();
  g_prof.nl.clear();
  g_prof.used = 0;
  g_prof.on = false;
  if (max_records <= 0) return SIREN_OK;
  g_prof.ev.resize(2 * (size_t)max_records);
  for (auto& e : g_prof.ev) SIREN_TRY(hipEventCreate(&e));
  g_prof.kind.assign(max_records, -1);
  g_prof.nl.assign(max_records, 1);
  g_prof.on = true;
  return SIREN_OK;
}

int siren_profile_reset(void) {
  g_prof.used = 0;
  return SIREN_OK;
}

int siren_profile_mask(uint32_t kinds) {
  g_prof.mask = kinds;
  return SIREN_OK;
}

int siren_profile_read(int32_t kind, double* total_ms, int64_t* count) {
  if (!total_ms || !count) return SIREN_ERR_NULL;
  double tot = 0.0;
  int64_t n = 0;
  for (int i = 0; i < g_prof.used; ++i) {
    if (g_prof.kind[i] != kind) continue;
    SIREN_TRY(hipEventSynchronize(g_prof.ev[2 * i + 1]));
    float ms = 0.f;
    SIREN_TRY(hipEventElapsedTime(&ms, g_prof.ev[2 * i], g_prof.ev[2 * i + 1]));
    tot += ms;
    n += g_prof.nl[i];
  }
  *total_ms = tot;
  *count = n;
  return SIREN_OK;
}

}  // extern "C"

// ---- KAN variant (kan.py, run.py:92-93) -----------------------------------
namespace {

constexpr int KAN_K1 = 9;  // A-columns per input feature: SiLU + 8 B-spline bases

int check_kan(const siren_kan_net* n) {
  if (!n) return SIREN_ERR_NULL;
  if (n->n_layers < 1 || n->n_layers > SIREN_KAN_MAX_LAYERS) return SIREN_ERR_CONFIG;
  for (int l = 0; l <= n->n_layers; ++l)
    if (n->width[l] < 1 || n->width[l] > 4096) return SIREN_ERR_SHAPE;
  for (int l = 0; l < n->n_layers; ++l)
    if (!n->grid[l] || !n->base_w[l] || !n->spline_w[l] || !n->scaler[l]) return SIREN_ERR_NULL;
  return SIREN_OK;
}

// Workspace carve-up (floats, each piece 64-float aligned):
//   X[l] rows x w[l] for l = 1..L (X[L] = the output row vector);  W[l] w[l+1] x 9 w[l] and its
//   transpose WT[l];
//   dW w_max_out x 9 w_max_in;  slab splits x that;  G[2] rows x w_max;
//   sse/gsum/gmax partials 3 x ceil(rows/256);  one zero float.
// (No expansion A or dA: the fused kernels recompute the bases -- kan.hip.)
struct KanWs {
  float* X[SIREN_KAN_MAX_LAYERS + 1];
  float* W[SIREN_KAN_MAX_LAYERS];
  float* WT[SIREN_KAN_MAX_LAYERS];  // W transposed, [9 in][out] (the dX kernel's operand)
  float *dW, *slab, *G[2], *sse_part, *gsum_part, *gmax_part, *zero;
  int64_t slab_floats, total;
};

inline int64_t al64(int64_t x) { return (x + 63) / 64 * 64; }

KanWs kan_layout(const siren_kan_net* n, int64_t rows, int splits, float* base) {
  KanWs w = {};
  int64_t off = 0;
  auto take = [&](int64_t floats) {
    float* p = base ? base + off : nullptr;
    off += al64(floats);
    return p;
  };
  int64_t wmax = 1, wk = 1;
  for (int l = 0; l < n->n_layers; ++l) {
    w.W[l] = take((int64_t)n->width[l + 1] * KAN_K1 * n->width[l]);
    w.WT[l] = take((int64_t)n->width[l + 1] * KAN_K1 * n->width[l]);
    const int64_t kw = (int64_t)n->width[l + 1] * KAN_K1 * n->width[l];
    if (kw > wk) wk = kw;
    if (n->width[l] > wmax) wmax = n->width[l];
  }
  for (int l = 1; l <= n->n_layers; ++l) w.X[l] = take(rows * n->width[l]);
  w.dW = take(wk);
  // split-K slabs: splits x (out x 9 in) for the fused weight gradient, 4 splits x 9 in for the
  // last layer's wave partials
  int64_t slab = wk * splits;
  for (int l = 0; l < n->n_layers; ++l)
    if (n->width[l + 1] == 1 && 4LL * splits * KAN_K1 * n->width[l] > slab) slab = 4LL * splits * KAN_K1 * n->width[l];
  w.slab = take(slab);
  w.slab_floats = slab;
  w.G[0] = take(rows * wmax);
  w.G[1] = take(rows * wmax);
  const int64_t np = (rows + 255) / 256;
  w.sse_part = take(np);
  w.gsum_part = take(np);
  w.gmax_part = take(np);
  w.zero = take(1);
  w.total = off;
  return w;
}

// layers 0 .. nl-1 (nl = n_layers for inference)
hipError_t kan_run_forward(const siren_kan_net* n, const siren_kan_batch* b, const KanWs& w, hipStream_t s, int nl) {
  const int64_t R = b->rows;
  const float* x = b->coords;
  for (int l = 0; l < nl; ++l) {
    const int in = n->width[l], out = n->width[l + 1];
    SIREN_PROF(SIREN_PROF_KAN_MISC, s, kan_combine(n->base_w[l], n->spline_w[l], n->scaler[l], out, in, w.W[l], w.WT[l], s));
    // X[l+1][r][o] = sum_k A[r][k] W[o][k], A = [SiLU(x) | bases(x)] recomputed in LDS
    if (out == 1 && in <= 64)
      SIREN_PROF(SIREN_PROF_KAN_FWD, s, kan_head_fwd(x, n->grid[l], w.W[l], R, in, w.X[l + 1], s));
    else
      SIREN_PROF(SIREN_PROF_KAN_FWD, s, kan_fwd_fused(x, n->grid[l], w.W[l], R, in, out, w.X[l + 1], s));
    x = w.X[l + 1];
  }
  return hipSuccess;
}

// backward of layers l_top .. 0 from G = dLoss/dX[l_top + 1] ([R][out]); the layer inputs X[l] and
// the combined weights are the workspace's from the forward.  grad_coords != NULL: also dLoss/dcoords
// ([R][width[0]]), the first layer's input gradient (the fit itself never needs it).
hipError_t kan_run_backward(const siren_kan_net* net, const siren_kan_grads* gr, const siren_kan_batch* b,
                            const KanWs& w, hipStream_t s, const float* G, int l_top, int cur, float* grad_coords) {
  const int64_t R = b->rows;
  for (int l = l_top; l >= 0; --l) {
    const int in = net->width[l], out = net->width[l + 1];
    const float* xl = l == 0 ? b->coords : w.X[l];
    const int64_t max_splits = w.slab_floats / ((int64_t)out * KAN_K1 * in);
    float* gin = l > 0 ? w.G[cur] : grad_coords;
    if (out <= 64 && gin) {
      // dW and dX = SiLU' dA_base + sum_c B'_c dA_c in one pass (bases and G read once)
      SIREN_PROF(SIREN_PROF_KAN_DX, s, kan_bwd_fused(xl, net->grid[l], G, w.WT[l], R, in, out, max_splits, w.slab,
                                                     w.dW, gin, s));
      SIREN_PROF(SIREN_PROF_KAN_MISC, s, kan_param_grads(w.dW, net->spline_w[l], net->scaler[l], out, in, 1,
                                                         gr->base_w[l], gr->spline_w[l], gr->scaler[l], s));
      G = gin;
      cur ^= 1;
      continue;
    }
    // dW[o][k] = sum_r G[r][o] A[r][k]  (split-K over the coordinates, bases recomputed)
    SIREN_PROF(SIREN_PROF_KAN_DW, s, kan_dw_fused(xl, net->grid[l], G, R, in, out, max_splits, w.slab, w.dW, s));
    SIREN_PROF(SIREN_PROF_KAN_MISC, s, kan_param_grads(w.dW, net->spline_w[l], net->scaler[l], out, in, 1,
                                                       gr->base_w[l], gr->spline_w[l], gr->scaler[l], s));
    if (!gin) break;  // layer 0 without a coordinate gradient
    // dX = SiLU' dA_base + sum_c B'_c dA_spline_c with dA = G W formed per chunk in LDS
    SIREN_PROF(SIREN_PROF_KAN_DX, s, kan_dx_fused(xl, net->grid[l], G, w.WT[l], R, in, out, gin, s));
    G = gin;
    cur ^= 1;
  }
  return hipSuccess;
}

}  // namespace

extern "C" {

int64_t siren_kan_workspace_floats(const siren_kan_net* net, int32_t rows, int32_t splits) {
  if (check_kan(net) || rows < 1 || splits < 1) return -1;
  return kan_layout(net, rows, splits, nullptr).total;
}

int siren_kan_forward(const siren_kan_net* net, siren_kan_batch* b, void* stream) {
  int st = check_kan(net);
  if (st) return st;
  if (!b) return SIREN_ERR_NULL;
  if (!b->coords || !b->out || !b->g || !b->ws) return SIREN_ERR_NULL;
  if (b->rows < 1 || b->splits < 1) return SIREN_ERR_SHAPE;
  hipStream_t s = S(stream);
  const KanWs w = kan_layout(net, b->rows, b->splits, b->ws);
  SIREN_TRY(hipMemsetAsync(w.zero, 0, sizeof(float), s));
  SIREN_TRY(kan_run_forward(net, b, w, s, net->n_layers));
  const int wl = net->width[net->n_layers];
  if (wl != 1)  // a lone KANLinear / a KAN with a wide last layer: out = X[L] as it stands
    return (int)hipMemcpyAsync(b->out, w.X[net->n_layers], (size_t)b->rows * wl * sizeof(float),
                               hipMemcpyDeviceToDevice, s);
  SIREN_TRY(head_loss(w.X[net->n_layers], 1, b->rows, w.zero, b->out, 0, 0.f, b->out, b->g, w.sse_part,
                      w.gsum_part, nullptr, s));
  return SIREN_OK;
}

int siren_kan_train_step(const siren_kan_net* net, const siren_kan_grads* gr, siren_kan_batch* b, void* stream) {
  int st = check_kan(net);
  if (st) return st;
  if (!b || !gr || !gr->sse) return SIREN_ERR_NULL;
  if (!b->coords || !b->target || !b->out || !b->g || !b->ws) return SIREN_ERR_NULL;
  if (b->rows < 1 || b->splits < 1 || b->n_valid < 0 || b->n_valid > b->rows || b->n_total <= 0)
    return SIREN_ERR_SHAPE;
  for (int l = 0; l < net->n_layers; ++l)
    if (!gr->base_w[l] || !gr->spline_w[l] || !gr->scaler[l]) return SIREN_ERR_NULL;
  if (net->width[net->n_layers] != 1) return SIREN_ERR_SHAPE;  // MSELoss on a scalar output
  hipStream_t s = S(stream);
  const int64_t R = b->rows;
  const KanWs w = kan_layout(net, R, b->splits, b->ws);
  if (b->zero_grads && gr->flat) SIREN_TRY(hipMemsetAsync(gr->flat, 0, gr->flat_len * sizeof(float), s));
  SIREN_TRY(hipMemsetAsync(w.zero, 0, sizeof(float), s));
  const int L = net->n_layers;
  // a last layer of width in <= 64 after a hidden layer runs its forward, the MSE gradient and its
  // backward in one pass (kan_head_train); otherwise forward, head_loss, backward
  const bool head_train = L > 1 && net->width[L - 1] <= 64;
  const float gfac = (float)(2.0 / b->n_total);
  const float* G = b->g;
  int cur = 0, l_top = L - 1;
  if (head_train) {
    const int in = net->width[L - 1];
    SIREN_TRY(kan_run_forward(net, b, w, s, L - 1));
    SIREN_PROF(SIREN_PROF_KAN_MISC, s, kan_combine(net->base_w[L - 1], net->spline_w[L - 1], net->scaler[L - 1], 1, in,
                                                   w.W[L - 1], w.WT[L - 1], s));
    int nparts = 0;
    SIREN_PROF(SIREN_PROF_KAN_DW, s, kan_head_train(w.X[L - 1], net->grid[L - 1], w.W[L - 1], b->target, R, in,
                                                    b->n_valid, gfac, w.slab_floats / (KAN_K1 * in), (R + 255) / 256,
                                                    b->out, b->g, w.sse_part, w.slab, w.dW, w.G[cur], &nparts, s));
    SIREN_PROF(SIREN_PROF_KAN_MISC, s, sum_to(w.sse_part, nparts, gr->sse, 1, s));
    SIREN_PROF(SIREN_PROF_KAN_MISC, s, kan_param_grads(w.dW, net->spline_w[L - 1], net->scaler[L - 1], 1, in, 1,
                                                       gr->base_w[L - 1], gr->spline_w[L - 1], gr->scaler[L - 1], s));
    G = w.G[cur];
    cur ^= 1;
    l_top = L - 2;
  } else {
    SIREN_TRY(kan_run_forward(net, b, w, s, L));
    // MSELoss (run.py:168): out, g = 2(out - y)/N_total, squared-error partials
    SIREN_PROF(SIREN_PROF_KAN_MISC, s, head_loss(w.X[L], 1, b->rows, w.zero, b->target, b->n_valid, gfac, b->out, b->g,
                                                 w.sse_part, w.gsum_part, w.gmax_part, s));
    SIREN_PROF(SIREN_PROF_KAN_MISC, s, sum_to(w.sse_part, (int)((R + 255) / 256), gr->sse, 1, s));
  }
  // backward (autograd of run.py:185): G = dLoss/dX[l+1], [R][out]
  SIREN_TRY(kan_run_backward(net, gr, b, w, s, G, l_top, cur, nullptr));
  return SIREN_OK;
}

int siren_kan_backward(const siren_kan_net* net, const siren_kan_grads* gr, siren_kan_batch* b,
                       float* grad_coords, void* stream) {
  int st = check_kan(net);
  if (st) return st;
  if (!b || !gr) return SIREN_ERR_NULL;
  if (!b->coords || !b->g || !b->ws) return SIREN_ERR_NULL;
  if (b->rows < 1 || b->splits < 1) return SIREN_ERR_SHAPE;
  for (int l = 0; l < net->n_layers; ++l)
    if (!gr->base_w[l] || !gr->spline_w[l] || !gr->scaler[l]) return SIREN_ERR_NULL;
  hipStream_t s = S(stream);
  const KanWs w = kan_layout(net, b->rows, b->splits, b->ws);
  if (b->zero_grads && gr->flat) SIREN_TRY(hipMemsetAsync(gr->flat, 0, gr->flat_len * sizeof(float), s));
  SIREN_TRY(kan_run_backward(net, gr, b, w, s, b->g, net->n_layers - 1, 0, grad_coords));
  return SIREN_OK;
}

}  // extern "C"
