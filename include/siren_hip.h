/*
 * siren_hip.h -- C-ABI of libsiren_hip.so, the MI355X (gfx950) SIREN audio-fitting path.
 *
 * The reference (senyuanfan/inr-for-audio) is pure PyTorch and has no FFI; each entry point
 * below replaces the torch eager work behind one reference interface, cited as file:line
 * into the reference tree.  Conventions:
 *   - every pointer is a DEVICE pointer owned by the caller (torch allocates; the library
 *     never allocates, frees or synchronises the host);
 *   - 16-bit tensors (activations, cosines, weight shadows, pre-activation gradients) are
 *     IEEE fp16 passed as uint16_t*, row-major (DESIGN.md "Storage precision": fp16 keeps
 *     the fit at the fp32 reference's quality where bf16 costs ~1.3 dB); fp32 weights use
 *     the nn.Linear layout [out_features][in_features];
 *   - backward pre-activation gradients dZ are stored multiplied by a power-of-two scale
 *     S = gscale[0] (siren_grad_scale); every fp32 gradient leaves unscaled;
 *   - `stream` is a hipStream_t (e.g. torch.cuda.current_stream().cuda_stream);
 *   - every function returns 0 on success, or a non-zero siren_status / hipError_t code
 *     (see siren_status_string), and never aborts the process.
 */
#ifndef SIREN_HIP_H
#define SIREN_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SIREN_ABI_VERSION 12
#define SIREN_MAX_INNER 16  /* max hidden layers (num_sine + num_snake + num_tanh) */
/* hidden widths: 128, 256, 512, 1024, then multiples of 1024 up to this (run as 1024-column
 * windows; models.py pads any other width to the next of these) */
#define SIREN_MAX_HIDDEN 4096
#define SIREN_ROW_TILE 128  /* coordinate rows are padded to a multiple of this */
/* ints in one tile-queue counter set (siren_batch.tileq, siren_inner_fwd's tileq): the
 * hidden-layer forward GEMM's persistent blocks pull their tiles from it.  Caller-owned device
 * memory, any content: the library zeroes it on the stream before every launch that uses it.
 * One set serves every launch of one stream in order; launches that may run concurrently
 * (other streams, other devices, replays of other captured graphs) need sets of their own. */
#define SIREN_TILEQ_INTS 768

enum siren_status {
  SIREN_OK = 0,
  SIREN_ERR_SHAPE = 1001,   /* unsupported / inconsistent shape            */
  SIREN_ERR_NULL = 1002,    /* required pointer missing                    */
  SIREN_ERR_CONFIG = 1003   /* unsupported configuration (e.g. in_dim > 2) */
};

int siren_abi_version(void);
/* ABI 12: hex SHA-256 of the sources this library was compiled from (the .hip and .h files of csrc and this
 * header) and of its compile defines -- the binding compares it with the sources beside it, so a
 * stale or foreign library is refused instead of trusted by file time */
const char* siren_build_id(void);
/* sizeof of the ABI structs, for binding checks: 0 siren_net, 1 siren_grads, 2 siren_batch,
 * 3 siren_opt_state, 4 siren_kan_net, 5 siren_kan_grads, 6 siren_kan_batch, 7 siren_guard
 * (-1: unknown) */
int64_t siren_struct_size(int32_t which);
const char* siren_status_string(int status);

/* ---- device-resident optimizer state: torch.optim.Adam + ReduceLROnPlateau ------------
 * run.py:116-117 (Adam(lr), ReduceLROnPlateau(mode='min', factor=0.8, patience=200,
 * min_lr=min_learning_rate)).  Layout shared with the Python mirror. */
typedef struct siren_opt_state {
  double lr, best, step;
  int32_t num_bad, last_epoch;
  double min_lr, factor, threshold, eps_lr;
  int32_t patience, pad0;
  double beta1, beta2, eps;
} siren_opt_state;

/* ---- fp16 backward range guard (device-resident, optional) ---------------------------
 * The backward stores dZ in fp16 times a power-of-two scale S (siren_grad_scale) chosen so
 * that the head's bound lands under 2^headroom.  siren_apply_update checks the reduced fp32
 * gradients: if any is non-finite while the loss is finite (an fp16 overflow of dZ*S, which
 * fp32 autograd in the reference never has), the Adam and scheduler updates are SKIPPED
 * (nothing advances: no step, no history entry), headroom drops by 4, and the caller's next
 * step recomputes the same gradients with a 16x smaller S -- GradScaler-style, but with no
 * optimizer step lost.  After 1000 clean steps headroom grows back by 1 (up to its initial
 * value).  Zero-initialise it and set headroom = 6 (the fixed value used when NULL).
 * ABI 12: `stalls` counts hand-off waits of the fused last layer (siren_train_step with
 * SIREN_OPT_HEAD_FUSE) that gave up because a band partner never published its head partial (a
 * partner kept off the chip, e.g. CUs held by another process).  Such a step's loss and gradients
 * are void: while stalls != 0 siren_apply_update skips Adam and the scheduler (no step, no history
 * entry, headroom untouched) -- the counter is sticky, the caller reads it, reports the failure and
 * zeroes it before training on. */
typedef struct siren_guard {
  int32_t flag;        /* this step: non-finite gradients seen (written by apply_update)  */
  int32_t headroom;    /* S exponent target: max|g| max|w_head| omega S < 2^headroom       */
  int32_t clean;       /* consecutive clean steps since the last overflow                   */
  int32_t overflows;   /* steps skipped and recomputed so far                               */
  int32_t headroom0;   /* initial / maximum headroom                                       */
  int32_t stalls;      /* fused last layer: timed-out hand-off waits (sticky; ABI 12)       */
} siren_guard;

/* ---- one L x H network (SirenWithSnakeTanh, models.py:306-394) ------------------------
 * net.0 = SineLayer(in, H, is_first, omega0); then L inner layers H -> H, each a
 * SineLayer(H, H, omega) (models.py:114-115), a Linear + Snake(a) (models.py:356-364,
 * 235-241) or a Linear + Tanh (models.py:366-372), in the reference's order (num_sine
 * sines, then num_snake Snakes, then num_tanh Tanhs); last: Linear(H, 1).  act[i] says
 * which (siren_act); a[i] is the Snake's per-channel a [H]. */
enum siren_act { SIREN_ACT_SINE = 0, SIREN_ACT_SNAKE = 1, SIREN_ACT_TANH = 2 };
typedef struct siren_net {
  int32_t in_dim, hidden, n_inner, pad0;
  float omega0, omega;
  const float* W0;                          /* [H][in]  fp32 */
  const float* b0;                          /* [H]           */
  const float* b[SIREN_MAX_INNER];          /* [H]           */
  const uint16_t* Wh[SIREN_MAX_INNER];      /* [H][H] fp16 shadow of W_i   */
  const uint16_t* WTh[SIREN_MAX_INNER];     /* [H][H] fp16 shadow of W_i^T */
  const float* w_head;                      /* [H] (last Linear's weight[0]) */
  const float* b_head;                      /* [1]                          */
  int32_t act[SIREN_MAX_INNER];             /* siren_act of inner layer i   */
  const float* a[SIREN_MAX_INNER];          /* [H] Snake a (SNAKE layers)   */
  /* first_linear=True (models.py:330-333): net.0 is Linear(in, H) + Snake(a0) instead of the
   * first SineLayer (omega0 unused); last_linear=False (models.py:383-385): the last layer is
   * SineLayer(H, 1, head_omega) -- out = sin(head_omega (Y w^T + b)); 0 = the final Linear */
  int32_t first_snake, pad1;
  const float* a0;                          /* [H] (first_snake)            */
  float head_omega, pad2;
} siren_net;

/* gradient destinations (fp32, accumulated into: zero them, or set zero_grads) */
typedef struct siren_grads {
  float* W0; float* b0;
  float* W[SIREN_MAX_INNER]; float* b[SIREN_MAX_INNER];
  float* w_head; float* b_head;
  float* sse;                               /* [2] sum of squared errors of valid rows, then (ABI 12)
                                               the fused hand-off's stall flag: both accumulate like the
                                               gradients and ride the same all-reduce */
  float* flat; int64_t flat_len;            /* if flat != NULL and zero_grads: memset   */
  float* a[SIREN_MAX_INNER];                /* [H] Snake a gradients (SNAKE layers)     */
  float* a0;                                /* [H] first-layer Snake a (first_snake)    */
} siren_grads;

/* per-micro-batch activations and workspace; sizes from siren_workspace_floats() */
typedef struct siren_batch {
  int32_t rows;          /* padded rows, multiple of SIREN_ROW_TILE          */
  int32_t n_valid;       /* valid rows (<= rows)                             */
  double n_total;        /* global coordinate count: MSE mean denominator    */
  int32_t splits;        /* split-K slices of the weight-gradient GEMM       */
  int32_t zero_grads;    /* 1: zero `grads.flat` before accumulating         */
  const float* coords;   /* [rows][in]  */
  const float* target;   /* [rows]      */
  uint16_t* Y[SIREN_MAX_INNER + 1];  /* Y[0..L] fp16 [rows][H]: layer outputs          */
  uint16_t* C[SIREN_MAX_INNER + 1];  /* C[0..L] fp16 [rows][H]: cos(.) of a sine layer,
                                        dY/dz of a Snake / Tanh layer                 */
  uint16_t* dZ[2];       /* fp16 [rows][H] ping-pong pre-activation gradients x S */
  float* out;            /* [rows] model output                                 */
  float* g;              /* [rows] dLoss/dout                                   */
  float* head_part;      /* [H/128][rows]                                       */
  float* sse_part;       /* [rows/256]                                          */
  float* gsum_part;      /* [rows/256]                                          */
  float* gmax_part;      /* [rows/256]  max |g| per block (train / backward)    */
  float* gscale;         /* [2]  {S, 1/S} of this micro-batch's backward        */
  float* col_part;       /* [rows/128][max(2, 2+in)][H]                         */
  float* col_part2;      /* [rows/128][H]                                       */
  float* red_tmp;        /* [4][64][H]  (ABI 10; was [64][H])                   */
  float* slab;           /* [splits][H][H]                                      */
  uint16_t* E[SIREN_MAX_INNER + 1];  /* E[i+1] fp16 [rows][H]: dY/da of Snake inner layer
                                        i; E[0]: of a Linear + Snake first layer (NULL
                                        for other layers)                              */
  /* optional gradient-ready events (hipEvent_t, NULL = none), recorded on `stream` as soon
   * as a bucket's gradients are final in this call -- set them on the LAST micro-batch so a
   * data-parallel caller can all-reduce each bucket on a communication stream while the rest
   * of the backward runs.  [i < L]: inner layer i (W_i, b_i, Snake a_i);
   * [L]: the first layer (W0, b0); [L+1]: the head (w_head, b_head) and `sse`. */
  void* grad_ready[SIREN_MAX_INNER + 2];
  /* run.py:161-169 loss_mode: 0 = MSELoss (sse = sum err^2, g = 2 err / n_total), 1 = L1Loss
   * ('mae': sse slot = sum |err|, g = sign(err) / n_total) */
  int32_t loss_mode;
  /* ABI 11: 1 = gmax_part holds the max|g| partials of a previous siren_train_step /
   * siren_backward on this workspace (same rows).  A Snake last layer then runs fused with the
   * head (the backward scale S must be fixed before the forward, and |Y_L| has no bound, so S is
   * taken from those partials; the range guard catches a step whose |g| outgrew it).  0: a Snake
   * last layer runs unfused.  Sine / Tanh last layers ignore it. */
  int32_t head_scale_prev;
  /* range guard (NULL: fixed headroom 6, no overflow recovery, and the last layer runs unfused).
   * ABI 12: not const -- a fused last layer whose hand-off wait times out counts it in
   * guard->stalls, which voids the step */
  siren_guard* guard;
  int32_t* tileq;            /* SIREN_TILEQ_INTS ints of tile-queue counters on the device of the
                                activations (NULL: the forward GEMM's static tile walk) */
} siren_batch;

/* Workspace sizing / tiling helpers.  siren_nt_tile: tile edge the NT GEMMs use for
 * `rows` coordinates (partial-sum buffers then hold rows/tile rows and head partials
 * hidden/tile rows); siren_dw_tile: tile edge of the weight-gradient GEMM. */
int32_t siren_nt_tile(int32_t rows, int32_t hidden);
int32_t siren_dw_tile(int32_t rows, int32_t hidden);
int32_t siren_default_splits(int32_t rows, int32_t hidden);
int64_t siren_slab_floats(int32_t hidden, int32_t splits);

/* ---- fused path ---------------------------------------------------------------------
 * siren_forward:     run.py:158 / :255  model(model_input) -> batch.out (inference only).
 * siren_train_step:  run.py:158-185     forward + MSELoss + loss.backward() for one
 *                    micro-batch; gradients ACCUMULATE into `grads` (global-N scaling).
 * siren_apply_update:run.py:186-187     optimizer.step() + scheduler.step(loss), then the
 *                    fp16 weight shadows are refreshed.  (`params`, `grads_flat`, `exp_avg`,
 *                    `exp_avg_sq` are the flat fp32 vectors of length n_params.)          */
int siren_forward(const siren_net* net, siren_batch* batch, void* stream);
int siren_train_step(const siren_net* net, const siren_grads* grads, siren_batch* batch,
                     void* stream);
/* loss.backward() through the network for an arbitrary upstream gradient: batch->g holds
 * dLoss/dout (zero on pad rows) and batch->Y/C the activations of a prior siren_forward. */
int siren_backward(const siren_net* net, const siren_grads* grads, siren_batch* batch,
                   void* stream);
int siren_apply_update(const siren_net* net, float* params, const float* grads_flat,
                       float* exp_avg, float* exp_avg_sq, int64_t n_params,
                       float* const* W_fp32 /* [n_inner] views into params */,
                       uint16_t* const* Wh, uint16_t* const* WTh,
                       siren_opt_state* state, const float* sse, double n_total,
                       float* loss_hist, double* lr_hist, int64_t hist_cap,
                       siren_guard* guard /* NULL: no range check */, void* stream);
/* (siren_apply_update: `sse` is siren_grads.sse after any all-reduce -- sse[1] != 0 marks the guard
 * stalled, so every rank skips a step any rank's fused hand-off voided) */

/* ---- individual kernels (parity tests call these one by one) ------------------------ */
/* utils.py:99-109 get_coord: torch.linspace(-1,1,n_total) at [offset, offset+rows) */
int siren_coords_fill(float* t, int64_t rows, int64_t offset, int64_t n_total, void* stream);
/* utils.py:211-220 MultiWaveformFitting grid, rows [offset, offset+rows) of the height-major
 * (time, channel) grid: xy[r] = (linspace(-1,1,height)[k / width], ch[k % width]) with
 * k = offset + r, ch = linspace(-1,1,width) (all 0 when width == 1); rows past
 * height*width are (0, 0).  Bit-exact with torch.linspace. */
int siren_coords_fill_grid(float* xy, int64_t rows, int64_t offset, int64_t height, int32_t width,
                           void* stream);
/* models.py:114-115 first SineLayer: a0 = omega0*(t W0^T + b0) in fp32, Y0 = sin a0 and
 * C0 = cos a0 (one fp32 sincosf range reduction) -> fp16 */
int siren_first_fwd(const float* t, int32_t in_dim, const float* W0, const float* b0, float omega0,
                    int32_t rows, int32_t hidden, uint16_t* Y0, uint16_t* C0, void* stream);
/* models.py:114-115 hidden SineLayer: Y = sin(omega(X W^T + b)), C = cos(.); optional head
 * partial dot (models.py:374-381) when head_w != NULL; tileq: SIREN_TILEQ_INTS ints for the
 * dynamic tile queue (NULL: static tile walk; results are identical) */
int siren_inner_fwd(const uint16_t* X, const uint16_t* Wh, const float* b, float omega, int32_t rows,
                    int32_t hidden, uint16_t* Y, uint16_t* C, const float* head_w, float* head_part,
                    int32_t* tileq, void* stream);
/* siren_train_step's fused last layer (SIREN_OPT_HEAD_FUSE): models.py:114-115 hidden SineLayer,
 * the head (models.py:374-381), MSELoss / L1Loss gradient (run.py:161-169, loss_mode as
 * siren_batch) and the head backward in one launch -- out, g = dLoss/d(head linear output),
 * 256-row sse / gsum partials (as siren_head_loss), dZ = dZ_L x gscale[0] (as siren_head_bwd) and
 * part[rows/256][2][hidden] = column partials of db_L and dw_head.  Y / C are not written.  Needs
 * rows % 256 == 0 and the 256x256 ping-pong NT tiles (else SIREN_ERR_CONFIG); head_part is
 * [hidden/256][rows] scratch. */
int siren_head_fused_fwd(const uint16_t* X, const uint16_t* Wh, const float* b, float omega, int32_t rows,
                         int32_t hidden, const float* w_head, const float* b_head, float head_omega, const float* y,
                         int32_t n_valid, double n_total, int32_t loss_mode, const float* gscale, float* head_part,
                         float* out, float* g, float* sse_part, float* gsum_part, uint16_t* dZ, float* part,
                         void* stream);
/* ABI 11: siren_head_fused_fwd for a last inner layer of any kind (act, siren_act): SINE as
 * siren_head_fused_fwd; SNAKE (models.py:235-241, a = its [hidden] a) and TANH (models.py:366-372)
 * with their derivative in place of the cosine (omega unused) -- dZ, out, g and the partials as
 * siren_inner_fwd_act -> siren_head_loss -> siren_head_bwd compute them at the same gscale;
 * part[rows/256][2][hidden] (db_L, dw_head), Snake part[rows/256][3][hidden] (+ da_L);
 * gmax_part (nullable): [rows/256] max|g| per 256 rows, as siren_head_loss writes it; E (Snake,
 * else ignored): fp16 [rows][hidden], receives the layer's dY/da as siren_inner_fwd_act writes it
 * (the kernel reads it back for the da_L partials) */
int siren_head_fused_fwd_act(const uint16_t* X, const uint16_t* Wh, const float* b, int32_t act, float omega,
                             const float* a, int32_t rows, int32_t hidden, const float* w_head, const float* b_head,
                             float head_omega, const float* y, int32_t n_valid, double n_total, int32_t loss_mode,
                             const float* gscale, float* head_part, float* out, float* g, float* sse_part,
                             float* gsum_part, float* gmax_part, uint16_t* dZ, float* part, uint16_t* E,
                             void* stream);
/* the fused head's backward scale, fixed before the forward: gscale = {S, 1/S} from a bound of
 * max|g| (MSE: (sum|w_head| + |b_head| + max|y|) 2/n_total, or 1 + max|y| through a final sine of
 * head_omega; L1: 1/n_total; x head_omega) x max|w_head| x act_bound (|dY/dz| bound of the last
 * layer); max|y| over the n_valid target rows, ymax_part = (n_valid+255)/256 floats of scratch */
int siren_grad_scale_bound(const float* y, int32_t n_valid, float* ymax_part, const float* w_head,
                           const float* b_head, int32_t hidden, double n_total, float head_omega, int32_t loss_mode,
                           float act_bound, float* gscale, void* stream);
/* any inner layer kind: SINE as siren_inner_fwd; SNAKE (models.py:235-241): z = X W^T + b,
 * Y = z + sin^2(a z)/a, C = 1 + sin(2az), E = (z sin(2az) - sin^2(az)/a)/a; TANH
 * (models.py:366-372): Y = tanh z, C = 1 - Y^2 (a, E unused) */
int siren_inner_fwd_act(const uint16_t* X, const uint16_t* Wh, const float* b, int32_t act,
                        float omega, const float* a, int32_t rows, int32_t hidden, uint16_t* Y,
                        uint16_t* C, uint16_t* E, const float* head_w, float* head_part,
                        int32_t* tileq, void* stream);
/* run.py:125,168 MSELoss + final Linear bias: out, g = 2(out-y)/n_total, partial sums
 * (gmax_part may be NULL); the L1Loss of loss_mode 1 is reached through siren_train_step */
int siren_head_loss(const float* head_part, int32_t nparts, int32_t rows, const float* b_head,
                    const float* y, int32_t n_valid, double n_total, float* out, float* g,
                    float* sse_part, float* gsum_part, float* gmax_part, void* stream);
/* backward storage scale: gscale = {S, 1/S}, S = 2^k with max|g|*max|w_head|*omega*S < 2^6,
 * from the nparts = rows/256 max |g| partials of siren_head_loss (siren_train_step takes the
 * exponent from batch->guard->headroom instead of 6) */
int siren_grad_scale(const float* gmax_part, int32_t nparts, const float* w_head, int32_t hidden,
                     float omega, float* gscale, void* stream);
/* autograd of Linear(H,1) + the last layer's activation: dZ_L = g w_head omega C (x S),
 * db_L partials, dw_head partials (unscaled); gscale NULL = S 1.  Snake / Tanh last layer:
 * omega = 1 (C is their derivative); Snake also passes E and gets da_part (else NULL) */
int siren_head_bwd(const uint16_t* C, const uint16_t* Y, const float* g, const float* w_head,
                   float omega, int32_t rows, int32_t hidden, const float* gscale, uint16_t* dZ,
                   float* db_part, float* dwh_part, const uint16_t* E, float* da_part, void* stream);
/* autograd addmm dX + sin/omega backward of the layer below: dZprev = omega*cos*(dZ W)
 * (carries dZ's scale); db partials multiplied by 1/S (gscale NULL = unscaled) */
int siren_inner_bwd_dx(const uint16_t* dZ, const uint16_t* WTh, const uint16_t* Cprev, float omega_prev,
                       int32_t rows, int32_t hidden, const float* gscale, uint16_t* dZprev,
                       float* db_part, void* stream);
/* the same into a layer below of any kind (act_prev): SINE as above; TANH: dZprev = C (dZ W);
 * SNAKE: dZprev = D (dZ W) and part [rows/tile][2][H] = partials of db and of da = sum (dZ W) E
 * (x 1/S) */
int siren_inner_bwd_dx_act(const uint16_t* dZ, const uint16_t* WTh, const uint16_t* Cprev,
                           const uint16_t* Eprev, int32_t act_prev, float omega_prev, int32_t rows,
                           int32_t hidden, const float* gscale, uint16_t* dZprev, float* part,
                           void* stream);
/* same into the fp32 first layer (C0 from siren_first_fwd): partials [rows/128][1+in][H]
 * of dZ0 and dZ0*t_j (x 1/S); dZ0 itself is never stored */
int siren_first_bwd_dx(const uint16_t* dZ1, const uint16_t* WTh1, const uint16_t* C0, const float* t,
                       int32_t in_dim, float omega0, int32_t rows, int32_t hidden, const float* gscale,
                       float* part, void* stream);
/* autograd addmm dW: slab[s] = partial dZ^T Y over coordinate slice s, tile edge 128/256
 * (0 = siren_dw_tile(rows, hidden)); siren_dw_reduce must get the same tile. */
int siren_inner_bwd_dw(const uint16_t* Y, const uint16_t* dZ, int32_t rows, int32_t hidden,
                       int32_t splits, int32_t tile, float* slab, void* stream);
/* grad (+)= (sum_s slab[s]) * gscale[1]  (gscale NULL = 1) */
int siren_dw_reduce(const float* slab, int32_t splits, int32_t hidden, int32_t tile, float* grad,
                    int32_t accumulate, const float* gscale, void* stream);
int siren_col_reduce(const float* part, int64_t row_stride, int32_t nrows, int32_t ncols, float* out,
                     int32_t out_stride, int32_t accumulate, float* tmp, void* stream);
/* torch.optim.Adam step over a flat fp32 vector (run.py:186) */
int siren_adam_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                    const siren_opt_state* state, void* stream);
/* ReduceLROnPlateau.step(loss) (run.py:187); also increments state->step.  The history slot
 * is state->last_epoch (scheduler steps of this run), not the Adam step: a run resumed from a
 * checkpoint (run.py:84-106) restores the Adam step but builds a fresh scheduler. */
int siren_plateau_step(siren_opt_state* state, const float* sse, double n_total, float* loss_hist,
                       double* lr_hist, int64_t hist_cap, void* stream);
/* fp16 shadows W and W^T of a fp32 [H_out][H_in] weight */
int siren_cast_weight(const float* W, int32_t h_out, int32_t h_in, uint16_t* Wh, uint16_t* WTh,
                      void* stream);

/* ---- unfused fp32 layers: the module API outside the fused step ------------------------
 * A lone SineLayer (models.py:114-120: forward, forward_with_intermediate), nn.Linear, Snake
 * (models.py:235-241) and nn.Tanh -- what SirenWithSnakeTanh.forward_with_activations
 * (models.py:396-423) walks -- in fp32 like the reference (the fused path stores fp16).
 * x [rows][in], W [out][in] (nn.Linear layout), b [out] or NULL; all fp32, row-major. */
enum siren_fp32_act { SIREN_FP32_IDENTITY = 0, SIREN_FP32_SIN = 1, SIREN_FP32_TANH = 2, SIREN_FP32_SNAKE = 3 };
/* pre = omega * (x W^T + b)  (models.py:115 `self.omega_0 * self.linear(input)`; omega 1: nn.Linear) */
int siren_fp32_linear(const float* x, int64_t rows, int32_t in, int32_t out, const float* W, const float* b,
                      float omega, float* pre, void* stream);
/* y = act(x) elementwise over [rows][cols]: sin (models.py:115), tanh, Snake x + sin^2(a x)/a with a [cols] */
int siren_fp32_act(int32_t act, const float* x, int64_t rows, int32_t cols, const float* a, float* y, void* stream);
/* autograd of siren_fp32_act for dL/dy = gy: gx = gy * act'(x); Snake also da [cols] = column sums of
 * gy * dy/da (da_prod: rows*cols floats of scratch, tmp: 64*cols floats; both NULL otherwise) */
int siren_fp32_act_bwd(int32_t act, const float* x, int64_t rows, int32_t cols, const float* a, const float* gy,
                       float* gx, float* da, float* da_prod, float* tmp, void* stream);
/* autograd of siren_fp32_linear for dL/dpre = gpre (overwritten with omega * gpre): gW [out][in] via
 * `splits` split-K slices over the rows into `slab` (splits*out*in floats), gb [out] and gx [rows][in]
 * (either NULL: not computed); tmp: 64*out floats */
int siren_fp32_linear_bwd(const float* x, int64_t rows, int32_t in, int32_t out, const float* W, float omega,
                          float* gpre, float* gx, float* gW, float* gb, float* slab, int32_t splits, float* tmp,
                          void* stream);

/* ---- KAN variant: run.py:92-93 KAN([in, H, H, 1]) of kan.py:169-285 ----------
 * Layer l maps width[l] -> width[l+1] as efficient-KAN's KANLinear (kan.py:6-166) with
 * grid_size 5, spline_order 3, SiLU base: out = SiLU(x) base_w^T + B(x) (spline_w*scaler)^T,
 * B = the 8 order-3 B-spline bases on the layer's `grid` buffer [in][12].  fp32 throughout.
 * siren_kan_forward / _backward take any last width (out is then [rows][last width]); the fused
 * fit step (siren_kan_train_step) needs last width 1.  Workspace: one caller-owned fp32 buffer of
 * siren_kan_workspace_floats(net, rows, splits) floats (activations, combined weights,
 * gradients of the layer outputs, split-K slabs -- the expansions are never stored). */
#define SIREN_KAN_MAX_LAYERS 8
typedef struct siren_kan_net {
  int32_t n_layers, pad0;
  int32_t width[SIREN_KAN_MAX_LAYERS + 1];
  const float* grid[SIREN_KAN_MAX_LAYERS];      /* [in][12]     buffer layers.l.grid        */
  const float* base_w[SIREN_KAN_MAX_LAYERS];    /* [out][in]    layers.l.base_weight        */
  const float* spline_w[SIREN_KAN_MAX_LAYERS];  /* [out][in][8] layers.l.spline_weight      */
  const float* scaler[SIREN_KAN_MAX_LAYERS];    /* [out][in]    layers.l.spline_scaler      */
} siren_kan_net;
typedef struct siren_kan_grads {
  float* base_w[SIREN_KAN_MAX_LAYERS];
  float* spline_w[SIREN_KAN_MAX_LAYERS];
  float* scaler[SIREN_KAN_MAX_LAYERS];
  float* sse;                               /* [2] sum of squared errors of valid rows, then (ABI 12)
                                               the fused hand-off's stall flag: both accumulate like the
                                               gradients and ride the same all-reduce */
  float* flat; int64_t flat_len;            /* if flat != NULL and zero_grads: memset   */
} siren_kan_grads;
typedef struct siren_kan_batch {
  int32_t rows, n_valid;    /* rows: any count >= n_valid (no padding needed)      */
  double n_total;           /* global coordinate count (MSE mean denominator)      */
  int32_t splits;           /* split-K slices of the weight-gradient GEMMs (>= 1)  */
  int32_t zero_grads;
  const float* coords;      /* [rows][width[0]]  */
  const float* target;      /* [rows]            */
  float* out;               /* [rows] model output                                */
  float* g;                 /* [rows] dLoss/dout                                  */
  float* ws;                /* workspace, siren_kan_workspace_floats() floats     */
} siren_kan_batch;
int64_t siren_kan_workspace_floats(const siren_kan_net* net, int32_t rows, int32_t splits);
/* run.py:255 model(model_input) for arch='kan' */
int siren_kan_forward(const siren_kan_net* net, siren_kan_batch* batch, void* stream);
/* run.py:158-185 for arch='kan': forward + MSELoss + backward; gradients ACCUMULATE (last width 1) */
int siren_kan_train_step(const siren_kan_net* net, const siren_kan_grads* grads, siren_kan_batch* batch,
                         void* stream);
/* autograd of siren_kan_forward (kan.py:153-166, 268-273) for an arbitrary upstream gradient:
 * batch->g holds dLoss/dout [rows][last width] and batch->ws the workspace of a siren_kan_forward
 * of the same coords, rows and splits; gradients ACCUMULATE (zero_grads + flat: memset first);
 * grad_coords != NULL also receives dLoss/dcoords [rows][width[0]] (grads->sse is not used). */
int siren_kan_backward(const siren_kan_net* net, const siren_kan_grads* grads, siren_kan_batch* batch,
                       float* grad_coords, void* stream);

/* ---- per-launch HIP-event profiling of the fused path (bench.py) --------------------
 * siren_profile_enable(n) creates 2n hipEvents; while enabled every launch made by
 * siren_train_step / siren_backward / siren_forward / siren_apply_update (and the KAN
 * entry points, kinds 8..11) is bracketed
 * by events on its stream (eager launches only; not meant for graph capture).
 * siren_profile_read sums the elapsed time of all records of one kind (synchronises). */
enum siren_prof_kind {
  SIREN_PROF_FIRST_FWD = 0, SIREN_PROF_INNER_FWD = 1, SIREN_PROF_HEAD = 2, SIREN_PROF_BWD_DW = 3,
  SIREN_PROF_BWD_DX = 4, SIREN_PROF_BWD_DX0 = 5, SIREN_PROF_REDUCE = 6, SIREN_PROF_UPDATE = 7,
  /* KAN variant (siren_kan_train_step / siren_kan_forward): KAN_FWD the fused forward layers
   * (and the inference head); KAN_DW the last layer's training pass (forward, MSE gradient,
   * backward) and the first layer's weight gradient (+ slab reduces); KAN_DX the hidden layers'
   * one-pass backward (dW and dX); KAN_MISC the small rest */
  SIREN_PROF_KAN_FWD = 8, SIREN_PROF_KAN_DW = 9, SIREN_PROF_KAN_DX = 10, SIREN_PROF_KAN_MISC = 11,
  /* the last hidden layer fused with the head, the loss gradient and the head backward
   * (siren_train_step with SIREN_OPT_HEAD_FUSE; counted apart from INNER_FWD) */
  SIREN_PROF_HEAD_FWD = 12,
  SIREN_PROF_NKINDS = 13
};
/* tuning knobs for in-process A/B measurement (process-global; 0 = automatic):
 * SIREN_OPT_NT_TILE / SIREN_OPT_TN_TILE = 128 or 256 forces the GEMM tile edge;
 * SIREN_OPT_NT_PIPE = 256x256 NT GEMM K-loop: -1 automatic (4), 0 BK 64 one tile per block,
 * 1 BK 64 persistent double buffer, 4 BK 64 persistent with two wave groups in ping-pong; the
 * plain forward (no head) also takes the one-wave-per-SIMD measurement kernels 5 (128x256 tiles,
 * the epilogue under the next tile's MFMAs), 6 (256x256, BK 32, 4-stage ring) and 7 (pipe 5's K loop
 * with the epilogue at the tile's end), bit-identical to 4; other modes take 4;
 * SIREN_OPT_TN_PIPE = -1..4 selects the 256x256 dW K-loop (-1 automatic = 4; 0: BK 64 double
 * buffer, 1: BK 32 4-slot ring, 2: BK 32 5-slot ring, 3: BK 64 ping-pong in 16-MFMA phases,
 * 4: BK 64 ping-pong in 32-MFMA segments);
 * SIREN_OPT_NT_GRID = persistent NT grid size (0 = one block per CU; tests use small
 * values so every block walks several tiles);
 * SIREN_OPT_NT_DIAG = measurement-only NT ablations, accepted only by libraries built with
 *   -DSIREN_DIAG (__graft_entry__.build_diagnostic; the product library returns
 *   SIREN_ERR_CONFIG for any non-zero value); results are WRONG while set: bit 0 reads the X
 *   operand from the first 4 row bands only (L2-resident operand), bit 3 from the first 256 row bands
 *   (an X of 128 MB: Infinity-Cache-resident, not L2); ping-pong K-loop only: bit 2
 *   reads W from column tile 0 only (L2-resident W), bit 9 runs no tiles, bit 10 skips the
 *   epilogue (its compute and stores);
 * SIREN_OPT_NT_QUEUE = 1 (default): the ping-pong NT GEMM's persistent blocks take their tiles
 * from the caller's tile-queue set (siren_batch.tileq; 8 shard heads, agent-scope atomics) in the
 * forward modes, 2: in every mode, 0: never (the static walk b, b + G, ...).  Results are
 * identical.  (Options 5 and 7, the round-2 start stagger and X L2-prefetch distance, were
 * measured neutral or slower and retired with their kernels: they return SIREN_ERR_CONFIG.)
 * SIREN_OPT_HB_FAULT = measurement / test hook of the fused last layer's hand-off, accepted only by
 *   -DSIREN_DIAG libraries (product: SIREN_ERR_CONFIG for non-zero): bit 0 -- the blocks of column
 *   tile 1 never publish their head partials; value >> 8 (when non-zero) -- the wait's poll limit
 *   (default 2^23 polls of s_sleep 1, ~1.3 s).  Used to drive the timeout branch in tests.
 * SIREN_OPT_HEAD_FUSE = 1 (default): siren_train_step runs a sine last layer on 256x256
 * ping-pong tiles as one launch with the head, the loss gradient and the head backward
 * (dZ_L is written instead of Y_L / C_L; the backward scale S then comes from a bound of
 * max|g| known before the forward); 0: separate forward, head_loss and head_bwd launches. */
enum siren_option {
  SIREN_OPT_NT_TILE = 0, SIREN_OPT_TN_TILE = 1, SIREN_OPT_NT_PIPE = 2, SIREN_OPT_TN_PIPE = 3,
  SIREN_OPT_NT_GRID = 4, SIREN_OPT_NT_DIAG = 6, SIREN_OPT_NT_QUEUE = 8, SIREN_OPT_HEAD_FUSE = 9,
  SIREN_OPT_HB_FAULT = 10
};
int siren_set_option(int32_t option, int32_t value);
int siren_profile_enable(int32_t max_records);
int siren_profile_reset(void);
/* bit k set: launches of kind k are bracketed (default all).  bench.py times its steps with only
 * the dominant kind bracketed, so the events cost the timed region ~2 records per launch of that
 * kind instead of ~2 per launch of the step (measured: all kinds add 2-13% to a step). */
int siren_profile_mask(uint32_t kinds);
int siren_profile_read(int32_t kind, double* total_ms, int64_t* count);

#ifdef __cplusplus
}
#endif
#endif /* SIREN_HIP_H */
