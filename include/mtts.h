/*
 * mtts.h — C ABI of libmtts.so, the MI355X (gfx950) kernels behind the
 * MambaTTSDecoder hot path of whcorkran/mamba-TTS-project.
 *
 * Boundary: the reference decoder calls `mamba_ssm.Mamba` (mamba_decoder.py:4,
 * :29, :61, :63), whose CUDA extension entry points are what these functions
 * replace.  The [upstream] mamba-ssm / causal-conv1d packages are neither
 * vendored nor pinned by the reference (environment.yml:1-150, README.md:29),
 * so the "reference interface" column below names the upstream pybind
 * function each entry point stands in for, plus the reference call site.
 *
 * Conventions
 *  - Plain C: pointers, sizes, element strides.  No torch types.
 *  - Every tensor is caller-allocated device memory; the library never
 *    allocates, frees or synchronises (safe inside hipGraph capture).
 *  - Work is enqueued on `stream` (a hipStream_t; NULL = legacy default).
 *  - Return 0 on success, a negative MTTS_E* code on failure; the message is
 *    in mtts_last_error() (thread-local).
 *  - Activations are CHANNEL-LAST: element (b, t, c) of a (B, L, C) tensor is
 *    at  ptr[b*bstride + t*lstride + c]  (channel stride 1).  This is the
 *    layout the projections produce; mamba-ssm's (B, D, L) layout is a
 *    permutation of it (the math is identical).
 *  - dtype codes: MTTS_F32 / MTTS_BF16 for activations; states, A, D,
 *    biases, reductions and all accumulation are fp32.
 */
#ifndef MTTS_H
#define MTTS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MTTS_ABI_VERSION 14

enum { MTTS_F32 = 0, MTTS_BF16 = 1 };
enum {
  MTTS_OK = 0,
  MTTS_EINVAL = -22,       /* bad shape / stride / dtype / null pointer   */
  MTTS_EUNSUPPORTED = -95, /* valid but not on a built fast path          */
  MTTS_ELAUNCH = -5        /* hipGetLastError after the launch             */
};

int mtts_abi_version(void);
const char* mtts_last_error(void);

/* Kernel-path overrides (test and measurement hooks; no reference
 * counterpart).  Every key defaults to MTTS_OVR_AUTO (-1): the library picks
 * the path from the shapes.  A value forces a path so the tests can reach
 * kernels the C2 / north-star shapes never select (the narrow-stride scan,
 * the P-lane scan at large B*D, the generic attention kernels, ...).  The
 * table is process-wide: set it between launches, never while another
 * thread launches.  Returns the previous value, or MTTS_EINVAL for an
 * unknown key. */
enum {
  MTTS_OVR_AUTO = -1,
  MTTS_OVR_SCAN_PATH = 0,     /* forward: 1 one-lane-per-channel (c1), 2 LDS-DMA P-lane (w2), 3 narrow */
  MTTS_OVR_SCAN_P = 1,        /* lanes per channel of the P-lane kernels: 2 or 4 */
  MTTS_OVR_SCAN_SEGS = 2,     /* forward L segments (>= 1) */
  MTTS_OVR_SCAN_BWD_SEGS = 3, /* backward L segments (>= 1) */
  MTTS_OVR_GEMM_NARROW = 4,   /* 1: the single-group GEMM kernel with 8-byte epilogue stores */
  MTTS_OVR_ATTN_CHUNKS = 5,   /* attention backward query chunks (>= 1) */
  MTTS_OVR_ATTN_BWD = 6,      /* attention backward: 1 fused one-pass kernel, 2 split dQ + dK/dV passes */
  MTTS_OVR_ATTN_GENERIC = 7,  /* 1: generic MFMA attention kernels only (no short-key / long-key / q_len-1 kernels) */
  MTTS_OVR_CONV_UNTILED = 8,  /* 1: the untiled causal-conv kernels */
  MTTS_OVR_GEMM_TILE = 9,     /* NT bf16 GEMM: 1 eight-wave ping-pong tile, 2 four-wave 128x128-per-wave tile */
  MTTS_OVR_ATTN_DQ_DMA = 10,  /* long-key attention dQ pass (bf16 hd 64): 1 K / V blocks by LDS-DMA, else registers */
  MTTS_OVR_COUNT = 11
};
int mtts_set_override(int key, int value);
int mtts_get_override(int key);

/* ------------------------------------------------------------------------
 * Selective scan.  Replaces [upstream] selective_scan_cuda.fwd / .bwd
 * (mamba_ssm/ops/selective_scan_interface.py: SelectiveScanFn), reached from
 * the reference at mamba_decoder.py:61 (full sequence) / :63 (with state).
 *
 *   delta <- softplus(delta + delta_bias)          (if delta_softplus)
 *   h_t    = exp(delta_t * A) h_{t-1} + delta_t B_t u_t ,  h_{-1} = h0 or 0
 *   y_t    = <h_t, C_t> + D u_t ;   out_t = y_t * silu(z_t)  (if z)
 * u, delta, z, out : (B, L, D) channel-last, dtype `dtype_io`
 * Bm, Cm           : (B, L, N) with N stride 1, dtype `dtype_bc`
 * A                : (D, N) fp32, D/delta_bias : (D) fp32, h0/last_state :
 * (B, D, N) fp32.  dstate N must be 16 (mamba-ssm default d_state).
 * ckpt (optional)  : (B, ceil(L/ckpt_chunk), D, N) fp32 — h at the START of
 *                    every chunk of `ckpt_chunk` steps (the backward's
 *                    restart points; upstream saves `x` chunk states too).
 * ------------------------------------------------------------------------ */
typedef struct {
  int batch, dim, seqlen, dstate;
  int dtype_io, dtype_bc;
  int delta_softplus;
  int ckpt_chunk;                 /* 16 iff ckpt != NULL (the backward chunk) */
  int a_is_log;                   /* 1: `A` holds A_log and A = -exp(A_log) is formed in-kernel;
                                     the backward's dA is then d/dA_log (= dA * A) */
  int reserved_;
  int64_t u_bs, u_ls;             /* element strides (batch, time)       */
  int64_t delta_bs, delta_ls;
  int64_t z_bs, z_ls;
  int64_t out_bs, out_ls;
  int64_t B_bs, B_ls;
  int64_t C_bs, C_ls;
  const void* u;
  const void* delta;
  const float* A;
  const void* Bm;
  const void* Cm;
  const float* D;          /* optional */
  const void* z;           /* optional */
  const float* delta_bias; /* optional */
  const float* h0;         /* optional */
  void* out;
  float* last_state;       /* optional */
  float* ckpt;             /* optional */
  void* workspace;         /* mtts_selective_scan_fwd_workspace() bytes */
} MttsScanFwdArgs;

/* Scratch for the sequence-segment pass (0 bytes when B*D fills the chip). */
int64_t mtts_selective_scan_fwd_workspace(int batch, int dim, int seqlen, int dstate);
int mtts_selective_scan_fwd(const MttsScanFwdArgs* a, void* stream);

/* Backward of the forward above (requires the forward's ckpt).
 * dout : (B, L, D) dtype_io.  Outputs (caller-allocated):
 *   du, ddelta, dz : (B, L, D) dtype_io (dz only if z; ddelta is w.r.t. the
 *                    RAW delta, i.e. through softplus and delta_bias)
 *   dB, dC         : (B, L, N) fp32 with strides dB_bs/dB_ls (N stride 1)
 *   dA             : (D, N) fp32   dD, ddelta_bias : (D) fp32  (overwritten)
 *   dh0            : optional (B, D, N) fp32 gradient w.r.t. h0
 *   workspace      : mtts_selective_scan_bwd_workspace() bytes            */
typedef struct {
  MttsScanFwdArgs f;      /* same tensors / shapes as the forward call */
  const void* dout;
  int64_t dout_bs, dout_ls;
  void* du;      int64_t du_bs, du_ls;
  void* ddelta;  int64_t ddelta_bs, ddelta_ls;
  void* dz;      int64_t dz_bs, dz_ls;
  float* dB;     int64_t dB_bs, dB_ls;
  float* dC;     int64_t dC_bs, dC_ls;
  float* dA;
  float* dD;
  float* ddelta_bias;
  float* dh0;
  void* workspace;
} MttsScanBwdArgs;

int64_t mtts_selective_scan_bwd_workspace(int batch, int dim, int seqlen, int dstate);
int mtts_selective_scan_bwd(const MttsScanBwdArgs* a, void* stream);

/* ------------------------------------------------------------------------
 * Causal depthwise conv1d (width K <= 4) + bias + optional SiLU.
 * Replaces [upstream] causal_conv1d_cuda.causal_conv1d_fwd / _bwd
 * (causal-conv1d package; torch fallback HF:81-101), reached through
 * Mamba.forward from mamba_decoder.py:61/:63.
 *   out[b,t,c] = act( sum_k w[c,k] * xx[b, t-(K-1)+k, c] + bias[c] )
 * where xx is x preceded by the K pre-conv inputs in conv_state_in
 * (B, D, K) (zeros when NULL).  conv_state_out (B, D, K), optional, receives
 * the last K inputs of [conv_state_in ‖ x] (mamba-ssm prefill semantics).
 * ------------------------------------------------------------------------ */
typedef struct {
  int batch, dim, seqlen, width;
  int dtype;                      /* x / out / dx / dout */
  int silu;
  int64_t x_bs, x_ls, out_bs, out_ls;
  const void* x;
  const float* w;                 /* (D, K) */
  const float* bias;              /* optional (D) */
  const float* conv_state_in;     /* optional (B, D, K) */
  void* out;
  float* conv_state_out;          /* optional (B, D, K) */
} MttsConvFwdArgs;

int mtts_causal_conv1d_fwd(const MttsConvFwdArgs* a, void* stream);

typedef struct {
  MttsConvFwdArgs f;
  const void* dout; int64_t dout_bs, dout_ls;
  void* dx;         int64_t dx_bs, dx_ls;
  float* dw;        /* (D, K)  overwritten */
  float* dbias;     /* (D)     overwritten, optional */
  void* workspace;  /* mtts_causal_conv1d_bwd_workspace() bytes */
} MttsConvBwdArgs;

int64_t mtts_causal_conv1d_bwd_workspace(int batch, int dim, int seqlen, int width);
int mtts_causal_conv1d_bwd(const MttsConvBwdArgs* a, void* stream);

/* ------------------------------------------------------------------------
 * Decode step (L = 1).  Replaces [upstream] causal_conv1d_update and
 * selective_state_update (Mamba.step; HF:61-78, HF:128-171), reached from
 * mamba_decoder.py:63 via decode_step (:188-256).  Both update the state
 * tensors IN PLACE (as upstream does) — safe for hipGraph replay.
 * ------------------------------------------------------------------------ */
typedef struct {
  int batch, dim, width, dtype, silu;
  int64_t x_bs, out_bs;
  const void* x;       /* (B, D) */
  float* conv_state;   /* (B, D, K) in/out */
  const float* w;      /* (D, K) */
  const float* bias;   /* optional */
  void* out;           /* (B, D) */
} MttsConvUpdateArgs;

int mtts_causal_conv1d_update(const MttsConvUpdateArgs* a, void* stream);

typedef struct {
  int batch, dim, dstate, dtype_io, dtype_bc, dt_softplus;
  int64_t x_bs, dt_bs, z_bs, out_bs, B_bs, C_bs;
  float* state;              /* (B, D, N) in/out */
  const void* x;             /* (B, D) */
  const void* dt;            /* (B, D) raw delta */
  const float* A;            /* (D, N) */
  const void* Bm;            /* (B, N) */
  const void* Cm;            /* (B, N) */
  const float* D;            /* optional */
  const void* z;             /* optional */
  const float* dt_bias;      /* optional */
  void* out;                 /* (B, D) */
  /* optional fused dt_proj (Mamba.step: dt = dt_proj(x_db[:, :dt_rank])):
   * with dt_rank > 0, `dt` is the (B, dt_rank) low-rank input (row stride
   * dt_bs, dtype_io) and raw delta[b, c] = sum_r dt[b, r] * dt_w[c, r],
   * dt_w (D, dt_rank) row-major, dtype_io. */
  int dt_rank;
  const void* dt_w;
  /* optional: out also written as a packed activation image (xpk_index;
   * batch <= 32, dim % 32 == 0, bf16) for the out_proj projection; out may
   * then be NULL */
  void* out_packed;
} MttsStateUpdateArgs;

int mtts_selective_state_update(const MttsStateUpdateArgs* a, void* stream);


/* ------------------------------------------------------------------------
 * LayerNorm (eps) with optional fused FiLM, optional fused residual add.
 * Replaces torch nn.LayerNorm at mamba_decoder.py:59,67,81,184 and the FiLM
 * modulation h = gamma*h + beta of mamba_decoder.py:82-86.
 *   if res:   xs = x + res   (xs written to x_sum when x_sum != NULL)
 *   y = LN(xs) * w + b ;  if gamma: y = gamma[row / rows_per_group] * y
 *                                     + beta[row / rows_per_group]
 * x/res/x_sum/y: (M, N) rows with row strides; gamma/beta: (G, N) with row
 * stride gb_stride (fp32 or dtype).  mean/rstd: (M) fp32, saved for bwd.
 * ------------------------------------------------------------------------ */
typedef struct {
  int rows, cols, dtype, rows_per_group;
  float eps;
  int64_t x_rs, res_rs, xsum_rs, y_rs, gb_rs;
  const void* x;
  const void* res;         /* optional */
  void* x_sum;             /* optional, written when res != NULL */
  const float* w;
  const float* b;
  const void* gamma;       /* optional */
  const void* beta;        /* optional (required iff gamma) */
  int gb_dtype;
  void* y;
  float* mean;
  float* rstd;
} MttsLNArgs;

int mtts_layernorm_fwd(const MttsLNArgs* a, void* stream);

/* Decode-step LayerNorm(+FiLM) of <= 32 rows straight into the packed
 * activation image of the next projection (csrc/gemv.hip): y_packed =
 * image of bf16(LN(x) * w + b [, gamma * . + beta]) (bf16 x, gamma, beta;
 * rows_per_group 1; cols % 32 == 0; a->y / res / mean / rstd unused). */
int mtts_layernorm_rows_packed(const MttsLNArgs* a, void* y_packed, void* stream);

/* Backward: dy (M, N) -> dx (M, N) [+= dx_acc if given: dx = dx_acc + LN'],
 * dw, db (N) fp32, dgamma/dbeta (G, N) fp32 (when gamma; row stride dgb_rs,
 * 0 = N, so both can live in one (G, 2N) gamma|beta gradient).  Uses the
 * saved mean/rstd and the normalised input (x, or x_sum when res was fused).
 * dx_colsum (optional, N fp32): the column sums of dx over all M rows, as
 * stored (dtype-rounded) -- the bias gradient of the linear layer whose
 * output is this LayerNorm's input (mamba_decoder.py:77/:88 out_proj / ff[2]
 * bias), so that layer needs no column-sum launch of its own. */
typedef struct {
  MttsLNArgs f;
  const void* dy;   int64_t dy_rs;
  const void* dx_acc; int64_t dxacc_rs;   /* optional residual-stream grad */
  void* dx;         int64_t dx_rs;
  float* dw;
  float* db;
  float* dgamma;
  float* dbeta;
  void* workspace;  /* mtts_layernorm_bwd_workspace() bytes */
  float* dx_colsum; /* optional (ABI 9) */
  int64_t dgb_rs;   /* row stride of dgamma / dbeta (ABI 9; 0 = cols) */
} MttsLNBwdArgs;

int64_t mtts_layernorm_bwd_workspace(int rows, int cols, int rows_per_group);
int mtts_layernorm_bwd(const MttsLNBwdArgs* a, void* stream);

/* ------------------------------------------------------------------------
 * Column sums over row-major rows: out[g*out_gstride + c] = sum over rows r
 * of group g (rows_per_group consecutive rows) of in[r*row_stride + c], fp32
 * accumulation, deterministic order.  Used for bias gradients (sum of dy over
 * tokens; torch Linear/MHA bias grads at mamba_decoder.py:32-48) and FiLM
 * gradients.  dtype: MTTS_F32 / MTTS_BF16 input.
 * ------------------------------------------------------------------------ */
int64_t mtts_colsum_workspace(int rows, int cols, int rows_per_group);
int mtts_colsum(const void* in, int dtype, int rows, int cols, int64_t row_stride, int rows_per_group, float* out,
                int64_t out_gstride, void* workspace, void* stream);

/* ------------------------------------------------------------------------
 * Multi-head cross-attention core (no projections):
 *   out[b, t, h*hd:(h+1)*hd] = softmax_s(scale * q_h[t] . k_h[s] + mask) v_h
 * Replaces the attention inside nn.MultiheadAttention(batch_first=True) as
 * called at mamba_decoder.py:72-77 (decoder -> [ref ‖ text]) and
 * style_cross_attention.py:125-131,270-276 (torch's
 * F.multi_head_attention_forward / scaled_dot_product_attention).
 * q (B, Tq, H*hd), k/v (B, Tk, H*hd) channel-last with unit channel stride;
 * key_padding_mask (B, Tk) bytes, nonzero = ignore the key (torch's
 * key_padding_mask=True), NULL = none.  A query whose keys are ALL masked
 * yields NaN, as torch MHA does.  lse (B, H, Tq) fp32 receives
 * ln sum_s exp(scale * q.k_s) (-inf for fully masked rows); the backward
 * needs it.  hd in {16, 32, 64, 128}; bf16 uses bf16 MFMA, f32 uses f32 MFMA.
 * Strides and q/k/v/out base pointers must be 16-byte aligned.
 * ------------------------------------------------------------------------ */
typedef struct {
  int batch, heads, head_dim, q_len, kv_len;
  int dtype;                 /* MTTS_F32 / MTTS_BF16 for q, k, v, out */
  float scale;               /* usually 1/sqrt(head_dim) */
  int64_t q_bs, q_ls, k_bs, k_ls, v_bs, v_ls, o_bs, o_ls;  /* element strides */
  int64_t mask_bs;           /* key_padding_mask batch stride (bytes) */
  const void* q;
  const void* k;
  const void* v;
  const uint8_t* key_padding_mask;
  void* out;
  float* lse;                /* may be NULL (inference) */
  /* q_len == 1 only, optional: out also written as a packed activation
   * image of (batch, heads * head_dim) (xpk_index; batch <= 32, bf16) for
   * the output projection; out may then be NULL */
  void* out_packed;
  /* q_len == 1 only, optional: element stride between heads of k / v
   * (0 = head_dim, heads contiguous inside a row).  With k / v stored
   * head-major (B, H, S, hd): k_bs = v_bs = H*S*hd, k_ls = v_ls = hd,
   * kv_hs = S*hd, so each (batch, head) reads one contiguous K and V block. */
  int64_t kv_hs;
} MttsAttnFwdArgs;

int mtts_attention_fwd(const MttsAttnFwdArgs* a, void* stream);

/* Single-query cross-attention with the query projection fused in
 * (csrc/attn.hip, ABI 10; the decode step, mamba_decoder.py:72-77 ->
 * nn.MultiheadAttention's q = LN_cross(x) Wq^T + bq): per (batch, head)
 * q_h = bf16(LN(x_b) Wq_h^T + bq_h) with LN(x) = bf16((x - mean) rstd w + b)
 * (two-pass statistics, as the projection kernels' LayerNorm prologue), then
 * the single-pass decode attention of mtts_attention_fwd.  f.q is ignored;
 * bf16, q_len 1, head_dim 64 / 128, batch <= 32, the single-pass key range;
 * d_model <= 2048.  out and / or out_packed as mtts_attention_fwd. */
typedef struct {
  MttsAttnFwdArgs f;
  const void* x;       /* (batch, d_model) bf16 residual rows, row stride x_rs */
  int64_t x_rs;
  const void* wq;      /* (heads * head_dim, d_model) bf16 row-major (16-byte aligned) */
  const void* bq;      /* (heads * head_dim) bf16, or NULL */
  const float* ln_w;   /* (d_model) */
  const float* ln_b;
  float eps;
  int d_model;
} MttsAttnQProjArgs;
int mtts_attention_decode_qproj(const MttsAttnQProjArgs* a, void* stream);

/* Backward: dout -> dq, dk, dv (same dtype as q).  f.out / f.lse must hold
 * the forward's results.  Deterministic (no atomics). */
typedef struct {
  MttsAttnFwdArgs f;
  const void* dout; int64_t do_bs, do_ls;
  void* dq;         int64_t dq_bs, dq_ls;
  void* dk;         int64_t dk_bs, dk_ls;
  void* dv;         int64_t dv_bs, dv_ls;
  void* workspace;           /* mtts_attention_bwd_workspace() bytes */
} MttsAttnBwdArgs;

int64_t mtts_attention_bwd_workspace(int batch, int heads, int head_dim, int q_len, int kv_len, int dtype);
int mtts_attention_bwd(const MttsAttnBwdArgs* a, void* stream);

/* ------------------------------------------------------------------------
 * Length regulator (phoneme -> frame expansion).  Replaces the Python loop of
 * style_cross_attention.py:156-198 (LengthRegulator.forward: round, clamp
 * >= 0, repeat rows, one .item() per (b, phoneme)) and its autograd.
 *   dur[b,t]   = max(round_half_even(durations[b,t]), 0)
 *   lengths[b] = sum_t dur[b,t]                       (int64, pre-truncation)
 *   out[b,f,:] = hidden[b, t(f), :] for f < min(lengths[b], max_len), else 0
 * with t(f) the phoneme whose interval [end_{t-1}, end_t) of running duration
 * sums holds f.  The backward writes every row of dhidden:
 *   dhidden[b,t,:] = sum_{f in [end_{t-1}, min(end_t, max_len))} dout[b,f,:]
 * (fp32 accumulation, fixed order).  durations: fp32 (B, T) with batch stride
 * dur_bs; hidden/out/dout/dhidden: (B, rows, D) with unit element stride,
 * dtype MTTS_F32 / MTTS_BF16.  T <= 4096.
 * ------------------------------------------------------------------------ */
int mtts_length_regulate_lengths(const float* durations, int64_t dur_bs, int batch, int T, int64_t* lengths,
                                 void* stream);
int mtts_length_regulate_fwd(const void* hidden, int dtype, int batch, int T, int D, int64_t h_bs, int64_t h_ls,
                             const float* durations, int64_t dur_bs, int max_len, void* out, int64_t o_bs,
                             int64_t o_ls, void* stream);
int mtts_length_regulate_bwd(const void* dout, int dtype, int batch, int T, int D, int64_t do_bs, int64_t do_ls,
                             const float* durations, int64_t dur_bs, int max_len, void* dhidden, int64_t dh_bs,
                             int64_t dh_ls, void* stream);

/* ------------------------------------------------------------------------
 * Compute-dtype weight copies for the decoder's GEMMs, one launch per step:
 * for every descriptor, the contiguous fp32 master src (rows x cols) is
 * rounded (RNE) to bf16 into dst (rows x cols, contiguous) and, when dstT is
 * not NULL, into dstT = src^T (cols x rows, contiguous).  Stands in for the
 * per-parameter `.to(bfloat16)` casts an autocast region would make of the
 * reference's fp32 nn.Linear / nn.MultiheadAttention weights
 * (mamba_decoder.py:26-48, mamba_ssm Mamba projections); dstT feeds the
 * data-gradient GEMMs.  `descs` is a DEVICE array of n descriptors sorted
 * by tile0, where tile0 is the running sum of mtts_cast_tiles(rows, cols)
 * of the descriptors before it; total_tiles is the sum over all.
 * ------------------------------------------------------------------------ */
typedef struct {
  const float* src;
  void* dst;
  void* dstT;       /* may be NULL */
  int rows, cols;
  int64_t tile0;
} MttsCastDesc;

int64_t mtts_cast_tiles(int rows, int cols);
int mtts_cast_bf16_multi(const MttsCastDesc* descs, int n, int64_t total_tiles, void* stream);

/* ------------------------------------------------------------------------
 * Fused gradient clipping + Adam over a parameter list (train.py:232-235:
 * torch.nn.utils.clip_grad_norm_(params, max_norm) then torch.optim.Adam
 * .step(), default Adam: L2 weight_decay, no amsgrad).  With max_norm > 0
 * the update uses g * min(1, max_norm / (||g||_2 + 1e-6)) (gradients are not
 * rewritten); max_norm <= 0 disables clipping.  `tensors` is a DEVICE array
 * of n fp32 tensors (p, g, exp_avg, exp_avg_sq: numel each), sorted by
 * chunk0 = running sum of mtts_adam_chunks(numel).  step_counter (device
 * int32) holds the steps taken; the call increments it and derives the bias
 * corrections from it on the device (graph-replayable).  norm_out (device,
 * 4 floats) receives {total grad norm, clip coefficient, lr/(1-b1^t),
 * sqrt(1-b2^t)}.  Deterministic.
 * ------------------------------------------------------------------------ */
typedef struct {
  float* p;
  const float* g;
  float* m;
  float* v;
  int64_t n;
  int64_t chunk0;
} MttsAdamTensor;

int64_t mtts_adam_chunks(int64_t numel);
int64_t mtts_adam_workspace(int64_t total_chunks);
int mtts_clip_adam(const MttsAdamTensor* tensors, int ntensors, int64_t total_chunks, int* step_counter, float lr,
                   float beta1, float beta2, float eps, float weight_decay, float max_norm, void* workspace,
                   float* norm_out, void* stream);

/* ------------------------------------------------------------------------
 * Embedding sum of the decoder prologue (mamba_decoder.py:167-171:
 * token_embed(tokens) + pos_embed(arange(T)) + quant_embed(quant_ids)) and of
 * the reference-voice path (train.py:115-131 embed_codec_tokens: positions
 * arange(T_ref).repeat(Q), quantizers arange(Q).repeat_interleave(T_ref)):
 *   out[b,l,:] = tok_w[tokens[b,l]] + q_w[quant_ids[l]] + pos_w[pos_ids[l]]
 * tokens int64 (B, L) with batch stride tok_bs; quant_ids / pos_ids int32
 * (L) shared by the batch; tables fp32 contiguous (rows x d), d % 4 == 0;
 * out (B, L, d) contiguous rows, batch stride out_bs, dtype MTTS_F32/BF16.
 * A token outside [0, vocab) sets *err_flag = 1 (device int32, caller
 * zeroed) and leaves its row unwritten (nn.Embedding raises).
 * ------------------------------------------------------------------------ */
int mtts_embed_sum(const int64_t* tokens, int64_t tok_bs, const int* quant_ids, const int* pos_ids,
                   const float* tok_w, const float* q_w, const float* pos_w, int batch, int L, int d, int vocab,
                   void* out, int dtype, int64_t out_bs, int* err_flag, void* stream);

/* Gradient of a small embedding table (ABI 14; csrc/regulate.hip): the
 * token-embedding backward of mamba_decoder.py:167 (token_embed) and
 * train.py:115-131 (the reference embedding through the same table) for the
 * codec vocabulary (train.py's 10 codes):
 *   out[v, c] = sum over rows r with ids[r] == v of g[r * g_rs + c]   (fp32)
 * ids int64 (n), g (n, d) MTTS_F32 / MTTS_BF16 rows of whole 16-byte pieces
 * (d and g_rs multiples of 4 / 8, g 16-byte aligned), vocab <= 16; ids
 * outside [0, vocab) contribute nothing (the forward flags them).  One pass
 * over g, fixed-order sums (bitwise reproducible).  workspace: at least
 * mtts_embed_table_grad_workspace(n, d, vocab) bytes. */
int64_t mtts_embed_table_grad_workspace(int64_t n, int d, int vocab);
int mtts_embed_table_grad(const int64_t* ids, int64_t n, const void* g, int dtype, int64_t g_rs, int d, int vocab,
                          float* out, void* workspace, void* stream);

/* ------------------------------------------------------------------------
 * Decode-step projections (MambaTTSDecoder.decode_step, mamba_decoder.py:
 * 188-256 -> Mamba.step in_proj/x_proj/out_proj, the cross-attention q/out
 * projections, the FFN and the head of every step):
 *   y = act(x W^T + bias), act 0 = identity, 1 = GELU (exact erf, F.gelu)
 * bf16 in / out, fp32 accumulation; x is M x K (M <= 32 rows, row stride
 * ldx), W is N x K (the nn.Linear weight, row stride ldw), bias bf16 or
 * NULL, y M x N (row stride ldy).  K % 64 == 0; x, W 16-byte aligned.
 * Optional fusions (they remove the LayerNorm and conv-update launches of
 * the step):
 *  - ln_w != NULL, LayerNorm prologue: the x operand is first replaced by
 *    bf16(LN(x) * ln_w + ln_b) (fp32 ln_w / ln_b of length K, eps ln_eps),
 *    then gamma * . + beta per row when gamma != NULL (bf16 (M, K), row
 *    stride ld_gb): exactly mtts_layernorm_fwd's output (mamba_decoder.py:
 *    59,67,81,184 and the FiLM of :82-86) consumed in place.  K <= 2048.
 *  - res != NULL, residual epilogue: y = bf16(bf16(product) + res) (bf16
 *    (M, N), row stride ld_res): the residual-stream value that
 *    mtts_layernorm_fwd writes to x_sum.
 *  - conv_dim > 0 (a multiple of 32; not with res): columns c < conv_dim
 *    also go through Mamba.step's causal_conv1d_update (width 4) + SiLU on
 *    the bf16 value of y[:, c]: conv_state (M, conv_dim, 4) fp32 shifted in
 *    place, u[:, c] (bf16, row stride ldu) = silu(conv_state . conv_w[c] +
 *    conv_b[c]).
 * ------------------------------------------------------------------------ */
typedef struct {
  int M, N, K, act;
  int64_t ldx, ldw, ldy;
  const void* x;
  const void* W;
  const void* bias;          /* optional */
  void* y;
  int conv_dim;              /* 0 = no conv epilogue */
  float* conv_state;
  const float* conv_w;
  const float* conv_b;       /* optional */
  void* u;
  int64_t ldu;
  const float* ln_w;         /* NULL = no LayerNorm prologue */
  const float* ln_b;
  float ln_eps;
  const void* gamma;         /* optional FiLM */
  const void* beta;
  int64_t ld_gb;
  const void* res;           /* NULL = no residual epilogue */
  int64_t ld_res;
  /* kgroups > 1: the K range is also split over kgroups workgroups per
   * 32-column tile (K % (64 * kgroups) == 0, kgroups <= 32); fp32 partials
   * go to splitk_slab (ceil(N / 32) * kgroups * 1024 floats) and the last
   * workgroup of a tile (one ticket per tile in splitk_count, ceil(N / 32)
   * ints that must be ZERO before the first launch; the kernel resets them)
   * sums them in fixed order and runs the epilogue. */
  int kgroups;
  float* splitk_slab;
  int* splitk_count;
  /* w_packed = 1: W is mtts_pack_rows_weight's image of the (N, K) weight
   * (ldw ignored, kgroups must be <= 1): one 16-column tile per workgroup,
   * the K range over up to 8 waves, every weight load a coalesced KiB
   * (csrc/gemv.hip).  Needs K / 32 = KS * S, KS <= 8 a power of 2,
   * S in {1, 2, 4, 8, 16}; the fusions above all apply, LayerNorm at any
   * such K. */
  int w_packed;
  /* Packed activations (csrc/common.h xpk_index: the B-fragment order of the
   * packed kernel, 32 * K elements, M <= 32, K % 32 == 0):
   *  x_packed = 1: x is such an image (ldx ignored; w_packed required)
   *                -> coalesced KiB operand loads; with the LayerNorm
   *                prologue the FiLM gamma / beta are images too (ld_gb
   *                ignored);
   *  y_packed != NULL: y is also written as an image of (M, N) (N % 32 == 0;
   *                y may then be NULL), for the next projection;
   *  u_packed != NULL: u of the conv epilogue also written as an image. */
  int x_packed;
  void* y_packed;
  void* u_packed;
} MttsRowsArgs;

int mtts_gemm_rows(const MttsRowsArgs* a, void* stream);

/* ------------------------------------------------------------------------
 * Codec-token cross-entropy with ignore index: replaces train.py:31-42
 * codec_ce_loss = F.cross_entropy(logits.view(B*T, V), targets.view(B*T),
 * ignore_index=pad_id) (mean over the non-ignored rows; NaN when all are
 * ignored, as torch).  logits (rows, vocab) with row stride ld, F32 or BF16;
 * targets int64 (rows).  Forward: loss[0] = mean loss, loss[1] = count,
 * lse (rows) fp32 saved; workspace mtts_cross_entropy_workspace(rows) bytes.
 * Backward: dlogits = (softmax - onehot) * grad_loss[0] / count on the
 * non-ignored rows, 0 elsewhere (grad_loss read on the device). fp32 math,
 * fixed-order reductions (deterministic).
 * ------------------------------------------------------------------------ */
typedef struct {
  int64_t rows;
  int vocab;
  int dtype;                 /* MTTS_F32 / MTTS_BF16 logits (and dlogits) */
  int64_t ld;
  const void* logits;
  const int64_t* targets;
  int ignore_index;
  float* loss;               /* 2 floats: mean loss, non-ignored count */
  float* lse;                /* rows */
  float* workspace;
} MttsCrossEntropyArgs;

int64_t mtts_cross_entropy_workspace(int64_t rows);
int mtts_cross_entropy_fwd(const MttsCrossEntropyArgs* a, void* stream);
int mtts_cross_entropy_bwd(const MttsCrossEntropyArgs* a, const float* grad_loss, void* dlogits, int64_t ld_dlogits,
                           void* stream);

/* Packed image of a bf16 decode weight W (N, K), row stride ldw (K % 64 == 0,
 * 16-byte aligned): for 16-column tile t and k-step s, the 64 lanes'
 * v_mfma_f32_16x16x32_bf16 A fragments W[16t + l%16][32s + 8(l/16) .. +8]
 * are one contiguous KiB; rows past N are zero.  out holds
 * mtts_pack_rows_bytes(N, K) bytes (16-byte aligned).  Made once per decode
 * context (DecodeEngine), stream-ordered. */
int64_t mtts_pack_rows_bytes(int N, int K);
int mtts_pack_rows_weight(const void* W, int64_t ldw, int N, int K, void* out, void* stream);


/* ------------------------------------------------------------------------
 * Training-path GEMM (replaces the nn.Linear / Mamba in_proj, x_proj,
 * dt_proj, out_proj / MHA in/out projection / FFN matmuls of
 * mamba_decoder.py:29-43 as applied at :61-88, forward and backward).
 * bf16 operands, fp32 accumulation on v_mfma_f32_16x16x32_bf16.
 *   layout NT: C[m,n] = A[m,k] . B[n,k]^T  (A, B k-contiguous; row strides
 *              lda, ldb): forward x W^T, data gradient dy (W^T)^T
 *   layout TN: C[m,n] = A[k,m]^T . B[k,n]  (A, B m/n-contiguous): weight
 *              gradient dy^T x; fp32 out, no epilogue, optional split-K
 *              (splits > 1: fp32 partial slabs in `workspace`,
 *              mtts_gemm_workspace() bytes, summed in fixed order)
 * out_dtype 0 = fp32 (C = AB + beta C), 1 = bf16 with epilogues:
 *   BIAS  : + bias[n] (bias_dtype 0 fp32 / 1 bf16)
 *   GELU  : aux[m,n] = bf16(AB (+bias)) (pre-activation, for the backward),
 *           C = bf16(gelu(aux))  (exact erf; F.gelu on the bf16 value)
 *   DGELU : C = bf16(bf16(AB) * gelu'(aux[m,n]))  (GELU backward fused into
 *           the data gradient of the layer that consumes the activation)
 * Requirements: k % (64 * splits) == 0, n % 8 == 0 (TN: m % 8 == 0 too),
 * A/B 16-byte aligned with row strides a multiple of 8 elements, C 16-byte
 * aligned with ldc % 4 == 0.
 * ------------------------------------------------------------------------ */
#define MTTS_GEMM_NT 0
#define MTTS_GEMM_TN 1
#define MTTS_GEMM_EPI_BIAS 1
#define MTTS_GEMM_EPI_GELU 2
#define MTTS_GEMM_EPI_DGELU 4
typedef struct {
  int m, n, k;
  int layout;                /* MTTS_GEMM_NT / MTTS_GEMM_TN */
  int splits;                /* TN split-K factor (1 = none) */
  int epilogue;              /* MTTS_GEMM_EPI_* flags (bf16 out only) */
  int out_dtype;             /* 0 fp32, 1 bf16 */
  int bias_dtype;            /* 0 fp32, 1 bf16 */
  int64_t lda, ldb, ldc, ld_aux;
  const void* a;
  const void* b;
  void* c;
  const void* bias;          /* optional */
  void* aux;                 /* GELU / DGELU pre-activation (bf16 m x n) */
  void* workspace;           /* split-K slabs */
  float beta;                /* fp32 out: C = AB + beta C */
} MttsGemmArgs;

int64_t mtts_gemm_workspace(const MttsGemmArgs* a);
int mtts_gemm(const MttsGemmArgs* a, void* stream);

/* Grouped weight gradients (ABI 9; 24 problems since ABI 10): `n` (1..24) TN problems, each C_i =
 * A_i^T B_i (+ C_i when beta_i = 1) with fp32 out, no epilogue, no split-K,
 * in ONE launch; every output tile reduces its problem's whole K in one
 * workgroup (no partial slabs, no reduce pass).  Put the longest-K problems
 * first.  The deferred weight-gradient engine (mtts/wgrad.py) gathers a decoder
 * layer's projection weight gradients (mamba_decoder.py:29-43 in/out_proj,
 * MHA q/kv/out, FFN) into one such launch. */
int mtts_gemm_grouped(const MttsGemmArgs* probs, int n, void* stream);

/* ------------------------------------------------------------------------
 * fp32 MFMA GEMM over WINDOWED row matrices (csrc/convgemm.hip, ABI 10): the
 * text encoder's / duration predictor's convolutions as direct implicit-GEMM
 * convolutions (FastSpeech2 PositionwiseFeedForward Conv1d k = 9 / 1 and
 * VariancePredictor Conv k = 3; reference text_encoder.py:80-85, 118-122,
 * 131-209 -> the un-vendored FastSpeech2 modules; replaces nn.Conv1d there).
 * Row r of an operand starts at ptr + (r / seg_rows) * seg_stride +
 * (r % seg_rows) * row_stride (elements) and is contiguous; on a zero-padded
 * channel-last activation (B, T + 2p, C) with seg_rows = T, seg_stride =
 * (T + 2p) C, row_stride = C, a row of K*C elements is the conv window.
 *   NT: C[m,n] = sum_k A[row m][k] B[row n][k]
 *   TN: C[m,n] = sum_k A[row k][m] B[row k][n]
 *   NN: C[m,n] = sum_k A[row m][k] B[row k][n]  (MTTS_CONVGEMM_NN: the data
 *       gradient straight from the forward's weight layout, no transpose)
 * C rows through the same map (n contiguous).  fp32 everywhere, exact-f32
 * MFMA products, fp32 accumulation.  n % 4 == 0; NT k % 4 == 0, TN m % 4 ==
 * 0; 16-byte aligned pointers, strides multiples of 4 elements.  Epilogues
 * (bf16 GEMM's not reused: fp32 out): + bias[n]; ReLU; ReLU backward
 * (C = result where aux[row m][n] > 0, else 0); beta: C = result + beta C.
 * ------------------------------------------------------------------------ */
#define MTTS_CONVGEMM_NN 2   /* convgemm only: C[m,n] = sum_k A[row m][k] B[row k][n] */
#define MTTS_CONVGEMM_BIAS 1
#define MTTS_CONVGEMM_RELU 2
#define MTTS_CONVGEMM_DRELU 4
typedef struct {
  const void* ptr;
  int64_t seg_rows, seg_stride, row_stride;
  /* halo_c > 0 (a 'same' convolution's window over the UNPADDED activation,
   * (B, T, C) with seg_rows = T, seg_stride = T C, row_stride = C, halo_c = C,
   * halo_p = p): row r = (b, t) starts at ptr + b seg_stride + (t - p) C and
   * its element e reads 0 where tap t - p + e / C falls outside [0, T) -- the
   * zero padding without a padded copy.  Only on NT / NN operand A and TN
   * operand B, halo_c % 32 == 0. */
  int32_t halo_c, halo_p;
} MttsRowMap;
typedef struct {
  int layout;                /* MTTS_GEMM_NT / MTTS_GEMM_TN / MTTS_CONVGEMM_NN */
  int m, n, k;
  MttsRowMap a, b, c, aux;   /* aux: the ReLU output for MTTS_CONVGEMM_DRELU */
  const float* bias;
  int epilogue;              /* MTTS_CONVGEMM_* bits */
  float beta;
  int splits;                /* > 1: K split over workgroups, fp32 partial slabs summed in fixed order */
  void* workspace;           /* splits > 1: mtts_convgemm_workspace() bytes */
  float* colsum_a;           /* TN only, optional (ABI 12): colsum_a[m] = sum_k A[row k][m] -- with A = dy,
                                the bias gradient, summed by the weight-gradient kernel from its own A tiles */
} MttsConvGemmArgs;
int64_t mtts_convgemm_workspace(const MttsConvGemmArgs* a);
int mtts_convgemm(const MttsConvGemmArgs* a, void* stream);

/* ------------------------------------------------------------------------
 * Skinny bf16 GEMMs of the Mamba mixer's inner projections (csrc/skinny.hip).
 * Replace the x_proj / dt_proj matmuls of [upstream] mamba_inner_fn
 * (x_dbl = F.linear(u, x_proj.weight); delta = dt_proj.weight @ dt^T, and
 * their data gradients), reached from the reference at mamba_decoder.py:61
 * through Mamba(d_model) (:29).
 *   C[m,n] = A[m,k] . B[n,k]^T + beta * C     (A, B bf16, k-contiguous rows)
 *   mode SKINNY_N  : n <= 128 (one workgroup per row block, K split over its
 *                    4 waves, fixed-order sum)
 *   mode SMALL_K   : k <= 128 (64 x 256 output tiles)
 * k % 32 == 0, n % 4 == 0; A / B 16-byte aligned, lda / ldb multiples of 8;
 * C bf16 (8-byte aligned) or fp32 (16-byte aligned), ldc % 4 == 0;
 * beta 0 or 1 (accumulate into C, e.g. du += d(x_dbl) W_x).
 *   mode SKINNY_TN : C[m,n] = A[k,m]^T . B[k,n] (both token-major), the
 *                    x_proj / dt_proj weight gradients: n <= 128, n % 8 == 0,
 *                    m % 128 == 0, fp32 C contiguous (ldc = n, or = m with
 *                    trans_c: C^T (n x m) is written), beta = 0; chunk
 *                    partials in `workspace` (mtts_gemm_skinny_workspace()
 *                    bytes), summed in fixed order.
 * ------------------------------------------------------------------------ */
#define MTTS_SKINNY_N 0
#define MTTS_SKINNY_SMALL_K 1
#define MTTS_SKINNY_TN 2
typedef struct {
  int mode;                  /* MTTS_SKINNY_N / MTTS_SKINNY_SMALL_K / MTTS_SKINNY_TN */
  int m, n, k;
  int c_dtype;               /* MTTS_F32 / MTTS_BF16 */
  float beta;
  int64_t lda, ldb, ldc;
  const void* a;
  const void* b;
  void* c;
  void* workspace;           /* SKINNY_TN only */
  int trans_c;               /* SKINNY_TN: write C^T */
  int reserved_;
} MttsSkinnyArgs;

int64_t mtts_gemm_skinny_workspace(const MttsSkinnyArgs* a);
int mtts_gemm_skinny(const MttsSkinnyArgs* a, void* stream);

/* ------------------------------------------------------------------------
 * Dropout (ABI 13; csrc/dropout.hip).  Replaces nn.Dropout / F.dropout in
 * the training paths of style_cross_attention.py (:38-46, 100-109, 133,
 * 246-255, 278) and of the text encoder's FastSpeech2 blocks
 * (text_encoder.py:80-85, 168).
 *   y[i] = x[i] * keep(i) / (1 - p),  keep(i) = hash(seed, i) >= p * 2^32
 * a counter-based mask: the backward passes the SAME seed and regenerates
 * it (dx = dy * keep / (1 - p)); no mask is stored.  With `pre` (bf16, n
 * elements): y = bf16(bf16(x * keep / (1 - p)) * gelu'(pre)), the backward of
 * dropout(gelu(pre)) in one pass (exact-erf GELU, torch's GeluBackward).
 * `group` > 1: one mask draw per `group` consecutive elements (index i /
 * group; a multiple of 8 for bf16, 4 for fp32): attention-weight dropout
 * over a single key, one draw per (batch, head, query) shared by the head's
 * channels.  Contiguous x / y / pre, 16-byte aligned; n % 8 == 0;
 * 0 <= p < 1; x == y allowed (in place).
 * `x_rep` > 1 (ABI 14): x is broadcast over a middle dimension -- y is
 * (n / (x_rep * x_inner), x_rep, x_inner), x is (n / (x_rep * x_inner),
 * x_inner) and y[o, r, c] drops x[o, c] (x_inner a multiple of 8 / 4; no
 * `pre`, not in place): the single-key attention's value row expanded over
 * the queries without a materialised copy.  `seed_in` (optional, device
 * int64): added to `seed` -- a base that a captured step advances, so a
 * replayed hipGraph draws fresh masks; `seed_out` (optional) receives the
 * base the forward used, for its backward's `seed_in`.
 * ------------------------------------------------------------------------ */
typedef struct {
  int64_t n;
  int dtype;                 /* MTTS_F32 / MTTS_BF16 (x and y) */
  float p;
  uint64_t seed;
  const void* x;
  void* y;
  const void* pre;           /* optional bf16 GELU pre-activation (DGELU form) */
  int group;                 /* elements per mask draw (0 / 1: every element) */
  int x_rep;                 /* ABI 14: > 1 = x broadcast x_rep times over the middle dimension */
  int x_inner;               /* ABI 14: the broadcast rows' length (elements) */
  int reserved_;
  const int64_t* seed_in;    /* ABI 14, optional: device int64 added to `seed` (graph-replayable base) */
  int64_t* seed_out;         /* ABI 14, optional: receives *seed_in (the forward's record for its backward) */
} MttsDropoutArgs;

int mtts_dropout(const MttsDropoutArgs* a, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MTTS_H */
