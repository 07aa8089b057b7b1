// Decode-step projections on PACKED weights (decode_step, reference
// mamba_decoder.py:188-256; C4: 32 sequences, one token each).
//
// The step's projections are weight-streaming problems: 32 rows of x against
// 2-8 MB of bf16 weights, each weight byte read once per step.  What bounds
// them is how fast the whole matrix can be put in flight, not arithmetic:
//  * the weights are re-laid ONCE per decode context (mtts_pack_rows_weight)
//    into v_mfma_f32_16x16x32_bf16 A-fragment order: for a 16-column tile t
//    and a 32-deep k-step s, the 64 lanes' 16-byte fragments are one
//    contiguous KiB, so every weight load of a wave is a fully coalesced 1 KiB
//    (the row-major layout touched 32 rows x 32 B per instruction);
//  * one 16-column tile per workgroup (N = 1024 -> 64 workgroups, N = 4096 ->
//    256), the K range split over KS <= 8 waves, each issuing ALL of its
//    S <= 16 weight loads and x loads up front (no trips: one memory latency
//    per launch instead of one per trip);
//  * x (L2-resident, just written by the previous launch) is the B operand,
//    rows 0-15 and 16-31 as two MFMAs per k-step sharing the weight fragment;
//  * the KS partial 16x32 tiles are summed through LDS in fixed wave order
//    (deterministic) by 128 threads that own 4 consecutive columns of one row
//    each, with the epilogues of csrc/rows.hip: bias, exact-erf GELU, the
//    residual add (y = bf16(bf16(xW^T + b) + res)), the causal-conv1d update
//    + SiLU of Mamba.step on in_proj's x half; and the LayerNorm(+FiLM)
//    prologue with row statistics from the operand registers (per-wave
//    partials summed through LDS in fixed order).
#include "common.h"

namespace mtts {
namespace {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kMaxKS = 8;   // 512-thread workgroups: 256 VGPRs per lane

__device__ __forceinline__ f32x4 mfma16(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

// packed[((t * nsteps + s) * 64 + lane) * 8 + q] = W[16 t + lane % 16][32 s + 8 (lane / 16) + q]
// (zero for rows >= N); one thread per 16-byte fragment
__global__ void pack_rows_kernel(const bf16_t* __restrict__ W, int64_t ldw, int N, int K, uint4* __restrict__ out,
                                 int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int nsteps = K >> 5;
  const int lane = (int)(idx & 63);
  const int64_t ts = idx >> 6;
  const int s = (int)(ts % nsteps);
  const int t = (int)(ts / nsteps);
  const int n = t * 16 + (lane & 15), k = s * 32 + 8 * (lane >> 4);
  uint4 v = make_uint4(0, 0, 0, 0);
  if (n < N) v = *reinterpret_cast<const uint4*>(W + (int64_t)n * ldw + k);
  out[idx] = v;
}

__device__ __forceinline__ float gelu_erf(float s) { return 0.5f * s * (1.f + erff(s * 0.70710678118654752f)); }

// S: k-steps per wave (K = 32 * S * KS, KS = blockDim.x / 64); LNM:
// 0 none, 1 LayerNorm prologue, 2 LayerNorm + FiLM; CONV: conv-update
// epilogue operands present
template <int S, int LNM, bool CONV, bool XP>
__global__ __launch_bounds__(64 * kMaxKS) void gemv16_kernel(const MttsRowsArgs a) {
  constexpr bool LNP = LNM > 0, FILM = LNM == 2;

  __shared__ __attribute__((aligned(16))) f32x4 red[kMaxKS][2][64];
  __shared__ float psum[LNP ? kMaxKS : 1][32], psq[LNP ? kMaxKS : 1][32];
  const int KS = blockDim.x >> 6;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int tile = blockIdx.x, n0 = tile * 16;
  const int M = a.M, N = a.N;
  const int nsteps = a.K >> 5;
  const int s0 = wave * S;
  const bool two = M > 16;

  // ---- x fragments (B operand): rows r and 16 + r, k = 32 (s0 + j) + 8 g.
  // Rows >= M read row 0: they only feed output rows that are never stored.
  const int kx = 32 * s0 + 8 * g;
  const bf16_t* x0 = (const bf16_t*)a.x + (int64_t)(r < M ? r : 0) * a.ldx + kx;
  const bf16_t* x1 = (const bf16_t*)a.x + (int64_t)(16 + r < M ? 16 + r : 0) * a.ldx + kx;
  s16x8 xf0[S], xf1[S];
#pragma unroll
  for (int j = 0; j < S; ++j) {
#ifdef GEMV_DIAG_NOX   // timing-only build: no x operand loads
    xf0[j] = s16x8{(short)j, 1, 2, 3, 4, 5, 6, (short)r};
    xf1[j] = xf0[j];
#else
    if constexpr (XP) {   // packed image: the two halves of k-step s0 + j are consecutive KiB
      const s16x8* xp = reinterpret_cast<const s16x8*>(a.x) + (int64_t)(s0 + j) * 128 + lane;
      xf0[j] = xp[0];
      xf1[j] = xp[64];
    } else {
      xf0[j] = *reinterpret_cast<const s16x8*>(x0 + 32 * j);
      xf1[j] = *reinterpret_cast<const s16x8*>(x1 + 32 * j);   // unconditional: a branch here drains vmcnt
    }
#endif
  }

  // ---- LayerNorm parameters / FiLM rows, also ahead of the weights: vmcnt
  // retires in issue order, so anything the prologue waits for must be
  // issued before the weight loads or the prologue waits for the weights
  float4 lw[LNP ? S : 1][2], lb[LNP ? S : 1][2];
  s16x8 ga0[FILM ? S : 1], ba0[FILM ? S : 1], ga1[FILM ? S : 1], ba1[FILM ? S : 1];
  if constexpr (LNP) {
    const bf16_t* gp = (const bf16_t*)a.gamma;
    const bf16_t* bp = (const bf16_t*)a.beta;
    const int64_t o0 = (int64_t)(r < M ? r : 0) * a.ld_gb + kx, o1 = (int64_t)(16 + r < M ? 16 + r : 0) * a.ld_gb + kx;
#ifdef GEMV_DIAG_NOLNP   // timing-only build: no LayerNorm parameter / FiLM loads
    const float4 one4 = make_float4(1.f, 1.f, 1.f, (float)r);
#pragma unroll
    for (int j = 0; j < S; ++j) {
      lw[j][0] = lw[j][1] = lb[j][0] = lb[j][1] = one4;
      if constexpr (FILM) ga0[j] = ba0[j] = ga1[j] = ba1[j] = s16x8{1, 2, 3, 4, 5, 6, 7, (short)j};
    }
    if (false)
#endif
#pragma unroll
    for (int j = 0; j < S; ++j) {
      lw[j][0] = *reinterpret_cast<const float4*>(a.ln_w + kx + 32 * j);
      lw[j][1] = *reinterpret_cast<const float4*>(a.ln_w + kx + 32 * j + 4);
      lb[j][0] = *reinterpret_cast<const float4*>(a.ln_b + kx + 32 * j);
      lb[j][1] = *reinterpret_cast<const float4*>(a.ln_b + kx + 32 * j + 4);
      if constexpr (FILM && XP) {   // packed FiLM images: coalesced KiB like x
        const int64_t o = (int64_t)(s0 + j) * 128 * 8 + lane * 8;
        ga0[j] = *reinterpret_cast<const s16x8*>(gp + o);
        ba0[j] = *reinterpret_cast<const s16x8*>(bp + o);
        ga1[j] = *reinterpret_cast<const s16x8*>(gp + o + 512);
        ba1[j] = *reinterpret_cast<const s16x8*>(bp + o + 512);
      } else if constexpr (FILM) {
        ga0[j] = *reinterpret_cast<const s16x8*>(gp + o0 + 32 * j);
        ba0[j] = *reinterpret_cast<const s16x8*>(bp + o0 + 32 * j);
        ga1[j] = *reinterpret_cast<const s16x8*>(gp + o1 + 32 * j);
        ba1[j] = *reinterpret_cast<const s16x8*>(bp + o1 + 32 * j);
      }
    }
  }
  // ---- all of this wave's weight fragments: S contiguous KiB
  const s16x8* wp = reinterpret_cast<const s16x8*>(a.W) + ((int64_t)tile * nsteps + s0) * 64 + lane;
  s16x8 wf[S];
#pragma unroll
  for (int j = 0; j < S; ++j) {
#ifdef GEMV_DIAG_NOW   // timing-only build (tools/diag_build.sh): no weight stream
    wf[j] = xf0[j];
#else
    // non-temporal: every weight byte is read once per step and the step's
    // ~0.4 GB of weights exceed the Infinity Cache (decode p50 0.775 ->
    // 0.755 ms, C4, three interleaved rounds; hot-cache per-call timings equal)
    wf[j] = __builtin_nontemporal_load(wp + j * 64);
#endif
  }
  // ---- epilogue operands, fetched before the product (threads < 128:
  // half = row block, 4 consecutive columns nb..nb+3 of row m)
  const int et = threadIdx.x;
  const bool epi = et < (two ? 128 : 64);
  const int half = (et >> 6) & 1, el = et & 63;
  const int m = 16 * half + (el & 15), nb = n0 + 4 * (el >> 4);
  const bool mok = epi && m < M;
  // every load below is unconditional (clamped indices, dummy pointers for
  // absent operands, selects afterwards): a branch around a load makes the
  // compiler drain vmcnt, i.e. wait for the weights in flight
  // (a select after the load is sunk into a branch by the compiler: the
  // absent operands are masked bitwise instead)
  // (dummy: the output row 0 / its packed image, valid for every column < N)
  const int mc = m < M ? m : M - 1;
  const bf16_t* dummy = (const bf16_t*)(a.y ? a.y : a.y_packed);
  const bf16_t* bias = a.bias ? (const bf16_t*)a.bias : dummy;
  const bf16_t* res = a.res ? (const bf16_t*)a.res + (int64_t)mc * a.ld_res : dummy;
  const uint32_t bmask = a.bias ? 0xffff0000u : 0u, rmask = a.res ? 0xffff0000u : 0u;
  float bv[4], rv[4];
  float4 cst[4], cwv[4];
  float cbv[4];
  const bool conv_tile = CONV && n0 < a.conv_dim;   // conv_dim % 32 == 0: whole tiles
  const float* cbp = a.conv_b ? a.conv_b : a.conv_w;
  const uint32_t cmask = a.conv_b ? 0xffffffffu : 0u;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = nb + q < N ? nb + q : N - 1;
    bv[q] = __uint_as_float(((uint32_t)bias[c] << 16) & bmask);
    rv[q] = __uint_as_float(((uint32_t)res[c] << 16) & rmask);
    if constexpr (CONV) {
      const int cc = c < a.conv_dim ? c : a.conv_dim - 1;
      cst[q] = *reinterpret_cast<const float4*>(a.conv_state + ((int64_t)mc * a.conv_dim + cc) * 4);
      cwv[q] = *reinterpret_cast<const float4*>(a.conv_w + (int64_t)cc * 4);
      cbv[q] = __uint_as_float(__float_as_uint(cbp[cc]) & cmask);
    }
  }

  if constexpr (LNP) {
    // operand = bf16(LN(x) * ln_w + ln_b [, gamma * . + beta]) exactly as
    // mtts_layernorm_fwd rounds it; statistics of the full row from the
    // wave's registers (lanes r, r+16, r+32, r+48 share row r), then over the
    // KS waves in fixed order; two passes (mean, then squared deviations)
#ifdef GEMV_DIAG_NOSTATS   // timing-only build: no row statistics (no barriers)
    const float ma = 0.f, mb = 0.f, ra = 1.f, rb = 1.f;
#else
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int j = 0; j < S; ++j)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        sa += bf2f((bf16_t)xf0[j][q]);
        sb += bf2f((bf16_t)xf1[j][q]);
      }
    sa = sum_xor32(sum_xor16(sa));
    sb = sum_xor32(sum_xor16(sb));
    if (g == 0) { psum[wave][r] = sa; psum[wave][16 + r] = sb; }
    block_sync();
    float ma = 0.f, mb = 0.f;
    for (int w = 0; w < KS; ++w) { ma += psum[w][r]; mb += psum[w][16 + r]; }
    ma /= a.K;
    mb /= a.K;
    float qa = 0.f, qb = 0.f;
#pragma unroll
    for (int j = 0; j < S; ++j)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float da = bf2f((bf16_t)xf0[j][q]) - ma, db = bf2f((bf16_t)xf1[j][q]) - mb;
        qa = fmaf(da, da, qa);
        qb = fmaf(db, db, qb);
      }
    qa = sum_xor32(sum_xor16(qa));
    qb = sum_xor32(sum_xor16(qb));
    if (g == 0) { psq[wave][r] = qa; psq[wave][16 + r] = qb; }
    block_sync();
    float va = 0.f, vb = 0.f;
    for (int w = 0; w < KS; ++w) { va += psq[w][r]; vb += psq[w][16 + r]; }
    const float ra = 1.f / sqrtf(va / a.K + a.ln_eps), rb = 1.f / sqrtf(vb / a.K + a.ln_eps);
#endif
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const float w8[8] = {lw[j][0].x, lw[j][0].y, lw[j][0].z, lw[j][0].w, lw[j][1].x, lw[j][1].y, lw[j][1].z, lw[j][1].w};
      const float b8[8] = {lb[j][0].x, lb[j][0].y, lb[j][0].z, lb[j][0].w, lb[j][1].x, lb[j][1].y, lb[j][1].z, lb[j][1].w};
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float va_ = fmaf((bf2f((bf16_t)xf0[j][q]) - ma) * ra, w8[q], b8[q]);
        float vb_ = fmaf((bf2f((bf16_t)xf1[j][q]) - mb) * rb, w8[q], b8[q]);
        if constexpr (FILM) {
          va_ = fmaf(bf2f((bf16_t)ga0[j][q]), va_, bf2f((bf16_t)ba0[j][q]));
          vb_ = fmaf(bf2f((bf16_t)ga1[j][q]), vb_, bf2f((bf16_t)ba1[j][q]));
        }
        xf0[j][q] = (short)f2bf(va_);
        xf1[j][q] = (short)f2bf(vb_);
      }
    }
  }

  // ---- product: D[n][m] (lane: n = n0 + 4 g + q, m = r (+16))
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < S; ++j) acc0 = mfma16(wf[j], xf0[j], acc0);
  if (two) {
#pragma unroll
    for (int j = 0; j < S; ++j) acc1 = mfma16(wf[j], xf1[j], acc1);
  }
  red[wave][0][lane] = acc0;
  if (two) red[wave][1][lane] = acc1;
  block_sync();
  if (!mok) return;

  // ---- fixed-order sum over the KS waves + epilogue
  f32x4 s = red[0][half][el];
  for (int w = 1; w < KS; ++w) s += red[w][half][el];
  bf16_t out[4];
  float yv[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float v = s[q] + bv[q];
    if (a.act == 1) v = gelu_erf(v);
    const bf16_t sb = f2bf(v);
    yv[q] = bf2f(sb);
    out[q] = a.res ? f2bf(yv[q] + rv[q]) : sb;
  }
  if (a.y) {
    bf16_t* yrow = (bf16_t*)a.y + (int64_t)m * a.ldy;
    if (nb + 3 < N && ((uintptr_t)(yrow + nb) & 7) == 0) {
      uint2 w2;
      w2.x = (uint32_t)out[0] | ((uint32_t)out[1] << 16);
      w2.y = (uint32_t)out[2] | ((uint32_t)out[3] << 16);
      *reinterpret_cast<uint2*>(yrow + nb) = w2;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (nb + q < N) yrow[nb + q] = out[q];
    }
  }
  if (a.y_packed) {   // N % 32 == 0: columns nb..nb+3 are 4 consecutive elements of the image
    uint2 w2;
    w2.x = (uint32_t)out[0] | ((uint32_t)out[1] << 16);
    w2.y = (uint32_t)out[2] | ((uint32_t)out[3] << 16);
    *reinterpret_cast<uint2*>((bf16_t*)a.y_packed + xpk_index(m, nb)) = w2;
  }
  if (conv_tile) {   // causal_conv1d_update (width 4) + SiLU on the bf16-rounded column
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = nb + q;
      float4 st = make_float4(cst[q].y, cst[q].z, cst[q].w, yv[q]);
      *reinterpret_cast<float4*>(a.conv_state + ((int64_t)m * a.conv_dim + c) * 4) = st;
      const float4 w = cwv[q];
      const float v = fmaf(w.x, st.x, fmaf(w.y, st.y, fmaf(w.z, st.z, fmaf(w.w, st.w, cbv[q]))));
      out[q] = f2bf(silu_f(v));
      ((bf16_t*)a.u)[(int64_t)m * a.ldu + c] = out[q];
    }
    if (a.u_packed) {
      uint2 w2;
      w2.x = (uint32_t)out[0] | ((uint32_t)out[1] << 16);
      w2.y = (uint32_t)out[2] | ((uint32_t)out[3] << 16);
      *reinterpret_cast<uint2*>((bf16_t*)a.u_packed + xpk_index(m, nb)) = w2;
    }
  }
}

template <int S, int LNM>
void launch_gemv2(const MttsRowsArgs* a, const dim3 grid, const dim3 block, hipStream_t st) {
  if (a->x_packed) {
    if (a->conv_dim > 0) hipLaunchKernelGGL((gemv16_kernel<S, LNM, true, true>), grid, block, 0, st, *a);
    else hipLaunchKernelGGL((gemv16_kernel<S, LNM, false, true>), grid, block, 0, st, *a);
    return;
  }
  if (a->conv_dim > 0) hipLaunchKernelGGL((gemv16_kernel<S, LNM, true, false>), grid, block, 0, st, *a);
  else hipLaunchKernelGGL((gemv16_kernel<S, LNM, false, false>), grid, block, 0, st, *a);
}

template <int S>
void launch_gemv(const MttsRowsArgs* a, int ks, hipStream_t st) {
  const dim3 grid((a->N + 15) / 16), block(64 * ks);
  if constexpr (S <= 8) {
    if (a->ln_w) {
      if (a->gamma) launch_gemv2<S, 2>(a, grid, block, st);
      else launch_gemv2<S, 1>(a, grid, block, st);
      return;
    }
  }
  launch_gemv2<S, 0>(a, grid, block, st);
}

// One wave per row (<= 32 rows): two-pass statistics over the row in
// registers, the same arithmetic and summation order as ln_fwd_kernel
// (csrc/ln.hip, VEC 8), so bf16(LN(x) * w + b [, gamma * . + beta]) is bit
// identical to mtts_layernorm_fwd's y; written as 16-byte pieces of the
// packed activation image.
template <bool FILM, int NC>
__global__ __launch_bounds__(256) void ln_rows_packed_kernel(const MttsLNArgs a, bf16_t* __restrict__ yp) {
  // NC 16-byte chunks per lane (cols <= 512 NC); every load is issued up
  // front and unconditionally (clamped chunk index, masked afterwards):
  // branches around loads would drain vmcnt between them
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.rows) return;
  const int C = a.cols;
  const bf16_t* x = (const bf16_t*)a.x + (int64_t)row * a.x_rs;
  float v[NC][8], w[NC][8], b[NC][8], gm[FILM ? NC : 1][8], bt[FILM ? NC : 1][8];
  bool ok[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int k0 = 8 * (lane + 64 * i);
    ok[i] = k0 < C;
    const int k = ok[i] ? k0 : 0;
    ld_vec<bf16_t, 8>(x + k, v[i]);
    ld_vec<float, 4>(a.w + k, *reinterpret_cast<float(*)[4]>(w[i]));
    ld_vec<float, 4>(a.w + k + 4, *reinterpret_cast<float(*)[4]>(w[i] + 4));
    ld_vec<float, 4>(a.b + k, *reinterpret_cast<float(*)[4]>(b[i]));
    ld_vec<float, 4>(a.b + k + 4, *reinterpret_cast<float(*)[4]>(b[i] + 4));
    if constexpr (FILM) {
      ld_vec<bf16_t, 8>((const bf16_t*)a.gamma + (int64_t)row * a.gb_rs + k, gm[i]);
      ld_vec<bf16_t, 8>((const bf16_t*)a.beta + (int64_t)row * a.gb_rs + k, bt[i]);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q) s += ok[i] ? v[i][q] : 0.f;
  const float mean = wave_sum(s) / C;
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q) { const float d = ok[i] ? v[i][q] - mean : 0.f; sq = fmaf(d, d, sq); }
  const float rstd = 1.f / sqrtf(wave_sum(sq) / C + a.eps);
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    float o[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      o[q] = fmaf((v[i][q] - mean) * rstd, w[i][q], b[i][q]);
      if constexpr (FILM) o[q] = fmaf(gm[i][q], o[q], bt[i][q]);
    }
    if (ok[i]) st_vec<bf16_t, 8>(yp + xpk_index(row, 8 * (lane + 64 * i)), o);
  }
}

template <bool FILM>
void launch_ln_rows(const MttsLNArgs* a, bf16_t* yp, hipStream_t st) {
  const dim3 grid((a->rows + 3) / 4), block(256);
  const int nc = (a->cols + 511) / 512;
  switch (nc) {
    case 1: hipLaunchKernelGGL((ln_rows_packed_kernel<FILM, 1>), grid, block, 0, st, *a, yp); break;
    case 2: hipLaunchKernelGGL((ln_rows_packed_kernel<FILM, 2>), grid, block, 0, st, *a, yp); break;
    case 3:
    case 4: hipLaunchKernelGGL((ln_rows_packed_kernel<FILM, 4>), grid, block, 0, st, *a, yp); break;
    default: hipLaunchKernelGGL((ln_rows_packed_kernel<FILM, 8>), grid, block, 0, st, *a, yp); break;
  }
}

}  // namespace

// wave split of the packed launch: KS waves x S k-steps, K = 32 * S * KS
int gemv_split(int K, int* ks_out, int* s_out) {
  const int nsteps = K / 32;
  int ks = 1;
  while (ks < kMaxKS && nsteps % (2 * ks) == 0) ks *= 2;
  const int s = nsteps / ks;
  if (s != 1 && s != 2 && s != 4 && s != 8 && s != 16) return 0;
  *ks_out = ks;
  *s_out = s;
  return 1;
}

int launch_gemv_packed(const MttsRowsArgs* a, hipStream_t st) {
  int ks, s;
  if (a->K % 64 != 0 || !gemv_split(a->K, &ks, &s)) {
    set_error("gemm_rows: packed weights need K %% 64 == 0 and K / 32 = KS * S with KS <= 8 a power of 2, "
              "S in {1, 2, 4, 8, 16} (K=%d)", a->K);
    return MTTS_EUNSUPPORTED;
  }
  if ((a->y_packed && a->N % 32) || (a->x_packed && a->K % 32) || (!a->y && !a->y_packed)) {
    set_error("gemm_rows: packed activation images need N / K %% 32 == 0 (N=%d K=%d), and some output", a->N, a->K);
    return MTTS_EINVAL;
  }
  if (a->ln_w && s > 8) {
    set_error("gemm_rows: packed weights with the LayerNorm prologue need at most 8 k-steps per wave, "
              "K <= 256 * waves = 2048 (K=%d, %d waves)", a->K, ks);
    return MTTS_EUNSUPPORTED;
  }
  switch (s) {
    case 1: launch_gemv<1>(a, ks, st); break;
    case 2: launch_gemv<2>(a, ks, st); break;
    case 4: launch_gemv<4>(a, ks, st); break;
    case 8: launch_gemv<8>(a, ks, st); break;
    default: launch_gemv<16>(a, ks, st); break;
  }
  MTTS_LAUNCH_CHECK("gemm_rows (packed)");
  return MTTS_OK;
}

}  // namespace mtts

using namespace mtts;

extern "C" int64_t mtts_pack_rows_bytes(int N, int K) {
  if (N <= 0 || K <= 0 || K % 32) return -1;
  return (int64_t)((N + 15) / 16) * 16 * K * 2;
}

extern "C" int mtts_pack_rows_weight(const void* W, int64_t ldw, int N, int K, void* out, void* stream) {
  MTTS_CHECK(W && out, "pack_rows_weight: null pointer");
  MTTS_CHECK(N > 0 && K > 0 && K % 64 == 0, "pack_rows_weight: N=%d K=%d (K must be a positive multiple of 64)", N, K);
  MTTS_CHECK(ldw >= K && ldw % 8 == 0 && (uintptr_t)W % 16 == 0 && (uintptr_t)out % 16 == 0,
             "pack_rows_weight: W / out must be 16-byte aligned with a row stride >= K, multiple of 8");
  const int64_t total = (int64_t)((N + 15) / 16) * (K / 32) * 64;
  const int threads = 256;
  hipLaunchKernelGGL(pack_rows_kernel, dim3((unsigned)((total + threads - 1) / threads)), dim3(threads), 0,
                     (hipStream_t)stream, (const bf16_t*)W, ldw, N, K, (uint4*)out, total);
  MTTS_LAUNCH_CHECK("pack_rows_weight");
  return MTTS_OK;
}

extern "C" int mtts_layernorm_rows_packed(const MttsLNArgs* a, void* y_packed, void* stream) {
  MTTS_CHECK(a && a->x && a->w && a->b && y_packed, "layernorm_rows_packed: null pointer");
  MTTS_CHECK(a->rows > 0 && a->rows <= 32 && a->cols > 0 && a->cols % 32 == 0 && a->cols <= 4096,
             "layernorm_rows_packed: rows=%d must be in [1, 32], cols=%d a multiple of 32 <= 4096", a->rows, a->cols);
  MTTS_CHECK(a->dtype == MTTS_BF16 && (!a->gamma || (a->beta && a->gb_dtype == MTTS_BF16 && a->rows_per_group <= 1)),
             "layernorm_rows_packed: bf16 rows, FiLM rows bf16 with one row per group");
  MTTS_CHECK(((uintptr_t)a->x | (uintptr_t)a->w | (uintptr_t)a->b | (uintptr_t)y_packed) % 16 == 0 &&
                 a->x_rs % 8 == 0 && (!a->gamma || (((uintptr_t)a->gamma | (uintptr_t)a->beta) % 16 == 0 &&
                                                    a->gb_rs % 8 == 0)),
             "layernorm_rows_packed: operands must be 16-byte aligned with 16-byte row strides");
  if (a->gamma) launch_ln_rows<true>(a, (bf16_t*)y_packed, (hipStream_t)stream);
  else launch_ln_rows<false>(a, (bf16_t*)y_packed, (hipStream_t)stream);
  MTTS_LAUNCH_CHECK("layernorm_rows_packed");
  return MTTS_OK;
}
