// Projections of the incremental decode step (decode_step, reference
// mamba_decoder.py:188-256; C4: 32 sequences, one token each): y = x W^T (+
// bias, optional exact-erf GELU), x (M <= 32 rows) bf16, W (N x K) bf16.
// hipBLASLt picks 32x32 / 16x32 macro tiles for M = 32 and streams the
// weights at < 1 TB/s (11 us for the 8 MB in_proj weight); these GEMVs are
// weight-streaming problems.  Here one 32-column output tile per workgroup,
// the K range split over KS waves: every wave streams its slice of 32 weight
// rows straight from HBM into v_mfma_f32_32x32x16_bf16 B fragments (lane =
// output column, 8 consecutive k = 16 contiguous bytes of a weight row; no
// LDS), x fragments come from L2, and the KS partial 32x32 tiles are summed
// through LDS in a fixed order with bias / GELU fused into the store.
// Optional epilogue: the causal-conv1d state update + SiLU on the x half of
// in_proj (Mamba.step), which removes the conv-update launch.  (A residual +
// LayerNorm tail run by the last workgroup to finish was measured and
// dropped: the agent-scope release/acquire it needs costs more than the
// LayerNorm launch it saves, 15 us per use; DESIGN.md.)
#include "common.h"

namespace mtts {
namespace {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// SK: the K range is also split over a.kgroups workgroups per 32-column tile
// (grid = tiles * kgroups), each writing its fp32 32x32 partial to a slab;
// the last to arrive (agent-scope release / acquire around one ticket per
// tile, the counter reset by it) sums the kgroups slabs in fixed order and
// runs the epilogue.  With the LayerNorm prologue every workgroup derives
// the full-row statistics itself from the (L2-resident) x rows.
template <int KS, int U, bool LNP, bool SK>
__global__ __launch_bounds__(64 * KS) void gemm_rows_kernel(const MttsRowsArgs a) {
  __shared__ float red[KS][32][33];
  __shared__ float psum[LNP ? (SK ? 2 * KS : KS) : 1][32], psq[LNP ? (SK ? 2 * KS : KS) : 1][32];
  __shared__ __attribute__((aligned(16))) float slw[LNP ? 2048 : 4], slb[LNP ? 2048 : 4];
  __shared__ int s_last;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int KG = SK ? a.kgroups : 1;
  int tile = blockIdx.x, kg = 0;
  if constexpr (SK) {
    const int tiles = gridDim.x / KG;
    if (tiles % 8 == 0) {   // a tile's K groups on one XCD (round-robin dispatch): same-XCD slab reads
      const int xcd = blockIdx.x % 8, q = blockIdx.x / 8;
      tile = xcd + 8 * (q / KG);
      kg = q % KG;
    } else {
      tile = blockIdx.x / KG;
      kg = blockIdx.x % KG;
    }
  }
  const int n0 = tile * 32;
  const int M = a.M, N = a.N;
  const int kc = a.K / (KS * KG), kb = (kg * KS + wave) * kc;
  const bool rowok = i < M, colok = n0 + i < N;
  const bf16_t* xr = (const bf16_t*)a.x + (int64_t)(rowok ? i : 0) * a.ldx + kb + 8 * h;
  const bf16_t* wr = (const bf16_t*)a.W + (int64_t)(colok ? n0 + i : 0) * a.ldw + kb + 8 * h;
  // conv epilogue operands do not depend on the product: fetch them first
  constexpr int E = 1024 / (64 * KS), EP = KS >= 4 ? E : 1;
  const bool conv_tile = n0 < a.conv_dim;   // conv_dim % 32 == 0: whole tiles
  float4 cst[EP], cwv[EP];
  float cbv[EP];
  if constexpr (KS >= 4) {
    if (conv_tile) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int idx = threadIdx.x + e * 64 * KS, row = idx >> 5, c = n0 + (idx & 31);
        if (row < M) {
          cst[e] = *reinterpret_cast<const float4*>(a.conv_state + ((int64_t)row * a.conv_dim + c) * 4);
          cwv[e] = *reinterpret_cast<const float4*>(a.conv_w + (int64_t)c * 4);
          cbv[e] = a.conv_b ? a.conv_b[c] : 0.f;
        }
      }
    }
  }
  // bias / residual of the epilogue elements, fetched before the product too
  float bv[E], rv[E];
  const bf16_t* bias = (const bf16_t*)a.bias;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int idx = threadIdx.x + e * 64 * KS, row = idx >> 5, c = n0 + (idx & 31);
    const bool ok = row < M && c < N;
    bv[e] = bias && ok ? bf2f(bias[c]) : 0.f;
    rv[e] = a.res && ok ? bf2f(((const bf16_t*)a.res)[(int64_t)row * a.ld_res + c]) : 0.f;
  }
  f32x16 acc = {};
  s16x8 xa[U], wb[U];
  auto load_w = [&](int k) {
#pragma unroll
    for (int u = 0; u < U; ++u) wb[u] = *reinterpret_cast<const s16x8*>(wr + k + 16 * u);
  };
  auto load_x = [&](int k) {
#pragma unroll
    for (int u = 0; u < U; ++u) xa[u] = *reinterpret_cast<const s16x8*>(xr + k + 16 * u);
  };
  if constexpr (LNP) {
    // LayerNorm prologue, one trip (host: K == KS * 16 * U): the wave's x
    // fragments hold all of its k slice, so the row statistics come from
    // registers (per-wave partials, fixed-order sums through LDS) while the
    // weights, FiLM rows and LN parameters (-> LDS) are in flight.
    for (int c = threadIdx.x * 4; c < a.K; c += 64 * KS * 4) {
      *reinterpret_cast<float4*>(slw + c) = *reinterpret_cast<const float4*>(a.ln_w + c);
      *reinterpret_cast<float4*>(slb + c) = *reinterpret_cast<const float4*>(a.ln_b + c);
    }
    load_w(0);
    load_x(0);
    s16x8 ga[U], ba[U];
    if (a.gamma) {
      const int64_t ro = (int64_t)(rowok ? i : 0) * a.ld_gb + kb + 8 * h;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ga[u] = *reinterpret_cast<const s16x8*>((const bf16_t*)a.gamma + ro + 16 * u);
        ba[u] = *reinterpret_cast<const s16x8*>((const bf16_t*)a.beta + ro + 16 * u);
      }
    }
    float mean, rstd;
    if constexpr (!SK) {
      float sx = 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int q = 0; q < 8; ++q) sx += bf2f((bf16_t)xa[u][q]);
      sx += __shfl_xor(sx, 32);
      if (lane < 32) psum[wave][i] = sx;
      block_sync();
      mean = 0.f;
#pragma unroll
      for (int w = 0; w < KS; ++w) mean += psum[w][i];
      mean /= a.K;
      float sq = 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int q = 0; q < 8; ++q) { const float d = bf2f((bf16_t)xa[u][q]) - mean; sq = fmaf(d, d, sq); }
      sq += __shfl_xor(sq, 32);
      if (lane < 32) psq[wave][i] = sq;
      block_sync();
      float var = 0.f;
#pragma unroll
      for (int w = 0; w < KS; ++w) var += psq[w][i];
      rstd = 1.f / sqrtf(var / a.K + a.ln_eps);
    } else {
      // full-row statistics from x itself (L2-resident; the weights are
      // already in flight): thread (row r, part p) covers K / (2 KS) columns;
      // two passes (mean, then sum of squared deviations) as the LayerNorm
      // kernel does, fixed-order combines through LDS
      const int r = threadIdx.x & 31, part = threadIdx.x >> 5, np = 2 * KS;
      const bf16_t* xrow = (const bf16_t*)a.x + (int64_t)(r < M ? r : 0) * a.ldx;
      const int span = a.K / np;
      float s1 = 0.f;
#pragma unroll 4
      for (int c = part * span; c < (part + 1) * span; c += 8) {
        const s16x8 v = *reinterpret_cast<const s16x8*>(xrow + c);
#pragma unroll
        for (int q = 0; q < 8; ++q) s1 += bf2f((bf16_t)v[q]);
      }
      psum[part][r] = s1;
      block_sync();
      float t1 = 0.f;
      for (int w = 0; w < np; ++w) t1 += psum[w][r];
      const float mr = t1 / a.K;
      float s2 = 0.f;
#pragma unroll 4
      for (int c = part * span; c < (part + 1) * span; c += 8) {
        const s16x8 v = *reinterpret_cast<const s16x8*>(xrow + c);
#pragma unroll
        for (int q = 0; q < 8; ++q) { const float d = bf2f((bf16_t)v[q]) - mr; s2 = fmaf(d, d, s2); }
      }
      psq[part][r] = s2;
      block_sync();
      float t2 = 0.f;
      mean = 0.f;
      for (int w = 0; w < np; ++w) { mean += psum[w][i]; t2 += psq[w][i]; }
      mean /= a.K;
      const float var = t2 / a.K;
      rstd = 1.f / sqrtf(var + a.ln_eps);
    }
    // operand = bf16(LN(x) * w + b [, gamma * . + beta]) as mtts_layernorm_fwd rounds it
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c0 = kb + 16 * u + 8 * h;
      const float4 w0 = *reinterpret_cast<const float4*>(slw + c0), w1 = *reinterpret_cast<const float4*>(slw + c0 + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(slb + c0), b1 = *reinterpret_cast<const float4*>(slb + c0 + 4);
      const float lw[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      const float lb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float v = fmaf((bf2f((bf16_t)xa[u][q]) - mean) * rstd, lw[q], lb[q]);
        if (a.gamma) v = fmaf(bf2f((bf16_t)ga[u][q]), v, bf2f((bf16_t)ba[u][q]));
        xa[u][q] = (short)f2bf(v);
      }
    }
  }
  for (int k = 0; k < kc; k += 16 * U) {   // U k-steps per trip, all loads issued first
    if constexpr (!LNP) {
      load_w(k);
      load_x(k);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!rowok) xa[u] = s16x8{};
      if (!colok) wb[u] = s16x8{};
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, xa[u]),
                                                    __builtin_bit_cast(bf16x8, wb[u]), acc, 0, 0, 0);
    }
  }
  // acc register r: output row (batch) acc_row(r, h), column n0 + i
#pragma unroll
  for (int r = 0; r < 16; ++r) red[wave][acc_row(r, h)][i] = acc[r];
  block_sync();
  float part[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int idx = threadIdx.x + e * 64 * KS, row = idx >> 5, col = idx & 31;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < KS; ++w) s += red[w][row][col];
    part[e] = s;
  }
  if constexpr (SK) {
    if (KG > 1) {
      // write-through (sc1) slab stores, drained by every wave, then ONE
      // agent-scope RELEASE ticket per workgroup; the last arriver runs an
      // agent-scope ACQUIRE fence before it reads the slabs (HIP memory model;
      // the sc1 loads alone would rest on hardware behaviour)
      float* slab = a.splitk_slab + (int64_t)tile * KG * 1024;
#pragma unroll
      for (int e = 0; e < E; ++e)
        __hip_atomic_store(slab + kg * 1024 + threadIdx.x + e * 64 * KS, part[e], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      block_sync();
      if (threadIdx.x == 0) {
        const int old = __hip_atomic_fetch_add(a.splitk_count + tile, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == KG - 1;
        if (last) __hip_atomic_store(a.splitk_count + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = last;
      }
      block_sync();
      if (!s_last) return;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // invalidates this CU's L1: other CUs' slabs
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int e = 0; e < E; ++e) {
        float v[32];
#pragma unroll
        for (int g = 0; g < 32; ++g)
          if (g < KG) v[g] = __hip_atomic_load(slab + g * 1024 + threadIdx.x + e * 64 * KS, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
        float s = 0.f;
#pragma unroll
        for (int g = 0; g < 32; ++g)
          if (g < KG) s += v[g];
        part[e] = s;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int idx = threadIdx.x + e * 64 * KS, row = idx >> 5, col = idx & 31, c = n0 + col;
    if (row >= M || c >= N) continue;
    float s = part[e];
    s += bv[e];
    if (a.act == 1) s = 0.5f * s * (1.f + erff(s * 0.70710678118654752f));   // F.gelu (exact erf)
    const bf16_t sb = f2bf(s);
    // residual epilogue: y = bf16(bf16(product) + res), the stream value mtts_layernorm_fwd writes to x_sum
    ((bf16_t*)a.y)[(int64_t)row * a.ldy + c] = a.res ? f2bf(bf2f(sb) + rv[e]) : sb;
    if (conv_tile) {   // causal_conv1d_update (width 4) + SiLU on the bf16-rounded column
      float4* stp = reinterpret_cast<float4*>(a.conv_state + ((int64_t)row * a.conv_dim + c) * 4);
      float4 st, w;
      float cb;
      if constexpr (KS >= 4) {
        st = cst[e], w = cwv[e], cb = cbv[e];
      } else {
        st = *stp, w = *reinterpret_cast<const float4*>(a.conv_w + (int64_t)c * 4), cb = a.conv_b ? a.conv_b[c] : 0.f;
      }
      st = make_float4(st.y, st.z, st.w, bf2f(sb));
      *stp = st;
      const float v = fmaf(w.x, st.x, fmaf(w.y, st.y, fmaf(w.z, st.z, fmaf(w.w, st.w, cb))));
      ((bf16_t*)a.u)[(int64_t)row * a.ldu + c] = f2bf(silu_f(v));
    }
  }
}

template <int KS, int U>
void launch_rows(const MttsRowsArgs* a, int tiles, hipStream_t st) {
  const bool sk = a->kgroups > 1;
  const dim3 grid(tiles * (sk ? a->kgroups : 1));
  if constexpr (KS <= 8) {
    if (a->ln_w) {
      if (sk) hipLaunchKernelGGL((gemm_rows_kernel<KS, U, true, true>), grid, dim3(64 * KS), 0, st, *a);
      else hipLaunchKernelGGL((gemm_rows_kernel<KS, U, true, false>), grid, dim3(64 * KS), 0, st, *a);
      return;
    }
  }
  if (sk) hipLaunchKernelGGL((gemm_rows_kernel<KS, U, false, true>), grid, dim3(64 * KS), 0, st, *a);
  else hipLaunchKernelGGL((gemm_rows_kernel<KS, U, false, false>), grid, dim3(64 * KS), 0, st, *a);
}

}  // namespace
}  // namespace mtts

using namespace mtts;

extern "C" int mtts_gemm_rows(const MttsRowsArgs* a, void* stream) {
  MTTS_CHECK(a && a->x && a->W && (a->y || (a->w_packed && a->y_packed)), "gemm_rows: null pointer");
  const int M = a->M, N = a->N, K = a->K;
  MTTS_CHECK(M >= 0 && M <= 32 && N > 0 && K > 0, "gemm_rows: M=%d must be in [0, 32], N, K > 0", M);
  MTTS_CHECK(K % 64 == 0, "gemm_rows: K=%d must be a multiple of 64", K);
  MTTS_CHECK(a->act == 0 || a->act == 1, "gemm_rows: act must be 0 (none) or 1 (gelu)");
  MTTS_CHECK(((uintptr_t)a->x | (uintptr_t)a->W) % 16 == 0 && a->ldx % 8 == 0 && (a->w_packed || a->ldw % 8 == 0),
             "gemm_rows: x / W must be 16-byte aligned with 16-byte row strides");
  MTTS_CHECK(a->conv_dim >= 0 && a->conv_dim <= N && a->conv_dim % 32 == 0,
             "gemm_rows: conv_dim=%d must be a multiple of 32 in [0, N]", a->conv_dim);
  MTTS_CHECK(a->conv_dim == 0 || (a->conv_state && a->conv_w && a->u && (uintptr_t)a->conv_state % 16 == 0 &&
                                  (uintptr_t)a->conv_w % 16 == 0),
             "gemm_rows: conv epilogue needs 16-byte aligned conv_state / conv_w and u");
  if (a->ln_w) {
    MTTS_CHECK(a->ln_b && (!a->gamma || a->beta), "gemm_rows: LayerNorm prologue needs ln_b, and beta with gamma");
    MTTS_CHECK((uintptr_t)a->ln_w % 16 == 0 && (uintptr_t)a->ln_b % 16 == 0 &&
                   (!a->gamma || ((uintptr_t)a->gamma % 16 == 0 && (uintptr_t)a->beta % 16 == 0 && a->ld_gb % 8 == 0)),
               "gemm_rows: LayerNorm prologue operands must be 16-byte aligned");
  }
  MTTS_CHECK(!a->res || a->conv_dim == 0, "gemm_rows: residual and conv epilogues are exclusive");
  if (a->w_packed) {
    MTTS_CHECK(a->kgroups <= 1, "gemm_rows: packed weights take no split-K");
    if (M == 0) return MTTS_OK;
    return launch_gemv_packed(a, (hipStream_t)stream);
  }
  if (M == 0) return MTTS_OK;
  hipStream_t st = (hipStream_t)stream;
  const int tiles = (N + 31) / 32;
  // K split over ks = 8 waves of one workgroup (fewer where K is short),
  // each streaming its k slice in trips of 4 MFMA k-steps with all loads of
  // a trip in flight.  Measured on the C4 step (tools/decode_ab.py, p50 ms):
  // ks = 8 everywhere 1.20; 4 / 8 / 16 by tile count 1.23; ks = 4 1.25;
  // ks = 2 1.44; one 8-step trip per wave with up to 16 waves 1.28.
  const int KG = a->kgroups > 1 ? a->kgroups : 1;
  if (KG > 1) {
    MTTS_CHECK(a->splitk_slab && a->splitk_count && K % (64 * KG) == 0 && KG <= 32,
               "gemm_rows: split-K over %d workgroups needs slab / counters and K %% (64 * kgroups) == 0", KG);
    if (a->ln_w && K > 2048) {
      set_error("gemm_rows: LayerNorm prologue needs K <= 2048 (LN parameters staged in LDS; K=%d)", K);
      return MTTS_EUNSUPPORTED;
    }
  }
  const int Kw = K / KG;   // per-workgroup K range
  int U = 4;
  int ks = Kw % (64 * 8) == 0 ? 8 : Kw % (64 * 4) == 0 ? 4 : Kw % (64 * 2) == 0 ? 2 : 1;
  int u8 = U == 8;
  if (a->ln_w) {   // LayerNorm prologue: exactly one trip per wave (Kw == ks * 16 * U), ks <= 8
    int f = 0;
    for (int c = 8; c >= 1 && !f; c >>= 1) {
      if (Kw == c * 64) f = c, u8 = 0;
      else if (Kw == c * 128) f = c, u8 = 1;
    }
    if (!f || (KG == 1 && K > 2048)) {
      set_error("gemm_rows: LayerNorm prologue needs K / kgroups = 64 * {1,2,4,8} or 128 * {1,..,8} (K=%d)", K);
      return MTTS_EUNSUPPORTED;
    }
    ks = f;
  }
  if (u8) {
    switch (ks) {
      case 16: launch_rows<16, 8>(a, tiles, st); break;
      case 8: launch_rows<8, 8>(a, tiles, st); break;
      case 4: launch_rows<4, 8>(a, tiles, st); break;
      case 2: launch_rows<2, 8>(a, tiles, st); break;
      default: launch_rows<1, 8>(a, tiles, st); break;
    }
  } else {
    switch (ks) {
      case 16: launch_rows<16, 4>(a, tiles, st); break;
      case 8: launch_rows<8, 4>(a, tiles, st); break;
      case 4: launch_rows<4, 4>(a, tiles, st); break;
      case 2: launch_rows<2, 4>(a, tiles, st); break;
      default: launch_rows<1, 4>(a, tiles, st); break;
    }
  }
  MTTS_LAUNCH_CHECK("gemm_rows");
  return MTTS_OK;
}
