// Skinny bf16 MFMA GEMMs for the Mamba mixer's inner projections (gfx950):
// x_proj (d_inner -> dt_rank + 2 d_state = 96 columns) and dt_proj
// (dt_rank = 64 -> d_inner), forward and data gradient, which the 256x256
// projection kernel (gemm.hip) cannot fill the chip with.
// Reference sites: [upstream] mamba_simple.Mamba x_proj / dt_proj (the
// reference's Mamba(d_model) at /root/reference/mamba_decoder.py:29, applied
// at :61), inside mamba_inner_fn:  x_dbl = x_proj(u);  delta = dt_proj.W @ dt.
//
// Both compute C[m, n] = A[m, k] . B[n, k]^T (+ beta C) with fp32 accumulation
// on v_mfma_f32_16x16x32_bf16, operands straight from global memory into
// registers (16-byte loads: a lane owns one row's 8-element k-chunk; the
// B fragment goes first in the MFMA so a lane's accumulator holds 4
// consecutive output columns of one row).
//
//  * SKINNY_N (n <= 128): a workgroup owns RB rows and all n columns; its 4
//    waves split the K range (k-steps of 32 dealt round-robin), each keeping
//    a register double buffer of the next k-step's fragments; the 4 partial
//    tiles are summed through LDS in a fixed order ((w0 + w2) + (w1 + w3)).
//    Reads A once (the activation, HBM) and B once per workgroup (the weight,
//    L2-resident).  x_proj forward (A = u), dt_proj data gradient
//    (A = d delta, B = W_dt^T).
//  * SMALL_K (k <= 128): a workgroup owns 64 rows x 256 columns, a wave
//    64 x 64; all of A's and B's fragments are loaded up front (k/32 steps).
//    Output-bound (writes m x n, reads it too with beta = 1).  dt_proj
//    forward (A = x_dbl[:, :dt_rank], B = W_dt), x_proj data gradient
//    accumulated into du (A = d x_dbl, B = W_x^T, beta = 1).
#include "common.h"

namespace mtts {
namespace {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16(const uint4& x, const uint4& y, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, x), __builtin_bit_cast(bf16x8, y), c, 0, 0,
                                                 0);
}

struct SkinnyP {
  const bf16_t* a;
  const bf16_t* b;
  void* c;
  int64_t lda, ldb, ldc;
  int m, n, k;
  int c_f32;
  float beta;
};

// 4 consecutive columns of one row of C: + beta * old, store (bf16 8 B / fp32 16 B)
__device__ __forceinline__ void store4(const SkinnyP& p, int row, int col, f32x4 v) {
  if (row >= p.m || col >= p.n) return;   // n % 4 == 0 (host): a lane's 4 columns are all in or all out
  if (p.c_f32) {
    float* cp = (float*)p.c + (int64_t)row * p.ldc + col;
    if (p.beta != 0.f) v += p.beta * *(const f32x4*)cp;
    *(f32x4*)cp = v;
  } else {
    bf16_t* cp = (bf16_t*)p.c + (int64_t)row * p.ldc + col;
    if (p.beta != 0.f) {
      const uint2 o = *(const uint2*)cp;
      v[0] += p.beta * __uint_as_float(o.x << 16);
      v[1] += p.beta * __uint_as_float(o.x & 0xffff0000u);
      v[2] += p.beta * __uint_as_float(o.y << 16);
      v[3] += p.beta * __uint_as_float(o.y & 0xffff0000u);
    }
    *(uint2*)cp = make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                             (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
  }
}

// A fragments PA k-steps ahead (HBM latency), B fragments one ahead (L2)
template <int MB, int NB>
__global__ __launch_bounds__(256) void skinny_n_kernel(SkinnyP p) {
  constexpr int RB = MB * 16;
  constexpr int PA = 4;
  __shared__ __attribute__((aligned(16))) f32x4 red[2][MB * NB][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row0 = blockIdx.x * RB;
  const int li = lane & 15, kq = (lane >> 4) * 8;
  const bf16_t* ap[MB];
  const bf16_t* bp[NB];
#pragma unroll
  for (int i = 0; i < MB; ++i) ap[i] = p.a + (int64_t)min(row0 + i * 16 + li, p.m - 1) * p.lda + kq + wave * 32;
#pragma unroll
  for (int j = 0; j < NB; ++j) bp[j] = p.b + (int64_t)min(j * 16 + li, p.n - 1) * p.ldb + kq + wave * 32;
  f32x4 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // this wave's k-steps: wave, wave + 4, ...  (index i: element offset i * 128)
  const int ni = (p.k / 32 - wave + 3) / 4;
  uint4 fa[PA][MB], fb[2][NB];
  auto load_a = [&](int i, int st) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < MB; ++r) fa[st][r] = *(const uint4*)(ap[r] + i * 128);
  };
  auto load_b = [&](int i, int st) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < NB; ++j) fb[st][j] = *(const uint4*)(bp[j] + i * 128);
  };
#pragma unroll
  for (int j = 0; j < PA; ++j)
    if (j < ni) load_a(j, j);
  if (ni > 0) load_b(0, 0);
  for (int i0 = 0; i0 < ni; i0 += PA) {
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const int i = i0 + j;
      if (i < ni) {
        if (i + 1 < ni) load_b(i + 1, (j + 1) & 1);
#pragma unroll
        for (int r = 0; r < MB; ++r)
#pragma unroll
          for (int c = 0; c < NB; ++c) acc[r][c] = mfma16(fb[j & 1][c], fa[j][r], acc[r][c]);
        if (i + PA < ni) load_a(i + PA, j);
      }
    }
  }
  // fixed-order sum of the 4 K-quarter tiles: (w0 + w2) + (w1 + w3)
  if (wave >= 2) {
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) red[wave - 2][i * NB + j][lane] = acc[i][j];
  }
  block_sync();
  if (wave < 2) {
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[i][j] += red[wave][i * NB + j][lane];
  }
  block_sync();
  if (wave == 1) {
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) red[0][i * NB + j][lane] = acc[i][j];
  }
  block_sync();
  if (wave == 0) {
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) store4(p, row0 + i * 16 + li, j * 16 + (lane >> 4) * 4, acc[i][j] + red[0][i * NB + j][lane]);
  }
}

// all operand fragments up front; with beta the old C values are loaded in
// one batch before the products; stores are 16-byte (bf16: a permlane16 swap
// pairs the 4-column groups of neighbouring 16-column blocks)
template <int KS>
__global__ __launch_bounds__(256) void small_k_kernel(SkinnyP p) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row0 = blockIdx.y * 64;
  const int col0 = blockIdx.x * 256 + wave * 64;
  if (col0 >= p.n) return;
  const int li = lane & 15, kq = (lane >> 4) * 8;
  const int g = lane >> 4;
  // bf16 C: a lane's 8 consecutive columns per (row block, column pair) start
  // at cw; with beta the old values are requested first (their latency then
  // overlaps the operand loads and the products)
  const int cw_off = (g & 1) * 16 + 8 * (g >> 1);
  uint4 old16[4][2];
  f32x4 old32[4][4];
  if (p.beta != 0.f) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = row0 + i * 16 + li;
      if (p.c_f32) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int col = col0 + j * 16 + 4 * g;
          old32[i][j] = (row < p.m && col < p.n) ? *(const f32x4*)((const float*)p.c + (int64_t)row * p.ldc + col)
                                                 : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      } else {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int cw = col0 + q * 32 + cw_off;
          old16[i][q] = (row < p.m && cw < p.n) ? *(const uint4*)((const bf16_t*)p.c + (int64_t)row * p.ldc + cw)
                                                : make_uint4(0, 0, 0, 0);
        }
      }
    }
  }
  uint4 fa[4][KS], fb[4][KS];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bf16_t* ap = p.a + (int64_t)min(row0 + i * 16 + li, p.m - 1) * p.lda + kq;
#pragma unroll
    for (int s = 0; s < KS; ++s) fa[i][s] = *(const uint4*)(ap + s * 32);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bf16_t* bp = p.b + (int64_t)min(col0 + j * 16 + li, p.n - 1) * p.ldb + kq;
#pragma unroll
    for (int s = 0; s < KS; ++s) fb[j][s] = *(const uint4*)(bp + s * 32);
  }
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) acc[i][j] = mfma16(fb[j][s], fa[i][s], acc[i][j]);
    }
  if (p.c_f32) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = row0 + i * 16 + li;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = col0 + j * 16 + 4 * g;
        f32x4 v = acc[i][j];
        if (p.beta != 0.f) v += p.beta * old32[i][j];
        if (row < p.m && col < p.n) *(f32x4*)((float*)p.c + (int64_t)row * p.ldc + col) = v;
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = row0 + i * 16 + li;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      // after the swap, even 16-lane groups hold block 2q's columns
      // 8(g>>1)..+7, odd groups block 2q+1's
      float v8[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * q][e]),
                                                        __float_as_uint(acc[i][2 * q + 1][e]), false, false);
        v8[e] = __uint_as_float(r[0]);
        v8[4 + e] = __uint_as_float(r[1]);
      }
      if (p.beta != 0.f) {
        const uint32_t ow[4] = {old16[i][q].x, old16[i][q].y, old16[i][q].z, old16[i][q].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v8[2 * e] += p.beta * __uint_as_float(ow[e] << 16);
          v8[2 * e + 1] += p.beta * __uint_as_float(ow[e] & 0xffff0000u);
        }
      }
      uint32_t w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = (uint32_t)f2bf(v8[2 * e]) | ((uint32_t)f2bf(v8[2 * e + 1]) << 16);
      const int cw = col0 + q * 32 + cw_off;
      if (row < p.m && cw < p.n) *(uint4*)((bf16_t*)p.c + (int64_t)row * p.ldc + cw) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

// ---------------------------------------------------------------------------
// SKINNY_TN: C[m, n] = A[k, m]^T . B[k, n] (fp32, optionally stored as C^T)
// with n <= 128 narrow and m % 128 == 0 wide -- the x_proj / dt_proj weight
// gradients (dW_dt = d(delta)^T dt: m = d_inner, n = dt_rank; dW_x^T =
// u^T d(x_dbl): m = d_inner, n = dt_rank + 2 d_state), K = tokens.
// Both operands are token-major (k = the row index), so the MFMA fragments
// (8 consecutive k of one column per lane) come from ds_read_b64_tr_b16 over a
// row-major LDS image: a workgroup (8 waves) owns 128 columns of A (one
// 16-column block per wave) x all n and a chunk of kc tokens; 64-token tiles
// of A (64 x 128) and B (64 x 128, zero-padded past n) are staged through a
// double-buffered LDS image (plain 256-B rows, 16-B chunk swizzle
// ch ^ (((row&3)<<2) | ((row>>2)&3)): conflict-free transposed reads), the
// next tile's rows loaded into registers while the current one computes.
// The chunks' fp32 partial tiles go to a slab summed in fixed order
// (colsum).  HBM-bound: A is read once, B once per 128 columns (L2).
constexpr int kTnRows = 64;   // tokens per LDS tile
__device__ __forceinline__ int tn_off(int row, int ch) {   // byte offset of 16-B chunk ch of row `row`
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
// lane's transposed fragment of the image: column block cb (16 columns), k rows 32 ks + 8 g .. +7
__device__ __forceinline__ uint4 tn_frag(const char* img, int cb, int ks, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  s16x4 r[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = ks * 32 + 8 * g + 4 * h + q;
    const int off = tn_off(row, cb * 2 + (pp >> 1)) + 8 * (pp & 1);
    r[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + off));
  }
  s16x8 v{r[0][0], r[0][1], r[0][2], r[0][3], r[1][0], r[1][1], r[1][2], r[1][3]};
  return __builtin_bit_cast(uint4, v);
}

struct TnP {
  const bf16_t* a;   // (k, m) row stride lda
  const bf16_t* b;   // (k, n) row stride ldb
  float* slab;       // (chunks, m, n) or (chunks, n, m) with TRANS
  int64_t lda, ldb;
  int m, n, k, kc;
};

template <int NB, bool TRANS>
__global__ __launch_bounds__(512) void tn_skinny_kernel(TnP p) {
  __shared__ __attribute__((aligned(16))) char sa[2][kTnRows * 256];
  __shared__ __attribute__((aligned(16))) char sb[2][kTnRows * 256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c0 = blockIdx.x * 128;
  const int k0 = blockIdx.y * p.kc, k1 = min(p.k, k0 + p.kc);
  const int ntile = (k1 - k0 + kTnRows - 1) / kTnRows;
  // this thread's two 16-B chunks of each 64 x 128 tile: rows tid/16 and tid/16 + 32, chunk tid % 16
  const int ch = tid & 15, r0 = tid >> 4;
  const bool bok = ch * 8 < p.n;   // n % 8 == 0 (host): a chunk is all in or all out
  uint4 ra[2], rb[2];
  auto load = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int row = k0 + t * kTnRows + r0 + 32 * s;
      const bool ok = row < k1;
      const int rr = ok ? row : k0;
      ra[s] = *(const uint4*)(p.a + (int64_t)rr * p.lda + c0 + ch * 8);
      rb[s] = *(const uint4*)(p.b + (int64_t)rr * p.ldb + (bok ? ch * 8 : 0));
      if (!ok) ra[s] = make_uint4(0, 0, 0, 0);
      if (!ok || !bok) rb[s] = make_uint4(0, 0, 0, 0);
    }
  };
  auto store = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      *(uint4*)(sa[buf] + tn_off(r0 + 32 * s, ch)) = ra[s];
      *(uint4*)(sb[buf] + tn_off(r0 + 32 * s, ch)) = rb[s];
    }
  };
  f32x4 acc[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (ntile > 0) {
    load(0);
    store(0);
  }
  block_sync();
  // (a two-deep register ring measured equal / slower: tools/skinny_ab.py)
  for (int t = 0; t < ntile; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntile) load(t + 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const uint4 fa = tn_frag(sa[buf], wave, ks, lane);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const uint4 fb = tn_frag(sb[buf], j, ks, lane);
        // !TRANS: lane ends with 4 consecutive n of one m; TRANS: 4 consecutive m of one n
        acc[j] = TRANS ? mfma16(fa, fb, acc[j]) : mfma16(fb, fa, acc[j]);
      }
    }
    if (t + 1 < ntile) store(buf ^ 1);
    block_sync();
  }
  float* sl = p.slab + (int64_t)blockIdx.y * p.m * p.n;
  const int li = lane & 15, g4 = (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    if constexpr (TRANS) {   // C^T[n][m]: n = 16 j + li, m = c0 + 16 wave + g4 .. +3
      const int nn = j * 16 + li;
      if (nn < p.n) *(f32x4*)(sl + (int64_t)nn * p.m + c0 + wave * 16 + g4) = acc[j];
    } else {                 // C[m][n]: m = c0 + 16 wave + li, n = 16 j + g4 .. +3
      const int nn = j * 16 + g4;
      if (nn < p.n) *(f32x4*)(sl + (int64_t)(c0 + wave * 16 + li) * p.n + nn) = acc[j];
    }
  }
}

template <int MB>
void launch_skinny_n(const SkinnyP& p, hipStream_t st) {
  const int nb = (p.n + 15) / 16;
  const dim3 grid((p.m + MB * 16 - 1) / (MB * 16));
  switch (nb) {
#define SK_(N) case N: hipLaunchKernelGGL((skinny_n_kernel<MB, N>), grid, dim3(256), 0, st, p); break;
    SK_(1) SK_(2) SK_(3) SK_(4) SK_(5) SK_(6) SK_(7) SK_(8)
#undef SK_
  }
}

}  // namespace
}  // namespace mtts

using namespace mtts;

static int tn_chunk(int k) { return k >= 8192 ? 512 : 256; }   // tokens per workgroup (>= 512 workgroups at C2)

extern "C" int64_t mtts_gemm_skinny_workspace(const MttsSkinnyArgs* a) {
  if (!a || a->mode != MTTS_SKINNY_TN || a->k <= 0) return 0;
  const int kc = tn_chunk(a->k);
  return (int64_t)((a->k + kc - 1) / kc) * a->m * a->n * 4 + 256;
}

static int skinny_tn(const MttsSkinnyArgs* a, hipStream_t st) {
  MTTS_CHECK(a->m % 128 == 0 && a->n <= 128 && a->n % 8 == 0,
             "gemm_skinny TN: needs m %% 128 == 0 and n <= 128, n %% 8 == 0 (m=%d n=%d)", a->m, a->n);
  MTTS_CHECK(a->c_dtype == MTTS_F32 && a->beta == 0.f, "gemm_skinny TN: fp32 output, beta = 0");
  MTTS_CHECK(a->workspace, "gemm_skinny TN: workspace required (mtts_gemm_skinny_workspace)");
  MTTS_CHECK(a->ldc == (a->trans_c ? a->m : a->n), "gemm_skinny TN: C must be contiguous (ldc = %d)",
             a->trans_c ? a->m : a->n);
  MTTS_CHECK(a->lda >= a->m && a->ldb >= a->n, "gemm_skinny TN: leading dimension too small");
  TnP p;
  p.a = (const bf16_t*)a->a; p.b = (const bf16_t*)a->b; p.slab = (float*)a->workspace;
  p.lda = a->lda; p.ldb = a->ldb; p.m = a->m; p.n = a->n; p.k = a->k; p.kc = tn_chunk(a->k);
  const int chunks = (a->k + p.kc - 1) / p.kc;
  const dim3 grid(a->m / 128, chunks);
  const int nb = (a->n + 15) / 16;
#define TN_(N)                                                                                        \
  case N:                                                                                             \
    if (a->trans_c) hipLaunchKernelGGL((tn_skinny_kernel<N, true>), grid, dim3(512), 0, st, p);      \
    else hipLaunchKernelGGL((tn_skinny_kernel<N, false>), grid, dim3(512), 0, st, p);                \
    break;
  switch (nb) { TN_(1) TN_(2) TN_(3) TN_(4) TN_(5) TN_(6) TN_(7) TN_(8) }
#undef TN_
  MTTS_LAUNCH_CHECK("gemm_skinny TN");
  const int ncols = a->m * a->n;
  colsum(p.slab, chunks, chunks, ncols, ncols, (float*)a->c, 0, st);
  MTTS_LAUNCH_CHECK("gemm_skinny TN chunk sum");
  return MTTS_OK;
}

extern "C" int mtts_gemm_skinny(const MttsSkinnyArgs* a, void* stream) {
  MTTS_CHECK(a && a->a && a->b && a->c, "gemm_skinny: null pointer");
  MTTS_CHECK(a->mode == MTTS_SKINNY_N || a->mode == MTTS_SKINNY_SMALL_K || a->mode == MTTS_SKINNY_TN,
             "gemm_skinny: bad mode %d", a->mode);
  MTTS_CHECK(a->m > 0 && a->n > 0 && a->k > 0, "gemm_skinny: m=%d n=%d k=%d must be positive", a->m, a->n, a->k);
  if (a->mode == MTTS_SKINNY_TN) {
    MTTS_CHECK(((uintptr_t)a->a | (uintptr_t)a->b | (uintptr_t)a->c) % 16 == 0 && a->lda % 8 == 0 && a->ldb % 8 == 0,
               "gemm_skinny TN: A / B / C must be 16-byte aligned with row strides a multiple of 8 elements");
    return skinny_tn(a, (hipStream_t)stream);
  }
  MTTS_CHECK(a->k % 32 == 0, "gemm_skinny: k=%d must be a multiple of 32", a->k);
  MTTS_CHECK(a->n % 4 == 0, "gemm_skinny: n=%d must be a multiple of 4", a->n);
  MTTS_CHECK(a->mode != MTTS_SKINNY_N || a->n <= 128, "gemm_skinny: SKINNY_N needs n <= 128 (n=%d)", a->n);
  MTTS_CHECK(a->mode != MTTS_SKINNY_SMALL_K || a->k <= 128, "gemm_skinny: SMALL_K needs k <= 128 (k=%d)", a->k);
  MTTS_CHECK(((uintptr_t)a->a | (uintptr_t)a->b) % 16 == 0 && a->lda % 8 == 0 && a->ldb % 8 == 0,
             "gemm_skinny: A / B must be 16-byte aligned with row strides a multiple of 8 elements");
  MTTS_CHECK(a->lda >= a->k && a->ldb >= a->k && a->ldc >= a->n, "gemm_skinny: leading dimension too small");
  MTTS_CHECK(a->c_dtype == MTTS_F32 || a->c_dtype == MTTS_BF16, "gemm_skinny: bad c_dtype");
  const int ces = a->c_dtype == MTTS_F32 ? 4 : 2;
  MTTS_CHECK((uintptr_t)a->c % (4 * ces) == 0 && a->ldc % 4 == 0,
             "gemm_skinny: C must be %d-byte aligned with ldc a multiple of 4", 4 * ces);
  // SMALL_K with bf16 C moves 8 consecutive columns (16 bytes) per lane
  MTTS_CHECK(a->mode != MTTS_SKINNY_SMALL_K || ces == 4 ||
                 (a->n % 8 == 0 && a->ldc % 8 == 0 && (uintptr_t)a->c % 16 == 0),
             "gemm_skinny: SMALL_K with bf16 C needs n %% 8 == 0, ldc %% 8 == 0 and a 16-byte aligned C "
             "(n=%d ldc=%d)", a->n, a->ldc);
  SkinnyP p;
  p.a = (const bf16_t*)a->a; p.b = (const bf16_t*)a->b; p.c = a->c;
  p.lda = a->lda; p.ldb = a->ldb; p.ldc = a->ldc;
  p.m = a->m; p.n = a->n; p.k = a->k;
  p.c_f32 = a->c_dtype == MTTS_F32;
  p.beta = a->beta;
  hipStream_t st = (hipStream_t)stream;
  if (a->mode == MTTS_SKINNY_N) {
    launch_skinny_n<4>(p, st);   // 64 rows per workgroup (tools/skinny_ab.py: 4 row-blocks beat 1 / 2)
  } else {
    const dim3 grid((a->n + 255) / 256, (a->m + 63) / 64);
    switch (a->k / 32) {
      case 1: hipLaunchKernelGGL((small_k_kernel<1>), grid, dim3(256), 0, st, p); break;
      case 2: hipLaunchKernelGGL((small_k_kernel<2>), grid, dim3(256), 0, st, p); break;
      case 3: hipLaunchKernelGGL((small_k_kernel<3>), grid, dim3(256), 0, st, p); break;
      default: hipLaunchKernelGGL((small_k_kernel<4>), grid, dim3(256), 0, st, p); break;
    }
  }
  MTTS_LAUNCH_CHECK("gemm_skinny");
  return MTTS_OK;
}
