// LayerNorm (+ fused residual add, + fused FiLM) forward / backward, gfx950.
//
// Replaces nn.LayerNorm at mamba_decoder.py:59,67,81,184 and the FiLM of
// mamba_decoder.py:82-86 (h = gamma*LN(x) + beta, gamma/beta per batch row,
// no "1+gamma").  One wave per row: the row stays in registers (16-byte
// vector loads), statistics by DPP/permlane wave reductions; HBM-bound.
// Parameter-gradient sums over rows go to per-block partials reduced by a
// second deterministic kernel (no atomics).
#include "common.h"

namespace mtts {

constexpr int kLnWaves = 4;
constexpr int kMaxVec = 8;  // elements per 16-byte vector (bf16)


// NV = vectors per lane (cols = 64 * VEC * NV)
template <typename T, typename TG, int VEC, int NV>
__global__ __launch_bounds__(64 * kLnWaves) void ln_fwd_kernel(const MttsLNArgs a) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kLnWaves + (threadIdx.x >> 6);
  if (row >= a.rows) return;
  const int n = a.cols;
  float v[NV][VEC];
  const T* x = (const T*)a.x + (int64_t)row * a.x_rs;
#pragma unroll
  for (int k = 0; k < NV; ++k) ld_vec<T, VEC>(x + (k * 64 + lane) * VEC, v[k]);
  if (a.res) {
    const T* r = (const T*)a.res + (int64_t)row * a.res_rs;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      float t[VEC];
      ld_vec<T, VEC>(r + (k * 64 + lane) * VEC, t);
#pragma unroll
      for (int q = 0; q < VEC; ++q) v[k][q] += t[q];
    }
    if (a.x_sum) {
      T* xs = (T*)a.x_sum + (int64_t)row * a.xsum_rs;
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        // round to the storage dtype (in registers) so fwd/bwd see the same stream value
        st_vec<T, VEC>(xs + (k * 64 + lane) * VEC, v[k]);
        if constexpr (sizeof(T) == 2) {
#pragma unroll
          for (int q = 0; q < VEC; ++q) v[k][q] = bf2f(f2bf(v[k][q]));
        }
      }
    }
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k)
#pragma unroll
    for (int q = 0; q < VEC; ++q) s += v[k][q];
  const float mean = wave_sum(s) / n;
  float s2 = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k)
#pragma unroll
    for (int q = 0; q < VEC; ++q) { const float d = v[k][q] - mean; s2 = fmaf(d, d, s2); }
  const float var = wave_sum(s2) / n;
  const float rstd = 1.f / sqrtf(var + a.eps);
  if (lane == 0) { a.mean[row] = mean; a.rstd[row] = rstd; }
  const int grp = a.gamma ? row / a.rows_per_group : 0;
  T* y = (T*)a.y + (int64_t)row * a.y_rs;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c0 = (k * 64 + lane) * VEC;
    float o[VEC];
#pragma unroll
    for (int q = 0; q < VEC; ++q) o[q] = fmaf((v[k][q] - mean) * rstd, a.w[c0 + q], a.b[c0 + q]);
    if (a.gamma) {
      float g[VEC], be[VEC];
      ld_vec<TG, VEC>((const TG*)a.gamma + (int64_t)grp * a.gb_rs + c0, g);
      ld_vec<TG, VEC>((const TG*)a.beta + (int64_t)grp * a.gb_rs + c0, be);
#pragma unroll
      for (int q = 0; q < VEC; ++q) o[q] = fmaf(g[q], o[q], be[q]);
    }
    st_vec<T, VEC>(y + c0, o);
  }
}

// Each block handles RB consecutive rows (all in one FiLM group); partials
// per block: dw, db (cols each) and dgamma, dbeta (cols each).
// 8 waves per block for rows of <= 16 elements per lane (2 per SIMD at one
// block per CU; wider rows keep 4 waves to stay in registers) and the next
// row's x / dy loads issued before the current row's math: the 4-wave,
// load-then-compute form ran at ~55 % of HBM (one 16-B load pair in flight
// per wave).
template <int VEC, int NV>
constexpr int ln_bwd_waves() { return VEC * NV <= 16 ? 8 : 4; }
template <typename T, typename TG, int VEC, int NV>
__global__ __launch_bounds__((64 * ln_bwd_waves<VEC, NV>())) void ln_bwd_kernel(const MttsLNBwdArgs a, int RB,
                                                                  float* __restrict__ part) {
  constexpr int kLnBwdWaves = ln_bwd_waves<VEC, NV>();
  const MttsLNArgs& f = a.f;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int n = f.cols;
  const int row0 = blockIdx.x * RB;
  const bool film = f.gamma != nullptr;
  const int grp = film ? row0 / f.rows_per_group : 0;
  const bool csum = a.dx_colsum != nullptr;
  // Parameter-gradient partials from TWO running sums per column (round 6):
  // the block's RB rows lie in one FiLM group (ln_rb), so gamma_g is a
  // constant per column and, with A = sum dy * xhat, S = sum dy over the rows:
  //   dw = gamma_g A, db = gamma_g S (no FiLM: gamma_g = 1),
  //   dgamma = w A + b S, dbeta = S
  // -- 32 fewer accumulator VGPRs than four running sums, which pays for the
  // residual-gradient row (dx_acc) prefetched with x / dy one row ahead.
  float wv[NV][VEC], bv[NV][VEC], gv[NV][VEC];
  float pA[NV][VEC], pS[NV][VEC], pdx[NV][VEC];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c0 = (k * 64 + lane) * VEC;
    ld_vec<float, VEC>(f.w + c0, wv[k]);
    ld_vec<float, VEC>(f.b + c0, bv[k]);
    if (film) ld_vec<TG, VEC>((const TG*)f.gamma + (int64_t)grp * f.gb_rs + c0, gv[k]);
#pragma unroll
    for (int q = 0; q < VEC; ++q) {
      if (!film) gv[k][q] = 1.f;
      pA[k][q] = pS[k][q] = pdx[k][q] = 0.f;
    }
  }
  const T* xsrc = (const T*)((f.res && f.x_sum) ? f.x_sum : f.x);
  const int64_t xrs = (f.res && f.x_sum) ? f.xsum_rs : f.x_rs;
  const int rend = min(RB, f.rows - row0);
  const bool acc = a.dx_acc != nullptr;
  // raw 16-byte pieces of the residual-gradient row when a vector holds 16 bytes
  constexpr bool kRawAcc = VEC * sizeof(T) == 16;
  float nxv[NV][VEC], ndy[NV][VEC];
  uint4 nacc[kRawAcc ? NV : 1];
  auto load_row = [&](int rr) __attribute__((always_inline)) {
    const int row = row0 + rr;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c0 = (k * 64 + lane) * VEC;
      ld_vec<T, VEC>(xsrc + (int64_t)row * xrs + c0, nxv[k]);
      ld_vec<T, VEC>((const T*)a.dy + (int64_t)row * a.dy_rs + c0, ndy[k]);
      if constexpr (kRawAcc) {
        if (acc) nacc[k] = *reinterpret_cast<const uint4*>((const T*)a.dx_acc + (int64_t)row * a.dxacc_rs + c0);
      }
    }
  };
  if (wave < rend) load_row(wave);
  for (int r = wave; r < rend; r += kLnBwdWaves) {
    const int row = row0 + r;
    const float mean = f.mean[row], rstd = f.rstd[row];
    float cxv[NV][VEC], cdy[NV][VEC];
    uint4 cacc[kRawAcc ? NV : 1];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
#pragma unroll
      for (int q = 0; q < VEC; ++q) { cxv[k][q] = nxv[k][q]; cdy[k][q] = ndy[k][q]; }
      if constexpr (kRawAcc) cacc[k] = nacc[k];
    }
    if (r + kLnBwdWaves < rend) load_row(r + kLnBwdWaves);
    float xh[NV][VEC], dxh[NV][VEC];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
#pragma unroll
      for (int q = 0; q < VEC; ++q) {
        const float h = (cxv[k][q] - mean) * rstd;
        xh[k][q] = h;
        const float dy = cdy[k][q];
        pA[k][q] = fmaf(dy, h, pA[k][q]);
        pS[k][q] += dy;
        const float d = dy * gv[k][q] * wv[k][q];
        dxh[k][q] = d;
        s1 += d;
        s2 = fmaf(d, h, s2);
      }
    }
    const float m1 = wave_sum(s1) / n, m2 = wave_sum(s2) / n;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c0 = (k * 64 + lane) * VEC;
      float o[VEC];
#pragma unroll
      for (int q = 0; q < VEC; ++q) o[q] = rstd * (dxh[k][q] - m1 - xh[k][q] * m2);
      if (acc) {
        float t[VEC];
        if constexpr (kRawAcc) {
          if constexpr (sizeof(T) == 2) {
            const uint32_t w4[4] = {cacc[k].x, cacc[k].y, cacc[k].z, cacc[k].w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              t[2 * q] = __uint_as_float(w4[q] << 16);
              t[2 * q + 1] = __uint_as_float(w4[q] & 0xffff0000u);
            }
          } else {
            t[0] = __uint_as_float(cacc[k].x); t[1] = __uint_as_float(cacc[k].y);
            t[2] = __uint_as_float(cacc[k].z); t[3] = __uint_as_float(cacc[k].w);
          }
        } else {
          ld_vec<T, VEC>((const T*)a.dx_acc + (int64_t)row * a.dxacc_rs + c0, t);
        }
#pragma unroll
        for (int q = 0; q < VEC; ++q) o[q] += t[q];
      }
      st_vec<T, VEC>((T*)a.dx + (int64_t)row * a.dx_rs + c0, o);
      if (csum) {   // column sums of dx as stored (the upstream linear's bias gradient)
#pragma unroll
        for (int q = 0; q < VEC; ++q) pdx[k][q] += sizeof(T) == 2 ? bf2f(f2bf(o[q])) : o[q];
      }
    }
  }
  // block partials: reduce the waves through LDS, then one write per column
  // slabs: 0 dw, 1 db, 2 dgamma, 3 dbeta (FiLM), 4 dx column sums (dx_colsum)
  extern __shared__ float sm[];  // [kLnBwdWaves][cols]
  for (int which = 0; which < 5; ++which) {
    if ((which == 2 || which == 3) && !film) continue;   // block-uniform
    if (which == 4 && !csum) continue;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c0 = (k * 64 + lane) * VEC;
#pragma unroll
      for (int q = 0; q < VEC; ++q) {
        const float A = pA[k][q], S = pS[k][q];
        const float val = which == 0 ? gv[k][q] * A : which == 1 ? gv[k][q] * S
                        : which == 2 ? fmaf(wv[k][q], A, bv[k][q] * S) : which == 3 ? S : pdx[k][q];
        sm[wave * n + c0 + q] = val;
      }
    }
    block_sync();
    for (int c = threadIdx.x; c < n; c += 64 * kLnBwdWaves) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < kLnBwdWaves; ++w) s += sm[w * n + c];
      part[((int64_t)which * gridDim.x + blockIdx.x) * n + c] = s;
    }
    block_sync();
  }
}

static int ln_rb(const MttsLNArgs* a) {
  if (!a->gamma) {   // 64 rows per block; short inputs (the text encoder's 1024 rows: 16 blocks) down to 8
    int rb = 64;
    while (rb > 8 && (a->rows + rb - 1) / rb < 256) rb >>= 1;
    return rb;
  }
  for (int rb = 64; rb > 1; rb >>= 1)
    if (a->rows_per_group % rb == 0) return rb;
  return 1;
}

template <typename T, typename TG, int VEC, int NV>
static void launch_fwd(const MttsLNArgs* a, hipStream_t st) {
  hipLaunchKernelGGL((ln_fwd_kernel<T, TG, VEC, NV>), dim3((a->rows + kLnWaves - 1) / kLnWaves), dim3(64 * kLnWaves), 0,
                     st, *a);
}
template <typename T, typename TG, int VEC, int NV>
static void launch_bwd(const MttsLNBwdArgs* a, int rb, float* part, hipStream_t st) {
  const int nblk = (a->f.rows + rb - 1) / rb;
  constexpr int W = ln_bwd_waves<VEC, NV>();
  hipLaunchKernelGGL((ln_bwd_kernel<T, TG, VEC, NV>), dim3(nblk), dim3(64 * W), W * a->f.cols * sizeof(float), st, *a,
                     rb, part);
}

// dispatch on (dtype, gamma dtype, cols)
template <template <typename, typename, int, int> class F, typename... Args>
static int dispatch_ln(const MttsLNArgs* a, Args... args) {
  const int n = a->cols;
  auto go = [&](auto tag_t, auto tag_g) -> int {
    using T = typename decltype(tag_t)::type;
    using TG = typename decltype(tag_g)::type;
    constexpr int VEC = 16 / sizeof(T);
    const bool vec_ok = n % (64 * VEC) == 0 && (a->x_rs * (int64_t)sizeof(T)) % 16 == 0 &&
                        (a->y_rs * (int64_t)sizeof(T)) % 16 == 0 && (uintptr_t)a->x % 16 == 0 &&
                        (uintptr_t)a->y % 16 == 0 &&
                        (!a->res || ((uintptr_t)a->res % 16 == 0 && (a->res_rs * (int64_t)sizeof(T)) % 16 == 0)) &&
                        (!a->gamma || ((uintptr_t)a->gamma % 16 == 0 && (a->gb_rs * (int64_t)sizeof(TG)) % 16 == 0 &&
                                       (uintptr_t)a->beta % 16 == 0));
    if (vec_ok) {
      switch (n / (64 * VEC)) {
        case 1: F<T, TG, VEC, 1>::run(a, args...); return MTTS_OK;
        case 2: F<T, TG, VEC, 2>::run(a, args...); return MTTS_OK;
        case 3: F<T, TG, VEC, 3>::run(a, args...); return MTTS_OK;
        case 4: F<T, TG, VEC, 4>::run(a, args...); return MTTS_OK;
        case 6: F<T, TG, VEC, 6>::run(a, args...); return MTTS_OK;
        case 8: F<T, TG, VEC, 8>::run(a, args...); return MTTS_OK;
        default: break;
      }
    }
    if (n % 64 == 0) {
      switch (n / 64) {
        case 1: F<T, TG, 1, 1>::run(a, args...); return MTTS_OK;
        case 2: F<T, TG, 1, 2>::run(a, args...); return MTTS_OK;
        case 3: F<T, TG, 1, 3>::run(a, args...); return MTTS_OK;
        case 4: F<T, TG, 1, 4>::run(a, args...); return MTTS_OK;
        case 6: F<T, TG, 1, 6>::run(a, args...); return MTTS_OK;
        case 8: F<T, TG, 1, 8>::run(a, args...); return MTTS_OK;
        case 16: F<T, TG, 1, 16>::run(a, args...); return MTTS_OK;
        default: break;
      }
    }
    set_error("layernorm: cols=%d unsupported", n);
    return MTTS_EUNSUPPORTED;
  };
  struct F32 { using type = float; };
  struct BF { using type = bf16_t; };
  const bool gf = !a->gamma || a->gb_dtype == MTTS_F32;
  if (a->dtype == MTTS_F32) return gf ? go(F32{}, F32{}) : go(F32{}, BF{});
  return gf ? go(BF{}, F32{}) : go(BF{}, BF{});
}

template <typename T, typename TG, int VEC, int NV>
struct FwdRunner {
  static void run(const MttsLNArgs* a, hipStream_t st) { launch_fwd<T, TG, VEC, NV>(a, st); }
};
template <typename T, typename TG, int VEC, int NV>
struct BwdRunner {
  static void run(const MttsLNArgs* a, const MttsLNBwdArgs* b, int rb, float* part, hipStream_t st) {
    (void)a;
    launch_bwd<T, TG, VEC, NV>(b, rb, part, st);
  }
};

static int check_ln(const MttsLNArgs* a) {
  MTTS_CHECK(a && a->x && a->w && a->b && a->y && a->mean && a->rstd, "layernorm: null tensor");
  MTTS_CHECK(a->rows >= 0 && a->cols > 0, "layernorm: bad sizes");
  MTTS_CHECK(a->dtype == MTTS_F32 || a->dtype == MTTS_BF16, "layernorm: bad dtype");
  MTTS_CHECK(!a->gamma || (a->beta && a->rows_per_group > 0), "layernorm: FiLM needs beta and rows_per_group");
  return MTTS_OK;
}

}  // namespace mtts

using namespace mtts;

extern "C" int mtts_layernorm_fwd(const MttsLNArgs* a, void* stream) {
  int rc = check_ln(a);
  if (rc) return rc;
  if (a->rows == 0) return MTTS_OK;
  rc = dispatch_ln<FwdRunner>(a, (hipStream_t)stream);
  if (rc) return rc;
  MTTS_LAUNCH_CHECK("layernorm_fwd");
  return MTTS_OK;
}

extern "C" int64_t mtts_layernorm_bwd_workspace(int rows, int cols, int rows_per_group) {
  MttsLNArgs t{};
  t.gamma = rows_per_group > 0 ? (const void*)1 : nullptr;
  t.rows_per_group = rows_per_group;
  t.rows = rows;
  const int rb = ln_rb(&t);
  const int64_t nblk = (rows + rb - 1) / rb;
  return 5 * nblk * cols * 4 + 256;
}

extern "C" int mtts_layernorm_bwd(const MttsLNBwdArgs* a, void* stream) {
  MTTS_CHECK(a, "layernorm_bwd: null args");
  int rc = check_ln(&a->f);
  if (rc) return rc;
  MTTS_CHECK(a->dy && a->dx && a->dw && a->db && a->workspace, "layernorm_bwd: null tensor");
  MTTS_CHECK(!a->f.gamma || (a->dgamma && a->dbeta), "layernorm_bwd: FiLM needs dgamma/dbeta");
  const MttsLNArgs& f = a->f;
  hipStream_t st = (hipStream_t)stream;
  MTTS_CHECK(a->dgb_rs == 0 || a->dgb_rs >= f.cols, "layernorm_bwd: dgb_rs < cols");
  if (f.rows == 0) {
    (void)hipMemsetAsync(a->dw, 0, f.cols * 4, st);
    (void)hipMemsetAsync(a->db, 0, f.cols * 4, st);
    if (a->dx_colsum) (void)hipMemsetAsync(a->dx_colsum, 0, f.cols * 4, st);
    return MTTS_OK;
  }
  const int rb = ln_rb(&f);
  float* part = (float*)a->workspace;
  rc = dispatch_ln<BwdRunner>(&f, a, rb, part, st);
  if (rc) return rc;
  MTTS_LAUNCH_CHECK("layernorm_bwd");
  const int nblk = (f.rows + rb - 1) / rb;
  const int64_t slab = (int64_t)nblk * f.cols;
  // dw, db (and dgamma, dbeta per FiLM row group) in one launch
  ColsumJob jobs[5] = {{part, a->dw, nblk, nblk, 0}, {part + slab, a->db, nblk, nblk, 0}};
  int nj = 2;
  if (f.gamma) {
    const int bpg = f.rows_per_group / rb;
    const int64_t gs = a->dgb_rs > 0 ? a->dgb_rs : (int64_t)f.cols;
    jobs[nj++] = {part + 2 * slab, a->dgamma, nblk, bpg, gs};
    jobs[nj++] = {part + 3 * slab, a->dbeta, nblk, bpg, gs};
  }
  if (a->dx_colsum) jobs[nj++] = {part + 4 * slab, a->dx_colsum, nblk, nblk, 0};
  colsum_multi(jobs, nj, f.cols, f.cols, st);
  MTTS_LAUNCH_CHECK("layernorm_bwd_reduce");
  return MTTS_OK;
}
