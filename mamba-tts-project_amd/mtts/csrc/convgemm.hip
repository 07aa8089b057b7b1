// fp32 MFMA GEMM over WINDOWED row matrices: the text encoder's and duration
// predictor's convolutions (FastSpeech2 PositionwiseFeedForward k = 9 / 1,
// VariancePredictor k = 3: reference text_encoder.py:80-85, 118-122, 131-209)
// as direct implicit-GEMM convolutions, with no unfold copy.
//
// An operand is a matrix whose row r starts at
//     ptr + (r / seg_rows) * seg_stride + (r % seg_rows) * row_stride
// and holds its elements contiguously.  On a channel-last (B, T + 2p, C)
// zero-padded activation, rows = B*T tokens, seg_rows = T, seg_stride =
// (T + 2p) C, row_stride = C and a row of K*C elements IS the conv window
// x[b, t .. t+K-1, :] (rows overlap), so
//   y  = conv(x, W)      : NT, A = window(x_pad),  B = W as (O, K*C) [o][k][c]
//   dx = conv^T(dy, W)   : NT, A = window(dy_pad), B = W flipped as (C, K*O)
//   dW = dy^T window(x)  : TN, A = dy (tokens x O), B = window(x_pad)
// (2p = K - 1).  fp32 in, fp32 out, exact-f32 products (v_mfma_f32_16x16x4_f32)
// with fp32 accumulation: the reference's fp32 convolution arithmetic.
//
// Tile: 128 x 128 outputs per 256-thread workgroup, 4 waves of 64 x 64 (4 x 4
// MFMA blocks, 64 accumulator registers): a 32-deep K-step is 128 MFMAs
// (4096 cycles) per wave against 8 fragment reads, and fp32 operands cost
// 32 flop per byte staged (a 64 x 64 tile: 16, which L2 cannot feed at the
// fp32 MFMA rate).  Operands are register-staged (four float4 per thread and
// operand, loaded one K-step ahead) into a double-buffered LDS image sized
// for the TN tile (2 x 2 x 32 x 144 floats = 72 KiB per workgroup; two
// workgroups per CU fit gfx950's 160 KiB of LDS -- above the 64 KiB per
// workgroup of gfx942-class parts, a gfx950-only tile): NT tiles [row][32 k] with 16-B chunk c of row r at
// c ^ (r & 7) (conflict-free ds_read_b128: a lane group's 16 rows hit 16
// distinct slots), TN tiles [k][128 + 16] floats (the pad puts k-rows 0 / 1
// on disjoint banks for ds_read_b32).  MFMA operands are swapped (B fragment
// first) so a lane holds 4 consecutive output columns: float4 row stores.
// The text encoder's GEMMs have 16-64 such tiles, so K is split over up to
// 16 workgroups (`splits`): each writes its fp32 partial tile to a slab and a
// second kernel sums the slabs in fixed order (deterministic) and applies the
// epilogue.  Epilogues: + bias, ReLU, ReLU-backward (x (aux > 0)), beta
// accumulate.
#include "common.h"

#include <algorithm>
#include <climits>

namespace mtts {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kT = 256;     // threads
constexpr int kBM = 128, kBN = 128, kBK = 32;
constexpr int kLd = 4;                      // float4 loads per thread and operand per K-step
constexpr int kNtTile = kBM * kBK;          // floats per NT operand tile
constexpr int kTnPitch = kBM + 16;          // floats per k-row of a TN tile
constexpr int kTnTile = kBK * kTnPitch;
// the double-buffered A / B image of convgemm_kernel, two workgroups per CU
// (__launch_bounds__(kT, 2)) within gfx950's 160 KiB LDS
static_assert(2 * 2 * std::max(kNtTile, kTnTile) * sizeof(float) * 2 <= 160 * 1024,
              "convgemm: two workgroups' LDS images exceed gfx950's 160 KiB");

struct RowMap {
  const float* p;        // halo maps: already moved back by halo_p rows (host)
  int64_t seg_stride, row_stride;
  uint32_t seg_rows;     // host-checked < 2^31 (32-bit division on the device)
  int halo_c, halo_p;    // halo_c > 0: taps outside the segment read 0 (mtts.h)
  __device__ __forceinline__ const float* row(int r) const {
    const uint32_t s = (uint32_t)r / seg_rows;
    return p + (int64_t)s * seg_stride + (int64_t)((uint32_t)r - s * seg_rows) * row_stride;
  }
  __device__ __forceinline__ int pos(int r) const { return (int)((uint32_t)r % seg_rows); }
};

struct Params {
  RowMap a, b, aux;
  float* c;
  int64_t c_seg_stride, c_row_stride;
  uint32_t c_seg_rows;
  const float* bias;
  float* slabs;          // splits > 1: (splits, m, n) fp32 partials, then (splits, m) column-sum partials
  float* colsum;         // TN: sum over k of A's columns (n-tile 0's workgroups sum their A tiles)
  int m, n, k, tiles_n, tiles, splits, kper;
  int layout, epi;
  float beta;
};

// the epilogue on 4 consecutive columns n .. n+3 of row m
__device__ __forceinline__ void epi_store(const Params& p, int m, int n, f32x4 v) {
  const uint32_t s = (uint32_t)m / p.c_seg_rows;
  float* crow = p.c + (int64_t)s * p.c_seg_stride + (int64_t)((uint32_t)m - s * p.c_seg_rows) * p.c_row_stride;
  if (p.epi & MTTS_CONVGEMM_BIAS) v += *(const f32x4*)(p.bias + n);
  if (p.epi & MTTS_CONVGEMM_RELU) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
  }
  if (p.epi & MTTS_CONVGEMM_DRELU) {
    const f32x4 h = *(const f32x4*)(p.aux.row(m) + n);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = h[e] > 0.f ? v[e] : 0.f;
  }
  if (p.beta != 0.f) v += p.beta * *(const f32x4*)(crow + n);
  *(f32x4*)(crow + n) = v;
}

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// NT operand tile (rows r0.. of a k-contiguous matrix, K-step k0): thread t
// holds float4 t + 256 i (i < kLd) of the 128 x 32 tile
struct NtLoad {
  const float* rp[kLd];
  int chunk[kLd], lrow[kLd], tpos[kLd];
  bool rok[kLd];
  __device__ void init(const RowMap& mp, int r0, int rows, int tid) {
#pragma unroll
    for (int i = 0; i < kLd; ++i) {
      const int idx = tid + i * kT;
      lrow[i] = idx >> 3;
      chunk[i] = idx & 7;
      const int r = r0 + lrow[i];
      rok[i] = r < rows;
      rp[i] = mp.row(rok[i] ? r : 0);
      tpos[i] = mp.pos(rok[i] ? r : 0);
    }
  }
  // halo: the K-step's 32 columns are one tap j = k0 / halo_c (halo_c % 32 ==
  // 0, K-steps 32-aligned), valid on rows with 0 <= t - p + j < T
  __device__ __forceinline__ void load(f32x4 (&v)[kLd], int k0, int K, const RowMap& mp) const {
    int lo = INT_MIN, hi = INT_MAX;
    if (mp.halo_c > 0) {
      const int j = __builtin_amdgcn_readfirstlane(k0 / mp.halo_c);   // uniform: scalar division
      lo = mp.halo_p - j;
      hi = (int)mp.seg_rows + mp.halo_p - j;
    }
#pragma unroll
    for (int i = 0; i < kLd; ++i) {
      const int kk = k0 + chunk[i] * 4;
      v[i] = (rok[i] && kk < K && tpos[i] >= lo && tpos[i] < hi) ? *(const f32x4*)(rp[i] + kk)
                                                                : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  __device__ __forceinline__ void store(float* tile, const f32x4 (&v)[kLd]) const {
#pragma unroll
    for (int i = 0; i < kLd; ++i)
      *(f32x4*)(tile + lrow[i] * kBK + ((chunk[i] ^ (lrow[i] & 7)) << 2)) = v[i];
  }
};

// TN operand tile (k-rows k0.. of a matrix whose rows hold the m / n index
// contiguously, columns c0..c0+127): thread t holds float4 t + 256 i.  The
// row pointers walk the map incrementally (K-steps are consecutive within a
// split), so there is no 32-bit division per load and step.
struct TnLoad {
  int krow[kLd];
  bool cok[kLd];
  int tap[kLd];          // halo: the column's tap - p (fixed per thread: c0 is per workgroup)
  const float* rp[kLd];  // row k0 + krow[i] of the current step, at the thread's column
  uint32_t t[kLd];       // that row's position in its segment
  __device__ void init(int tid, const RowMap& mp, int c0, int cols, int k0) {
#pragma unroll
    for (int i = 0; i < kLd; ++i) {
      const int idx = tid + i * kT;
      krow[i] = idx >> 5;
      const int cc = c0 + (idx & 31) * 4;
      cok[i] = cc < cols;
      tap[i] = mp.halo_c > 0 ? cc / mp.halo_c - mp.halo_p : 0;
      const uint32_t kr = (uint32_t)(k0 + krow[i]);
      const uint32_t sg = kr / mp.seg_rows;
      t[i] = kr - sg * mp.seg_rows;
      rp[i] = mp.p + (int64_t)sg * mp.seg_stride + (int64_t)t[i] * mp.row_stride + cc;
    }
  }
  // halo (operand B of TN: rows = tokens, column cc = tap * C + channel):
  // token t contributes to tap j only where 0 <= t - p + j < T
  __device__ __forceinline__ void load(f32x4 (&v)[kLd], const RowMap& mp, int k0, int K) const {
#pragma unroll
    for (int i = 0; i < kLd; ++i) {
      bool ok = k0 + krow[i] < K && cok[i];
      if (mp.halo_c > 0) ok = ok && (uint32_t)((int)t[i] + tap[i]) < mp.seg_rows;
      v[i] = ok ? *(const f32x4*)rp[i] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  __device__ __forceinline__ void advance(const RowMap& mp) {   // to the next K-step's rows
#pragma unroll
    for (int i = 0; i < kLd; ++i) {
      t[i] += kBK;
      rp[i] += kBK * mp.row_stride;
      while (t[i] >= mp.seg_rows) {
        t[i] -= mp.seg_rows;
        rp[i] += mp.seg_stride - (int64_t)mp.seg_rows * mp.row_stride;
      }
    }
  }
  __device__ __forceinline__ void store(float* tile, const f32x4 (&v)[kLd]) const {
#pragma unroll
    for (int i = 0; i < kLd; ++i) *(f32x4*)(tile + krow[i] * kTnPitch + ((threadIdx.x + i * kT) & 31) * 4) = v[i];
  }
};

template <int LAYOUT>
__global__ __launch_bounds__(kT, 2) void convgemm_kernel(Params p) {
  constexpr bool NT = LAYOUT == MTTS_GEMM_NT;
  constexpr bool NN = LAYOUT == MTTS_CONVGEMM_NN;   // A as NT, B as TN
  constexpr int kTile = NT ? kNtTile : kTnTile;     // NN: A uses the first kNtTile floats
  __shared__ __attribute__((aligned(16))) float lds[2][2][kTile];   // [buffer][A / B]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int tile = blockIdx.x % p.tiles, split = blockIdx.x / p.tiles;
  const int m0 = (tile / p.tiles_n) * kBM, n0 = (tile % p.tiles_n) * kBN;
  const int kbeg = split * p.kper;
  const int kend = min(p.k, kbeg + p.kper);
  const int nk = (kend - kbeg + kBK - 1) / kBK;

  NtLoad na, nb;
  TnLoad ta_l, tb_l;   // TN operand A, TN / NN operand B
  if constexpr (NT || NN) na.init(p.a, m0, p.m, tid);
  if constexpr (NT) nb.init(p.b, n0, p.n, tid);
  if constexpr (!NT && !NN) ta_l.init(tid, p.a, m0, p.m, kbeg);
  if constexpr (!NT) tb_l.init(tid, p.b, n0, p.n, kbeg);
  f32x4 va[kLd], vb[kLd];
  auto load = [&](int kt) {   // called for kt = 0, 1, 2, ... in order (the TN row walk)
    const int k0 = kbeg + kt * kBK;
    if constexpr (NT || NN) na.load(va, k0, kend, p.a);
    else { ta_l.load(va, p.a, k0, kend); ta_l.advance(p.a); }
    if constexpr (NT) nb.load(vb, k0, kend, p.b);
    else { tb_l.load(vb, p.b, k0, kend); tb_l.advance(p.b); }
  };
  auto store = [&](int buf) {
    if constexpr (NT || NN) na.store(lds[buf][0], va);
    else ta_l.store(lds[buf][0], va);
    if constexpr (NT) nb.store(lds[buf][1], vb);
    else tb_l.store(lds[buf][1], vb);
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // TN column sums of A (the bias gradient when A = dy): the first n-tile's
  // workgroups add up the A tiles they stage anyway, thread t column t & 127
  // over k-rows 16 (t >> 7) .. +15 of each step (~16 LDS reads against 128
  // MFMAs per wave and step)
  const bool do_cs = !NT && !NN && p.colsum != nullptr && tile % p.tiles_n == 0;
  float cs = 0.f;

  load(0);
  store(0);
  if (nk > 1) load(1);
  block_sync();
  const int r16 = lane & 15, q = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) {
      store((kt + 1) & 1);   // the other buffer: its last reads were before the previous barrier
      if (kt + 2 < nk) load(kt + 2);
    }
    const float* ta = lds[kt & 1][0];
    const float* tb = lds[kt & 1][1];
    if constexpr (NT) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x4 fa[4], fb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ra = wr * 64 + i * 16 + r16, rb = wc * 64 + i * 16 + r16;
          fa[i] = *(const f32x4*)(ta + ra * kBK + (((h * 4 + q) ^ (ra & 7)) << 2));
          fb[i] = *(const f32x4*)(tb + rb * kBK + (((h * 4 + q) ^ (rb & 7)) << 2));
        }
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfma4(fb[j][s], fa[i][s], acc[i][j]);
      }
    } else if constexpr (NN) {
      // A from the swizzled NT image by float4 (as NT: lane group q's element
      // s is k = 16h + 4q + s), B from the TN image at those k-rows
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x4 fa[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ra = wr * 64 + i * 16 + r16;
          fa[i] = *(const f32x4*)(ta + ra * kBK + (((h * 4 + q) ^ (ra & 7)) << 2));
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          float fb[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) fb[j] = tb[(16 * h + 4 * q + s) * kTnPitch + wc * 64 + j * 16 + r16];
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfma4(fb[j], fa[i][s], acc[i][j]);
        }
      }
    } else {
      if (do_cs) {
#pragma unroll
        for (int r = 0; r < 16; ++r) cs += ta[((tid >> 7) * 16 + r) * kTnPitch + (tid & 127)];
      }
#pragma unroll
      for (int s = 0; s < kBK / 4; ++s) {
        const int kr = s * 4 + q;
        float fa[4], fb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          fa[i] = ta[kr * kTnPitch + wr * 64 + i * 16 + r16];
          fb[i] = tb[kr * kTnPitch + wc * 64 + i * 16 + r16];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma4(fb[j], fa[i], acc[i][j]);
      }
    }
    block_sync();
  }

  if (do_cs) {   // halves of the k-rows -> one sum per column (fixed order), then the split's slab or colsum
    float* red = lds[0][0];   // free: every step's reads precede the loop's last barrier
    if (tid >= 128) red[tid - 128] = cs;
    block_sync();
    const int m = m0 + tid;
    if (tid < 128 && m < p.m) {
      const float v = cs + red[tid];
      if (p.splits > 1) p.slabs[(int64_t)p.splits * p.m * p.n + (int64_t)split * p.m + m] = v;
      else p.colsum[m] = v;
    }
  }

  // lane holds C[m][n .. n+3], m = .. + (lane & 15), n = .. + 4 (lane >> 4)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wr * 64 + i * 16 + r16;
    if (m >= p.m) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wc * 64 + j * 16 + 4 * q;
      if (n >= p.n) continue;
      if (p.splits > 1)
        *(f32x4*)(p.slabs + ((int64_t)split * p.m + m) * p.n + n) = acc[i][j];
      else
        epi_store(p, m, n, acc[i][j]);
    }
  }
}

// split-K: C = epilogue(sum over splits of the slabs, fixed order)
__global__ __launch_bounds__(256) void convgemm_reduce_kernel(Params p) {
  const int n4 = p.n / 4;
  const int64_t total = (int64_t)p.m * n4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int m = (int)(i / n4), n = (int)(i % n4) * 4;
    const float* sp = p.slabs + (int64_t)m * p.n + n;
    f32x4 v = *(const f32x4*)sp;
    for (int s = 1; s < p.splits; ++s) v += *(const f32x4*)(sp + (int64_t)s * p.m * p.n);
    epi_store(p, m, n, v);
  }
  if (p.colsum) {   // the column-sum partials, in split order
    const float* cp = p.slabs + (int64_t)p.splits * p.m * p.n;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < p.m; i += gridDim.x * blockDim.x) {
      float v = cp[i];
      for (int s = 1; s < p.splits; ++s) v += cp[(int64_t)s * p.m + i];
      p.colsum[i] = v;
    }
  }
}

bool map_ok(const MttsRowMap& r, bool halo_ok = false) {
  if (r.halo_c != 0 && !(halo_ok && r.halo_c > 0 && r.halo_c % 32 == 0 && r.halo_p >= 0))
    return false;
  return r.ptr && r.seg_rows > 0 && r.seg_rows < (1ll << 31) && r.seg_stride % 4 == 0 && r.row_stride % 4 == 0 &&
         (uintptr_t)r.ptr % 16 == 0;
}

}  // namespace
}  // namespace mtts

using namespace mtts;

extern "C" int mtts_convgemm(const MttsConvGemmArgs* a, void* stream) {
  MTTS_CHECK(a, "convgemm: null args");
  MTTS_CHECK(a->m > 0 && a->n > 0 && a->k > 0, "convgemm: m=%d n=%d k=%d must be positive", a->m, a->n, a->k);
  MTTS_CHECK(a->layout == MTTS_GEMM_NT || a->layout == MTTS_GEMM_TN || a->layout == MTTS_CONVGEMM_NN,
             "convgemm: layout must be NT (0), TN (1) or NN (2)");
  const bool nt = a->layout == MTTS_GEMM_NT, nn = a->layout == MTTS_CONVGEMM_NN;
  MTTS_CHECK(map_ok(a->a, nt || nn) && map_ok(a->b, !nt && !nn) && map_ok(a->c),
             "convgemm: operands need a pointer, seg_rows > 0, 16-byte alignment and strides a multiple of 4 "
             "(halo maps: NT / NN operand A or TN operand B only, halo_c %% 32 == 0, halo_p >= 0)");
  MTTS_CHECK(a->n % 4 == 0, "convgemm: n=%d must be a multiple of 4", a->n);
  MTTS_CHECK((nt || nn) ? a->k % 4 == 0 : a->m % 4 == 0, "convgemm: %s must be a multiple of 4",
             (nt || nn) ? "k" : "m");
  MTTS_CHECK(!(a->epilogue & MTTS_CONVGEMM_BIAS) || (a->bias && (uintptr_t)a->bias % 16 == 0),
             "convgemm: bias epilogue needs a 16-byte aligned bias");
  MTTS_CHECK(!(a->epilogue & MTTS_CONVGEMM_DRELU) || map_ok(a->aux), "convgemm: ReLU-backward epilogue needs aux");
  MTTS_CHECK(a->k % 32 == 0 || a->a.halo_c == 0, "convgemm: a halo operand A needs k %% 32 == 0");
  MTTS_CHECK(!((a->epilogue & MTTS_CONVGEMM_RELU) && (a->epilogue & MTTS_CONVGEMM_DRELU)),
             "convgemm: RELU and DRELU are exclusive");
  Params p{};
  auto rm = [](const MttsRowMap& r) {   // a halo map's rows start halo_p rows before t (never read there)
    return RowMap{(const float*)r.ptr - (int64_t)r.halo_p * r.row_stride, r.seg_stride, r.row_stride,
                  (uint32_t)r.seg_rows, r.halo_c, r.halo_p};
  };
  p.a = rm(a->a);
  p.b = rm(a->b);
  if (a->epilogue & MTTS_CONVGEMM_DRELU) p.aux = rm(a->aux);
  p.c = (float*)a->c.ptr;
  p.c_seg_rows = (uint32_t)a->c.seg_rows; p.c_seg_stride = a->c.seg_stride; p.c_row_stride = a->c.row_stride;
  p.bias = a->bias;
  p.m = a->m; p.n = a->n; p.k = a->k;
  p.tiles_n = (a->n + kBN - 1) / kBN;
  p.layout = a->layout; p.epi = a->epilogue; p.beta = a->beta;
  const int64_t tiles = (int64_t)((a->m + kBM - 1) / kBM) * p.tiles_n;
  const int splits = a->splits > 1 ? a->splits : 1;
  MTTS_CHECK(splits <= 64, "convgemm: splits=%d (at most 64)", splits);
  MTTS_CHECK(tiles * splits < (1ll << 31), "convgemm: too many tiles");
  MTTS_CHECK(splits == 1 || (a->workspace && (uintptr_t)a->workspace % 16 == 0),
             "convgemm: split-K needs the workspace (mtts_convgemm_workspace bytes, 16-byte aligned)");
  p.tiles = (int)tiles;
  p.splits = splits;
  p.kper = (int)(((int64_t)(a->k + splits - 1) / splits + kBK - 1) / kBK * kBK);
  p.slabs = (float*)a->workspace;
  MTTS_CHECK(!a->colsum_a || a->layout == MTTS_GEMM_TN, "convgemm: colsum_a is a TN option (A = dy)");
  p.colsum = a->colsum_a;
  hipStream_t st = (hipStream_t)stream;
  const unsigned grid = (unsigned)(tiles * splits);
  if (nt) hipLaunchKernelGGL(convgemm_kernel<MTTS_GEMM_NT>, dim3(grid), dim3(kT), 0, st, p);
  else if (nn) hipLaunchKernelGGL(convgemm_kernel<MTTS_CONVGEMM_NN>, dim3(grid), dim3(kT), 0, st, p);
  else hipLaunchKernelGGL(convgemm_kernel<MTTS_GEMM_TN>, dim3(grid), dim3(kT), 0, st, p);
  MTTS_LAUNCH_CHECK("convgemm");
  if (splits > 1) {
    const int64_t total = (int64_t)a->m * (a->n / 4);
    const int blocks = (int)std::min<int64_t>((total + 255) / 256, 2048);
    hipLaunchKernelGGL(convgemm_reduce_kernel, dim3(blocks), dim3(256), 0, st, p);
    MTTS_LAUNCH_CHECK("convgemm reduce");
  }
  return MTTS_OK;
}

extern "C" int64_t mtts_convgemm_workspace(const MttsConvGemmArgs* a) {
  if (!a || a->splits <= 1) return 0;
  return (int64_t)a->splits * a->m * (a->n + (a->colsum_a ? 1 : 0)) * 4;
}
