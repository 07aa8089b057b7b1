// bf16 MFMA GEMM for the decoder's training projections (gfx950).
//
// C[M,N] = epilogue( A·B ) with fp32 accumulation, two operand layouts:
//   NT (fwd y = x·Wᵀ, dgrad dx = dy·W on the cast kernel's Wᵀ copy):
//       A[M,K], B[N,K], both k-contiguous;
//   TN (wgrad dW = dyᵀ·x over the token axis):
//       A[K,M], B[K,N], both m/n-contiguous, fp32 out (master grads), split-K.
// Reference sites: the nn.Linear / in_proj / x_proj / dt_proj / out_proj / MHA
// projections of /root/reference/mamba_decoder.py:29-43 (Mamba, MHA, FFN)
// applied at :61-88.
//
// Structure (one 256x256 output tile per 512-thread workgroup, 8 waves as
// 2 (M) x 4 (N), 128x64 per wave, v_mfma_f32_16x16x32_bf16):
//  * a 64-deep K-tile of A and B is 64 KiB of LDS, split into four 16 KiB
//    REGIONS by the quadrant that reads them: A0/A1 = the A rows each wave
//    reads as its first/second 64-row half, B0/B1 = the B rows it reads as
//    its first/second 32-column half.  Two K-tile buffers = 128 KiB, ONE
//    __shared__ array.
//  * a K-tile is four PHASES, one 64x32 quadrant x K=64 per wave each
//    (16 MFMAs): (A0,B0) (A0,B1) (A1,B1) (A1,B0); A frags are read at
//    phases 0 and 2, B frags at phases 0 and 1 and kept in registers, so each
//    region's last LDS read is in phase 0, 0, 1 or 2.
//  * every phase stages exactly one region (2 LDS-DMA global_load_lds_dwordx4
//    per thread, 16 KiB per workgroup) of a LATER K-tile into a region whose
//    last read lies at least one barrier back: phase 0 stages A1 of tile t+1,
//    phases 1-3 stage A0, B0, B1 of tile t+2.  A region is first read 6 or 7
//    phases after it was staged, so each phase ends with s_waitcnt vmcnt(10)
//    (the 5 younger phases' 2 DMAs each stay in flight across the barrier) and
//    one raw s_barrier; the last two K-tiles wait vmcnt(0).
//  * the LDS images are lane-linear (the DMA writes base + 16*lane); bank
//    swizzles move to the SOURCE address (k-major: 16-B chunk c of row r at
//    c ^ ((r>>1)&7), conflict-free ds_read_b128 for 16 consecutive rows;
//    m/n-major: 32-B granule g of k-row r at g ^ ((r&3) | ((r>>3)&1)<<2),
//    conflict-free ds_read_b64_tr_b16 over a 32-lane half).
//  * MFMA operands are swapped (B fragment first) so a lane's accumulator
//    holds 4 consecutive output COLUMNS of one row: 8-byte (bf16) / 16-byte
//    (fp32) row-major stores.
//  * epilogues on the fp32 accumulator: + bias; GELU (exact erf) writing the
//    pre-activation too (for the backward); GELU backward (dgrad times
//    gelu'(pre-activation)); fp32 out with beta·C accumulate (wgrad).
#include "common.h"

#include <type_traits>

namespace mtts {
namespace {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) s16x8 lds_s16x8;

constexpr int kThreads = 512;
constexpr int kTile = 256;        // BM = BN
constexpr int kBK = 64;
constexpr int kRegion = 16384;    // bytes
constexpr int kBuf = 4 * kRegion; // one K-tile: A0 A1 B0 B1
constexpr int kLds = 2 * kBuf;    // 128 KiB

enum { R_A0 = 0, R_A1 = 1, R_B0 = 2, R_B1 = 3 };

struct GemmParams {
  const bf16_t* a;
  const bf16_t* b;
  void* c;
  const void* bias;
  void* aux;
  int64_t lda, ldb, ldc, ld_aux;
  int64_t split_stride;  // elements between split-K output slabs (fp32 out)
  int m, n, k;           // k: per-split K range length (multiple of 64)
  int tiles_m, tiles_n, splits;
  int group;             // tile rows per L2 group
  int epi;               // MTTS_GEMM_EPI_*
  int bias_bf16;
  int wide_out;          // bf16 out (and aux) rows 16-byte aligned: dwordx4 epilogue
  float beta;
};

// region-local row/column (0..127) -> tile row/column
__device__ __forceinline__ int a_map(int rr, int s) { return (rr >> 6) * 128 + s * 64 + (rr & 63); }
__device__ __forceinline__ int b_map(int rr, int s) { return (rr >> 5) * 64 + s * 32 + (rr & 31); }
template <bool IS_A>
__device__ __forceinline__ int rmap(int rr, int s) { return IS_A ? a_map(rr, s) : b_map(rr, s); }

// 16-byte LDS-DMA with a 32-bit per-lane offset from a wave-uniform base;
// invisible to the compiler's wait insertion (every consumer waits by hand).
__device__ __forceinline__ void glds16(const void* base, uint32_t voff, uint32_t lds_base) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(base), "s"(lds_base)
               : "memory", "m0");
#endif
}
template <int N>
__device__ __forceinline__ void wait_vm() {
#if defined(__HIP_DEVICE_COMPILE__)
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
#endif
}
// lgkmcnt(0) + s_barrier through the builtins (so the compiler's own wait
// bookkeeping sees the LDS reads retired: an inline-asm wait is invisible to
// it and it re-waits on the NEXT phase's prefetch reads), then a compiler
// fence so no LDS access moves across.
__device__ __forceinline__ void barrier() {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0); vmcnt / expcnt untouched
#ifndef MTTS_GEMM_DIAG_NOBAR
  __builtin_amdgcn_s_barrier();
#endif
  asm volatile("" ::: "memory");
#endif
}

__device__ __forceinline__ f32x4 mfma(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

// GELU epilogues (exact-erf F.gelu and its derivative) with one polynomial
// and one exp2, no branches: the tail h(x) = Phi(-|x|) = erfc(|x|/sqrt2)/2 is
// exp2(S(a) - a^2 log2(e)/2), a = min(|x|, 5.5), S a degree-10 polynomial
// (least-squares fit of log2 h + a^2 log2(e)/2 on [0, 5.5], reweighted to an
// equi-ripple error: 1.4e-7 relative in float64, 2.8e-6 evaluated in fp32,
// where exp2 of the ~-26 argument at a = 5.5 sets the floor); Phi(x) = x >= 0 ?
// 1 - h : h.  18 VALU per GELU (was 27: erf as two polynomial arms and a
// select), 21 per derivative (was 31).  Fit and check: DESIGN.md §3.
__device__ __forceinline__ float gelu_tail_s(float a) {
  float s = -1.7774024116e-08f;
  s = fmaf(s, a, 5.6194854933e-07f);
  s = fmaf(s, a, -7.6223902631e-06f);
  s = fmaf(s, a, 5.5893204013e-05f);
  s = fmaf(s, a, -2.0454518331e-04f);
  s = fmaf(s, a, -1.6655060660e-04f);
  s = fmaf(s, a, 7.1668288485e-03f);
  s = fmaf(s, a, -5.2604280745e-02f);
  s = fmaf(s, a, 2.6218665810e-01f);
  s = fmaf(s, a, -1.1511125488e+00f);
  s = fmaf(s, a, -9.9999981719e-01f);
  return s;
}
__device__ __forceinline__ float gelu_f(float x) {
  const float a = fminf(fabsf(x), 5.5f);
  const float h = __builtin_amdgcn_exp2f(fmaf(x * (-0.5f * kLog2e), x, gelu_tail_s(a)));
  return x * (x >= 0.f ? 1.f - h : h);
}
// The same two functions on two values at once: the polynomial and the
// argument arithmetic as packed f32 (v_pk_fma_f32 / v_pk_mul_f32, each lane's
// fma exactly the scalar one: bit-identical results at half the VALU issues)
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_tail_s2(f32x2 a) {
  f32x2 s = f32x2{-1.7774024116e-08f, -1.7774024116e-08f};
  const float c[10] = {5.6194854933e-07f, -7.6223902631e-06f, 5.5893204013e-05f, -2.0454518331e-04f,
                       -1.6655060660e-04f, 7.1668288485e-03f, -5.2604280745e-02f, 2.6218665810e-01f,
                       -1.1511125488e+00f, -9.9999981719e-01f};
#pragma unroll
  for (int i = 0; i < 10; ++i) s = __builtin_elementwise_fma(s, a, f32x2{c[i], c[i]});
  return s;
}
__device__ __forceinline__ f32x2 gelu_f2(f32x2 x) {
  const f32x2 a = __builtin_elementwise_min(__builtin_elementwise_abs(x), f32x2{5.5f, 5.5f});
  const f32x2 t = __builtin_elementwise_fma(x * f32x2{-0.5f * kLog2e, -0.5f * kLog2e}, x, gelu_tail_s2(a));
  const float h0 = __builtin_amdgcn_exp2f(t[0]), h1 = __builtin_amdgcn_exp2f(t[1]);
  return x * f32x2{x[0] >= 0.f ? 1.f - h0 : h0, x[1] >= 0.f ? 1.f - h1 : h1};
}
__device__ __forceinline__ f32x2 gelu_grad_f2(f32x2 x) {
  const f32x2 a = __builtin_elementwise_min(__builtin_elementwise_abs(x), f32x2{5.5f, 5.5f});
  const f32x2 m = x * f32x2{-0.5f * kLog2e, -0.5f * kLog2e} * x;
  const f32x2 u = m + gelu_tail_s2(a);
  const f32x2 e = f32x2{__builtin_amdgcn_exp2f(m[0]), __builtin_amdgcn_exp2f(m[1])};
  const f32x2 h = f32x2{__builtin_amdgcn_exp2f(u[0]), __builtin_amdgcn_exp2f(u[1])};
  return __builtin_elementwise_fma(x * f32x2{0.3989422804014327f, 0.3989422804014327f}, e,
                                   f32x2{x[0] >= 0.f ? 1.f - h[0] : h[0], x[1] >= 0.f ? 1.f - h[1] : h[1]});
}

// torch's GeluBackward: Phi(x) + x exp(-x^2/2) / sqrt(2 pi)
__device__ __forceinline__ float gelu_grad_f(float x) {
  const float a = fminf(fabsf(x), 5.5f);
  const float m = x * (-0.5f * kLog2e) * x;
  const float e = __builtin_amdgcn_exp2f(m);
  const float h = __builtin_amdgcn_exp2f(m + gelu_tail_s(a));
  return fmaf(x * 0.3989422804014327f, e, x >= 0.f ? 1.f - h : h);
}

// Per-thread source offsets (elements) of one region's two DMAs, relative to
// the operand's tile origin; k-major: rows of the tile, m/n-major: k-rows.
template <bool KMAJ, bool IS_A>
struct Loader {
  uint32_t off[2][2];  // [sub s][dma i], in bytes from the K-tile origin

  __device__ void init(int tid, int row0, int nrows, int64_t ld) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if constexpr (KMAJ) {
          const int rr = i * 64 + (tid >> 3), p = tid & 7;
          const int c = p ^ ((rr >> 1) & 7);
          int row = row0 + rmap<IS_A>(rr, s);
          row = row < nrows ? row : nrows - 1;
          off[s][i] = (uint32_t)((row * ld + c * 8) * 2);
        } else {
          const int kr = i * 32 + (tid >> 4), p = tid & 15;
          const int f = (kr & 3) | (((kr >> 3) & 1) << 2);
          const int c = p ^ (f << 1);                   // logical 16-B chunk (8 columns)
          int col = row0 + rmap<IS_A>(c * 8, s);
          col = col + 8 <= nrows ? col : ((nrows - 8) & ~7);
          off[s][i] = (uint32_t)((kr * ld + col) * 2);
        }
      }
  }
  // stage sub-part s of K-tile `kt` (origin pointer for that K-tile) into region `lds_region`
  __device__ __forceinline__ void stage1(const char* ktile, int s, uint32_t lds_region, int wave, int i) const {
    glds16(ktile, off[s][i], lds_region + i * 8192 + wave * 1024);
  }
};

// fragment for (region byte base, 16-row block at region-local row rb, k-step ks)
template <bool KMAJ>
__device__ __forceinline__ s16x8 frag(const char* region, int rb, int ks, int lane) {
#ifdef MTTS_GEMM_DIAG_NOREAD
  s16x8 z{};   // timing-only: no LDS reads
  asm volatile("" : "+v"(z));
  return z;
#endif
  if constexpr (KMAJ) {
    const int rr = rb + (lane & 15);
    const int c = (ks * 4 + (lane >> 4)) ^ ((rr >> 1) & 7);
    return *(const lds_s16x8*)(region + rr * 128 + c * 16);
  } else {
    // two ds_read_b64_tr_b16: k-rows ks*32 + 8g + 4h + q, columns rb + 4p .. +3
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int col = rb + 4 * p;
    s16x4 r[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int kr = ks * 32 + 8 * g + 4 * h + q;
      const int f = (kr & 3) | (((kr >> 3) & 1) << 2);
      const int chunk = (col >> 3) ^ (f << 1);
      r[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_s16x4*)(region + kr * 256 + chunk * 16 + (col & 7) * 2));
    }
    return s16x8{r[0][0], r[0][1], r[0][2], r[0][3], r[1][0], r[1][1], r[1][2], r[1][3]};
  }
}

// Epilogue shared by the kernels: the wave's 128x64 accumulator tile
// (acc[MB][NB], lane rows m = MB*16 + (lane&15), columns 4*(lane>>4) + j of
// block NB) -> bf16 (+bias / GELU / GELU-backward) or fp32 (split slab, beta).
template <int EPI, bool OUT_F32>
__device__ __forceinline__ void store_tile(const GemmParams& p, f32x4 (&acc)[8][4], int m0, int n0, int wr, int wc,
                                           int lane, int split) {
  // lane holds rows m = .. + (lane&15), columns n = .. + 4*(lane>>4) + j
  const int rl = lane & 15, cl = 4 * (lane >> 4);
  // wave-uniform: the wave's whole 128x64 sub-tile in bounds (no per-lane masks)
  const bool full = m0 + wr * 128 + 128 <= p.m && n0 + wc * 64 + 64 <= p.n;
  if constexpr (!OUT_F32) {
   if (p.wide_out) {
    // bf16 out: the 16-lane rows g and g^1 of the wave hold adjacent 4-column
    // groups of the same output rows; one v_permlane16_swap per dword of a
    // (NB, NB+1) pair gives each lane 8 consecutive columns, so the tile
    // leaves as 16 dwordx4 stores per lane instead of 32 dwordx2 (the store
    // tail is issue-bound: cdna_hip_programming.md T21).  After the swap the
    // even rows hold block 2pr columns 8(g>>1)..+7, the odd rows block 2pr+1.
    const int g = lane >> 4;
    const int cw0 = n0 + wc * 64 + (g & 1) * 16 + 8 * (g >> 1);
#pragma unroll
    for (int MB = 0; MB < 8; ++MB) {
      const int row = m0 + wr * 128 + MB * 16 + rl;
      if (!full && row >= p.m) continue;   // rows g and g^1 share `row`: the swap partners skip together
      uint32_t o2[4][2], h2[4][2];
#pragma unroll
      for (int NB = 0; NB < 4; ++NB) {
        const int col = n0 + wc * 64 + NB * 16 + cl;
        const bool cok = full || col < p.n;   // n % 8 == 0: a lane's 4 columns are all in or all out
        f32x4 v = acc[MB][NB];
        if (EPI & MTTS_GEMM_EPI_BIAS) {
          float bb[4] = {0.f, 0.f, 0.f, 0.f};
          if (cok) {
            if (p.bias_bf16) {
              const uint2 raw = *(const uint2*)((const bf16_t*)p.bias + col);
              bb[0] = __uint_as_float(raw.x << 16); bb[1] = __uint_as_float(raw.x & 0xffff0000u);
              bb[2] = __uint_as_float(raw.y << 16); bb[3] = __uint_as_float(raw.y & 0xffff0000u);
            } else {
              const f32x4 b4 = *(const f32x4*)((const float*)p.bias + col);
              bb[0] = b4[0]; bb[1] = b4[1]; bb[2] = b4[2]; bb[3] = b4[3];
            }
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] += bb[j];
        }
        bf16_t o[4];
        if constexpr ((EPI & MTTS_GEMM_EPI_GELU) != 0) {
          bf16_t hpre[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            hpre[j] = f2bf(v[j]);
            o[j] = f2bf(gelu_f(bf2f(hpre[j])));
          }
          h2[NB][0] = hpre[0] | ((uint32_t)hpre[1] << 16);
          h2[NB][1] = hpre[2] | ((uint32_t)hpre[3] << 16);
        } else if constexpr ((EPI & MTTS_GEMM_EPI_DGELU) != 0) {
          uint2 raw = make_uint2(0, 0);
          if (cok) raw = *(const uint2*)((const bf16_t*)p.aux + (int64_t)row * p.ld_aux + col);
          const float h[4] = {__uint_as_float(raw.x << 16), __uint_as_float(raw.x & 0xffff0000u),
                              __uint_as_float(raw.y << 16), __uint_as_float(raw.y & 0xffff0000u)};
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = f2bf(bf2f(f2bf(v[j])) * gelu_grad_f(h[j]));
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = f2bf(v[j]);
        }
        o2[NB][0] = o[0] | ((uint32_t)o[1] << 16);
        o2[NB][1] = o[2] | ((uint32_t)o[3] << 16);
      }
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        uint32_t w[4];
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const auto r = __builtin_amdgcn_permlane16_swap(o2[2 * pr][d], o2[2 * pr + 1][d], false, false);
          w[d] = r[0];
          w[2 + d] = r[1];
        }
        const int cw = cw0 + pr * 32;
        if (full || cw < p.n) {
          *(uint4*)((bf16_t*)p.c + (int64_t)row * p.ldc + cw) = make_uint4(w[0], w[1], w[2], w[3]);
        }
        if constexpr ((EPI & MTTS_GEMM_EPI_GELU) != 0) {
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            const auto r = __builtin_amdgcn_permlane16_swap(h2[2 * pr][d], h2[2 * pr + 1][d], false, false);
            w[d] = r[0];
            w[2 + d] = r[1];
          }
          if (full || cw < p.n)
            *(uint4*)((bf16_t*)p.aux + (int64_t)row * p.ld_aux + cw) = make_uint4(w[0], w[1], w[2], w[3]);
        }
      }
    }
    return;
   }
  }
#pragma unroll
  for (int MB = 0; MB < 8; ++MB) {
    const int row = m0 + wr * 128 + MB * 16 + rl;
    if (!full && row >= p.m) continue;
#pragma unroll
    for (int NB = 0; NB < 4; ++NB) {
      const int col = n0 + wc * 64 + NB * 16 + cl;
      if (!full && col >= p.n) continue;   // n % 8 == 0: a lane's 4 columns are all in or all out
      f32x4 v = acc[MB][NB];
      if constexpr (OUT_F32) {
        float* cp = (float*)p.c + (int64_t)split * p.split_stride + (int64_t)row * p.ldc + col;
        if (p.beta != 0.f) {
          const f32x4 o = *(const f32x4*)cp;
          v = v + p.beta * o;
        }
        *(f32x4*)cp = v;
      } else {
        if (EPI & MTTS_GEMM_EPI_BIAS) {
          float bb[4];
          if (p.bias_bf16) {
            const uint2 raw = *(const uint2*)((const bf16_t*)p.bias + col);
            bb[0] = __uint_as_float(raw.x << 16); bb[1] = __uint_as_float(raw.x & 0xffff0000u);
            bb[2] = __uint_as_float(raw.y << 16); bb[3] = __uint_as_float(raw.y & 0xffff0000u);
          } else {
            const f32x4 b4 = *(const f32x4*)((const float*)p.bias + col);
            bb[0] = b4[0]; bb[1] = b4[1]; bb[2] = b4[2]; bb[3] = b4[3];
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] += bb[j];
        }
        bf16_t o[4];
        if constexpr ((EPI & MTTS_GEMM_EPI_GELU) != 0) {
          bf16_t hpre[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            hpre[j] = f2bf(v[j]);
            o[j] = f2bf(gelu_f(bf2f(hpre[j])));
          }
          bf16_t* ap = (bf16_t*)p.aux + (int64_t)row * p.ld_aux + col;
          *(uint2*)ap = make_uint2(hpre[0] | ((uint32_t)hpre[1] << 16), hpre[2] | ((uint32_t)hpre[3] << 16));
        } else if constexpr ((EPI & MTTS_GEMM_EPI_DGELU) != 0) {
          const bf16_t* ap = (const bf16_t*)p.aux + (int64_t)row * p.ld_aux + col;
          const uint2 raw = *(const uint2*)ap;
          const float h[4] = {__uint_as_float(raw.x << 16), __uint_as_float(raw.x & 0xffff0000u),
                              __uint_as_float(raw.y << 16), __uint_as_float(raw.y & 0xffff0000u)};
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = f2bf(bf2f(f2bf(v[j])) * gelu_grad_f(h[j]));
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = f2bf(v[j]);
        }
        bf16_t* cp = (bf16_t*)p.c + (int64_t)row * p.ldc + col;
        *(uint2*)cp = make_uint2(o[0] | ((uint32_t)o[1] << 16), o[2] | ((uint32_t)o[3] << 16));
      }
    }
  }
}

template <bool AK, bool BKM, int EPI, bool OUT_F32>
__global__ __launch_bounds__(kThreads, 1) void gemm_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) char lds[kLds];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  // XCD-aware tile order: consecutive ids (one XCD's share) walk N fastest
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
  const int id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tiles = p.tiles_m * p.tiles_n;
  const int split = id / tiles;
  const int tile = id % tiles;
  // groups of `group` tile rows walked column by column: the ~32 tiles one
  // XCD runs at a time share a few A and B panels in its L2
  const int gsz = p.group * p.tiles_n;
  const int g0 = (tile / gsz) * p.group;
  const int gr = min(p.group, p.tiles_m - g0);
  const int tm = g0 + (tile % gsz) % gr, tn = (tile % gsz) / gr;
#ifdef MTTS_GEMM_DIAG_SAMETILE
  const int m0 = 0, n0 = 0;   // timing-only: every block streams tile (0, 0) (L2-resident)
#else
  const int m0 = tm * kTile, n0 = tn * kTile;
#endif

  // K-tile origins (bytes) for this split
  const int64_t k0 = (int64_t)split * p.k;
  const char* abase;
  const char* bbase;
  int64_t astep, bstep;  // bytes per K-tile
  if constexpr (AK) { abase = (const char*)(p.a + k0); astep = kBK * 2; }
  else { abase = (const char*)(p.a + k0 * p.lda); astep = kBK * p.lda * 2; }
  if constexpr (BKM) { bbase = (const char*)(p.b + k0); bstep = kBK * 2; }
  else { bbase = (const char*)(p.b + k0 * p.ldb); bstep = kBK * p.ldb * 2; }

  Loader<AK, true> la;
  Loader<BKM, false> lb;
  la.init(tid, m0, p.m, p.lda);
  lb.init(tid, n0, p.n, p.ldb);

  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds;
  auto region_addr = [&](int buf, int r) -> uint32_t { return lds0 + buf * kBuf + r * kRegion; };
  auto stage1 = [&](int kt, int r, int i) {
#ifdef MTTS_GEMM_DIAG_NODMA
    if (kt >= 0) return;   // timing-only: no operand traffic
#endif
    const int buf = kt & 1;
#ifdef MTTS_GEMM_DIAG_FIXK
    kt = buf;   // timing-only: every K-tile re-reads K-tiles 0/1 (L2-resident, per-block addresses)
#endif
    if (r == R_A0 || r == R_A1) la.stage1(abase + kt * astep, r - R_A0, region_addr(buf, r), wave, i);
    else lb.stage1(bbase + kt * bstep, r - R_B0, region_addr(buf, r), wave, i);
  };
  auto stage = [&](int kt, int r) { stage1(kt, r, 0); stage1(kt, r, 1); };

  const int nk = p.k / kBK;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Global phase P = 4t + q.  Tile j's regions are staged at phases
  // A0: 4j-9, B0: 4j-8, B1: 4j-7, A1: 4j-6 and first (and only) read — as
  // the next phase's fragments, prefetched — at A0: 4j-2, B0: 4j-1, B1: 4j,
  // A1: 4j+1: seven phases later for every region.  So the end of phase P
  // retires what was staged at P-6 (read from P+1 on): vmcnt = 2 x the
  // regions staged in phases P-5..P.  The last staged phase is 4nk-10.
  const int lv = 4 * nk - 10;
  auto wait_end = [&](int P) {
    int n = (P < lv ? P : lv) - P + 6;   // regions staged in P-5..P
    n = n < 0 ? 0 : n;
    switch (n) {
      case 6: wait_vm<12>(); break;
      case 5: wait_vm<10>(); break;
      case 4: wait_vm<8>(); break;
      case 3: wait_vm<6>(); break;
      case 2: wait_vm<4>(); break;
      case 1: wait_vm<2>(); break;
      default: wait_vm<0>(); break;
    }
    barrier();
  };
  // prologue: phases -9 .. -1
  // (A0(2), staged at phase -1 into tile 0's buffer, waits for the reads of
  // A0(0) and one barrier)
  stage(0, R_A0); stage(0, R_B0); stage(0, R_B1); stage(0, R_A1);
  if (nk > 1) { stage(1, R_A0); stage(1, R_B0); stage(1, R_B1); stage(1, R_A1); }
  if (nk > 1) wait_vm<10>(); else wait_vm<2>();   // A0(0) B0(0) B1(0) landed
  barrier();

  const char* lbase = lds;
  s16x8 a0[2][4], a1[2][4], b0[2][2], b1[2][2];  // [ks][block]
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) a0[ks][mb] = frag<AK>(lbase + R_A0 * kRegion, wr * 64 + mb * 16, ks, lane);
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) b0[ks][nb] = frag<BKM>(lbase + R_B0 * kRegion, wc * 32 + nb * 16, ks, lane);
  }
  barrier();
  if (nk > 2) stage(2, R_A0);

  // steady K-tiles (every phase stages; constant waits), then the tail.
  // Inside a phase the two DMAs sit between MFMA groups (pinned by
  // sched_barrier): a DMA holds its wave's issue for ~60-180 cycles, during
  // which the SIMD's other wave keeps the matrix pipe busy.
#define MFMA4(BF, AF, MO, NO, KS, MP)                                                         \
  _Pragma("unroll") for (int mb_ = 2 * (MP); mb_ < 2 * (MP) + 2; ++mb_)                      \
  _Pragma("unroll") for (int nb_ = 0; nb_ < 2; ++nb_)                                        \
      acc[(MO) + mb_][(NO) + nb_] = mfma(BF[KS][nb_], AF[KS][mb_], acc[(MO) + mb_][(NO) + nb_]);
#define PHASE_MFMA(BF, AF, MO, NO, DO_STAGE, KT, R)                                           \
  __builtin_amdgcn_s_setprio(1);                                                              \
  MFMA4(BF, AF, MO, NO, 0, 0)                                                                 \
  __builtin_amdgcn_sched_barrier(0);                                                          \
  if (DO_STAGE) stage1(KT, R, 0);                                                             \
  __builtin_amdgcn_sched_barrier(0);                                                          \
  MFMA4(BF, AF, MO, NO, 0, 1)                                                                 \
  __builtin_amdgcn_sched_barrier(0);                                                          \
  if (DO_STAGE) stage1(KT, R, 1);                                                             \
  __builtin_amdgcn_sched_barrier(0);                                                          \
  MFMA4(BF, AF, MO, NO, 1, 0)                                                                 \
  MFMA4(BF, AF, MO, NO, 1, 1)                                                                 \
  __builtin_amdgcn_s_setprio(0);
  auto ktile = [&](int t, auto steady) {
    constexpr bool ST = decltype(steady)::value;
    const char* bufp = lbase + (t & 1) * kBuf;
    const char* nxtp = lbase + ((t + 1) & 1) * kBuf;
    const int P = 4 * t;
    const bool more = ST || t + 1 < nk;
    // ---- phase 0: A0 x B0 | prefetch B1(t) | stage B0(t+2)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) b1[ks][nb] = frag<BKM>(bufp + R_B1 * kRegion, wc * 32 + nb * 16, ks, lane);
    PHASE_MFMA(b0, a0, 0, 0, (ST || P <= lv), t + 2, R_B0)
    if constexpr (ST) wait_vm<12>(), barrier(); else wait_end(P);
    // ---- phase 1: A0 x B1 | prefetch A1(t) | stage B1(t+2)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) a1[ks][mb] = frag<AK>(bufp + R_A1 * kRegion, wr * 64 + mb * 16, ks, lane);
    PHASE_MFMA(b1, a0, 0, 2, (ST || P + 1 <= lv), t + 2, R_B1)
    if constexpr (ST) wait_vm<12>(), barrier(); else wait_end(P + 1);
    // ---- phase 2: A1 x B1 | prefetch A0(t+1) | stage A1(t+2)
    if (more) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) a0[ks][mb] = frag<AK>(nxtp + R_A0 * kRegion, wr * 64 + mb * 16, ks, lane);
    }
    PHASE_MFMA(b1, a1, 4, 2, (ST || P + 2 <= lv), t + 2, R_A1)
    if constexpr (ST) wait_vm<12>(), barrier(); else wait_end(P + 2);
    // ---- phase 3: A1 x B0 | prefetch B0(t+1) | stage A0(t+3)
    s16x8 b0n[2][2];
    if (more) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) b0n[ks][nb] = frag<BKM>(nxtp + R_B0 * kRegion, wc * 32 + nb * 16, ks, lane);
    }
    PHASE_MFMA(b0, a1, 4, 0, (ST || P + 3 <= lv), t + 3, R_A0)
    if constexpr (ST) wait_vm<12>(), barrier(); else wait_end(P + 3);
    if (more) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) b0[ks][nb] = b0n[ks][nb];
    }
  };
#undef PHASE_MFMA
#undef MFMA4
  const int nsteady = nk > 3 ? nk - 3 : 0;
  for (int t = 0; t < nsteady; ++t) ktile(t, std::true_type{});
  for (int t = nsteady; t < nk; ++t) ktile(t, std::false_type{});

  store_tile<EPI, OUT_F32>(p, acc, m0, n0, wr, wc, lane, split);
}

// ---------------------------------------------------------------------------
// Ping-pong persistent form (default): the same 256x256 tile, regions,
// loaders, fragment reads and epilogue math, scheduled as two wave GROUPS
// (wr = 0: waves 0-3, wr = 1: waves 4-7; a workgroup's 8 waves land two per
// SIMD, one of each group) that run one barrier apart.  A phase of a wave is a
// READ segment (its fragment ds_reads for this phase + the phase's 2 LDS-DMAs
// + a counted vmcnt) and an MFMA segment (lgkmcnt(0), 16 MFMAs at
// s_setprio 1), each closed by a barrier; with the offset, every barrier
// interval pairs one group's MFMA segment with the other group's read segment
// on each SIMD, so the matrix pipe is fed while the partner issues its LDS
// reads and DMAs (MI355X_MICROARCH.md "Two waves per SIMD"; cdna_hip_
// programming.md §5 "256² 8-phase template").
//
// Fragment reads per phase (quadrants as gemm_kernel): q0 A0 + B0, q1 B1,
// q2 A1, q3 none (A1 and B0 stay in registers).  A region can be restaged two
// phases after its last read (the partner group retires its reads one barrier
// later); staging per phase of K-tile g:  q0 A1(g+1), q1 B1(g+1), q2 A0(g+2),
// q3 B0(g+2), read 6 / 4 / 6 / 5 phases later.  Each read segment ends with the
// wait for the NEXT phase's regions, counted in VMEM operations issued after
// the needed one (q0 -> B1(g): 6, q1 -> A1(g): 10, q3 -> A0/B0(g+1): 8, fewer
// at the end of the stream), and the barrier after it orders every wave's
// wait before any read.
// Every epilogue memory operation is a single-instruction buffer load /
// store: out-of-range rows and columns are dropped by the buffer's range
// check, not by branches.
template <int N>
__device__ __forceinline__ void wait_ops() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  wait_vm<N>();
}
template <int BASE>
__device__ __forceinline__ void wait_ops_rt(int n) {   // vmcnt(n), n in [0, 63]; BASE: the common value
  if (n == BASE) { wait_ops<BASE>(); return; }
  switch (n) {
#define W_(k) case k: wait_ops<k>(); break;
    W_(0) W_(1) W_(2) W_(3) W_(4) W_(5) W_(6) W_(7) W_(8) W_(9) W_(10) W_(11) W_(12) W_(13) W_(14) W_(15)
    W_(16) W_(17) W_(18) W_(19) W_(20) W_(21) W_(22) W_(23) W_(24) W_(25) W_(26) W_(27) W_(28) W_(29) W_(30)
    W_(31) W_(32) W_(33) W_(34) W_(35) W_(36) W_(37) W_(38) W_(39) W_(40) W_(41) W_(42) W_(43) W_(44) W_(45)
    W_(46) W_(47) W_(48) W_(49) W_(50) W_(51) W_(52) W_(53) W_(54) W_(55) W_(56) W_(57) W_(58) W_(59) W_(60)
    W_(61) W_(62)
#undef W_
    default: wait_ops<0>(); break;
  }
}
__device__ __forceinline__ void sbar() {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#endif
}

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
constexpr uint32_t kOOB = 0xFFFFFFF0u;   // a buffer offset past every range: the access is dropped / reads 0

__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

template <int EPI>
__device__ __forceinline__ void load_bias(const GemmParams& p, int n0, int wc, int lane, f32x4 (&bias)[4]) {
  if constexpr ((EPI & MTTS_GEMM_EPI_BIAS) != 0) {
    const int cl = 4 * (lane >> 4);
    const int es = p.bias_bf16 ? 2 : 4;
    const __amdgpu_buffer_rsrc_t r = brsrc(p.bias, (uint32_t)p.n * es);
#pragma unroll
    for (int NB = 0; NB < 4; ++NB) {
      const int col = n0 + wc * 64 + NB * 16 + cl;
      const uint32_t off = col < p.n ? (uint32_t)col * es : kOOB;
      if (p.bias_bf16) {
        const i32x2 raw = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
        bias[NB] = f32x4{__uint_as_float((uint32_t)raw.x << 16), __uint_as_float((uint32_t)raw.x & 0xffff0000u),
                         __uint_as_float((uint32_t)raw.y << 16), __uint_as_float((uint32_t)raw.y & 0xffff0000u)};
      } else {
        bias[NB] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
      }
    }
  }
}

// store_tile with buffer stores (beta == 0 for fp32 out): the same VMEM
// instructions whatever the bounds
template <int EPI, bool OUT_F32>
__device__ __forceinline__ void store_tile_buf(const GemmParams& p, f32x4 (&acc)[8][4], const f32x4 (&bias)[4],
                                               int m0, int n0, int wr, int wc, int lane, int split) {
  const int rl = lane & 15, cl = 4 * (lane >> 4);
  if constexpr (OUT_F32) {
    const __amdgpu_buffer_rsrc_t r = brsrc((const float*)p.c + (int64_t)split * p.split_stride,
                                           (uint32_t)((int64_t)p.m * p.ldc * 4));
    const bool acc_old = p.beta != 0.f;   // uniform: C = beta C + A B (splits == 1 only)
#pragma unroll
    for (int MB = 0; MB < 8; ++MB) {
      const int row = m0 + wr * 128 + MB * 16 + rl;
      f32x4 old[4];
      if (acc_old) {
#pragma unroll
        for (int NB = 0; NB < 4; ++NB) {
          const int col = n0 + wc * 64 + NB * 16 + cl;
          const uint32_t off = (row < p.m && col < p.n) ? (uint32_t)((row * p.ldc + col) * 4) : kOOB;
          old[NB] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
        }
      }
#pragma unroll
      for (int NB = 0; NB < 4; ++NB) {
        const int col = n0 + wc * 64 + NB * 16 + cl;
        const uint32_t off = (row < p.m && col < p.n) ? (uint32_t)((row * p.ldc + col) * 4) : kOOB;
        f32x4 v = acc[MB][NB];
        if (acc_old) v += p.beta * old[NB];
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, v), r, off, 0, 0);
      }
    }
  } else {
    const int g = lane >> 4;
    const int cw0 = n0 + wc * 64 + (g & 1) * 16 + 8 * (g >> 1);
    const __amdgpu_buffer_rsrc_t rc = brsrc(p.c, (uint32_t)((int64_t)p.m * p.ldc * 2));
    const __amdgpu_buffer_rsrc_t ra = brsrc(p.aux, (uint32_t)((int64_t)p.m * p.ld_aux * 2));
#pragma unroll
    for (int MB = 0; MB < 8; ++MB) {
      const int row = m0 + wr * 128 + MB * 16 + rl;
      const bool rok = row < p.m;
      uint32_t o2[4][2], h2[4][2];
      i32x2 auxv[4];
      if constexpr ((EPI & MTTS_GEMM_EPI_DGELU) != 0) {
#pragma unroll
        for (int NB = 0; NB < 4; ++NB) {
          const int col = n0 + wc * 64 + NB * 16 + cl;
          const uint32_t off = (rok && col < p.n) ? (uint32_t)((row * p.ld_aux + col) * 2) : kOOB;
          auxv[NB] = __builtin_amdgcn_raw_buffer_load_b64(ra, off, 0, 0);
        }
      }
#pragma unroll
      for (int NB = 0; NB < 4; ++NB) {
        f32x4 v = acc[MB][NB];
        if constexpr ((EPI & MTTS_GEMM_EPI_BIAS) != 0) v += bias[NB];
        bf16_t o[4];
        if constexpr ((EPI & MTTS_GEMM_EPI_GELU) != 0) {
          bf16_t hpre[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) hpre[j] = f2bf(v[j]);
#pragma unroll
          for (int j = 0; j < 4; j += 2) {
            const f32x2 g = gelu_f2(f32x2{bf2f(hpre[j]), bf2f(hpre[j + 1])});
            o[j] = f2bf(g[0]);
            o[j + 1] = f2bf(g[1]);
          }
          h2[NB][0] = hpre[0] | ((uint32_t)hpre[1] << 16);
          h2[NB][1] = hpre[2] | ((uint32_t)hpre[3] << 16);
        } else if constexpr ((EPI & MTTS_GEMM_EPI_DGELU) != 0) {
          const uint32_t x = (uint32_t)auxv[NB].x, y = (uint32_t)auxv[NB].y;
          const float h[4] = {__uint_as_float(x << 16), __uint_as_float(x & 0xffff0000u), __uint_as_float(y << 16),
                              __uint_as_float(y & 0xffff0000u)};
#pragma unroll
          for (int j = 0; j < 4; j += 2) {
            const f32x2 gg = gelu_grad_f2(f32x2{h[j], h[j + 1]});
            o[j] = f2bf(bf2f(f2bf(v[j])) * gg[0]);
            o[j + 1] = f2bf(bf2f(f2bf(v[j + 1])) * gg[1]);
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = f2bf(v[j]);
        }
        o2[NB][0] = o[0] | ((uint32_t)o[1] << 16);
        o2[NB][1] = o[2] | ((uint32_t)o[3] << 16);
      }
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        uint32_t w[4];
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const auto r = __builtin_amdgcn_permlane16_swap(o2[2 * pr][d], o2[2 * pr + 1][d], false, false);
          w[d] = r[0];
          w[2 + d] = r[1];
        }
        const int cw = cw0 + pr * 32;
        const bool ok = rok && cw < p.n;   // n % 8 == 0: a lane's 8 columns are all in or all out
        __builtin_amdgcn_raw_buffer_store_b128(i32x4{(int)w[0], (int)w[1], (int)w[2], (int)w[3]}, rc,
                                               ok ? (uint32_t)((row * p.ldc + cw) * 2) : kOOB, 0, 0);
        if constexpr ((EPI & MTTS_GEMM_EPI_GELU) != 0) {
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            const auto r = __builtin_amdgcn_permlane16_swap(h2[2 * pr][d], h2[2 * pr + 1][d], false, false);
            w[d] = r[0];
            w[2 + d] = r[1];
          }
          __builtin_amdgcn_raw_buffer_store_b128(i32x4{(int)w[0], (int)w[1], (int)w[2], (int)w[3]}, ra,
                                                 ok ? (uint32_t)((row * p.ld_aux + cw) * 2) : kOOB, 0, 0);
        }
      }
    }
  }
}

struct WorkItem {
  int m0, n0, split;
};
__device__ __forceinline__ WorkItem work_item(const GemmParams& p, int id) {
  const int tiles = p.tiles_m * p.tiles_n;
  const int split = id / tiles;
  const int tile = id % tiles;
  const int gsz = p.group * p.tiles_n;
  const int g0 = (tile / gsz) * p.group;
  const int gr = min(p.group, p.tiles_m - g0);
  const int tm = g0 + (tile % gsz) % gr, tn = (tile % gsz) / gr;
  return WorkItem{tm * kTile, tn * kTile, split};
}

// per-thread LDS-DMA source offsets of one operand, recomputed per tile from
// the tile origin (row0) and kept relative to the K-tile origin pointer
template <bool KMAJ, bool IS_A>
struct PLoader {
  uint32_t fixed[2];   // [dma i]: k-major: chunk byte offset; m/n-major: k-row byte offset
  int rm[2][2];        // [sub s][dma i]: region-local row / column -> tile row / column
  __device__ void init(int tid, int64_t ld) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if constexpr (KMAJ) {
        const int rr = i * 64 + (tid >> 3), pp = tid & 7;
        fixed[i] = (uint32_t)(((pp ^ ((rr >> 1) & 7)) * 8) * 2);
#pragma unroll
        for (int s = 0; s < 2; ++s) rm[s][i] = rmap<IS_A>(rr, s);
      } else {
        const int kr = i * 32 + (tid >> 4), pp = tid & 15;
        const int f = (kr & 3) | (((kr >> 3) & 1) << 2);
        const int c = pp ^ (f << 1);
        fixed[i] = (uint32_t)(kr * ld * 2);
#pragma unroll
        for (int s = 0; s < 2; ++s) rm[s][i] = rmap<IS_A>(c * 8, s);
      }
    }
  }
  __device__ __forceinline__ uint32_t off(int row0, int nrows, int64_t ld, int s, int i) const {
    if constexpr (KMAJ) {
      int row = row0 + rm[s][i];
      row = row < nrows ? row : nrows - 1;
      return (uint32_t)(row * ld * 2) + fixed[i];
    } else {
      int col = row0 + rm[s][i];
      col = col + 8 <= nrows ? col : ((nrows - 8) & ~7);
      return fixed[i] + (uint32_t)col * 2;
    }
  }
};

// XCD-aware work order: the ids one XCD holds at a time are consecutive
__device__ __forceinline__ int xcd_work_id() {
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
}

// the ping-pong tile of work item `wid` of problem `p` (the kernels below)
template <bool AK, bool BKM, int EPI, bool OUT_F32>
__device__ __forceinline__ void gemm_pp_body(const GemmParams& p, const int wid) {
  __shared__ __attribute__((aligned(16))) char lds[kLds];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int nk = p.k / kBK;
  const int G = nk;                                                  // K-tiles of the item

  PLoader<AK, true> la;
  PLoader<BKM, false> lb;
  la.init(tid, p.lda);
  lb.init(tid, p.ldb);
  const int64_t astep = AK ? kBK * 2 : kBK * p.lda * 2;   // bytes per K-tile
  const int64_t bstep = BKM ? kBK * 2 : kBK * p.ldb * 2;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds;

  // the item's K-tile-0 operand origins (wave-uniform) and 8 per-thread DMA
  // offsets (A0/A1 x 2, B0/B1 x 2), made once: a DMA's address register is
  // never recomputed right behind the DMA that reads it.  (A persistent form
  // looping over items, the next item's K-tiles staged into the current
  // item's tail, measured 0-7 % slower and was removed in round 4.)
  struct Src {
    const char* a;
    const char* b;
    uint32_t o[8];
  };
  auto source = [&](const WorkItem& it, Src& sr) {
    const int64_t k0 = (int64_t)it.split * p.k;
    sr.a = (const char*)(AK ? p.a + k0 : p.a + k0 * p.lda);
    sr.b = (const char*)(BKM ? p.b + k0 : p.b + k0 * p.ldb);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        sr.o[s * 2 + i] = la.off(it.m0, p.m, p.lda, s, i);
        sr.o[4 + s * 2 + i] = lb.off(it.n0, p.n, p.ldb, s, i);
      }
  };
  const WorkItem cur = work_item(p, wid);
  Src scur;
  source(cur, scur);
  auto stage = [&](int kt, int r) {
    const uint32_t reg = lds0 + (kt & 1) * kBuf + r * kRegion;
    const int oi = (r == R_A0 ? 0 : r == R_A1 ? 2 : r == R_B0 ? 4 : 6);
    const bool isa = r == R_A0 || r == R_A1;
    const char* base = isa ? scur.a + kt * astep : scur.b + kt * bstep;
    glds16(base, scur.o[oi], reg + wave * 1024);
    glds16(base, scur.o[oi + 1], reg + 8192 + wave * 1024);
  };

  f32x4 bias[4] = {};
  load_bias<EPI>(p, cur.n0, wc, lane, bias);   // older than every DMA: outside the counts

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: all of K-tile 0, A0 / B0 of K-tile 1
  stage(0, R_A0); stage(0, R_B0); stage(0, R_B1); stage(0, R_A1);
  if (G > 1) { stage(1, R_A0); stage(1, R_B0); }
  if (G > 1) wait_ops<8>(); else wait_ops<4>();   // A0(0), B0(0) landed
  sbar();
  if (wr == 1) sbar();   // group 1 runs one barrier behind

  const char* lbase = lds;
  s16x8 af[2][4], b0f[2][2], b1f[2][2];   // [ks][block]
#define PP_MFMA(BF, MO, NO)                                                                   \
  __builtin_amdgcn_sched_barrier(0);                                                        \
  __builtin_amdgcn_s_waitcnt(0xC07F);                                                        \
  __builtin_amdgcn_sched_barrier(0);                                                        \
  __builtin_amdgcn_s_setprio(1);                                                            \
  _Pragma("unroll") for (int ks_ = 0; ks_ < 2; ++ks_)                                        \
  _Pragma("unroll") for (int mb_ = 0; mb_ < 4; ++mb_)                                        \
  _Pragma("unroll") for (int nb_ = 0; nb_ < 2; ++nb_)                                        \
      acc[(MO) + mb_][(NO) + nb_] = mfma(BF[ks_][nb_], af[ks_][mb_], acc[(MO) + mb_][(NO) + nb_]); \
  __builtin_amdgcn_s_setprio(0);                                                            \
  __builtin_amdgcn_sched_barrier(0);                                                        \
  sbar();
  // Wait counts (VMEM ops younger than the needed region): steady 6 / 10 / 8;
  // the first K-tile 8 / 8 / 8; the last two fewer.  One uniform branch per wait.
  for (int g = 0; g < G; ++g) {
    const bool steady = g > 0 && g + 2 < G;
    const bool n1 = g + 1 < G, n2 = g + 2 < G;
    const char* bufp = lbase + (g & 1) * kBuf;
    // ---- q0: A0 x B0 | stage A1(g+1) | wait B1(g)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) b0f[ks][nb] = frag<BKM>(bufp + R_B0 * kRegion, wc * 32 + nb * 16, ks, lane);
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) af[ks][mb] = frag<AK>(bufp + R_A0 * kRegion, wr * 64 + mb * 16, ks, lane);
    }
    if (n1) stage(g + 1, R_A1);
    if (steady) wait_ops<6>();
    else wait_ops_rt<6>(g == 0 ? (n1 ? 8 : 2) : (n1 ? 6 : 0));
    sbar();
    PP_MFMA(b0f, 0, 0)
    // ---- q1: A0 x B1 | stage B1(g+1) | wait A1(g)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) b1f[ks][nb] = frag<BKM>(bufp + R_B1 * kRegion, wc * 32 + nb * 16, ks, lane);
    if (n1) stage(g + 1, R_B1);
    if (steady) wait_ops<10>();
    else wait_ops_rt<10>(g == 0 ? (n1 ? 8 : 0) : (n1 ? 10 : 2));
    sbar();
    PP_MFMA(b1f, 0, 2)
    // ---- q2: A1 x B1 | stage A0(g+2)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) af[ks][mb] = frag<AK>(bufp + R_A1 * kRegion, wr * 64 + mb * 16, ks, lane);
    if (n2) stage(g + 2, R_A0);
    sbar();
    PP_MFMA(b1f, 4, 2)
    // ---- q3: A1 x B0 | stage B0(g+2) | wait A0 / B0(g+1)
    if (n2) stage(g + 2, R_B0);
    if (steady) wait_ops<8>();
    else if (n1) wait_ops_rt<8>((n2 ? 8 : 4));
    sbar();
    PP_MFMA(b0f, 4, 0)
  }
#undef PP_MFMA
  if (wr == 0) sbar();   // the same barrier count for both groups
  store_tile_buf<EPI, OUT_F32>(p, acc, bias, cur.m0, cur.n0, wr, wc, lane, cur.split);
}

template <bool AK, bool BKM, int EPI, bool OUT_F32>
__global__ __launch_bounds__(kThreads, 1) void gemm_pp_kernel(GemmParams p) {
  gemm_pp_body<AK, BKM, EPI, OUT_F32>(p, xcd_work_id());
}

// Grouped weight gradients (round 5): up to kGroupMax TN problems in ONE
// launch, each tile over the problem's WHOLE K (no split-K slabs, no
// split_reduce pass).  The host orders the problems longest-K first; tiles of
// a problem are consecutive work ids (an XCD walks one problem's tiles).
constexpr int kGroupMax = 24;   // 24 x 128-byte problems: kernel arguments stay under 4 KiB
struct GroupParams {
  GemmParams p[kGroupMax];
  int tile_end[kGroupMax];   // exclusive prefix sums of the problems' tile counts
  int n;
};

template <bool AK, bool BKM, int EPI, bool OUT_F32>
__global__ __launch_bounds__(kThreads, 1) void gemm_pp_grouped_kernel(const GroupParams G) {
  const int wid = xcd_work_id();
  int i = 0, t0 = 0;
#pragma unroll
  for (int j = 0; j + 1 < kGroupMax; ++j)
    if (j + 1 < G.n && wid >= G.tile_end[j]) { i = j + 1; t0 = G.tile_end[j]; }
  // static indices only (a dynamic index into the kernel-argument struct
  // would copy it to scratch)
  GemmParams q = G.p[0];
#pragma unroll
  for (int j = 1; j < kGroupMax; ++j)
    if (i == j) q = G.p[j];
  gemm_pp_body<AK, BKM, EPI, OUT_F32>(q, wid - t0);
}

// ---------------------------------------------------------------------------
// Four-wave form (round 5, NT): the same 256x256 output tile on 4 waves
// (2 M x 2 N, one per SIMD), 128x128 per wave (8x8 16x16 accumulator blocks,
// 256 registers), so a 32-deep K-step reads 8 A + 8 B fragments for 64 MFMAs:
// 0.25 fragment reads per MFMA against the 8-wave tile's 0.375.
//  * K-steps of 32 go by LDS-DMA into a ring of 4 stages of 32 KiB (A then B,
//    16 row-blocks of 16 rows x 64 B each); a wave stages row-blocks
//    4w..4w+3 of A and of B, one DMA per MFMA group.
//  * one barrier per K-step.  Top of step g: this wave's DMAs of step g+1
//    retired (counted vmcnt) and its fragment reads of step g retired
//    (lgkmcnt 0), barrier -> every wave's DMAs of g+1 have landed and every
//    read of step g's stage is done; then step g+4 is staged into step g's
//    stage and step g+1's fragments are read between step g's 64 MFMAs.
//  * bank swizzle of a row-block (16 rows of 4 16-B chunks): chunk c of row r
//    at slot 4r + (c ^ (-(r>>2) & 3)), written by the DMA's source address;
//    each ds_read_b128 lane group (rows 0-3 and 12-15 at chunk c, rows 4-11
//    at chunk c^1) then covers 16 distinct 16-B slots.
constexpr int kW4Threads = 256;
constexpr int kW4BK = 32;
constexpr int kW4Stages = 4;
constexpr int kW4Stage = 32768;

__device__ __forceinline__ int w4_slot(int r, int c) { return 4 * r + (c ^ (-(r >> 2) & 3)); }

template <int EPI>
__global__ __launch_bounds__(kW4Threads, 1) void gemm_w4_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) char lds[kW4Stages * kW4Stage];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int nk = p.k / kW4BK;
  const WorkItem it = work_item(p, xcd_work_id());
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds;

  // DMA source offsets: lane -> (row r, chunk c) of the slot 16*lane it writes
  uint32_t oa[4], ob[4];
  {
    const int r = lane >> 2;
    const int c = (lane & 3) ^ (-(r >> 2) & 3);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int row = it.m0 + (4 * wave + i) * 16 + r;
      row = row < p.m ? row : p.m - 1;
      oa[i] = (uint32_t)((int64_t)row * p.lda * 2) + c * 16;
      int col = it.n0 + (4 * wave + i) * 16 + r;
      col = col < p.n ? col : p.n - 1;
      ob[i] = (uint32_t)((int64_t)col * p.ldb * 2) + c * 16;
    }
  }
  const char* abase = (const char*)p.a;
  const char* bbase = (const char*)p.b;
  auto stage1 = [&](int g, int slot, int j) {   // DMA j (0-3: A block, 4-7: B block) of K-step g
    const uint32_t st = lds0 + slot * kW4Stage + wave * 4096;
    if (j < 4) glds16(abase + g * (kW4BK * 2), oa[j & 3], st + (j & 3) * 1024);
    else glds16(bbase + g * (kW4BK * 2), ob[j & 3], st + 16384 + (j & 3) * 1024);
  };
  // fragment addresses: one VGPR per operand, the block offset an immediate
  const char* fra = lds + wr * 8192 + w4_slot(lane & 15, lane >> 4) * 16;
  const char* frb = fra - wr * 8192 + 16384 + wc * 8192;
  auto fa = [&](int g, int mb) -> s16x8 { return *(const lds_s16x8*)(fra + (g & 3) * kW4Stage + mb * 1024); };
  auto fb = [&](int g, int nb) -> s16x8 { return *(const lds_s16x8*)(frb + (g & 3) * kW4Stage + nb * 1024); };

  f32x4 acc[2][8][4];   // [column half][16-row block][16-column block]
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[h][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int g = 0; g < kW4Stages; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j) stage1(g < nk ? g : nk - 1, g, j);
  wait_ops<24>();   // K-step 0 landed
  sbar();
  // A fragment j is dead after MFMA group j and is reloaded there with the
  // next K-step's; the B fragments serve every group: double-buffered
  s16x8 fA[8], fB[2][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    fA[j] = fa(0, j);
    fB[0][j] = fb(0, j);
  }

  // One uniform step (no tail code: a separate tail made the register
  // allocator shuttle the 256 accumulators between register files): K-step
  // g+4 is staged as min(g+4, nk-1) (the last steps re-stage K-step nk-1
  // into slots already consumed) and the next step's fragments are always
  // read (past the end: stale slots, never used), so every step issues 8
  // DMAs and waits with the same count; the loop ends with vmcnt(0).
  auto step = [&](int g, auto cur_c) {
    constexpr int CUR = decltype(cur_c)::value;
    wait_ops<16>();   // K-step g+1 landed (g+2, g+3 in flight)
    barrier();        // lgkmcnt(0) + s_barrier
    const int gs = g + 4 < nk ? g + 4 : nk - 1;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      __builtin_amdgcn_sched_barrier(0);
      stage1(gs, (g + 4) & 3, j);
#pragma unroll
      for (int nb = 0; nb < 8; ++nb)
        acc[nb >> 2][j][nb & 3] = mfma(fB[CUR][nb], fA[j], acc[nb >> 2][j][nb & 3]);
      fA[j] = fa(g + 1, j);
      fB[1 - CUR][j] = fb(g + 1, j);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int g = 0; g < nk; g += 2) {   // nk is even (K % 64 == 0)
    step(g, std::integral_constant<int, 0>{});
    step(g + 1, std::integral_constant<int, 1>{});
  }
  wait_ops<0>();   // the re-staged DMAs: none may land after the workgroup ends
  // pin the accumulators to the accumulator file across the loop exit (the
  // bias / GELU epilogues otherwise lead the allocator to shuttle them
  // between register files inside the loop)
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" : "+a"(acc[h][i][j]));
#pragma unroll
  for (int h = 0; h < 2; ++h) {   // every DMA retired: the bias loads are the only VMEM in flight
    f32x4 bias[4] = {};
    load_bias<EPI>(p, it.n0, 2 * wc + h, lane, bias);
    store_tile_buf<EPI, false>(p, acc[h], bias, it.m0, it.n0, wr, 2 * wc + h, lane, 0);
  }
}

// out[i] = beta*out[i] + sum_s slab[s][i] (fixed order); rows x cols with row strides
__global__ __launch_bounds__(256) void split_reduce_kernel(const float* __restrict__ slabs, int64_t sstride, int splits,
                                                           int rows, int cols, int64_t lds_, float* out, int64_t ldo,
                                                           float beta) {
  const int c4 = cols / 4;
  const int64_t total = (int64_t)rows * c4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / c4), c = (int)(i % c4) * 4;
    f32x4 s = *(const f32x4*)(slabs + (int64_t)r * lds_ + c);
    for (int k = 1; k < splits; ++k) s += *(const f32x4*)(slabs + k * sstride + (int64_t)r * lds_ + c);
    float* op = out + (int64_t)r * ldo + c;
    if (beta != 0.f) s += beta * *(const f32x4*)op;
    *(f32x4*)op = s;
  }
}

// Ping-pong kernel, one tile per workgroup (tools/gemm_pp_ab.py, C2 shapes,
// same box: 1078-1339 TF/s NT, 696-1110 TN vs 997-1321 / 684-1128 for the
// round-2 single-group kernel, which remains the fallback for 8-byte-aligned
// outputs, C / aux spans past 2 GiB and beta accumulate with split-K).
template <bool AK, bool BKM, int EPI, bool F32>
void launch(const GemmParams& p, int nwg, hipStream_t st) {
  // the ping-pong epilogue stores 16-byte bf16 pieces (wide_out) and
  // addresses C / aux / each slab with 31-bit buffer offsets
  const int64_t cbytes = F32 ? (int64_t)p.m * p.ldc * 4 : (int64_t)p.m * p.ldc * 2;
  const int64_t abytes = (EPI & (MTTS_GEMM_EPI_GELU | MTTS_GEMM_EPI_DGELU)) ? (int64_t)p.m * p.ld_aux * 2 : 0;
  const bool pp_ok = (F32 || p.wide_out) && cbytes < (1ll << 31) && abytes < (1ll << 31) &&
                     (!F32 || p.beta == 0.f || p.splits == 1) && override_of(MTTS_OVR_GEMM_NARROW) != 1;
  if (!pp_ok) {
    hipLaunchKernelGGL((gemm_kernel<AK, BKM, EPI, F32>), dim3(nwg), dim3(kThreads), 0, st, p);
    return;
  }
  if constexpr (AK && BKM && !F32) {
    if (override_of(MTTS_OVR_GEMM_TILE) == 2) {
      hipLaunchKernelGGL((gemm_w4_kernel<EPI>), dim3(nwg), dim3(kW4Threads), 0, st, p);
      return;
    }
  }
  hipLaunchKernelGGL((gemm_pp_kernel<AK, BKM, EPI, F32>), dim3(nwg), dim3(kThreads), 0, st, p);
}

}  // namespace
}  // namespace mtts

using namespace mtts;

extern "C" int64_t mtts_gemm_workspace(const MttsGemmArgs* a) {
  if (!a || a->layout != MTTS_GEMM_TN || a->splits <= 1) return 0;
  return (int64_t)a->splits * a->m * a->n * 4;
}

extern "C" int mtts_gemm(const MttsGemmArgs* a, void* stream) {
  MTTS_CHECK(a && a->a && a->b && a->c, "gemm: null pointer");
  const int M = a->m, N = a->n, K = a->k;
  MTTS_CHECK(M > 0 && N > 0 && K > 0, "gemm: m=%d n=%d k=%d must be positive", M, N, K);
  MTTS_CHECK(a->layout == MTTS_GEMM_NT || a->layout == MTTS_GEMM_TN, "gemm: layout must be NT (0) or TN (1)");
  const bool nt = a->layout == MTTS_GEMM_NT;
  const int splits = a->splits > 0 ? a->splits : 1;
  MTTS_CHECK(K % (kBK * splits) == 0, "gemm: k=%d must be a multiple of 64*splits (splits=%d)", K, splits);
  MTTS_CHECK(N % 8 == 0, "gemm: n=%d must be a multiple of 8", N);
  MTTS_CHECK(nt || M % 8 == 0, "gemm: TN needs m=%d a multiple of 8", M);
  MTTS_CHECK(((uintptr_t)a->a | (uintptr_t)a->b) % 16 == 0 && a->lda % 8 == 0 && a->ldb % 8 == 0,
             "gemm: A / B must be 16-byte aligned with row strides a multiple of 8 elements");
  MTTS_CHECK(a->ldc % 4 == 0 && (uintptr_t)a->c % 16 == 0, "gemm: C must be 16-byte aligned, ldc a multiple of 4");
  MTTS_CHECK(nt ? (a->lda >= K && a->ldb >= K) : (a->lda >= M && a->ldb >= N), "gemm: leading dimension too small");
  // 32-bit DMA offsets from the K-tile origin
  const int64_t aspan = nt ? (int64_t)(M - 1) * a->lda + K : (int64_t)(kBK - 1) * a->lda + M;
  const int64_t bspan = nt ? (int64_t)(N - 1) * a->ldb + K : (int64_t)(kBK - 1) * a->ldb + N;
  MTTS_CHECK(aspan * 2 < (1ll << 32) && bspan * 2 < (1ll << 32), "gemm: operand span exceeds 4 GiB");
  const int epi = a->epilogue;
  const bool f32out = a->out_dtype == 0;
  MTTS_CHECK(a->out_dtype == 0 || a->out_dtype == 1, "gemm: out_dtype must be 0 (f32) or 1 (bf16)");
  MTTS_CHECK(!f32out || epi == 0, "gemm: epilogues apply to bf16 output only");
  MTTS_CHECK(f32out || splits == 1, "gemm: split-K needs fp32 output");
  MTTS_CHECK(!(epi & MTTS_GEMM_EPI_BIAS) || a->bias, "gemm: bias epilogue without bias");
  // the epilogue reads the bias as f32x4 (fp32) / uint2 (bf16) and aux as uint2 / uint4
  MTTS_CHECK(!(epi & MTTS_GEMM_EPI_BIAS) || (uintptr_t)a->bias % (a->bias_dtype == 1 ? 8 : 16) == 0,
             "gemm: bias must be %d-byte aligned", a->bias_dtype == 1 ? 8 : 16);
  MTTS_CHECK(!(epi & (MTTS_GEMM_EPI_GELU | MTTS_GEMM_EPI_DGELU)) || (uintptr_t)a->aux % 8 == 0,
             "gemm: aux must be 8-byte aligned");
  MTTS_CHECK(!(epi & (MTTS_GEMM_EPI_GELU | MTTS_GEMM_EPI_DGELU)) || (a->aux && a->ld_aux % 4 == 0),
             "gemm: GELU epilogues need aux (ld_aux multiple of 4)");
  MTTS_CHECK((epi & (MTTS_GEMM_EPI_GELU | MTTS_GEMM_EPI_DGELU)) != (MTTS_GEMM_EPI_GELU | MTTS_GEMM_EPI_DGELU),
             "gemm: GELU and DGELU are exclusive");
  MTTS_CHECK(nt || (epi == 0 && f32out), "gemm: TN (weight gradient) runs fp32 out, no epilogue");
  MTTS_CHECK(splits == 1 || a->workspace, "gemm: split-K needs the workspace (mtts_gemm_workspace bytes)");

  GemmParams p{};
  p.a = (const bf16_t*)a->a; p.b = (const bf16_t*)a->b;
  p.bias = a->bias; p.aux = a->aux; p.bias_bf16 = a->bias_dtype == 1;
  p.lda = a->lda; p.ldb = a->ldb; p.ld_aux = a->ld_aux;
  p.m = M; p.n = N; p.k = K / splits;
  p.tiles_m = (M + kTile - 1) / kTile; p.tiles_n = (N + kTile - 1) / kTile;
  p.splits = splits; p.epi = epi;
  p.group = std::min(p.tiles_m, 4);
  if (splits > 1) {
    p.c = a->workspace; p.ldc = N; p.split_stride = (int64_t)M * N; p.beta = 0.f;
  } else {
    p.c = a->c; p.ldc = a->ldc; p.split_stride = 0; p.beta = a->beta;
  }
  p.wide_out = !f32out && a->ldc % 8 == 0 && (!(epi & (MTTS_GEMM_EPI_GELU | MTTS_GEMM_EPI_DGELU)) || a->ld_aux % 8 == 0) &&
               (!a->aux || (uintptr_t)a->aux % 16 == 0) && override_of(MTTS_OVR_GEMM_NARROW) != 1;
  const int nwg = p.tiles_m * p.tiles_n * splits;
  hipStream_t st = (hipStream_t)stream;
  if (!nt) {
    launch<false, false, 0, true>(p, nwg, st);
  } else if (f32out) {
    launch<true, true, 0, true>(p, nwg, st);
  } else {
    switch (epi) {
      case 0: launch<true, true, 0, false>(p, nwg, st); break;
      case MTTS_GEMM_EPI_BIAS: launch<true, true, MTTS_GEMM_EPI_BIAS, false>(p, nwg, st); break;
      case MTTS_GEMM_EPI_GELU: launch<true, true, MTTS_GEMM_EPI_GELU, false>(p, nwg, st); break;
      case MTTS_GEMM_EPI_BIAS | MTTS_GEMM_EPI_GELU:
        launch<true, true, MTTS_GEMM_EPI_BIAS | MTTS_GEMM_EPI_GELU, false>(p, nwg, st); break;
      case MTTS_GEMM_EPI_DGELU: launch<true, true, MTTS_GEMM_EPI_DGELU, false>(p, nwg, st); break;
      default: MTTS_CHECK(false, "gemm: unsupported epilogue combination %d", epi);
    }
  }
  MTTS_LAUNCH_CHECK("gemm");
  if (splits > 1) {
    const int64_t total = (int64_t)M * (N / 4);
    const int blocks = (int)std::min<int64_t>((total + 255) / 256, 2048);
    hipLaunchKernelGGL(split_reduce_kernel, dim3(blocks), dim3(256), 0, st, (const float*)a->workspace,
                       (int64_t)M * N, splits, M, N, (int64_t)N, (float*)a->c, a->ldc, a->beta);
    MTTS_LAUNCH_CHECK("gemm split reduce");
  }
  return MTTS_OK;
}

extern "C" int mtts_gemm_grouped(const MttsGemmArgs* probs, int n, void* stream) {
  using namespace mtts;
  MTTS_CHECK(probs && n >= 1 && n <= kGroupMax, "gemm_grouped: 1 <= n <= %d problems", kGroupMax);
  GroupParams G{};
  int tiles = 0;
  for (int i = 0; i < n; ++i) {
    const MttsGemmArgs* a = probs + i;
    MTTS_CHECK(a->a && a->b && a->c, "gemm_grouped[%d]: null pointer", i);
    const int M = a->m, N = a->n, K = a->k;
    MTTS_CHECK(a->layout == MTTS_GEMM_TN && a->out_dtype == 0 && a->epilogue == 0 && a->splits <= 1,
               "gemm_grouped[%d]: TN, fp32 out, no epilogue, no split-K only", i);
    MTTS_CHECK(M > 0 && N > 0 && K > 0 && K % kBK == 0, "gemm_grouped[%d]: m=%d n=%d k=%d (k %% 64 == 0)", i, M, N, K);
    MTTS_CHECK(N % 8 == 0 && M % 8 == 0, "gemm_grouped[%d]: m, n must be multiples of 8", i);
    MTTS_CHECK(((uintptr_t)a->a | (uintptr_t)a->b) % 16 == 0 && a->lda % 8 == 0 && a->ldb % 8 == 0 &&
               a->lda >= M && a->ldb >= N, "gemm_grouped[%d]: A / B alignment or leading dimension", i);
    MTTS_CHECK(a->ldc % 4 == 0 && (uintptr_t)a->c % 16 == 0 && a->ldc >= N, "gemm_grouped[%d]: C alignment / ldc", i);
    MTTS_CHECK(a->beta == 0.f || a->beta == 1.f, "gemm_grouped[%d]: beta must be 0 or 1", i);
    MTTS_CHECK((int64_t)(kBK - 1) * a->lda + M < (1ll << 31) && (int64_t)(kBK - 1) * a->ldb + N < (1ll << 31) &&
               (int64_t)M * a->ldc * 4 < (1ll << 31), "gemm_grouped[%d]: operand / C span exceeds the 32-bit offsets", i);
    GemmParams& p = G.p[i];
    p.a = (const bf16_t*)a->a; p.b = (const bf16_t*)a->b; p.c = a->c;
    p.lda = a->lda; p.ldb = a->ldb; p.ldc = a->ldc;
    p.m = M; p.n = N; p.k = K;
    p.tiles_m = (M + kTile - 1) / kTile; p.tiles_n = (N + kTile - 1) / kTile;
    p.splits = 1; p.split_stride = 0; p.beta = a->beta;
    p.group = std::min(p.tiles_m, 4);
    tiles += p.tiles_m * p.tiles_n;
    G.tile_end[i] = tiles;
  }
  G.n = n;
  hipLaunchKernelGGL((gemm_pp_grouped_kernel<false, false, 0, true>), dim3(tiles), dim3(kThreads), 0,
                     (hipStream_t)stream, G);
  MTTS_LAUNCH_CHECK("gemm_grouped");
  return MTTS_OK;
}
