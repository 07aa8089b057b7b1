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
#include "common.h"

namespace mtts {
namespace {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

template <int KS>
__global__ __launch_bounds__(64 * KS) void gemm_rows_kernel(const bf16_t* __restrict__ x, int64_t ldx, int M,
                                                            const bf16_t* __restrict__ W, int64_t ldw, int N, int K,
                                                            const bf16_t* __restrict__ bias, int act,
                                                            bf16_t* __restrict__ y, int64_t ldy) {
  __shared__ float red[KS][32][33];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.x * 32;
  const int kc = K / KS, kb = wave * kc;
  const bool rowok = i < M, colok = n0 + i < N;
  const bf16_t* xr = x + (int64_t)(rowok ? i : 0) * ldx + kb + 8 * h;
  const bf16_t* wr = W + (int64_t)(colok ? n0 + i : 0) * ldw + kb + 8 * h;
  f32x16 acc = {};
  for (int k = 0; k < kc; k += 64) {   // 4 k-steps per trip, all loads issued first
    s16x8 a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a[u] = *reinterpret_cast<const s16x8*>(xr + k + 16 * u);
      b[u] = *reinterpret_cast<const s16x8*>(wr + k + 16 * u);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (!rowok) a[u] = s16x8{};
      if (!colok) b[u] = s16x8{};
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a[u]), __builtin_bit_cast(bf16x8, b[u]),
                                                    acc, 0, 0, 0);
    }
  }
  // acc register r: output row (batch) acc_row(r, h), column n0 + i
#pragma unroll
  for (int r = 0; r < 16; ++r) red[wave][acc_row(r, h)][i] = acc[r];
  __syncthreads();
  for (int e = threadIdx.x; e < 32 * 32; e += 64 * KS) {
    const int row = e >> 5, col = e & 31;
    if (row >= M || n0 + col >= N) continue;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < KS; ++w) s += red[w][row][col];
    if (bias) s += bf2f(bias[n0 + col]);
    if (act == 1) s = 0.5f * s * (1.f + erff(s * 0.70710678118654752f));   // F.gelu (exact erf)
    y[(int64_t)row * ldy + n0 + col] = f2bf(s);
  }
}

}  // namespace
}  // namespace mtts

using namespace mtts;

extern "C" int mtts_gemm_rows_bf16(const void* x, int64_t ldx, int M, const void* W, int64_t ldw, int N, int K,
                                   const void* bias, int act, void* y, int64_t ldy, void* stream) {
  MTTS_CHECK(x && W && y, "gemm_rows: null pointer");
  MTTS_CHECK(M >= 0 && M <= 32 && N > 0 && K > 0, "gemm_rows: M=%d must be in [0, 32], N, K > 0", M);
  MTTS_CHECK(K % 64 == 0, "gemm_rows: K=%d must be a multiple of 64", K);
  MTTS_CHECK(act == 0 || act == 1, "gemm_rows: act must be 0 (none) or 1 (gelu)");
  MTTS_CHECK(((uintptr_t)x | (uintptr_t)W) % 16 == 0 && ldx % 8 == 0 && ldw % 8 == 0,
             "gemm_rows: x / W must be 16-byte aligned with 16-byte row strides");
  if (M == 0) return MTTS_OK;
  hipStream_t st = (hipStream_t)stream;
  const int tiles = (N + 31) / 32;
  // K split: enough waves to stream the weights (>= ~512 in flight), 64-multiple k slice each
  int ks = 1;
  if (K % (64 * 4) == 0) ks = 4;
  if (tiles < 128 && K % (64 * 8) == 0) ks = 8;
  if (tiles < 32 && K % (64 * 16) == 0) ks = 16;
  switch (ks) {
    case 16:
      hipLaunchKernelGGL((gemm_rows_kernel<16>), dim3(tiles), dim3(64 * 16), 0, st, (const bf16_t*)x, ldx, M,
                         (const bf16_t*)W, ldw, N, K, (const bf16_t*)bias, act, (bf16_t*)y, ldy);
      break;
    case 8:
      hipLaunchKernelGGL((gemm_rows_kernel<8>), dim3(tiles), dim3(64 * 8), 0, st, (const bf16_t*)x, ldx, M,
                         (const bf16_t*)W, ldw, N, K, (const bf16_t*)bias, act, (bf16_t*)y, ldy);
      break;
    case 4:
      hipLaunchKernelGGL((gemm_rows_kernel<4>), dim3(tiles), dim3(64 * 4), 0, st, (const bf16_t*)x, ldx, M,
                         (const bf16_t*)W, ldw, N, K, (const bf16_t*)bias, act, (bf16_t*)y, ldy);
      break;
    default:
      hipLaunchKernelGGL((gemm_rows_kernel<1>), dim3(tiles), dim3(64), 0, st, (const bf16_t*)x, ldx, M,
                         (const bf16_t*)W, ldw, N, K, (const bf16_t*)bias, act, (bf16_t*)y, ldy);
      break;
  }
  MTTS_LAUNCH_CHECK("gemm_rows");
  return MTTS_OK;
}
