// Dropout in HIP (training paths of style_cross_attention.py and
// text_encoder.py: nn.Dropout(0.1) after the style / FFT blocks' attention
// output, FFN activation and FFN output -- reference
// /root/reference/style_cross_attention.py:38-46, 100-109, 133, 246-255,
// 278; FastSpeech2's MultiHeadAttention / PositionwiseFeedForward /
// VariancePredictor dropouts behind /root/reference/text_encoder.py:80-85,
// 168).
//
// y = x * keep(i) / (1 - p), keep(i) = hash(seed, i) >= p * 2^32: a
// counter-based mask (no stored mask), so the backward regenerates it from
// the same seed: dx = dy * keep(i) / (1 - p).  The DGELU form fuses the
// GELU backward of the activation the dropout followed (FFN: dropout(gelu(pre))):
// d(pre) = bf16(bf16(dy * keep / (1 - p)) * gelu'(pre)).  The hash is splitmix64's
// finalizer of seed + i * golden, one 64-bit hash per element pair (its two
// 32-bit halves).  HBM-bound: 16-byte loads / stores, 8 (bf16) or 4 (fp32)
// elements per lane, a grid-stride loop over ~2 waves per SIMD.
// x_rep > 1 (round 6): x is broadcast over a middle dimension -- y is
// (outer, x_rep, x_inner) and x (outer, x_inner), read as x[o, c] for y[o, r, c]:
// the single-key attention's value row expanded over the queries and dropped in
// one pass (no materialised (B, Tq, d) copy).
// seed_in (ABI 14): a device int64 added to the scalar seed (the library's
// per-device base, advanced once per training step by a captured add, so a
// replayed hipGraph draws fresh masks); seed_out: the forward records the
// base it used, and the backward reads it back as its seed_in.
#include "common.h"

namespace mtts {
namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// keep bit of mask index j: half (j & 1) of the 64-bit hash of j >> 1
__device__ __forceinline__ bool keep1(uint64_t seed, int64_t j, uint32_t thresh) {
  const uint64_t h = mix64(seed + (uint64_t)(j >> 1) * 0x9E3779B97F4A7C15ull);
  return (uint32_t)(h >> (32 * (j & 1))) >= thresh;
}

// GELU'(x) for the DGELU form: the same exact-erf derivative as the GEMM
// epilogue's gelu_grad_f (gemm.hip), torch's GeluBackward.
__device__ __forceinline__ float gelu_tail(float a) {
  float s = -1.7774024116e-08f;
  const float c[10] = {5.6194854933e-07f, -7.6223902631e-06f, 5.5893204013e-05f, -2.0454518331e-04f,
                       -1.6655060660e-04f, 7.1668288485e-03f, -5.2604280745e-02f, 2.6218665810e-01f,
                       -1.1511125488e+00f, -9.9999981719e-01f};
#pragma unroll
  for (int i = 0; i < 10; ++i) s = fmaf(s, a, c[i]);
  return s;
}
__device__ __forceinline__ float gelu_grad(float x) {
  constexpr float kLog2e = 1.4426950408889634f;
  const float a = fminf(fabsf(x), 5.5f);
  const float m = x * (-0.5f * kLog2e) * x;
  const float e = __builtin_amdgcn_exp2f(m);
  const float h = __builtin_amdgcn_exp2f(m + gelu_tail(a));
  return fmaf(x * 0.3989422804014327f, e, x >= 0.f ? 1.f - h : h);
}

template <typename T, bool DGELU>
__global__ __launch_bounds__(256) void dropout_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                      const bf16_t* __restrict__ pre, int64_t n, uint64_t seed,
                                                      uint32_t thresh, float scale, int group, int x_rep,
                                                      int x_inner, const int64_t* __restrict__ seed_in,
                                                      int64_t* __restrict__ seed_out) {
  constexpr int V = 16 / sizeof(T);   // elements per 16-byte piece
  if (seed_in) {
    const int64_t base = *seed_in;
    if (seed_out && blockIdx.x == 0 && threadIdx.x == 0) *seed_out = base;
    seed += (uint64_t)base;
  }
  const int64_t nv = n / V;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t inner_v = x_inner / V, outer_v = (int64_t)x_rep * inner_v;   // in 16-byte pieces
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
    // source piece: v itself, or x[o, c] for a broadcast x
    const int64_t sv = x_rep > 1 ? (v / outer_v) * inner_v + v % inner_v : v;
    float f[V];
    if constexpr (sizeof(T) == 2) {
      const uint4 r = reinterpret_cast<const uint4*>(x)[sv];
      const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f[2 * q] = __uint_as_float(w[q] << 16);
        f[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
      }
    } else {
      const float4 r = reinterpret_cast<const float4*>(x)[sv];
      f[0] = r.x; f[1] = r.y; f[2] = r.z; f[3] = r.w;
    }
    float g[V];
    if constexpr (DGELU) {
      // pre-activation: bf16, V elements (8 bf16 = 16 B, or 4 bf16 = 8 B)
      if constexpr (V == 8) {
        const uint4 r = reinterpret_cast<const uint4*>(pre)[v];
        const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          g[2 * q] = gelu_grad(__uint_as_float(w[q] << 16));
          g[2 * q + 1] = gelu_grad(__uint_as_float(w[q] & 0xffff0000u));
        }
      } else {
        const uint2 r = reinterpret_cast<const uint2*>(pre)[v];
        const uint32_t w[2] = {r.x, r.y};
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          g[2 * q] = gelu_grad(__uint_as_float(w[q] << 16));
          g[2 * q + 1] = gelu_grad(__uint_as_float(w[q] & 0xffff0000u));
        }
      }
    }
    float o[V];
    if (group == 1) {   // one hash per element pair
#pragma unroll
      for (int q = 0; q < V / 2; ++q) {
        const uint64_t h = mix64(seed + (uint64_t)(v * (V / 2) + q) * 0x9E3779B97F4A7C15ull);
        o[2 * q] = (uint32_t)h >= thresh ? f[2 * q] * scale : 0.f;
        o[2 * q + 1] = (uint32_t)(h >> 32) >= thresh ? f[2 * q + 1] * scale : 0.f;
      }
    } else {            // mask index i / group (group % V == 0: one draw per piece)
      const bool k = keep1(seed, v * V / group, thresh);
#pragma unroll
      for (int q = 0; q < V; ++q) o[q] = k ? f[q] * scale : 0.f;
    }
    if constexpr (sizeof(T) == 2) {
      uint32_t w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float a = o[2 * q], b = o[2 * q + 1];
        if constexpr (DGELU) {   // bf16(bf16(dy * keep * scale) * gelu'(pre)), as dropout then GeluBackward
          a = bf2f(f2bf(a)) * g[2 * q];
          b = bf2f(f2bf(b)) * g[2 * q + 1];
        }
        w[q] = (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
      }
      reinterpret_cast<uint4*>(y)[v] = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
      if constexpr (DGELU) {
#pragma unroll
        for (int q = 0; q < V; ++q) o[q] *= g[q];
      }
      reinterpret_cast<float4*>(y)[v] = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
}

}  // namespace
}  // namespace mtts

using namespace mtts;

extern "C" int mtts_dropout(const MttsDropoutArgs* a, void* stream) {
  MTTS_CHECK(a && a->x && a->y, "dropout: null pointer");
  MTTS_CHECK(a->dtype == MTTS_F32 || a->dtype == MTTS_BF16, "dropout: dtype must be f32 or bf16");
  MTTS_CHECK(a->n >= 0 && a->n % 8 == 0, "dropout: n=%lld must be a non-negative multiple of 8", (long long)a->n);
  MTTS_CHECK(a->p >= 0.f && a->p < 1.f, "dropout: p=%f must be in [0, 1)", (double)a->p);
  MTTS_CHECK(((uintptr_t)a->x | (uintptr_t)a->y) % 16 == 0, "dropout: x / y must be 16-byte aligned");
  MTTS_CHECK(!a->pre || (uintptr_t)a->pre % 16 == 0, "dropout: pre must be 16-byte aligned");
  const int vlen = a->dtype == MTTS_F32 ? 4 : 8;
  const int group = a->group > 0 ? a->group : 1;
  MTTS_CHECK(group == 1 || group % vlen == 0, "dropout: group=%d must be 1 or a multiple of %d", group, vlen);
  const int x_rep = a->x_rep > 1 ? a->x_rep : 1;
  MTTS_CHECK(x_rep == 1 || (a->x_inner > 0 && a->x_inner % vlen == 0 && a->n % ((int64_t)x_rep * a->x_inner) == 0),
             "dropout: x_rep=%d needs x_inner=%d a multiple of %d dividing n / x_rep", x_rep, a->x_inner, vlen);
  MTTS_CHECK(x_rep == 1 || (!a->pre && a->x != a->y), "dropout: a broadcast x takes no pre and is not in place");
  if (a->n == 0) return MTTS_OK;
  const uint32_t thresh = (uint32_t)fmin((double)a->p * 4294967296.0, 4294967295.0);
  const float scale = 1.f / (1.f - a->p);
  const int64_t nv = a->n / (a->dtype == MTTS_F32 ? 4 : 8);
  const int blocks = (int)std::min<int64_t>((nv + 255) / 256, 2048);
  hipStream_t st = (hipStream_t)stream;
  if (a->dtype == MTTS_F32) {
    if (a->pre)
      hipLaunchKernelGGL((dropout_kernel<float, true>), dim3(blocks), dim3(256), 0, st, (const float*)a->x,
                         (float*)a->y, (const bf16_t*)a->pre, a->n, a->seed, thresh, scale, group, x_rep, a->x_inner, a->seed_in, a->seed_out);
    else
      hipLaunchKernelGGL((dropout_kernel<float, false>), dim3(blocks), dim3(256), 0, st, (const float*)a->x,
                         (float*)a->y, nullptr, a->n, a->seed, thresh, scale, group, x_rep, a->x_inner, a->seed_in, a->seed_out);
  } else {
    if (a->pre)
      hipLaunchKernelGGL((dropout_kernel<bf16_t, true>), dim3(blocks), dim3(256), 0, st, (const bf16_t*)a->x,
                         (bf16_t*)a->y, (const bf16_t*)a->pre, a->n, a->seed, thresh, scale, group, x_rep, a->x_inner, a->seed_in, a->seed_out);
    else
      hipLaunchKernelGGL((dropout_kernel<bf16_t, false>), dim3(blocks), dim3(256), 0, st, (const bf16_t*)a->x,
                         (bf16_t*)a->y, nullptr, a->n, a->seed, thresh, scale, group, x_rep, a->x_inner, a->seed_in, a->seed_out);
  }
  MTTS_LAUNCH_CHECK("dropout");
  return MTTS_OK;
}
