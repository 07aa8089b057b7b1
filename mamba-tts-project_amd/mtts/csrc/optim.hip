// Fused gradient-norm clipping + Adam over a whole parameter list (SURVEY.md
// §8f row 4; reference train.py:232-235: clip_grad_norm_(decoder.parameters(),
// 1.0) then torch.optim.Adam.step()).  Three launches per step, independent of
// the number of tensors:
//   1. per-chunk partial sums of g^2 (64 Ki elements per block, float4),
//   2. one block: total = sqrt(sum of partials) in a fixed order,
//      coef = min(1, max_norm / (total + 1e-6))   (clip_grad_norm_'s formula),
//      t = ++(*step_counter) and the bias corrections (device-side, so the
//      whole training step can be captured in a hipGraph and replayed),
//   3. per-chunk Adam on (p, g*coef, m, v) with torch's update:
//        m = b1 m + (1-b1) g ;  v = b2 v + (1-b2) g^2
//        p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// (plus L2 weight decay g += wd*p before the moments, as torch.optim.Adam).
// HBM: reads g twice and p, m, v once, writes p, m, v: 32 B per parameter
// (torch: foreach norm + clip rewrite + fused Adam = 40 B and more launches).
// Gradients are left unclipped (the update uses g*coef).
#include "common.h"

namespace mtts {

constexpr int64_t kAdamChunk = 65536;   // elements per block
constexpr int kAdamBlock = 256;

__device__ __forceinline__ int find_tensor(const MttsAdamTensor* __restrict__ t, int n, int64_t blk) {
  int lo = 0, hi = n - 1;  // last tensor with chunk0 <= blk
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (t[mid].chunk0 <= blk) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  block_sync();
  float s = 0.f;
  if (threadIdx.x == 0) {
    for (int i = 0; i < kAdamBlock / 64; ++i) s += red[i];
  }
  return s;
}

__global__ __launch_bounds__(kAdamBlock) void sumsq_kernel(const MttsAdamTensor* __restrict__ ts, int n,
                                                           float* __restrict__ partial) {
  __shared__ float red[kAdamBlock / 64];
  const int64_t blk = blockIdx.x;
  const MttsAdamTensor t = ts[find_tensor(ts, n, blk)];
  const int64_t e0 = (blk - t.chunk0) * kAdamChunk;
  const int64_t e1 = min(t.n, e0 + kAdamChunk);
  float s = 0.f;
  const bool vec = ((uintptr_t)t.g % 16) == 0;
  if (vec) {
    const int64_t v0 = e0 / 4, v1 = e1 / 4;  // e0 is a multiple of 4
    const float4* __restrict__ g4 = reinterpret_cast<const float4*>(t.g);
    for (int64_t i = v0 + threadIdx.x; i < v1; i += kAdamBlock) {
      const float4 g = g4[i];
      s = fmaf(g.x, g.x, fmaf(g.y, g.y, fmaf(g.z, g.z, fmaf(g.w, g.w, s))));
    }
    for (int64_t i = v1 * 4 + threadIdx.x; i < e1; i += kAdamBlock) s = fmaf(t.g[i], t.g[i], s);
  } else {
    for (int64_t i = e0 + threadIdx.x; i < e1; i += kAdamBlock) s = fmaf(t.g[i], t.g[i], s);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) partial[blk] = s;
}

struct AdamHyper {
  float lr, b1, b2, eps, wd;
};

// one block: total grad norm, clip coefficient, and the step's bias
// corrections from the device step counter (so a captured hipGraph replays
// correct steps): out = {total, coef, lr / (1 - b1^t), sqrt(1 - b2^t)}
__global__ __launch_bounds__(kAdamBlock) void norm_final_kernel(const float* __restrict__ partial, int64_t nchunks,
                                                                float max_norm, int* __restrict__ step_counter,
                                                                const AdamHyper h, float* __restrict__ out) {
  __shared__ float red[kAdamBlock / 64];
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < nchunks; i += kAdamBlock) s += partial[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    const float total = sqrtf(s);
    out[0] = total;
    out[1] = max_norm > 0.f ? fminf(1.f, max_norm / (total + 1e-6f)) : 1.f;
    const int t = step_counter[0] + 1;
    step_counter[0] = t;
    const double bc1 = 1.0 - pow((double)h.b1, (double)t), bc2 = 1.0 - pow((double)h.b2, (double)t);
    out[2] = (float)(h.lr / bc1);
    out[3] = (float)sqrt(bc2);
  }
}

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float coef, float step_size,
                                          float bc2_sqrt, const AdamHyper& h) {
  g *= coef;
  if (h.wd != 0.f) g = fmaf(h.wd, p, g);
  m = fmaf(h.b1, m, (1.f - h.b1) * g);
  v = fmaf(h.b2, v, (1.f - h.b2) * g * g);
  const float denom = sqrtf(v) / bc2_sqrt + h.eps;
  p -= step_size * (m / denom);
}

__global__ __launch_bounds__(kAdamBlock) void adam_kernel(const MttsAdamTensor* __restrict__ ts, int n,
                                                          const float* __restrict__ norm, const AdamHyper h) {
  const int64_t blk = blockIdx.x;
  const MttsAdamTensor t = ts[find_tensor(ts, n, blk)];
  const float coef = norm[1], step_size = norm[2], bc2_sqrt = norm[3];
  const int64_t e0 = (blk - t.chunk0) * kAdamChunk;
  const int64_t e1 = min(t.n, e0 + kAdamChunk);
  const bool vec = (((uintptr_t)t.p | (uintptr_t)t.g | (uintptr_t)t.m | (uintptr_t)t.v) % 16) == 0;
  int64_t tail = e0;
  if (vec) {
    const int64_t v0 = e0 / 4, v1 = e1 / 4;
    float4* p4 = reinterpret_cast<float4*>(t.p);
    const float4* g4 = reinterpret_cast<const float4*>(t.g);
    float4* m4 = reinterpret_cast<float4*>(t.m);
    float4* q4 = reinterpret_cast<float4*>(t.v);
    for (int64_t i = v0 + threadIdx.x; i < v1; i += kAdamBlock) {
      float4 p = p4[i], m = m4[i], v = q4[i];
      const float4 g = g4[i];
      adam_elem(p.x, g.x, m.x, v.x, coef, step_size, bc2_sqrt, h);
      adam_elem(p.y, g.y, m.y, v.y, coef, step_size, bc2_sqrt, h);
      adam_elem(p.z, g.z, m.z, v.z, coef, step_size, bc2_sqrt, h);
      adam_elem(p.w, g.w, m.w, v.w, coef, step_size, bc2_sqrt, h);
      p4[i] = p; m4[i] = m; q4[i] = v;
    }
    tail = v1 * 4;
  }
  for (int64_t i = tail + threadIdx.x; i < e1; i += kAdamBlock)
    adam_elem(t.p[i], t.g[i], t.m[i], t.v[i], coef, step_size, bc2_sqrt, h);
}

}  // namespace mtts

using namespace mtts;

extern "C" int64_t mtts_adam_chunks(int64_t numel) { return numel <= 0 ? 0 : (numel + kAdamChunk - 1) / kAdamChunk; }

extern "C" int64_t mtts_adam_workspace(int64_t total_chunks) { return total_chunks * 4 + 256; }

extern "C" int mtts_clip_adam(const MttsAdamTensor* tensors, int ntensors, int64_t total_chunks, int* step_counter,
                              float lr, float beta1, float beta2, float eps, float weight_decay, float max_norm,
                              void* workspace, float* norm_out, void* stream) {
  MTTS_CHECK(tensors && ntensors > 0 && total_chunks > 0 && workspace && step_counter && norm_out,
             "clip_adam: bad args");
  MTTS_CHECK(total_chunks < (1ll << 31), "clip_adam: too many chunks");
  hipStream_t st = (hipStream_t)stream;
  float* partial = (float*)workspace;
  if (max_norm > 0.f) {
    hipLaunchKernelGGL(sumsq_kernel, dim3((unsigned)total_chunks), dim3(kAdamBlock), 0, st, tensors, ntensors,
                       partial);
    MTTS_LAUNCH_CHECK("clip_adam sumsq");
  }
  AdamHyper h;
  h.lr = lr;
  h.b1 = beta1;
  h.b2 = beta2;
  h.eps = eps;
  h.wd = weight_decay;
  hipLaunchKernelGGL(norm_final_kernel, dim3(1), dim3(kAdamBlock), 0, st, partial, max_norm > 0.f ? total_chunks : 0,
                     max_norm, step_counter, h, norm_out);
  MTTS_LAUNCH_CHECK("clip_adam norm");
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)total_chunks), dim3(kAdamBlock), 0, st, tensors, ntensors, norm_out,
                     h);
  MTTS_LAUNCH_CHECK("clip_adam adam");
  return MTTS_OK;
}
