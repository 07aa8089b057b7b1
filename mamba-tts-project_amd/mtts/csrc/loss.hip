// Codec-token cross-entropy with an ignore index (train.py:31-42
// codec_ce_loss = F.cross_entropy(logits.view(B*T, V), targets.view(B*T),
// ignore_index=pad_id), mean over the non-ignored rows).
//   forward : one thread per row (V logits in registers / L1): row max, lse,
//             lse - x[target]; per-block partial (sum, count) written to the
//             workspace, one block sums the partials in fixed order
//             (deterministic), loss = sum / count (0/0 = NaN when every
//             target is ignored, as torch); lse per row saved.
//   backward: one thread per logit: (exp(x - lse) - [v == target]) * g /
//             count, 0 on ignored rows; g read from the device (no host
//             sync, hipGraph-capturable).
// fp32 math; logits / dlogits fp32 or bf16.
#include "common.h"

namespace mtts {
namespace {

constexpr int kCeBlock = 256;

template <typename T>
__global__ __launch_bounds__(kCeBlock) void ce_fwd_kernel(const T* __restrict__ x, int64_t rows, int V, int64_t ld,
                                                          const int64_t* __restrict__ tgt, int ignore,
                                                          float* __restrict__ lse_out, float* __restrict__ part) {
  const int64_t r = (int64_t)blockIdx.x * kCeBlock + threadIdx.x;
  float loss = 0.f, cnt = 0.f;
  if (r < rows) {
    const T* xr = x + r * ld;
    float m = -INFINITY;
    for (int v = 0; v < V; ++v) m = fmaxf(m, ldf(xr + v));
    float s = 0.f;
    for (int v = 0; v < V; ++v) s += expf(ldf(xr + v) - m);
    const float lse = m + logf(s);
    lse_out[r] = lse;
    const int64_t t = tgt[r];
    if (t != ignore) {   // a target outside [0, V) gives NaN (torch asserts), never an out-of-row read
      loss = (t >= 0 && t < V) ? lse - ldf(xr + t) : __builtin_nanf("");
      cnt = 1.f;
    }
  }
  // fixed-order block reduction: wave sums, then the 4 wave partials
  __shared__ float ws[kCeBlock / 64][2];
  loss = wave_sum(loss);
  cnt = wave_sum(cnt);
  if ((threadIdx.x & 63) == 0) {
    ws[threadIdx.x >> 6][0] = loss;
    ws[threadIdx.x >> 6][1] = cnt;
  }
  block_sync();
  if (threadIdx.x == 0) {
    float a = 0.f, c = 0.f;
    for (int w = 0; w < kCeBlock / 64; ++w) { a += ws[w][0]; c += ws[w][1]; }
    part[2 * blockIdx.x] = a;
    part[2 * blockIdx.x + 1] = c;
  }
}

// one block: sum of the nb partials in fixed order; out[0] = loss, out[1] = count
__global__ __launch_bounds__(kCeBlock) void ce_sum_kernel(const float* __restrict__ part, int nb,
                                                          float* __restrict__ out) {
  float a = 0.f, c = 0.f;
  for (int i = threadIdx.x; i < nb; i += kCeBlock) { a += part[2 * i]; c += part[2 * i + 1]; }
  __shared__ float ws[kCeBlock / 64][2];
  a = wave_sum(a);
  c = wave_sum(c);
  if ((threadIdx.x & 63) == 0) {
    ws[threadIdx.x >> 6][0] = a;
    ws[threadIdx.x >> 6][1] = c;
  }
  block_sync();
  if (threadIdx.x == 0) {
    float sa = 0.f, sc = 0.f;
    for (int w = 0; w < kCeBlock / 64; ++w) { sa += ws[w][0]; sc += ws[w][1]; }
    out[0] = sa / sc;   // 0 / 0 = NaN when every target is ignored (torch)
    out[1] = sc;
  }
}

template <typename T>
__global__ __launch_bounds__(kCeBlock) void ce_bwd_kernel(const T* __restrict__ x, int64_t rows, int V, int64_t ld,
                                                          const int64_t* __restrict__ tgt, int ignore,
                                                          const float* __restrict__ lse, const float* __restrict__ red,
                                                          const float* __restrict__ gout, T* __restrict__ dx,
                                                          int64_t ldd) {
  const int64_t i = (int64_t)blockIdx.x * kCeBlock + threadIdx.x;
  if (i >= rows * V) return;
  const int64_t r = i / V;
  const int v = (int)(i % V);
  const int64_t t = tgt[r];
  float d = 0.f;
  if (t != ignore) {
    const float p = expf(ldf(x + r * ld + v) - lse[r]);
    d = (p - (v == t ? 1.f : 0.f)) * (gout[0] / red[1]);
  }
  stf(dx + r * ldd + v, d);
}

template <typename T>
int ce_fwd(const MttsCrossEntropyArgs* a, hipStream_t st) {
  const int nb = (int)((a->rows + kCeBlock - 1) / kCeBlock);
  float* part = a->workspace;
  hipLaunchKernelGGL(ce_fwd_kernel<T>, dim3(nb), dim3(kCeBlock), 0, st, (const T*)a->logits, a->rows, a->vocab,
                     a->ld, a->targets, a->ignore_index, a->lse, part);
  hipLaunchKernelGGL(ce_sum_kernel, dim3(1), dim3(kCeBlock), 0, st, part, nb, a->loss);
  return MTTS_OK;
}

template <typename T>
int ce_bwd(const MttsCrossEntropyArgs* a, const float* gout, void* dlogits, int64_t ldd, hipStream_t st) {
  const int64_t n = a->rows * a->vocab;
  hipLaunchKernelGGL(ce_bwd_kernel<T>, dim3((unsigned)((n + kCeBlock - 1) / kCeBlock)), dim3(kCeBlock), 0, st,
                     (const T*)a->logits, a->rows, a->vocab, a->ld, a->targets, a->ignore_index, a->lse, a->loss,
                     gout, (T*)dlogits, ldd);
  return MTTS_OK;
}

int check_ce(const MttsCrossEntropyArgs* a) {
  MTTS_CHECK(a && a->logits && a->targets && a->loss && a->lse && a->workspace, "cross_entropy: null pointer");
  MTTS_CHECK(a->rows > 0 && a->vocab > 0 && a->ld >= a->vocab, "cross_entropy: rows=%lld vocab=%d ld=%lld",
             (long long)a->rows, a->vocab, (long long)a->ld);
  MTTS_CHECK(a->dtype == MTTS_F32 || a->dtype == MTTS_BF16, "cross_entropy: logits must be F32 or BF16");
  return MTTS_OK;
}

}  // namespace
}  // namespace mtts

using namespace mtts;

extern "C" int64_t mtts_cross_entropy_workspace(int64_t rows) {
  return ((rows + kCeBlock - 1) / kCeBlock) * 2 * (int64_t)sizeof(float) + 256;
}

extern "C" int mtts_cross_entropy_fwd(const MttsCrossEntropyArgs* a, void* stream) {
  int rc = check_ce(a);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  rc = a->dtype == MTTS_F32 ? ce_fwd<float>(a, st) : ce_fwd<bf16_t>(a, st);
  MTTS_LAUNCH_CHECK("cross_entropy_fwd");
  return rc;
}

extern "C" int mtts_cross_entropy_bwd(const MttsCrossEntropyArgs* a, const float* grad_loss, void* dlogits,
                                      int64_t ld_dlogits, void* stream) {
  int rc = check_ce(a);
  if (rc) return rc;
  MTTS_CHECK(grad_loss && dlogits && ld_dlogits >= a->vocab, "cross_entropy_bwd: null gradient / bad stride");
  hipStream_t st = (hipStream_t)stream;
  rc = a->dtype == MTTS_F32 ? ce_bwd<float>(a, grad_loss, dlogits, ld_dlogits, st)
                            : ce_bwd<bf16_t>(a, grad_loss, dlogits, ld_dlogits, st);
  MTTS_LAUNCH_CHECK("cross_entropy_bwd");
  return rc;
}
