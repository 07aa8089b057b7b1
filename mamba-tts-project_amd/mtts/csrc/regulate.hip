// Length regulator (phoneme -> frame expansion) for the style pipeline,
// replacing the reference's per-(b, phoneme) Python loop with one .item()
// each (style_cross_attention.py:156-198, LengthRegulator.forward):
//   dur[b,t]   = max(round_half_even(durations[b,t]), 0)
//   lengths[b] = sum_t dur[b,t]
//   out[b,f,:] = hidden[b, t(f), :] for f < min(lengths[b], max_len), else 0,
// t(f) = the phoneme whose cumulative-duration interval [end_{t-1}, end_t)
// holds f.  The backward is the matching segment sum: dhidden[b,t,:] =
// sum over f in [end_{t-1}, min(end_t, max_len)) of dout[b,f,:] (fixed order,
// deterministic).  Every block re-derives the running sums of its batch row
// in LDS (T <= 4096 phonemes), so there is no host round trip and no
// intermediate index tensor; rows move as 16-byte vectors.
#include "common.h"

namespace mtts {

constexpr int kRegMaxT = 4096;
constexpr int kRegBlock = 256;

// ends[t] = sum_{s <= t} dur[s] (int64) for one batch row, whole block.
__device__ void dur_scan(const float* __restrict__ dur, int T, long long* ends, long long* part) {
  const int i = threadIdx.x;
  const int per = (T + kRegBlock - 1) / kRegBlock;
  const int t0 = min(T, i * per), t1 = min(T, t0 + per);
  long long s = 0;
  for (int t = t0; t < t1; ++t) {
    const float r = fmaxf(rintf(dur[t]), 0.f);   // torch.round (half to even), clamp(min=0)
    s += (long long)r;
    ends[t] = s;
  }
  part[i] = s;
  block_sync();
  for (int off = 1; off < kRegBlock; off <<= 1) {
    const long long v = i >= off ? part[i - off] : 0;
    block_sync();
    part[i] += v;
    block_sync();
  }
  const long long base = i > 0 ? part[i - 1] : 0;
  for (int t = t0; t < t1; ++t) ends[t] += base;
  block_sync();
}

template <typename T, int EV>
struct alignas(EV == 1 ? sizeof(T) : 16) Vec {
  T v[EV];
};

__global__ __launch_bounds__(kRegBlock) void reg_lengths_kernel(const float* __restrict__ dur, int64_t dur_bs, int T,
                                                                int64_t* __restrict__ lengths) {
  __shared__ long long ends[kRegMaxT];
  __shared__ long long part[kRegBlock];
  const int b = blockIdx.x;
  dur_scan(dur + b * dur_bs, T, ends, part);
  if (threadIdx.x == 0) lengths[b] = T > 0 ? ends[T - 1] : 0;
}

// one wave per output frame (fpb frames per block)
template <typename T, int EV>
__global__ __launch_bounds__(kRegBlock) void reg_fwd_kernel(const T* __restrict__ h, int64_t h_bs, int64_t h_ls,
                                                            const float* __restrict__ dur, int64_t dur_bs, int nT,
                                                            int D, int max_len, T* __restrict__ out, int64_t o_bs,
                                                            int64_t o_ls, int fpb) {
  __shared__ long long ends[kRegMaxT];
  __shared__ long long part[kRegBlock];
  const int b = blockIdx.y;
  dur_scan(dur + b * dur_bs, nT, ends, part);
  const long long len = nT > 0 ? ends[nT - 1] : 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nv = D / EV;
  using V = Vec<T, EV>;
  const int f0 = blockIdx.x * fpb;
  const int f1 = min(max_len, f0 + fpb);
  for (int f = f0 + w; f < f1; f += kRegBlock / 64) {
    V* __restrict__ dst = reinterpret_cast<V*>(out + b * o_bs + (int64_t)f * o_ls);
    if (f < len) {
      int lo = 0, hi = nT;  // first t with ends[t] > f
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (ends[mid] <= f) lo = mid + 1;
        else hi = mid;
      }
      const V* __restrict__ src = reinterpret_cast<const V*>(h + b * h_bs + (int64_t)lo * h_ls);
      for (int c = lane; c < nv; c += 64) dst[c] = src[c];
    } else {
      V z;
      for (int e = 0; e < EV; ++e) reinterpret_cast<T*>(&z)[e] = T(0);
      for (int c = lane; c < nv; c += 64) dst[c] = z;
    }
  }
}

// one wave per phoneme (ppb phonemes per block); fp32 accumulation
template <typename T, int EV>
__global__ __launch_bounds__(kRegBlock) void reg_bwd_kernel(const T* __restrict__ dout, int64_t do_bs, int64_t do_ls,
                                                            const float* __restrict__ dur, int64_t dur_bs, int nT,
                                                            int D, int max_len, T* __restrict__ dh, int64_t dh_bs,
                                                            int64_t dh_ls, int ppb) {
  __shared__ long long ends[kRegMaxT];
  __shared__ long long part[kRegBlock];
  const int b = blockIdx.y;
  dur_scan(dur + b * dur_bs, nT, ends, part);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nv = D / EV;
  using V = Vec<T, EV>;
  const int t0 = blockIdx.x * ppb;
  const int t1 = min(nT, t0 + ppb);
  for (int t = t0 + w; t < t1; t += kRegBlock / 64) {
    const long long s = t > 0 ? ends[t - 1] : 0;
    const long long e = min(ends[t], (long long)max_len);
    V* __restrict__ dst = reinterpret_cast<V*>(dh + b * dh_bs + (int64_t)t * dh_ls);
    for (int c = lane; c < nv; c += 64) {
      float acc[EV];
#pragma unroll
      for (int q = 0; q < EV; ++q) acc[q] = 0.f;
      for (long long f = s; f < e; ++f) {
        const V v = reinterpret_cast<const V*>(dout + b * do_bs + f * do_ls)[c];
#pragma unroll
        for (int q = 0; q < EV; ++q) acc[q] += ldf(&v.v[q]);
      }
      V o;
#pragma unroll
      for (int q = 0; q < EV; ++q) stf(&o.v[q], acc[q]);
      dst[c] = o;
    }
  }
}

static bool vec_ok(int es, int D, std::initializer_list<const void*> ptrs, std::initializer_list<int64_t> strides) {
  const int ev = 16 / es;
  if (D % ev) return false;
  for (const void* p : ptrs)
    if ((uintptr_t)p % 16) return false;
  for (int64_t s : strides)
    if (s % ev) return false;
  return true;
}

}  // namespace mtts

using namespace mtts;

extern "C" int mtts_length_regulate_lengths(const float* durations, int64_t dur_bs, int batch, int T,
                                            int64_t* lengths, void* stream) {
  MTTS_CHECK(lengths && batch >= 0 && T >= 0 && (T == 0 || durations), "length_regulate: bad args");
  MTTS_CHECK(T <= kRegMaxT, "length_regulate: T=%d phonemes > %d", T, kRegMaxT);
  if (batch == 0) return MTTS_OK;
  hipLaunchKernelGGL(reg_lengths_kernel, dim3(batch), dim3(kRegBlock), 0, (hipStream_t)stream, durations, dur_bs, T,
                     lengths);
  MTTS_LAUNCH_CHECK("length_regulate_lengths");
  return MTTS_OK;
}

extern "C" int mtts_length_regulate_fwd(const void* hidden, int dtype, int batch, int T, int D, int64_t h_bs,
                                        int64_t h_ls, const float* durations, int64_t dur_bs, int max_len, void* out,
                                        int64_t o_bs, int64_t o_ls, void* stream) {
  MTTS_CHECK(batch >= 0 && T >= 0 && D > 0 && max_len >= 0, "length_regulate: bad args");
  MTTS_CHECK(out || batch == 0 || max_len == 0, "length_regulate: null output");
  MTTS_CHECK(T == 0 || (hidden && durations), "length_regulate: null input");
  MTTS_CHECK(T <= kRegMaxT, "length_regulate: T=%d phonemes > %d", T, kRegMaxT);
  MTTS_CHECK(dtype == MTTS_F32 || dtype == MTTS_BF16, "length_regulate: bad dtype");
  if (batch == 0 || max_len == 0) return MTTS_OK;
  const int fpb = 16;  // 4 frames per wave: >= 256 blocks already at B=4, 1000 frames
  dim3 grid((max_len + fpb - 1) / fpb, batch);
  hipStream_t st = (hipStream_t)stream;
  const int es = dtype == MTTS_F32 ? 4 : 2;
  const bool v = vec_ok(es, D, {hidden, out}, {h_bs, h_ls, o_bs, o_ls});
  if (dtype == MTTS_F32) {
    if (v)
      hipLaunchKernelGGL((reg_fwd_kernel<float, 4>), grid, dim3(kRegBlock), 0, st, (const float*)hidden, h_bs, h_ls,
                         durations, dur_bs, T, D, max_len, (float*)out, o_bs, o_ls, fpb);
    else
      hipLaunchKernelGGL((reg_fwd_kernel<float, 1>), grid, dim3(kRegBlock), 0, st, (const float*)hidden, h_bs, h_ls,
                         durations, dur_bs, T, D, max_len, (float*)out, o_bs, o_ls, fpb);
  } else {
    if (v)
      hipLaunchKernelGGL((reg_fwd_kernel<bf16_t, 8>), grid, dim3(kRegBlock), 0, st, (const bf16_t*)hidden, h_bs,
                         h_ls, durations, dur_bs, T, D, max_len, (bf16_t*)out, o_bs, o_ls, fpb);
    else
      hipLaunchKernelGGL((reg_fwd_kernel<bf16_t, 1>), grid, dim3(kRegBlock), 0, st, (const bf16_t*)hidden, h_bs,
                         h_ls, durations, dur_bs, T, D, max_len, (bf16_t*)out, o_bs, o_ls, fpb);
  }
  MTTS_LAUNCH_CHECK("length_regulate_fwd");
  return MTTS_OK;
}

extern "C" int mtts_length_regulate_bwd(const void* dout, int dtype, int batch, int T, int D, int64_t do_bs,
                                        int64_t do_ls, const float* durations, int64_t dur_bs, int max_len,
                                        void* dhidden, int64_t dh_bs, int64_t dh_ls, void* stream) {
  MTTS_CHECK(batch >= 0 && T >= 0 && D > 0 && max_len >= 0, "length_regulate_bwd: bad args");
  MTTS_CHECK(dhidden || batch == 0 || T == 0, "length_regulate_bwd: null output");
  MTTS_CHECK(T == 0 || durations, "length_regulate_bwd: null durations");
  MTTS_CHECK(max_len == 0 || dout, "length_regulate_bwd: null dout");
  MTTS_CHECK(T <= kRegMaxT, "length_regulate_bwd: T=%d phonemes > %d", T, kRegMaxT);
  MTTS_CHECK(dtype == MTTS_F32 || dtype == MTTS_BF16, "length_regulate_bwd: bad dtype");
  if (batch == 0 || T == 0) return MTTS_OK;
  const int ppb = 16;
  dim3 grid((T + ppb - 1) / ppb, batch);
  hipStream_t st = (hipStream_t)stream;
  const int es = dtype == MTTS_F32 ? 4 : 2;
  const bool v = vec_ok(es, D, {dout ? dout : dhidden, dhidden}, {do_bs, do_ls, dh_bs, dh_ls});
  if (dtype == MTTS_F32) {
    if (v)
      hipLaunchKernelGGL((reg_bwd_kernel<float, 4>), grid, dim3(kRegBlock), 0, st, (const float*)dout, do_bs, do_ls,
                         durations, dur_bs, T, D, max_len, (float*)dhidden, dh_bs, dh_ls, ppb);
    else
      hipLaunchKernelGGL((reg_bwd_kernel<float, 1>), grid, dim3(kRegBlock), 0, st, (const float*)dout, do_bs, do_ls,
                         durations, dur_bs, T, D, max_len, (float*)dhidden, dh_bs, dh_ls, ppb);
  } else {
    if (v)
      hipLaunchKernelGGL((reg_bwd_kernel<bf16_t, 8>), grid, dim3(kRegBlock), 0, st, (const bf16_t*)dout, do_bs,
                         do_ls, durations, dur_bs, T, D, max_len, (bf16_t*)dhidden, dh_bs, dh_ls, ppb);
    else
      hipLaunchKernelGGL((reg_bwd_kernel<bf16_t, 1>), grid, dim3(kRegBlock), 0, st, (const bf16_t*)dout, do_bs,
                         do_ls, durations, dur_bs, T, D, max_len, (bf16_t*)dhidden, dh_bs, dh_ls, ppb);
  }
  MTTS_LAUNCH_CHECK("length_regulate_bwd");
  return MTTS_OK;
}

// ---------------------------------------------------------------------------
// Embedding sum (mamba_decoder.py:167-171 prologue, train.py:115-131
// embed_codec_tokens):  out[b,l,:] = tok_w[tok[b,l]] + q_w[qid[l]] + pos_w[pid[l]]
// fp32 tables (the master parameters), int64 token ids, int32 per-position
// quantizer / position ids shared by the batch; one wave per output row,
// float4 table reads, fp32 sum, out in f32 or bf16.
namespace mtts {

template <typename T>
__global__ __launch_bounds__(256) void embed_sum_kernel(const int64_t* __restrict__ tok, int64_t tok_bs,
                                                        const int* __restrict__ qid, const int* __restrict__ pid,
                                                        const float* __restrict__ tw, const float* __restrict__ qw,
                                                        const float* __restrict__ pw, int L, int d, int V, int rpb,
                                                        T* __restrict__ out, int64_t o_bs, int* __restrict__ err) {
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int l0 = blockIdx.x * rpb;
  for (int l = l0 + w; l < min(L, l0 + rpb); l += 4) {
    const int64_t t = tok[b * tok_bs + l];
    T* __restrict__ o = out + b * o_bs + (int64_t)l * d;
    if (t < 0 || t >= V) {
      // nn.Embedding would raise; the host checks the flag (mtts.embed.check_errors,
      // the decode engine once per step).  The row is written as zeros so no
      // uninitialised memory flows on.
      if (lane == 0) err[0] = 1;
      for (int c = lane; c < d / 4; c += 64) {
        if constexpr (sizeof(T) == 4) reinterpret_cast<float4*>(o)[c] = make_float4(0.f, 0.f, 0.f, 0.f);
        else reinterpret_cast<uint2*>(o)[c] = make_uint2(0u, 0u);
      }
      continue;
    }
    const float4* __restrict__ a = reinterpret_cast<const float4*>(tw + t * d);
    const float4* __restrict__ q = reinterpret_cast<const float4*>(qw + (int64_t)qid[l] * d);
    const float4* __restrict__ p = reinterpret_cast<const float4*>(pw + (int64_t)pid[l] * d);
    for (int c = lane; c < d / 4; c += 64) {
      const float4 x = a[c], y = q[c], z = p[c];
      const float s0 = (x.x + z.x) + y.x, s1 = (x.y + z.y) + y.y, s2 = (x.z + z.z) + y.z, s3 = (x.w + z.w) + y.w;
      if constexpr (sizeof(T) == 4) {
        reinterpret_cast<float4*>(o)[c] = make_float4(s0, s1, s2, s3);
      } else {
        reinterpret_cast<uint2*>(o)[c] =
            make_uint2((uint32_t)f2bf(s0) | ((uint32_t)f2bf(s1) << 16), (uint32_t)f2bf(s2) | ((uint32_t)f2bf(s3) << 16));
      }
    }
  }
}

}  // namespace mtts

extern "C" int mtts_embed_sum(const int64_t* tokens, int64_t tok_bs, const int* quant_ids, const int* pos_ids,
                              const float* tok_w, const float* q_w, const float* pos_w, int batch, int L, int d,
                              int vocab, void* out, int dtype, int64_t out_bs, int* err_flag, void* stream) {
  MTTS_CHECK(batch >= 0 && L >= 0 && d > 0 && vocab > 0, "embed_sum: bad args");
  MTTS_CHECK(d % 4 == 0, "embed_sum: d_model %% 4 != 0");
  MTTS_CHECK(dtype == MTTS_F32 || dtype == MTTS_BF16, "embed_sum: bad dtype");
  if (batch == 0 || L == 0) return MTTS_OK;
  MTTS_CHECK(tokens && quant_ids && pos_ids && tok_w && q_w && pos_w && out && err_flag, "embed_sum: null pointer");
  MTTS_CHECK(((uintptr_t)tok_w | (uintptr_t)q_w | (uintptr_t)pos_w | (uintptr_t)out) % 16 == 0,
             "embed_sum: tables/out must be 16-byte aligned");
  const int rpb = 16;
  dim3 grid((L + rpb - 1) / rpb, batch);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == MTTS_F32)
    hipLaunchKernelGGL(embed_sum_kernel<float>, grid, dim3(256), 0, st, tokens, tok_bs, quant_ids, pos_ids, tok_w, q_w,
                       pos_w, L, d, vocab, rpb, (float*)out, out_bs, err_flag);
  else
    hipLaunchKernelGGL(embed_sum_kernel<bf16_t>, grid, dim3(256), 0, st, tokens, tok_bs, quant_ids, pos_ids, tok_w,
                       q_w, pos_w, L, d, vocab, rpb, (bf16_t*)out, out_bs, err_flag);
  MTTS_LAUNCH_CHECK("embed_sum");
  return MTTS_OK;
}

// ---------------------------------------------------------------------------
// Gradient of a small embedding table (the codec vocabulary, train.py's 10
// codes: mamba_decoder.py:167 token_embed and train.py:115-131's reference
// embedding share it):  out[v, :] = sum over rows r with ids[r] == v of g[r, :].
// nn.Embedding's backward sorts the ids and scatters; a one-hot GEMM
// (onehot^T g, K = all rows, M = V) runs as a long thin reduction on hipBLASLt
// (~91 us per C5 call).  Here one pass over g: a lane owns 16 bytes of a row
// (8 bf16 / 4 fp32 columns) and keeps V <= 16 bins of them in registers (an
// fma by (id == v) per bin: no dynamic register indexing, no atomics), a
// block's 4 waves combine in LDS in a fixed order, and the per-block (V, d)
// slabs are summed by the deterministic column sum.  HBM-bound: reads g once.
namespace mtts {

constexpr int kEmbGradVMax = 16;

template <typename T>
__global__ __launch_bounds__(256) void embed_table_grad_kernel(const int64_t* __restrict__ ids, int64_t n,
                                                               const T* __restrict__ g, int64_t g_rs, int d, int V,
                                                               int rpb, float* __restrict__ part) {
  constexpr int EPL = 16 / (int)sizeof(T);
  constexpr int CB = 64 * EPL;
  __shared__ float red[4][CB];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * CB + lane * EPL;
  const int64_t r0 = (int64_t)blockIdx.y * rpb, r1 = min(n, r0 + rpb);
  float acc[kEmbGradVMax][EPL];
#pragma unroll
  for (int v = 0; v < kEmbGradVMax; ++v)
#pragma unroll
    for (int q = 0; q < EPL; ++q) acc[v][q] = 0.f;
  if (c < d) {
    for (int64_t r = r0 + w; r < r1; r += 4) {
      const int64_t id = ids[r];
      const uint4 raw = *reinterpret_cast<const uint4*>(g + r * g_rs + c);
      float x[EPL];
      if constexpr (sizeof(T) == 2) {
        const uint32_t u[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          x[2 * q] = __uint_as_float(u[q] << 16);
          x[2 * q + 1] = __uint_as_float(u[q] & 0xffff0000u);
        }
      } else {
        x[0] = __uint_as_float(raw.x); x[1] = __uint_as_float(raw.y);
        x[2] = __uint_as_float(raw.z); x[3] = __uint_as_float(raw.w);
      }
#pragma unroll
      for (int v = 0; v < kEmbGradVMax; ++v) {
        const float m = id == v ? 1.f : 0.f;
#pragma unroll
        for (int q = 0; q < EPL; ++q) acc[v][q] = fmaf(m, x[q], acc[v][q]);
      }
    }
  }
  for (int v = 0; v < V; ++v) {   // block-uniform loop
#pragma unroll
    for (int q = 0; q < EPL; ++q) red[w][lane * EPL + q] = acc[v][q];
    block_sync();
    for (int k = threadIdx.x; k < CB; k += 256) {
      const int cc = blockIdx.x * CB + k;
      if (cc < d) part[((int64_t)blockIdx.y * V + v) * d + cc] = (red[0][k] + red[1][k]) + (red[2][k] + red[3][k]);
    }
    block_sync();
  }
}

static int emb_grad_blocks(int64_t n, int* rpb) {
  int r = (int)std::max<int64_t>(64, (n + 255) / 256);
  r = (r + 3) / 4 * 4;
  *rpb = r;
  return (int)((n + r - 1) / r);
}

}  // namespace mtts

extern "C" int64_t mtts_embed_table_grad_workspace(int64_t n, int d, int vocab) {
  int rpb = 0;
  const int nblk = mtts::emb_grad_blocks(n, &rpb);
  return (int64_t)nblk * vocab * d * 4 + 256;
}

extern "C" int mtts_embed_table_grad(const int64_t* ids, int64_t n, const void* g, int dtype, int64_t g_rs, int d,
                                     int vocab, float* out, void* workspace, void* stream) {
  using namespace mtts;
  MTTS_CHECK(n >= 0 && d > 0 && vocab > 0 && vocab <= kEmbGradVMax, "embed_table_grad: vocab=%d must be in [1, %d]",
             vocab, kEmbGradVMax);
  MTTS_CHECK(dtype == MTTS_F32 || dtype == MTTS_BF16, "embed_table_grad: bad dtype");
  MTTS_CHECK(out, "embed_table_grad: null output");
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    (void)hipMemsetAsync(out, 0, (size_t)vocab * d * 4, st);
    return MTTS_OK;
  }
  const int vl = dtype == MTTS_F32 ? 4 : 8;
  MTTS_CHECK(ids && g && workspace, "embed_table_grad: null pointer");
  MTTS_CHECK(d % vl == 0 && g_rs % vl == 0 && (uintptr_t)g % 16 == 0,
             "embed_table_grad: rows must be whole 16-byte pieces (d=%d, row stride=%lld)", d, (long long)g_rs);
  int rpb = 0;
  const int nblk = emb_grad_blocks(n, &rpb);
  float* part = (float*)workspace;
  const dim3 grid((d + 64 * vl - 1) / (64 * vl), nblk);
  if (dtype == MTTS_F32)
    hipLaunchKernelGGL(embed_table_grad_kernel<float>, grid, dim3(256), 0, st, ids, n, (const float*)g, g_rs, d, vocab,
                       rpb, part);
  else
    hipLaunchKernelGGL(embed_table_grad_kernel<bf16_t>, grid, dim3(256), 0, st, ids, n, (const bf16_t*)g, g_rs, d,
                       vocab, rpb, part);
  MTTS_LAUNCH_CHECK("embed_table_grad");
  colsum(part, nblk, nblk, (int64_t)vocab * d, vocab * d, out, 0, st);
  MTTS_LAUNCH_CHECK("embed_table_grad sum");
  return MTTS_OK;
}
