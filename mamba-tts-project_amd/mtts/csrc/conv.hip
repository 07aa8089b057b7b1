// Causal depthwise conv1d (width 4) + bias + SiLU, channel-last, gfx950.
//
// Replaces [upstream] causal-conv1d's causal_conv1d_fwd / _bwd CUDA kernels
// (torch fallback HF:81-101), used by Mamba.forward behind
// mamba_decoder.py:61/:63; oracle/mamba_ref.py::causal_conv1d_ref.
//
// Each thread owns CPT consecutive channels (one 16-byte vector: 4 fp32 or
// 8 bf16) and walks a tile of TT timesteps with a register sliding window,
// so every input is read once (plus a 3-step halo per tile) and every load /
// store is a coalesced 16-byte access.  HBM-bound.
#include "common.h"

namespace mtts {

constexpr int kK = 4;
constexpr int kTT = 32;

template <typename T, int CPT>
__device__ __forceinline__ void ldv(const T* p, float (&o)[CPT]) {
  if constexpr (sizeof(T) * CPT == 16) {
    uint4 v = *reinterpret_cast<const uint4*>(p);
    if constexpr (sizeof(T) == 4) {
      o[0] = __uint_as_float(v.x); o[1] = __uint_as_float(v.y); o[2] = __uint_as_float(v.z); o[3] = __uint_as_float(v.w);
    } else {
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) { o[2 * q] = __uint_as_float(w[q] << 16); o[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u); }
    }
  } else {
#pragma unroll
    for (int q = 0; q < CPT; ++q) o[q] = ldf(p + q);
  }
}
template <typename T, int CPT>
__device__ __forceinline__ void stv(T* p, const float (&v)[CPT]) {
  if constexpr (sizeof(T) * CPT == 16) {
    uint4 w;
    if constexpr (sizeof(T) == 4) {
      w = make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3]));
    } else {
      uint32_t q[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) q[k] = (uint32_t)f2bf(v[2 * k]) | ((uint32_t)f2bf(v[2 * k + 1]) << 16);
      w = make_uint4(q[0], q[1], q[2], q[3]);
    }
    *reinterpret_cast<uint4*>(p) = w;
  } else {
#pragma unroll
    for (int q = 0; q < CPT; ++q) stf(p + q, v[q]);
  }
}

// x value at time t (t may be negative -> conv_state_in or zeros)
template <typename T, int CPT>
__device__ __forceinline__ void load_x(const MttsConvFwdArgs& a, int b, int c0, int t, float (&o)[CPT]) {
  if (t >= 0) {
    ldv<T, CPT>((const T*)a.x + (int64_t)b * a.x_bs + (int64_t)t * a.x_ls + c0, o);
  } else if (a.conv_state_in) {
#pragma unroll
    for (int q = 0; q < CPT; ++q) o[q] = a.conv_state_in[((int64_t)b * a.dim + c0 + q) * kK + (kK + t)];
  } else {
#pragma unroll
    for (int q = 0; q < CPT; ++q) o[q] = 0.f;
  }
}

template <typename T, int CPT>
__global__ __launch_bounds__(256) void conv_fwd_kernel(const MttsConvFwdArgs a) {
  const int c0 = (blockIdx.x * 256 + threadIdx.x) * CPT;
  if (c0 >= a.dim) return;
  const int b = blockIdx.z;
  const int t0 = blockIdx.y * kTT;
  float w[kK][CPT], bias[CPT];
#pragma unroll
  for (int q = 0; q < CPT; ++q) {
#pragma unroll
    for (int k = 0; k < kK; ++k) w[k][q] = a.w[(c0 + q) * kK + k];
    bias[q] = a.bias ? a.bias[c0 + q] : 0.f;
  }
  float x0[CPT], x1[CPT], x2[CPT];
  load_x<T, CPT>(a, b, c0, t0 - 3, x0);
  load_x<T, CPT>(a, b, c0, t0 - 2, x1);
  load_x<T, CPT>(a, b, c0, t0 - 1, x2);
  const int tend = min(t0 + kTT, a.seqlen);
  T* out = (T*)a.out + (int64_t)b * a.out_bs + c0;
  for (int t = t0; t < tend; ++t) {
    float x3[CPT], o[CPT];
    load_x<T, CPT>(a, b, c0, t, x3);
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
      float v = fmaf(w[0][q], x0[q], fmaf(w[1][q], x1[q], fmaf(w[2][q], x2[q], fmaf(w[3][q], x3[q], bias[q]))));
      o[q] = a.silu ? silu_f(v) : v;
      x0[q] = x1[q]; x1[q] = x2[q]; x2[q] = x3[q];
    }
    stv<T, CPT>(out + (int64_t)t * a.out_ls, o);
  }
}

// conv_state_out[b, c, k] = last K inputs of [conv_state_in ‖ x]
template <typename T>
__global__ void conv_state_kernel(const MttsConvFwdArgs a) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)a.batch * a.dim * kK) return;
  const int k = idx % kK;
  const int c = (idx / kK) % a.dim;
  const int b = idx / ((int64_t)kK * a.dim);
  const int t = a.seqlen - kK + k;
  float v;
  if (t >= 0) v = ldf((const T*)a.x + (int64_t)b * a.x_bs + (int64_t)t * a.x_ls + c);
  else v = a.conv_state_in ? a.conv_state_in[((int64_t)b * a.dim + c) * kK + (kK + t)] : 0.f;
  a.conv_state_out[idx] = v;
}

// backward: g = dout * silu'(pre); dx[t] = sum_k w[k] g[t+3-k]; dw, db partials
template <typename T, int CPT>
__global__ __launch_bounds__(256) void conv_bwd_kernel(const MttsConvBwdArgs a, float* __restrict__ part) {
  const MttsConvFwdArgs& f = a.f;
  const int c0 = (blockIdx.x * 256 + threadIdx.x) * CPT;
  if (c0 >= f.dim) return;
  const int b = blockIdx.z;
  const int t0 = blockIdx.y * kTT;
  const int L = f.seqlen;
  float w[kK][CPT], bias[CPT];
#pragma unroll
  for (int q = 0; q < CPT; ++q) {
#pragma unroll
    for (int k = 0; k < kK; ++k) w[k][q] = f.w[(c0 + q) * kK + k];
    bias[q] = f.bias ? f.bias[c0 + q] : 0.f;
  }
  float x0[CPT], x1[CPT], x2[CPT];
  load_x<T, CPT>(f, b, c0, t0 - 3, x0);
  load_x<T, CPT>(f, b, c0, t0 - 2, x1);
  load_x<T, CPT>(f, b, c0, t0 - 1, x2);
  float g0[CPT], g1[CPT], g2[CPT];
  float dw[kK][CPT], db[CPT];
#pragma unroll
  for (int q = 0; q < CPT; ++q) {
    g0[q] = g1[q] = g2[q] = 0.f;
    db[q] = 0.f;
#pragma unroll
    for (int k = 0; k < kK; ++k) dw[k][q] = 0.f;
  }
  const T* dout = (const T*)a.dout + (int64_t)b * a.dout_bs + c0;
  T* dx = (T*)a.dx + (int64_t)b * a.dx_bs + c0;
  // g beyond L is zero; dx[t-3] needs g[t-3 .. t]
  const int tlast = min(t0 + kTT + 3, L + 3);
  const int town = min(t0 + kTT, L);
  // x / dout of step t+2 and t+1 are in flight while step t computes
  float px[2][CPT], pg[2][CPT];
  auto fetch = [&](int t, float (&xx)[CPT], float (&gg)[CPT]) __attribute__((always_inline)) {
    if (t < L && t < tlast) {
      load_x<T, CPT>(f, b, c0, t, xx);
      ldv<T, CPT>(dout + (int64_t)t * a.dout_ls, gg);
    } else {
#pragma unroll
      for (int q = 0; q < CPT; ++q) { xx[q] = 0.f; gg[q] = 0.f; }
    }
  };
  fetch(t0, px[0], pg[0]);
  fetch(t0 + 1, px[1], pg[1]);
#pragma unroll 2
  for (int t = t0; t < tlast; ++t) {
    float x3[CPT], go[CPT], g[CPT];
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
      x3[q] = px[0][q]; go[q] = pg[0][q];
      px[0][q] = px[1][q]; pg[0][q] = pg[1][q];
    }
    fetch(t + 2, px[1], pg[1]);
    const bool own = t < town;
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
      float v = fmaf(w[0][q], x0[q], fmaf(w[1][q], x1[q], fmaf(w[2][q], x2[q], fmaf(w[3][q], x3[q], bias[q]))));
      float gg = go[q];
      if (f.silu) {
        const float s = sigmoid_f(v);
        gg *= s * (1.f + v * (1.f - s));
      }
      g[q] = gg;
      if (own) {
        db[q] += gg;
        dw[0][q] = fmaf(gg, x0[q], dw[0][q]);
        dw[1][q] = fmaf(gg, x1[q], dw[1][q]);
        dw[2][q] = fmaf(gg, x2[q], dw[2][q]);
        dw[3][q] = fmaf(gg, x3[q], dw[3][q]);
      }
    }
    // dx at t-3 = w3 g[t-3] + w2 g[t-2] + w1 g[t-1] + w0 g[t]
    if (t - 3 >= t0) {
      float o[CPT];
#pragma unroll
      for (int q = 0; q < CPT; ++q) o[q] = fmaf(w[3][q], g0[q], fmaf(w[2][q], g1[q], fmaf(w[1][q], g2[q], w[0][q] * g[q])));
      stv<T, CPT>(dx + (int64_t)(t - 3) * a.dx_ls, o);
    }
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
      x0[q] = x1[q]; x1[q] = x2[q]; x2[q] = x3[q];
      g0[q] = g1[q]; g1[q] = g2[q]; g2[q] = g[q];
    }
  }
  float* pp = part + ((int64_t)(b * gridDim.y + blockIdx.y) * f.dim + c0) * (kK + 1);
#pragma unroll
  for (int q = 0; q < CPT; ++q) {
#pragma unroll
    for (int k = 0; k < kK; ++k) pp[q * (kK + 1) + k] = dw[k][q];
    pp[q * (kK + 1) + kK] = db[q];
  }
}

__global__ void conv_bwd_split(const float* __restrict__ sums, int dim, float* dw, float* db) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= dim * (kK + 1)) return;
  const int c = idx / (kK + 1), k = idx % (kK + 1);
  if (k < kK) dw[c * kK + k] = sums[idx];
  else if (db) db[c] = sums[idx];
}

template <typename T>
static bool vec_ok(const MttsConvFwdArgs* a, int cpt) {
  const int es = sizeof(T);
  return a->dim % cpt == 0 && (uintptr_t)a->x % 16 == 0 && (uintptr_t)a->out % 16 == 0 &&
         (a->x_ls * es) % 16 == 0 && (a->x_bs * es) % 16 == 0 && (a->out_ls * es) % 16 == 0 &&
         (a->out_bs * es) % 16 == 0;
}

static int check_conv(const MttsConvFwdArgs* a) {
  MTTS_CHECK(a && a->x && a->w && a->out, "conv1d: null tensor");
  MTTS_CHECK(a->batch > 0 && a->dim > 0 && a->seqlen >= 0, "conv1d: bad sizes");
  if (a->width != kK) {
    set_error("conv1d: width=%d unsupported (fast path needs 4)", a->width);
    return MTTS_EUNSUPPORTED;
  }
  MTTS_CHECK(a->dtype == MTTS_F32 || a->dtype == MTTS_BF16, "conv1d: bad dtype");
  return MTTS_OK;
}

template <typename T, int CPT>
static void launch_fwd(const MttsConvFwdArgs* a, hipStream_t st) {
  dim3 grid((a->dim / CPT + 255) / 256, (a->seqlen + kTT - 1) / kTT, a->batch);
  hipLaunchKernelGGL((conv_fwd_kernel<T, CPT>), grid, dim3(256), 0, st, *a);
}

}  // namespace mtts

using namespace mtts;

extern "C" int mtts_causal_conv1d_fwd(const MttsConvFwdArgs* a, void* stream) {
  int rc = check_conv(a);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (a->seqlen > 0) {
    if (a->dtype == MTTS_F32) {
      if (vec_ok<float>(a, 4)) launch_fwd<float, 4>(a, st);
      else launch_fwd<float, 1>(a, st);
    } else {
      if (vec_ok<bf16_t>(a, 8)) launch_fwd<bf16_t, 8>(a, st);
      else launch_fwd<bf16_t, 1>(a, st);
    }
    MTTS_LAUNCH_CHECK("causal_conv1d_fwd");
  }
  if (a->conv_state_out) {
    const int64_t n = (int64_t)a->batch * a->dim * kK;
    if (a->dtype == MTTS_F32) hipLaunchKernelGGL(conv_state_kernel<float>, dim3((n + 255) / 256), dim3(256), 0, st, *a);
    else hipLaunchKernelGGL(conv_state_kernel<bf16_t>, dim3((n + 255) / 256), dim3(256), 0, st, *a);
    MTTS_LAUNCH_CHECK("causal_conv1d_state");
  }
  return MTTS_OK;
}

extern "C" int64_t mtts_causal_conv1d_bwd_workspace(int batch, int dim, int seqlen, int width) {
  (void)width;
  const int64_t ntile = (seqlen + kTT - 1) / kTT;
  return ((int64_t)batch * ntile + 1) * dim * (kK + 1) * 4 + 256;
}

template <typename T, int CPT>
static void launch_bwd(const MttsConvBwdArgs* a, hipStream_t st, float* part) {
  dim3 grid((a->f.dim / CPT + 255) / 256, (a->f.seqlen + kTT - 1) / kTT, a->f.batch);
  hipLaunchKernelGGL((conv_bwd_kernel<T, CPT>), grid, dim3(256), 0, st, *a, part);
}

extern "C" int mtts_causal_conv1d_bwd(const MttsConvBwdArgs* a, void* stream) {
  MTTS_CHECK(a, "conv1d_bwd: null args");
  int rc = check_conv(&a->f);
  if (rc) return rc;
  MTTS_CHECK(a->dout && a->dx && a->dw && a->workspace, "conv1d_bwd: null tensor");
  const MttsConvFwdArgs& f = a->f;
  if (f.seqlen == 0) return MTTS_OK;
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)a->workspace;
  const int es = f.dtype == MTTS_F32 ? 4 : 2;
  const int cpt = f.dtype == MTTS_F32 ? 4 : 8;
  const bool vec = f.dim % cpt == 0 && (uintptr_t)f.x % 16 == 0 && (uintptr_t)a->dout % 16 == 0 &&
                   (uintptr_t)a->dx % 16 == 0 && (f.x_ls * es) % 16 == 0 && (f.x_bs * es) % 16 == 0 &&
                   (a->dout_ls * es) % 16 == 0 && (a->dout_bs * es) % 16 == 0 && (a->dx_ls * es) % 16 == 0 &&
                   (a->dx_bs * es) % 16 == 0;
  if (f.dtype == MTTS_F32) {
    if (vec) launch_bwd<float, 4>(a, st, part);
    else launch_bwd<float, 1>(a, st, part);
  } else {
    if (vec) launch_bwd<bf16_t, 8>(a, st, part);
    else launch_bwd<bf16_t, 1>(a, st, part);
  }
  MTTS_LAUNCH_CHECK("causal_conv1d_bwd");
  const int nparts = f.batch * ((f.seqlen + kTT - 1) / kTT);
  float* sums = part + (int64_t)nparts * f.dim * (kK + 1);
  colsum(part, nparts, nparts, (int64_t)f.dim * (kK + 1), f.dim * (kK + 1), sums, 0, st);
  hipLaunchKernelGGL(conv_bwd_split, dim3((f.dim * (kK + 1) + 255) / 256), dim3(256), 0, st, sums, f.dim, a->dw,
                     a->dbias);
  MTTS_LAUNCH_CHECK("causal_conv1d_bwd_reduce");
  return MTTS_OK;
}
