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

#include <type_traits>

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
  } else if constexpr (sizeof(T) == 2 && CPT == 4) {
    *reinterpret_cast<uint2*>(p) = make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                                              (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
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

// ---------------------------------------------------------------- tiled forms
// The kernels above walk a 32-step tile with one load per step: each load is
// issued behind the previous step's store (which may alias it), so a thread
// has one load in flight and the kernel runs latency-bound (C2: fwd 43 us,
// bwd 84 us per call for 67 MB per operand).  The tiled forms issue ALL of a
// tile's 16-byte row loads before any arithmetic or store (x rows t0-3 ..
// t0+TT-1 for the forward; x rows t0-3 .. t0+TT+2 and dout rows t0 .. t0+TT+2
// for the backward), so a wave keeps TT+3 (2TT+9) loads in flight.
//
// Backward block = 8 waves = 8 consecutive 8-step tiles of the same 64 x CPT
// channels: the dw / db partials of the 8 tiles are summed through LDS, so
// the partial slab has one row per 64 steps (C2: 10 MB instead of 21).

typedef int i32x4c __attribute__((ext_vector_type(4)));

template <typename T, int CPT>
using rawv_t = typename std::conditional<sizeof(T) * CPT == 16, uint4, uint2>::type;

template <typename T, int CPT>
__device__ __forceinline__ void unpack16(const uint2& v, float (&o)[CPT]) {   // 4 bf16 channels
  static_assert(sizeof(T) == 2 && CPT == 4, "8-byte rows: bf16 x 4");
  o[0] = __uint_as_float(v.x << 16); o[1] = __uint_as_float(v.x & 0xffff0000u);
  o[2] = __uint_as_float(v.y << 16); o[3] = __uint_as_float(v.y & 0xffff0000u);
}
template <typename T, int CPT>
__device__ __forceinline__ void unpack16(const uint4& v, float (&o)[CPT]) {
  if constexpr (sizeof(T) == 4) {
    o[0] = __uint_as_float(v.x); o[1] = __uint_as_float(v.y); o[2] = __uint_as_float(v.z); o[3] = __uint_as_float(v.w);
  } else {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) { o[2 * q] = __uint_as_float(w[q] << 16); o[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u); }
  }
}

// x value at t < 0: the conv_state_in history column (or 0)
template <int CPT>
__device__ __forceinline__ void hist_x(const MttsConvFwdArgs& a, int b, int c0, int t, float (&o)[CPT]) {
#pragma unroll
  for (int q = 0; q < CPT; ++q) o[q] = a.conv_state_in ? a.conv_state_in[((int64_t)b * a.dim + c0 + q) * kK + (kK + t)] : 0.f;
}

template <typename T, int CPT, int TT>
__global__ __launch_bounds__(256) void conv_fwd_tile_kernel(const MttsConvFwdArgs a) {
  const int c0 = (blockIdx.x * 256 + threadIdx.x) * CPT;
  if (c0 >= a.dim) return;
  const int b = blockIdx.z;
  const int t0 = blockIdx.y * TT;   // block-uniform: the row origins below are scalar offsets
  const int L = a.seqlen;
  // x rows t0-3 .. t0+TT-1 and the output rows as buffer accesses (round 5, as
  // the tiled backward): descriptors over the block's columns of the batch row,
  // the lane's column in the vector offset, the row origin in the scalar
  // offset.  gfx950's range check covers voffset + soffset without 32-bit
  // wrap (tools/ubench/buffer_oob_probe.hip, profiles/r05_buffer_oob_probe.txt):
  // rows before 0 / at or past L read 0 (rows < 0 are replaced by the prefix
  // state below) and stores past L are dropped -- no clamps or 64-bit row
  // arithmetic per access (host: row spans below 2 GiB)
  constexpr int ES = (int)sizeof(T);
  const int cb = blockIdx.x * 256 * CPT, ncol = min(256 * CPT, a.dim - cb);
  auto span = [&](int64_t ls) { return (int)(((int64_t)(L - 1) * ls + ncol) * ES); };
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<T*>((const T*)a.x + (int64_t)b * a.x_bs + cb), 0, span(a.x_ls), 0x00020000);
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
      (T*)a.out + (int64_t)b * a.out_bs + cb, 0, span(a.out_ls), 0x00020000);
  const uint32_t vcol = (uint32_t)((c0 - cb) * ES);
  const int xls = (int)a.x_ls * ES, ols = (int)a.out_ls * ES;
  uint4 raw[TT + 3];
#pragma unroll
  for (int i = 0; i < TT + 3; ++i)
    raw[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rx, vcol, (t0 - 3 + i) * xls, 0));
  float w[kK][CPT], bias[CPT];
#pragma unroll
  for (int q = 0; q < CPT; ++q) {
    const float4 wq = *reinterpret_cast<const float4*>(a.w + (c0 + q) * kK);
    w[0][q] = wq.x; w[1][q] = wq.y; w[2][q] = wq.z; w[3][q] = wq.w;
    bias[q] = a.bias ? a.bias[c0 + q] : 0.f;
  }
  float x0[CPT], x1[CPT], x2[CPT];
  if (t0 == 0) {
    hist_x<CPT>(a, b, c0, -3, x0);
    hist_x<CPT>(a, b, c0, -2, x1);
    hist_x<CPT>(a, b, c0, -1, x2);
  } else {
    unpack16<T, CPT>(raw[0], x0);
    unpack16<T, CPT>(raw[1], x1);
    unpack16<T, CPT>(raw[2], x2);
  }
#pragma unroll
  for (int s = 0; s < TT; ++s) {
    float x3[CPT], o[CPT];
    unpack16<T, CPT>(raw[s + 3], x3);
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
      const float v = fmaf(w[0][q], x0[q], fmaf(w[1][q], x1[q], fmaf(w[2][q], x2[q], fmaf(w[3][q], x3[q], bias[q]))));
      o[q] = a.silu ? silu_f(v) : v;
      x0[q] = x1[q]; x1[q] = x2[q]; x2[q] = x3[q];
    }
    uint4 wv;
    if constexpr (sizeof(T) == 4) {
      wv = make_uint4(__float_as_uint(o[0]), __float_as_uint(o[1]), __float_as_uint(o[2]), __float_as_uint(o[3]));
    } else {
      uint32_t qv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) qv[k] = (uint32_t)f2bf(o[2 * k]) | ((uint32_t)f2bf(o[2 * k + 1]) << 16);
      wv = make_uint4(qv[0], qv[1], qv[2], qv[3]);
    }
    // the row origin goes into the VECTOR offset for stores: with a register
    // soffset hipcc omits the wait states a VALU write of a >8-byte store's data
    // registers needs after the store, and on gfx950 lanes 12-15 of each 16
    // then stored the next row's values (the round-4 revert)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4c, wv), ro, vcol + (uint32_t)((t0 + s) * ols), 0, 0);
  }
}

template <typename T, int CPT, int TT>
__global__ __launch_bounds__(512) void conv_bwd_tile_kernel(const MttsConvBwdArgs a, float* __restrict__ part) {
  const MttsConvFwdArgs& f = a.f;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c0 = (blockIdx.x * 64 + lane) * CPT;
  const bool cok = c0 < f.dim;
  const int cc = cok ? c0 : 0;       // lanes past dim run on channel 0 and store nothing (no early exit: LDS sum below)
  const int b = blockIdx.z;
  const int t0 = __builtin_amdgcn_readfirstlane((blockIdx.y * 8 + wave) * TT);   // wave-uniform (scalar offsets)
  const int L = f.seqlen;
  // x rows t0-3 .. t0+TT+2, dout rows t0 .. t0+TT+2 as buffer loads (round
  // 4): descriptors over the block's columns of the batch row, the lane's
  // column in the vector offset, the row origin in the scalar offset; rows
  // before 0 or at / past L fall outside the range and read 0 (rows < 0 are
  // replaced by the prefix state below, rows >= L have g = 0) -- no clamps or
  // 64-bit row arithmetic per load (host: row spans below 2 GiB)
  using RV = rawv_t<T, CPT>;
  constexpr int ES = (int)sizeof(T);
  const int cb = blockIdx.x * 64 * CPT, ncol = min(64 * CPT, f.dim - cb);
  auto span = [&](int64_t ls) { return (int)(((int64_t)(L - 1) * ls + ncol) * ES); };
  const __amdgpu_buffer_rsrc_t rxs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<T*>((const T*)f.x + (int64_t)b * f.x_bs + cb), 0, span(f.x_ls), 0x00020000);
  const __amdgpu_buffer_rsrc_t rgs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<T*>((const T*)a.dout + (int64_t)b * a.dout_bs + cb), 0, span(a.dout_ls), 0x00020000);
  const uint32_t vcol = (uint32_t)(lane * CPT * ES);
  auto ld = [&](const __amdgpu_buffer_rsrc_t& r, int row, int64_t ls) __attribute__((always_inline)) -> RV {
    const int so = (int)(row * ls * ES);
    if constexpr (sizeof(RV) == 16) return __builtin_bit_cast(RV, __builtin_amdgcn_raw_buffer_load_b128(r, vcol, so, 0));
    else return __builtin_bit_cast(RV, __builtin_amdgcn_raw_buffer_load_b64(r, vcol, so, 0));
  };
  RV rx[TT + 6], rg[TT + 3];
#pragma unroll
  for (int i = 0; i < TT + 6; ++i) rx[i] = ld(rxs, t0 - 3 + i, f.x_ls);
#pragma unroll
  for (int i = 0; i < TT + 3; ++i) rg[i] = ld(rgs, t0 + i, a.dout_ls);
  float w[kK][CPT], bias[CPT];
#pragma unroll
  for (int q = 0; q < CPT; ++q) {
    const float4 wq = *reinterpret_cast<const float4*>(f.w + (cc + q) * kK);
    w[0][q] = wq.x; w[1][q] = wq.y; w[2][q] = wq.z; w[3][q] = wq.w;
    bias[q] = f.bias ? f.bias[cc + q] : 0.f;
  }
  float x0[CPT], x1[CPT], x2[CPT];
  if (t0 == 0) {
    hist_x<CPT>(f, b, cc, -3, x0);
    hist_x<CPT>(f, b, cc, -2, x1);
    hist_x<CPT>(f, b, cc, -1, x2);
  } else {
    unpack16<T, CPT>(rx[0], x0);
    unpack16<T, CPT>(rx[1], x1);
    unpack16<T, CPT>(rx[2], x2);
  }
  float g0[CPT], g1[CPT], g2[CPT], dw[kK][CPT], db[CPT];
#pragma unroll
  for (int q = 0; q < CPT; ++q) {
    g0[q] = g1[q] = g2[q] = 0.f;
    db[q] = 0.f;
#pragma unroll
    for (int k = 0; k < kK; ++k) dw[k][q] = 0.f;
  }
  T* dx = (T*)a.dx + (int64_t)b * a.dx_bs + cc;
  // step s (time t0 + s): g[t] = dout[t] * silu'(pre[t]) for t < L, else 0;
  // dx[t-3] = w3 g[t-3] + w2 g[t-2] + w1 g[t-1] + w0 g[t] for t-3 in the tile
#pragma unroll
  for (int s = 0; s < TT + 3; ++s) {
    const int t = t0 + s;
    const bool live = t < L;
    const bool own = s < TT && live;
    float x3[CPT], go[CPT], g[CPT];
    unpack16<T, CPT>(rx[s + 3], x3);
    unpack16<T, CPT>(rg[s], go);
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
      const float v = fmaf(w[0][q], x0[q], fmaf(w[1][q], x1[q], fmaf(w[2][q], x2[q], fmaf(w[3][q], x3[q], bias[q]))));
      float gg = live ? go[q] : 0.f;
      if (f.silu) {
        const float sg = sigmoid_f(v);
        gg *= sg * (1.f + v * (1.f - sg));
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
    if (s >= 3 && cok && t - 3 < L) {
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
  // sum the 8 waves' (time tiles') partials: (K + 1) * CPT values per lane
  constexpr int NV = (kK + 1) * CPT;
  __shared__ float red[7][NV][64];
  if (wave > 0) {
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
#pragma unroll
      for (int k = 0; k < kK; ++k) red[wave - 1][q * (kK + 1) + k][lane] = dw[k][q];
      red[wave - 1][q * (kK + 1) + kK][lane] = db[q];
    }
  }
  block_sync();
  if (wave == 0 && cok) {
    float* pp = part + ((int64_t)(b * gridDim.y + blockIdx.y) * f.dim + c0) * (kK + 1);
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
#pragma unroll
      for (int k = 0; k <= kK; ++k) {
        float v = k < kK ? dw[k][q] : db[q];
#pragma unroll
        for (int j = 0; j < 7; ++j) v += red[j][q * (kK + 1) + k][lane];
        pp[q * (kK + 1) + k] = v;
      }
    }
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

constexpr int kFwdTT = 16;   // tiled forward: steps per thread
constexpr int kBwdTT = 8;    // tiled backward: steps per wave (8 waves = 64 steps per block)

static bool tiled_off() { return override_of(MTTS_OVR_CONV_UNTILED) == 1; }

template <typename T, int CPT>
static void launch_fwd(const MttsConvFwdArgs* a, hipStream_t st) {
  if constexpr (sizeof(T) * CPT == 16) {
   // buffer-addressed rows: spans below 2 GiB
   auto fits = [&](int64_t ls) { return (int64_t)(a->seqlen + 16) * ls * (int64_t)sizeof(T) < (1ll << 31); };
   if (!tiled_off() && fits(a->x_ls) && fits(a->out_ls)) {
    dim3 grid((a->dim / CPT + 255) / 256, (a->seqlen + kFwdTT - 1) / kFwdTT, a->batch);
    hipLaunchKernelGGL((conv_fwd_tile_kernel<T, CPT, kFwdTT>), grid, dim3(256), 0, st, *a);
    return;
   }
  }
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
      if (vec_ok<float>(a, 4) && (uintptr_t)a->w % 16 == 0) launch_fwd<float, 4>(a, st);
      else launch_fwd<float, 1>(a, st);
    } else {
      if (vec_ok<bf16_t>(a, 8) && (uintptr_t)a->w % 16 == 0) launch_fwd<bf16_t, 8>(a, st);
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

// returns the number of partial rows written
template <typename T, int CPT>
static int launch_bwd(const MttsConvBwdArgs* a, hipStream_t st, float* part, bool tiled) {
  if constexpr (sizeof(T) * CPT >= 8) {
   if (tiled) {
    dim3 grid((a->f.dim / CPT + 63) / 64, (a->f.seqlen + 8 * kBwdTT - 1) / (8 * kBwdTT), a->f.batch);
    hipLaunchKernelGGL((conv_bwd_tile_kernel<T, CPT, kBwdTT>), grid, dim3(512), 0, st, *a, part);
    return (int)(grid.y * grid.z);
   }
  }
  dim3 grid((a->f.dim / CPT + 255) / 256, (a->f.seqlen + kTT - 1) / kTT, a->f.batch);
  hipLaunchKernelGGL((conv_bwd_kernel<T, CPT>), grid, dim3(256), 0, st, *a, part);
  return (int)(grid.y * grid.z);
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
  // the tiled backward reads rows through buffer descriptors: spans below 2 GiB
  auto fits = [&](int64_t ls) { return (int64_t)(f.seqlen + 16) * ls * es < (1ll << 31); };
  const bool tiled = vec && (uintptr_t)f.w % 16 == 0 && !tiled_off() && fits(f.x_ls) && fits(a->dout_ls);
  int nparts;
  if (f.dtype == MTTS_F32) {
    if (vec) nparts = launch_bwd<float, 4>(a, st, part, tiled);
    else nparts = launch_bwd<float, 1>(a, st, part, false);
  } else {
    if (tiled) nparts = launch_bwd<bf16_t, 4>(a, st, part, true);   // 8-byte rows: half the live registers
    else if (vec) nparts = launch_bwd<bf16_t, 8>(a, st, part, false);
    else nparts = launch_bwd<bf16_t, 1>(a, st, part, false);
  }
  MTTS_LAUNCH_CHECK("causal_conv1d_bwd");
  float* sums = part + (int64_t)nparts * f.dim * (kK + 1);
  colsum(part, nparts, nparts, (int64_t)f.dim * (kK + 1), f.dim * (kK + 1), sums, 0, st);
  hipLaunchKernelGGL(conv_bwd_split, dim3((f.dim * (kK + 1) + 255) / 256), dim3(256), 0, st, sums, f.dim, a->dw,
                     a->dbias);
  MTTS_LAUNCH_CHECK("causal_conv1d_bwd_reduce");
  return MTTS_OK;
}
