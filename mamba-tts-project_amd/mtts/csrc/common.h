// Shared device/host helpers for libmtts (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>

#include "mtts.h"

namespace mtts {

// ---------------------------------------------------------------- errors
void set_error(const char* fmt, ...);
// kernel-path override (mtts_set_override; MTTS_OVR_AUTO = -1 when unset)
int override_of(int key);

// out[g * out_gstride + c] = sum over partials p in [g*ppg, (g+1)*ppg) of part[p * pstride + c]
void colsum(const float* part, int nparts, int ppg, int64_t pstride, int ncols, float* out, int64_t out_gstride,
            hipStream_t st);
struct ColsumJob {
  const float* part;
  float* out;
  int nparts, ppg;
  int64_t out_gstride;
};
// up to 5 colsum jobs over slabs of one width and part stride, one launch
void colsum_multi(const ColsumJob* jobs, int n, int ncols, int64_t pstride, hipStream_t st);

#define MTTS_CHECK(cond, ...)                                                 \
  do {                                                                        \
    if (!(cond)) {                                                            \
      ::mtts::set_error(__VA_ARGS__);                                         \
      return MTTS_EINVAL;                                                     \
    }                                                                         \
  } while (0)

#define MTTS_LAUNCH_CHECK(name)                                               \
  do {                                                                        \
    hipError_t e_ = hipGetLastError();                                        \
    if (e_ != hipSuccess) {                                                   \
      ::mtts::set_error("%s: launch failed: %s", name, hipGetErrorString(e_)); \
      return MTTS_ELAUNCH;                                                    \
    }                                                                         \
  } while (0)

// decode projections on packed weights (gemv.hip), called by mtts_gemm_rows
int launch_gemv_packed(const MttsRowsArgs* a, hipStream_t st);

// Packed ACTIVATION image of a decode-step operand (<= 32 rows, K columns,
// K % 32 == 0): the v_mfma_f32_16x16x32_bf16 B fragments of the packed
// projection kernel in load order, so its operand loads are coalesced KiB
// like the weights': element (m, k) lives at
//   ((k / 32 * 2 + m / 16) * 64 + (k / 8 % 4) * 16 + m % 16) * 8 + k % 8.
// 32 * K elements; rows >= M are never written (they only feed output rows
// that are never stored).
__host__ __device__ __forceinline__ int64_t xpk_index(int m, int k) {
  return ((int64_t)((k >> 5) * 2 + (m >> 4)) * 64 + ((k >> 3) & 3) * 16 + (m & 15)) * 8 + (k & 7);
}

// ---------------------------------------------------------------- dtypes
typedef uint16_t bf16_t;

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 h = (__bf16)f;  // v_cvt_pk_bf16_f32 (RNE, NaN-preserving)
  return *reinterpret_cast<bf16_t*>(&h);
}

template <typename T> struct IO;
template <> struct IO<float> {
  static __device__ __forceinline__ float ld(const float* p) { return *p; }
  static __device__ __forceinline__ void st(float* p, float v) { *p = v; }
};
template <> struct IO<bf16_t> {
  static __device__ __forceinline__ float ld(const bf16_t* p) { return bf2f(*p); }
  static __device__ __forceinline__ void st(bf16_t* p, float v) { *p = f2bf(v); }
};
template <typename T> __device__ __forceinline__ float ldf(const T* p) { return IO<T>::ld(p); }
template <typename T> __device__ __forceinline__ void stf(T* p, float v) { IO<T>::st(p, v); }

// ---------------------------------------------------------------- math
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

__device__ __forceinline__ float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * kLog2e); }
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

// softplus with torch's threshold (x > 20 -> x); accurate for very negative x
__device__ __forceinline__ float softplus_f(float x) {
  float e = __builtin_amdgcn_exp2f(fminf(x, 20.f) * kLog2e);
  float lg = __builtin_amdgcn_logf(1.f + e) * kLn2;  // v_log_f32 is log2
  float sm = e * (1.f - 0.5f * e);                   // log1p(e) for tiny e
  float r = e < 1e-3f ? sm : lg;
  return x > 20.f ? x : r;
}
// d softplus / dx = sigmoid(x)  (1 for x > 20, matching torch's threshold)
__device__ __forceinline__ float softplus_grad(float x) {
  float s = fast_rcp(1.f + __builtin_amdgcn_exp2f(-x * kLog2e));
  return x > 20.f ? 1.f : s;
}
__device__ __forceinline__ float sigmoid_f(float x) { return fast_rcp(1.f + __builtin_amdgcn_exp2f(-x * kLog2e)); }
__device__ __forceinline__ float silu_f(float x) { return x * sigmoid_f(x); }

// ---------------------------------------------------------------- workgroup barrier
// Every workgroup barrier of the library: this wave's own LDS operations
// complete (lgkmcnt(0)), THEN s_barrier.  hipcc's __syncthreads() alone is a
// bare s_barrier on gfx950 (LLVM assumes every wave observes LDS operations in
// one global order and drops the wait), but a ds_write issued before it is
// not always visible to another wave's ds_read issued after it:
// tools/ubench/lds_order_probe.hip counted 836,032 stale neighbour-wave
// reads in 2.6e9 with the bare barrier and 0 with the wait
// (profiles/r05_lds_order_probe.txt), and the scan backward's carry kernel
// drifted from run to run under GPU sharing (tools/dbg/race_probe.py).
// vmcnt / expcnt are left alone (in-flight LDS-DMA keeps its own counted
// waits).
__device__ __forceinline__ void block_sync() {
  __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0); vmcnt(63), expcnt(7): no wait
  __syncthreads();
}

// ---------------------------------------------------------------- cross-lane
// DPP quad_perm controls
constexpr int kQuadXor1 = 0xB1;  // [1,0,3,2]
constexpr int kQuadXor2 = 0x4E;  // [2,3,0,1]
template <int L> constexpr int quad_bcast() { return L * 0x55; }
constexpr int kRowRor4 = 0x124;
constexpr int kRowRor8 = 0x128;
constexpr int kRowRor12 = 0x12C;

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
// v_permlane32_swap(v, v) returns {a, b}: a = v with its upper half replaced
// by the lower half, b = v with its lower half replaced by the upper half.
__device__ __forceinline__ float xor32(float v, int lane) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float((lane & 32) ? r[0] : r[1]);
}
// v_permlane16_swap(v, v): a = rows [0,0,2,2], b = rows [1,1,3,3] of v.
__device__ __forceinline__ float xor16(float v, int lane) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float((lane & 16) ? r[0] : r[1]);
}
// v + v[lane ^ 16] and v + v[lane ^ 32] without selects
__device__ __forceinline__ float sum_xor16(float v) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float sum_xor32(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// max(v, v[lane ^ 16]) / max(v, v[lane ^ 32]) without selects (both swap
// outputs are {own, partner})
__device__ __forceinline__ float max_xor16(float v) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float max_xor32(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
constexpr int kQuadRev = 0x1B;         // [3,2,1,0]: lane ^ 3
constexpr int kRowHalfMirror = 0x141;  // lane i <- lane 7 - i within 8: lane ^ 7
// lane ^ 4 = (lane ^ 3) ^ 7: two DPP movs, no select (the second one fuses
// into a following add / max as its DPP source)
__device__ __forceinline__ float xor4(float v, int lane) {
  (void)lane;
  return dpp<kRowHalfMirror>(dpp<kQuadRev>(v));
}
__device__ __forceinline__ float xor8(float v) { return dpp<kRowRor8>(v); }

__device__ __forceinline__ float wave_sum(float v) {
  v += dpp<kQuadXor1>(v);
  v += dpp<kQuadXor2>(v);
  v += xor4(v, threadIdx.x & 63);
  v += xor8(v);
  v = sum_xor16(v);
  v = sum_xor32(v);
  return v;
}

// 16-byte row pieces as fp32 (LayerNorm rows, the decode LayerNorm tail)
template <typename T, int VEC>
__device__ __forceinline__ void ld_vec(const T* p, float (&o)[VEC]) {
  if constexpr (VEC * sizeof(T) == 16) {
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
    for (int q = 0; q < VEC; ++q) o[q] = ldf(p + q);
  }
}
template <typename T, int VEC>
__device__ __forceinline__ void st_vec(T* p, const float (&v)[VEC]) {
  if constexpr (VEC * sizeof(T) == 16) {
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
    for (int q = 0; q < VEC; ++q) stf(p + q, v[q]);
  }
}

}  // namespace mtts
