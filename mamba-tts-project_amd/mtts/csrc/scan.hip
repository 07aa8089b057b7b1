// Selective scan forward / backward for gfx950.
//
// Replaces [upstream] mamba-ssm csrc/selective_scan (selective_scan_cuda.fwd
// / .bwd), reached from mamba_decoder.py:61/:63 through Mamba.forward.
// Math: SURVEY.md §8a rows a8/a9; oracle/mamba_ref.py::selective_scan_ref.
//
// Design (MI355X-first, not a port of the upstream CUDA BlockScan):
//  * Activations are channel-last (B, L, D), the layout the projections
//    produce, so a wave's 64 lanes read 64/P consecutive channels of ONE
//    timestep: every u/delta/z load and out store is coalesced.
//  * The recurrence runs SEQUENTIALLY along L inside each lane, with the
//    state h in registers; no cross-lane scan is needed.  The d_state = 16
//    states of a channel are split over P adjacent lanes (NS = 16/P each),
//    which multiplies the lane count by P for small B*D (C2: B*D = 16k).
//  * Per-channel scalar work (loads, softplus, silu gate, D skip, store) is
//    NOT replicated across the P lanes: the P lanes of a channel take P
//    consecutive timesteps each, and exchange delta / delta*u with DPP
//    quad_perm broadcasts; the per-step partial outputs are reduce-scattered
//    back with DPP so lane j finishes timestep t0+j.
//  * exp(delta*A) is one v_exp_f32 (log2(e) folded into A).
//  * Backward restarts from fwd checkpoints every SUB = 16 steps, replays the
//    chunk forward keeping h and exp(delta*A) in registers, then runs the
//    reverse recurrence.  dB/dC (sums over channels) are reduce-scattered
//    across the wave with DPP/permlane (no atomics), summed over the block's
//    waves in LDS, written as per-block slabs and reduced by a second
//    deterministic kernel.
#include "common.h"
#include <algorithm>
#include <utility>

namespace mtts {

constexpr int kN = 16;       // d_state
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kSub = 16;     // checkpoint chunk (timesteps)
constexpr int kBlock = 256;  // threads per block

// ------------------------------------------------------------- helpers
// static_for<N>(f): f(integral_constant<int, 0..N-1>) fully unrolled at compile time
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}
// A[c, n]: the fp32 tensor itself, or -exp(A_log[c, n]) when the caller
// passes A_log (a_is_log; the Mamba mixer's parameter, so no per-step
// exp / neg launches): one accurate expf per value, loaded once per thread
__device__ __forceinline__ float ld_A(const MttsScanFwdArgs& a, int64_t i) {
  const float v = a.A[i];
  return a.a_is_log ? -expf(v) : v;
}

template <int P, int S>
__device__ __forceinline__ float group_bcast(float v) {
  if constexpr (P == 1) {
    return v;
  } else if constexpr (P == 2) {
    return dpp<(S == 0 ? 0xA0 : 0xF5)>(v);  // [0,0,2,2] / [1,1,3,3]
  } else {
    return dpp<S * 0x55>(v);                // [S,S,S,S]
  }
}

// v[s] partial over this lane's states for step s -> lane j returns the
// full sum over the P lanes for step j.
template <int P>
__device__ __forceinline__ float group_reduce_scatter(const float (&v)[P], int j) {
  if constexpr (P == 1) {
    return v[0];
  } else if constexpr (P == 2) {
    float keep = j ? v[1] : v[0];
    float send = j ? v[0] : v[1];
    return keep + dpp<kQuadXor1>(send);
  } else {
    const bool hi = j & 2;
    float k0 = hi ? v[2] : v[0], k1 = hi ? v[3] : v[1];
    float s0 = hi ? v[0] : v[2], s1 = hi ? v[1] : v[3];
    k0 += dpp<kQuadXor2>(s0);
    k1 += dpp<kQuadXor2>(s1);
    const bool lo = j & 1;
    float keep = lo ? k1 : k0, send = lo ? k0 : k1;
    return keep + dpp<kQuadXor1>(send);
  }
}

template <int P>
__device__ __forceinline__ float group_allreduce(float v) {
  if constexpr (P >= 2) v += dpp<kQuadXor1>(v);
  if constexpr (P >= 4) v += dpp<kQuadXor2>(v);
  return v;
}

template <typename T, int NS>
__device__ __forceinline__ void load_vec(const T* p, float (&o)[NS]);

template <>
__device__ __forceinline__ void load_vec<float, 1>(const float* p, float (&o)[1]) { o[0] = *p; }
template <>
__device__ __forceinline__ void load_vec<float, 2>(const float* p, float (&o)[2]) {
  float2 v = *reinterpret_cast<const float2*>(p);
  o[0] = v.x; o[1] = v.y;
}
template <>
__device__ __forceinline__ void load_vec<bf16_t, 1>(const bf16_t* p, float (&o)[1]) { o[0] = bf2f(*p); }
template <>
__device__ __forceinline__ void load_vec<bf16_t, 2>(const bf16_t* p, float (&o)[2]) {
  const uint32_t w = *reinterpret_cast<const uint32_t*>(p);
  o[0] = __uint_as_float(w << 16); o[1] = __uint_as_float(w & 0xffff0000u);
}
template <>
__device__ __forceinline__ void load_vec<float, 4>(const float* p, float (&o)[4]) {
  float4 v = *reinterpret_cast<const float4*>(p);
  o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
template <>
__device__ __forceinline__ void load_vec<float, 8>(const float* p, float (&o)[8]) {
  float4 v = *reinterpret_cast<const float4*>(p);
  float4 w = *reinterpret_cast<const float4*>(p + 4);
  o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w; o[4] = w.x; o[5] = w.y; o[6] = w.z; o[7] = w.w;
}
template <>
__device__ __forceinline__ void load_vec<float, 16>(const float* p, float (&o)[16]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float4 v = *reinterpret_cast<const float4*>(p + 4 * q);
    o[4 * q] = v.x; o[4 * q + 1] = v.y; o[4 * q + 2] = v.z; o[4 * q + 3] = v.w;
  }
}
__device__ __forceinline__ void unpack_bf2(uint32_t w, float& a, float& b) {
  a = __uint_as_float(w << 16);
  b = __uint_as_float(w & 0xffff0000u);
}
template <>
__device__ __forceinline__ void load_vec<bf16_t, 4>(const bf16_t* p, float (&o)[4]) {
  uint2 v = *reinterpret_cast<const uint2*>(p);
  unpack_bf2(v.x, o[0], o[1]); unpack_bf2(v.y, o[2], o[3]);
}
template <>
__device__ __forceinline__ void load_vec<bf16_t, 8>(const bf16_t* p, float (&o)[8]) {
  uint4 v = *reinterpret_cast<const uint4*>(p);
  unpack_bf2(v.x, o[0], o[1]); unpack_bf2(v.y, o[2], o[3]);
  unpack_bf2(v.z, o[4], o[5]); unpack_bf2(v.w, o[6], o[7]);
}
template <>
__device__ __forceinline__ void load_vec<bf16_t, 16>(const bf16_t* p, float (&o)[16]) {
  uint4 v = *reinterpret_cast<const uint4*>(p);
  uint4 w = *reinterpret_cast<const uint4*>(p + 8);
  unpack_bf2(v.x, o[0], o[1]); unpack_bf2(v.y, o[2], o[3]);
  unpack_bf2(v.z, o[4], o[5]); unpack_bf2(v.w, o[6], o[7]);
  unpack_bf2(w.x, o[8], o[9]); unpack_bf2(w.y, o[10], o[11]);
  unpack_bf2(w.z, o[12], o[13]); unpack_bf2(w.w, o[14], o[15]);
}

template <int NS>
__device__ __forceinline__ void store_vec(float* p, const float (&v)[NS]) {
#pragma unroll
  for (int q = 0; q < NS / 4; ++q)
    *reinterpret_cast<float4*>(p + 4 * q) = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
}

// Prefetched activations stay in their storage format until used: converting
// right after the load would make the compiler wait for the load there (the
// prefetch would then cost a full memory latency per group).
template <typename T> struct RawT;
template <> struct RawT<float> { using type = float; };
template <> struct RawT<bf16_t> { using type = uint32_t; };
template <typename T> using raw_t = typename RawT<T>::type;
__device__ __forceinline__ float cvt_raw(float v) { return v; }
__device__ __forceinline__ float cvt_raw(uint32_t v) { return __uint_as_float(v << 16); }
template <typename T>
__device__ __forceinline__ raw_t<T> ldr(const T* p) { return (raw_t<T>)*p; }

// N consecutive elements as raw 32-bit words (one vector load), unpacked at use
template <typename T, int N>
struct RawVec {
  static constexpr int W = (N * (int)sizeof(T) + 3) / 4;
  static_assert(W == 1 || W == 2 || W == 4 || W == 8, "RawVec width");
  uint32_t w[W];
  __device__ __forceinline__ void load(const T* p) {
    if constexpr (N * sizeof(T) == 2) {
      w[0] = (uint32_t)*p;  // one bf16
    } else if constexpr (W == 1) {
      w[0] = *reinterpret_cast<const uint32_t*>(p);
    } else if constexpr (W == 2) {
      const uint2 v = *reinterpret_cast<const uint2*>(p);
      w[0] = v.x; w[1] = v.y;
    } else {
#pragma unroll
      for (int q = 0; q < W / 4; ++q) {
        const uint4 v = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint32_t*>(p) + 4 * q);
        w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
      }
    }
  }
  __device__ __forceinline__ void unpack(float (&o)[N]) const {
    if constexpr (N * sizeof(T) == 2) {
      o[0] = __uint_as_float(w[0] << 16);
    } else if constexpr (sizeof(T) == 4) {
#pragma unroll
      for (int i = 0; i < N; ++i) o[i] = __uint_as_float(w[i]);
    } else {
#pragma unroll
      for (int i = 0; i < W; ++i) unpack_bf2(w[i], o[2 * i], o[2 * i + 1]);
    }
  }
};

// ------------------------------------------------------------- forward
// L is cut into K segments of seg_len steps (K = 1 when B*D alone fills the
// chip).  MODE kState (pass 1) scans segments 0..K-2 from h = 0 and writes
// each segment's end state and sum(delta) to `seg`; MODE kFull (pass 2)
// seeds segment k with  H_k = exp(A*S_{k-1}) H_{k-1} + h_{k-1}  (H_0 = h0)
// and produces the outputs.  B/C tiles are staged once per block in LDS
// (fp32); u/delta/z of the next tile are prefetched into registers while the
// current tile computes.
enum { kFull = 0, kState = 1 };
constexpr int kTileG = 8;   // P-step groups per tile (carry kernel)
constexpr int kTileGF = 4;  // forward: groups per tile (kRing register sets live)
constexpr int kRing = 3;    // forward: register sets in the prefetch ring
using TrueT = std::integral_constant<bool, true>;
using FalseT = std::integral_constant<bool, false>;

template <int P, typename Tio, typename Tbc, int MODE, bool SP>
__global__ __launch_bounds__(kBlock, 4) void scan_fwd_kernel(const MttsScanFwdArgs a, const int seg_len,
                                                             float* __restrict__ seg) {
  constexpr int NS = kN / P;
  constexpr int G = kTileGF;
  constexpr int TT = G * P;                       // timesteps per tile
  constexpr int VPT = TT * 2 * kN / kBlock;       // staged B/C values per thread (= P)
  __shared__ __attribute__((aligned(16))) float sBC[2][TT * 2 * kN];

  const int j = threadIdx.x % P;
  // lanes past `dim` recompute channel dim-1 bit-identically (benign duplicate stores)
  const int c = min((int)(blockIdx.x * (kBlock / P) + threadIdx.x / P), a.dim - 1);
  const int b = blockIdx.y;
  const int k = blockIdx.z;
  const int L = a.seqlen;
  const int K = (L + seg_len - 1) / seg_len;
  const int t_begin = k * seg_len;
  const int t_end = min(L, t_begin + seg_len);

  // Addressing: uniform (SGPR) base per timestep + one 32-bit per-lane offset,
  // so loads/stores use the saddr form with no per-access VALU index math.
  const Tio* __restrict__ u0 = (const Tio*)a.u + (int64_t)b * a.u_bs;
  const Tio* __restrict__ d0 = (const Tio*)a.delta + (int64_t)b * a.delta_bs;
  const bool has_z = MODE == kFull && a.z != nullptr;
  // without z the z loads read u (never used): no conditional loads in the loop
  const Tio* __restrict__ z0 = has_z ? (const Tio*)a.z + (int64_t)b * a.z_bs : u0;
  const int64_t z_ls = has_z ? a.z_ls : a.u_ls;
  Tio* __restrict__ o0 = (Tio*)a.out + (int64_t)b * a.out_bs;
  const uint32_t lu = (uint32_t)(j * a.u_ls + c), ld = (uint32_t)(j * a.delta_ls + c);
  const uint32_t lz = (uint32_t)(j * z_ls + c), lo = (uint32_t)(j * a.out_ls + c);

  // this thread's slice of the cooperative B/C staging
  const int e0 = threadIdx.x * VPT;
  const int st_s = e0 / (2 * kN), st_col = e0 % (2 * kN);
  const Tbc* __restrict__ st0 = st_col < kN ? (const Tbc*)a.Bm + (int64_t)b * a.B_bs
                                            : (const Tbc*)a.Cm + (int64_t)b * a.C_bs;
  const int64_t st_ls = st_col < kN ? a.B_ls : a.C_ls;
  const uint32_t lst = (uint32_t)(st_s * st_ls + (st_col % kN));

  float A2[NS], h[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) A2[i] = ld_A(a, (int64_t)c * kN + j * NS + i) * kLog2e;
  const float Dc = a.D ? a.D[c] : 0.f;
  const float bias = a.delta_bias ? a.delta_bias[c] : 0.f;
  float S = 0.f;
  if constexpr (MODE == kFull) {
#pragma unroll
    for (int i = 0; i < NS; ++i) h[i] = a.h0 ? a.h0[((int64_t)b * a.dim + c) * kN + j * NS + i] : 0.f;
    for (int kk = 0; kk < k; ++kk) {
      const float* sp = seg + (((int64_t)b * K + kk) * a.dim + c) * (kN + 1);
      const float Sk = sp[kN];
#pragma unroll
      for (int i = 0; i < NS; ++i) h[i] = fmaf(__builtin_amdgcn_exp2f(A2[i] * Sk), h[i], sp[j * NS + i]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < NS; ++i) h[i] = 0.f;
  }
  const int nck = (MODE == kFull && a.ckpt) ? (L + a.ckpt_chunk - 1) / a.ckpt_chunk : 0;
  float* __restrict__ ck0 = nck ? a.ckpt + (int64_t)b * nck * a.dim * kN : nullptr;
  const uint32_t lck = (uint32_t)(c * kN + j * NS);

  using R = raw_t<Tio>;
  // one tile's inputs, raw; two sets (A/B) ping-pong so the loads for tile
  // i+1 are in flight during tile i with no register copies between them
  struct TileRegs {
    R u[G], d[G], z[G];
    RawVec<Tbc, VPT> st;
  };
  float diag_sink = 0.f;
  // TAIL: some timesteps of the tile are >= t_end -> clamp to the last valid one
  auto load_tile = [&](auto tail, int t0, TileRegs& X) __attribute__((always_inline)) {
    constexpr bool TAIL = decltype(tail)::value;
    if constexpr (TAIL) {
      X.st.load(st0 + (int64_t)min(t0 + st_s, L - 1) * st_ls + (st_col % kN));
    } else {
      X.st.load(st0 + (int64_t)t0 * st_ls + lst);
    }
#ifdef MTTS_DIAG_NOMEM
#pragma unroll
    for (int g = 0; g < G; ++g) {
      X.u[g] = (R)(0x3f80u + (uint32_t)(t0 & 7) + g);
      X.d[g] = (R)(0xbf00u + (uint32_t)g);
      X.z[g] = (R)(0x3f00u + (uint32_t)g);
    }
    return;
#endif
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int tg = t0 + g * P;
      if constexpr (TAIL) {
        const int ts = min(tg + j, L - 1);
        X.u[g] = ldr(u0 + (int64_t)ts * a.u_ls + c);
        X.d[g] = ldr(d0 + (int64_t)ts * a.delta_ls + c);
        if constexpr (MODE == kFull) X.z[g] = ldr(z0 + (int64_t)ts * z_ls + c);
      } else {
        X.u[g] = ldr(u0 + (int64_t)tg * a.u_ls + lu);
        X.d[g] = ldr(d0 + (int64_t)tg * a.delta_ls + ld);
        if constexpr (MODE == kFull) X.z[g] = ldr(z0 + (int64_t)tg * z_ls + lz);
        static_assert(sizeof(lu) == 4, "32-bit lane offsets -> saddr loads");
      }
    }
  };
  auto write_stage = [&](int buf, const TileRegs& X) __attribute__((always_inline)) {
    float v[VPT];
    X.st.unpack(v);
    if constexpr (VPT == 4) {
      *reinterpret_cast<float4*>(&sBC[buf][e0]) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
      for (int q = 0; q < VPT; ++q) sBC[buf][e0 + q] = v[q];
    }
  };
  auto compute_tile = [&](auto tail, int t0, int buf, const TileRegs& X) __attribute__((always_inline)) {
    constexpr bool TAIL = decltype(tail)::value;
    static_for<G>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      const int tg = t0 + g * P;
      // checkpoints every kSub steps (tg is wave-uniform: scalar test)
      if constexpr ((TT % kSub) != 0 || (g * P) % kSub == 0) {
        if (nck && (tg & (kSub - 1)) == 0 && (!TAIL || tg < t_end))
          store_vec<NS>(ck0 + (int64_t)(tg / kSub) * a.dim * kN + lck, h);
      }
      const bool tv = !TAIL || (tg + j < t_end);
      float dt = cvt_raw(X.d[g]) + bias;
      if constexpr (SP) dt = softplus_f(dt);
      if constexpr (TAIL) dt = tv ? dt : 0.f;  // padded steps are the identity map
      const float ug = cvt_raw(X.u[g]);
      const float dtu = dt * ug;
      if constexpr (MODE == kState) S += dt;
#ifdef MTTS_DIAG_NOCOMPUTE
      if constexpr (MODE == kFull) {
        const float y = dtu + cvt_raw(X.z[g]);
        if constexpr (TAIL) {
          if (tv) stf(o0 + (int64_t)(tg + j) * a.out_ls + c, y);
        } else {
          stf(o0 + (int64_t)tg * a.out_ls + lo, y);
        }
      }
      return;
#endif
      float yp[P];
#pragma unroll
      for (int s = 0; s < P; ++s) {
        float dts, dtus;
        if constexpr (P == 2) {
          dts = s == 0 ? group_bcast<2, 0>(dt) : group_bcast<2, 1>(dt);
          dtus = s == 0 ? group_bcast<2, 0>(dtu) : group_bcast<2, 1>(dtu);
        } else {
          dts = s == 0 ? group_bcast<4, 0>(dt) : s == 1 ? group_bcast<4, 1>(dt)
              : s == 2 ? group_bcast<4, 2>(dt) : group_bcast<4, 3>(dt);
          dtus = s == 0 ? group_bcast<4, 0>(dtu) : s == 1 ? group_bcast<4, 1>(dtu)
               : s == 2 ? group_bcast<4, 2>(dtu) : group_bcast<4, 3>(dtu);
        }
        // one broadcast per step into a register (not a DPP operand per use),
        // so the state math below can use packed f32 instructions
        asm volatile("" : "+v"(dts), "+v"(dtus));
        const f2 dts2 = {dts, dts}, dtus2 = {dtus, dtus};
        const float* bc = &sBC[buf][(g * P + s) * 2 * kN];
        f2 y2 = {0.f, 0.f};
#pragma unroll
        for (int q = 0; q < NS / 4; ++q) {
          const f4 vb = *reinterpret_cast<const f4*>(bc + j * NS + 4 * q);
          f4 vc = {};
          if constexpr (MODE == kFull) vc = *reinterpret_cast<const f4*>(bc + kN + j * NS + 4 * q);
#pragma unroll
          for (int p2 = 0; p2 < 2; ++p2) {
            const int i = 4 * q + 2 * p2;
            const f2 x = dts2 * f2{A2[i], A2[i + 1]};
            const f2 e = {__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
            const f2 bv = p2 ? f2{vb[2], vb[3]} : f2{vb[0], vb[1]};
            const f2 hn = __builtin_elementwise_fma(e, f2{h[i], h[i + 1]}, dtus2 * bv);
            h[i] = hn[0];
            h[i + 1] = hn[1];
            if constexpr (MODE == kFull) {
              const f2 cv = p2 ? f2{vc[2], vc[3]} : f2{vc[0], vc[1]};
              y2 = __builtin_elementwise_fma(cv, hn, y2);
            }
          }
        }
        yp[s] = y2[0] + y2[1];
      }
      if constexpr (MODE == kFull) {
        float y = group_reduce_scatter<P>(yp, j);
        y = fmaf(Dc, ug, y);
        if (has_z) y *= silu_f(cvt_raw(X.z[g]));
        if constexpr (TAIL) {
          if (tv) stf(o0 + (int64_t)(tg + j) * a.out_ls + c, y);
        } else {
#ifdef MTTS_DIAG_NOMEM
          diag_sink += y;
#else
          stf(o0 + (int64_t)tg * a.out_ls + lo, y);
#endif
        }
      }
      // materialise h here: otherwise (state-only mode) LLVM sinks every
      // h-update to the tile end and keeps all staged B values live (spills)
#pragma unroll
      for (int i = 0; i < NS; ++i) asm volatile("" : "+v"(h[i]));
      __builtin_amdgcn_sched_barrier(0);  // keep each group's LDS reads local
    });
  };

  const int nfull = (t_end - t_begin) / TT;
  const int ntiles = (t_end - t_begin + TT - 1) / TT;
  // ring of kRing register sets: tile it+kRing-1 is loading while tile it computes
  // (prefetch distance kRing-1 tiles); ring slots are compile-time indices
  constexpr int NR = P == 4 ? kRing : 2;  // P = 2 holds 8 states per lane: two sets fit
  TileRegs ring[NR];
  auto load_any = [&](int it, TileRegs& X) __attribute__((always_inline)) {
    const int t0 = __builtin_amdgcn_readfirstlane(t_begin + it * TT);
    if (it < nfull) load_tile(FalseT{}, t0, X);
    else if (it < ntiles) load_tile(TrueT{}, t0, X);
  };
  static_for<NR - 1>([&](auto rc) { load_any(decltype(rc)::value, ring[decltype(rc)::value]); });
  write_stage(0, ring[0]);
  for (int it0 = 0; it0 < ntiles; it0 += NR) {
    static_for<NR>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      const int it = it0 + r;
      if (it < ntiles) {
        block_sync();
        load_any(it + NR - 1, ring[(r + NR - 1) % NR]);
        const int t0 = __builtin_amdgcn_readfirstlane(t_begin + it * TT);
        if (it < nfull) compute_tile(FalseT{}, t0, it & 1, ring[r]);
        else compute_tile(TrueT{}, t0, it & 1, ring[r]);
        if (it + 1 < ntiles) write_stage((it + 1) & 1, ring[(r + 1) % NR]);
      }
    });
  }
#ifdef MTTS_DIAG_NOMEM
  if (diag_sink == 12345.f) o0[c] = 0;
#endif
  if constexpr (MODE == kFull) {
    if (k == K - 1 && a.last_state)
      store_vec<NS>(a.last_state + ((int64_t)b * a.dim + c) * kN + j * NS, h);
  } else {
    S = group_allreduce<P>(S);
    float* sp = seg + (((int64_t)b * K + k) * a.dim + c) * (kN + 1);
#pragma unroll
    for (int i = 0; i < NS; ++i) sp[j * NS + i] = h[i];
    if (j == 0) sp[kN] = S;
  }
}

// ------------------------------------------------------------- forward, wide I/O
// Same recurrence, lane mapping and L-segmentation as scan_fwd_kernel, but
// u / delta / z tiles arrive as whole 16-byte chunks of timestep rows (the
// block's CPB channels of one timestep are contiguous in the channel-last
// layout) and go through LDS, and the outputs leave the same way.  The
// per-lane 2-byte pattern of the narrow kernel issues 8x more memory
// instructions than the bytes need and caps bf16 streaming at ~2.6 TB/s on
// MI355X (memory-only timing build, tools/diag); 16-byte chunks do not.
// Host-checked requirements: 16-byte aligned bases and strides of u, delta,
// z, out and dim % (16 / sizeof(Tio)) == 0; otherwise the narrow kernel runs.
constexpr bool wide_rows_ok(int P, int W, int pitch) {
  for (int k1 = 0; k1 < P; ++k1)
    for (int k2 = k1 + 1; k2 < P; ++k2) {
      const int d = ((k2 - k1) * pitch) % 64;
      if (d < W || 64 - d < W) return false;
    }
  return true;
}
// LDS row pitch (dwords) such that the P rows one wave reads in a group
// (each W dwords wide) fall in disjoint banks; a multiple of 4 dwords.
constexpr int wide_pitch_dw(int P, int rowdw, int W) {
  for (int pad = 4; pad <= 64; pad += 4)
    if (wide_rows_ok(P, W, rowdw + pad)) return rowdw + pad;
  return rowdw + 4;
}

// ------------------------------------------------------------- forward, LDS-DMA tiles, software-pipelined
// Same tensors, lane mapping (P lanes per channel, NS = 16/P states each),
// tile image and L-segmentation as the round-1 wide kernel (removed), restructured after
// profiling it at ~5.7 SIMD cycles per VALU instruction (its groups
// were serial chains: B/C LDS read -> wait -> state update -> y, per step):
//  * u / delta / z tiles go HBM -> LDS by LDS-DMA (global_load_lds_dwordx4,
//    1 KiB per wave-instruction): no staging VGPRs, no ds_write, no VALU;
//    rows are XOR-swizzled through the SOURCE address (chunk cc of row r sits
//    at cc ^ f(r)) so the P rows one wave reads per group hit disjoint banks;
//  * a group's B/C reads issue first and all P*NS exponentials are formed
//    before the first B/C use, so the LDS latency hides under the exps;
//  * the per-channel scalar work (delta/u/z reads, softplus, delta*u, silu
//    gate) of group g+1 runs inside group g, off the recurrence chain;
//  * one barrier per tile: tile i's outputs (written over u in the image) are
//    stored right after the barrier that opens tile i+1, each chunk by the
//    lane whose DMA refills it next (the store's read precedes that DMA).
// 16-byte LDS-DMA: lane l's 16 bytes at g land at lds + 16*l (lds wave-uniform).
// Inline asm, not __builtin_amdgcn_global_load_lds: with the builtin hipcc puts
// an s_waitcnt vmcnt(0) in front of the next LDS read it cannot prove disjoint
// (any read of the other tile buffer), which serialises the prefetch with the
// compute.  The asm is invisible to the compiler's wait insertion, so every
// consumer of DMA'd bytes is preceded by an explicit wait_vmem() + barrier.
// M0 holds the LDS base (one wait state before the DMA reads it).
__device__ __forceinline__ void dma16(const void* g, void* lds) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t l = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds);
  // nt: the u / delta / z tiles are read once (north-star fp32 fwd 2.185 ->
  // 2.160 ms over three interleaved rounds; C2 shapes and bwd unchanged)
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off nt" ::"v"(g), "s"(l) : "memory", "m0");
#endif
}
// The same LDS-DMA as a buffer load (round 4): base / range in an SGPR
// descriptor, a lane-constant byte offset in voff and the tile's row origin
// in the scalar offset, so a DMA costs no per-lane address arithmetic; rows at
// or past the range read 0.
typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4 rsrc4(const void* p, uint32_t bytes) {   // p, bytes wave-uniform
  const uint64_t a = (uint64_t)(uintptr_t)p;
  return i32x4{__builtin_amdgcn_readfirstlane((int)(uint32_t)a), __builtin_amdgcn_readfirstlane((int)((a >> 32) & 0xffff)),
               __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000};
}
__device__ __forceinline__ uint32_t lds_u32(const void* lds) {   // wave-uniform LDS byte address
  return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void*)lds);
}
__device__ __forceinline__ void dma16b(const i32x4& rs, uint32_t voff, int soff, uint32_t lds) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, %3 offen nt lds"
               ::"v"(voff), "s"(lds), "s"(rs), "s"(soff) : "memory", "m0");
#endif
}
// W-dword global load into registers, invisible to the compiler's wait
// insertion (so a later LDS-DMA can stay in flight past its consumer);
// consume only after wait_vm<N>(regs) with the loads counted.
template <int W, bool HALF = false>
__device__ __forceinline__ void ldg_asm(uint32_t (&w)[W], const void* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (HALF) {
    static_assert(W == 1, "half-dword load");
    asm volatile("global_load_ushort %0, %1, off" : "=v"(w[0]) : "v"(p) : "memory");
  } else if constexpr (W == 1) {
    asm volatile("global_load_dword %0, %1, off" : "=v"(w[0]) : "v"(p) : "memory");
  } else if constexpr (W == 2) {
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    u2 v;
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    w[0] = v[0]; w[1] = v[1];
  } else {
    static_assert(W == 4, "ldg_asm width");
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    u4 v;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    w[0] = v[0]; w[1] = v[1]; w[2] = v[2]; w[3] = v[3];
  }
#endif
}
// s_waitcnt vmcnt(N) that also "redefines" the staged registers, so no use of
// them can be scheduled above the wait.
template <int N, int W>
__device__ __forceinline__ void wait_vm(uint32_t (&w)[W]) {
#if defined(__HIP_DEVICE_COMPILE__)
  static_assert(N == 0 || N == 2 || N == 3, "wait_vm count");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
#pragma unroll
  for (int q = 0; q < W; ++q) asm volatile("" : "+v"(w[q]));
#endif
}
// s_waitcnt vmcnt(N) for any N < 64 (gfx9 encoding: vmcnt[3:0] | vmcnt[5:4] << 14,
// expcnt 7, lgkmcnt 15), redefining the staged registers like wait_vm
template <int N, int W>
__device__ __forceinline__ void wait_vmn(uint32_t (&w)[W]) {
#if defined(__HIP_DEVICE_COMPILE__)
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
#pragma unroll
  for (int q = 0; q < W; ++q) asm volatile("" : "+v"(w[q]));
#endif
}
__device__ __forceinline__ void wait_vmem() {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
#endif
}

// timing-only diagnostic switches (tools/diag_build.sh); all 0 in the product
#ifndef MTTS_DIAG_NOSCALAR
#define MTTS_DIAG_NOSCALAR 0
#endif
#ifndef MTTS_DIAG_NODPP
#define MTTS_DIAG_NODPP 0
#endif
#ifndef MTTS_DIAG_NOEXP
#define MTTS_DIAG_NOEXP 0
#endif

// softplus(x) / ln2 for xl = x log2(e): the forward kernels carry dt' = dt / ln2
// and h' = h / ln2 (see scan_fwd_c1_kernel); torch's x > 20 -> x threshold
// falls out of the max, log1p's small-argument series covers e < 1e-3
__device__ __forceinline__ float softplus_l2(float xl) {
  const float e = __builtin_amdgcn_exp2f(fminf(xl, 64.f));
  const float lg = __builtin_amdgcn_logf(1.f + e);                  // log2(1 + e)
  const float sm = e * fmaf(e, -0.5f * kLog2e, kLog2e);              // log2(1 + e) for tiny e
  return fmaxf(e < 1e-3f ? sm : lg, xl);
}

template <int P, int ES>
struct DmaTile {
  static constexpr int CPB = kBlock / P;          // channels per block
  static constexpr int ROWB = CPB * ES;           // bytes of a block's timestep row
  static constexpr int TT = 4096 / ROWB;          // timesteps per tile: one 16-B chunk per thread per array
  static constexpr int CPR = ROWB / 16;           // chunks per row
  static constexpr int WB = (64 / P) * ES / 16;   // chunks one wave reads per row (>= 1)
  // chunk cc of row r lives at cc ^ swz(r)
  static constexpr __host__ __device__ int swz(int r) { return WB * (r % P); }
  static constexpr bool conflict_free() {
    if (WB < 1 || WB * P > CPR) return false;
    for (int cc = 0; cc < CPR; cc += WB)
      for (int j1 = 0; j1 < P; ++j1)
        for (int j2 = j1 + 1; j2 < P; ++j2) {
          const int s1 = (j1 * ROWB + ((cc ^ swz(j1)) * 16)) % 256;
          const int s2 = (j2 * ROWB + ((cc ^ swz(j2)) * 16)) % 256;
          const int d = (s2 - s1 + 256) % 256;
          if (d < WB * 16 || 256 - d < WB * 16) return false;
        }
    return true;
  }
};

template <int P, typename Tio, typename Tbc, int MODE, bool SP>
__global__ __launch_bounds__(kBlock, 2) void scan_fwd_w2_kernel(const MttsScanFwdArgs a, const int seg_len,
                                                                float* __restrict__ seg) {
  constexpr int NS = kN / P;
  constexpr int NP2 = NS / 2;
  constexpr int ES = (int)sizeof(Tio);
  using DT = DmaTile<P, ES>;
  constexpr int CPB = DT::CPB;
  constexpr int TT = DT::TT;
  constexpr int G = TT / P;
  constexpr int CPR = DT::CPR;
  constexpr int EPC = 16 / ES;
  constexpr int NA = MODE == kFull ? 3 : 2;
  constexpr int IMG = TT * CPR * EPC;             // elements of one array image (4 KiB)
  constexpr int VPT = TT * 2 * kN / kBlock;
  static_assert(G >= 1 && TT % P == 0 && (TT * 2 * kN) % kBlock == 0 && NS % 4 == 0, "tile shape");
  static_assert(TT * CPR == kBlock, "one chunk per thread per array");
  static_assert(DT::conflict_free(), "swizzle");
  // tile buffers: 3 (DMA two tiles ahead) when they fit 4 blocks per CU, else 2
#ifdef MTTS_FWD_NB
  constexpr int NB = MTTS_FWD_NB;  // timing builds: buffer count forced (LDS then sets blocks per CU)
#else
  constexpr int NB = (3 * NA * IMG * ES + 2 * TT * 2 * kN * 4 + 4096) <= 40960 ? 3 : 2;
#endif
  __shared__ __attribute__((aligned(16))) Tio sX[NB][NA][IMG];
  __shared__ __attribute__((aligned(16))) float sBC[2][TT * 2 * kN];
  // per-wave (delta, delta*u) exchange: the lane that formed step s of a
  // group writes its pair, every lane of the channel reads all P pairs
  __shared__ __attribute__((aligned(16))) float sS[kBlock / 64][2][64 / P][P][2];

  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int j = tid % P, cl = tid / P;
  const int cw = (tid & 63) / P;                  // channel within the wave
  const int c0 = blockIdx.x * CPB;
  const bool cvalid = c0 + cl < a.dim;
  const int c = cvalid ? c0 + cl : a.dim - 1;
  const int b = blockIdx.y;
  const int k = blockIdx.z;
  const int L = a.seqlen;
  const int K = (L + seg_len - 1) / seg_len;
  const int t_begin = k * seg_len;
  const int t_end = min(L, t_begin + seg_len);
  const bool has_z = MODE == kFull && a.z != nullptr;

  // this thread's DMA / store chunk: LDS chunk position tid = (row, cp), global chunk cc = cp ^ swz(row)
  const int lrow = tid / CPR;
  const int gcol = ((tid % CPR) ^ DT::swz(lrow)) * EPC;
  const bool lvalid = c0 + gcol < a.dim;           // whole chunk (dim % EPC == 0)
  const int gcol_c = lvalid ? gcol : 0;            // out-of-range chunks read column c0 (discarded)
  const int64_t z_ls = has_z ? a.z_ls : a.u_ls;
  // u / delta / z / out through buffer descriptors over the block's channel
  // columns of the batch row (as scan_fwd_c1_kernel; host: spans below 2 GiB):
  // a lane-constant byte offset + the tile's row origin in the scalar offset.
  // Rows at or past L read 0 (rows of a later segment read real values that
  // are never used); stores past the segment's last row are dropped.
  const int ncol = min(CPB, a.dim - c0);
  auto span = [&](int64_t ls, int rows) { return (uint32_t)(((int64_t)(rows - 1) * ls + ncol) * ES); };
  const i32x4 ru = rsrc4((const Tio*)a.u + (int64_t)b * a.u_bs + c0, span(a.u_ls, L));
  const i32x4 rd = rsrc4((const Tio*)a.delta + (int64_t)b * a.delta_bs + c0, span(a.delta_ls, L));
  const i32x4 rz = has_z ? rsrc4((const Tio*)a.z + (int64_t)b * a.z_bs + c0, span(a.z_ls, L)) : ru;
  const uint32_t vu = (uint32_t)((lrow * a.u_ls + gcol_c) * ES), vd = (uint32_t)((lrow * a.delta_ls + gcol_c) * ES);
  const uint32_t vz = (uint32_t)((lrow * z_ls + gcol_c) * ES);
  const uint64_t opp = (uint64_t)(uintptr_t)((Tio*)a.out + (int64_t)b * a.out_bs + c0);
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(   // wave-uniform: no waterfall
      (void*)(uintptr_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(opp >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)opp)),
      0, __builtin_amdgcn_readfirstlane((int)span(a.out_ls, t_end)), 0x00020000);
  // lanes past dim store nothing (a branch, not an out-of-range voffset: with
  // the row origin in the scalar offset, voffset + soffset would wrap back into
  // range -- tools/ubench/buffer_oob_probe.hip)
  const uint32_t vo = (uint32_t)((lrow * a.out_ls + gcol_c) * ES);

  const int e0 = tid * VPT;
  const int st_s = e0 / (2 * kN), st_col = e0 % (2 * kN);
  const Tbc* __restrict__ st0 = st_col < kN ? (const Tbc*)a.Bm + (int64_t)b * a.B_bs
                                            : (const Tbc*)a.Cm + (int64_t)b * a.C_bs;
  const int64_t st_ls = st_col < kN ? a.B_ls : a.C_ls;

  f2 A2[NP2], h[NP2];
#pragma unroll
  for (int p = 0; p < NP2; ++p) {
    const int64_t ai = (int64_t)c * kN + j * NS + 2 * p;
    A2[p] = f2{ld_A(a, ai), ld_A(a, ai + 1)};   // log2 domain (scan_fwd_c1_kernel): exp2(dt' A)
  }
  const float Dc2 = a.D ? a.D[c] * kLog2e : 0.f;
  const float bias2 = a.delta_bias ? a.delta_bias[c] * kLog2e : 0.f;
  float S = 0.f;
  if constexpr (MODE == kFull) {
#pragma unroll
    for (int p = 0; p < NP2; ++p) {
      const int64_t o = ((int64_t)b * a.dim + c) * kN + j * NS + 2 * p;
      h[p] = a.h0 ? f2{a.h0[o] * kLog2e, a.h0[o + 1] * kLog2e} : f2{0.f, 0.f};   // h' = h / ln2
    }
    for (int kk = 0; kk < k; ++kk) {
      const float* sp = seg + (((int64_t)b * K + kk) * a.dim + c) * (kN + 1);
      const float Sk = sp[kN];
#pragma unroll
      for (int p = 0; p < NP2; ++p) {
        const f2 x = A2[p] * Sk;
        const f2 e = {__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
        h[p] = __builtin_elementwise_fma(e, h[p], f2{sp[j * NS + 2 * p], sp[j * NS + 2 * p + 1]});
      }
    }
  } else {
#pragma unroll
    for (int p = 0; p < NP2; ++p) h[p] = f2{0.f, 0.f};
  }
  const int nck = (MODE == kFull && a.ckpt) ? (L + kSub - 1) / kSub : 0;
  float* __restrict__ ck0 = nck ? a.ckpt + (int64_t)b * nck * a.dim * kN : nullptr;
  const uint32_t lck = (uint32_t)(c * kN + j * NS);

  constexpr int SW = RawVec<Tbc, VPT>::W;     // staging dwords per thread
  constexpr bool SHALF = VPT * (int)sizeof(Tbc) == 2;  // a single bf16
  static_assert(SHALF || VPT * (int)sizeof(Tbc) == 4 * SW, "B/C staging is whole dwords");
  uint32_t stg[SW];
  auto load_bc = [&](int t0) __attribute__((always_inline)) {
    ldg_asm<SW, SHALF>(stg, st0 + (int64_t)min(t0 + st_s, L - 1) * st_ls + (st_col % kN));
  };
  auto dma_tile = [&](int t0, int buf) __attribute__((always_inline)) {
    auto lds = [&](int q) { return lds_u32(&sX[buf][q][wave * 64 * EPC]); };
#ifdef MTTS_DIAG_NOMEM
    return;  // timing-only build: the tile images keep stale contents
#endif
    dma16b(ru, vu, (int)(t0 * a.u_ls * ES), lds(0));
    dma16b(rd, vd, (int)(t0 * a.delta_ls * ES), lds(1));
    if constexpr (NA == 3) dma16b(rz, vz, (int)(t0 * z_ls * ES), lds(2));
  };
  auto stage_bc = [&](int buf) __attribute__((always_inline)) {
    float v[VPT];
    if constexpr (sizeof(Tbc) == 4) {
#pragma unroll
      for (int q = 0; q < VPT; ++q) v[q] = __uint_as_float(stg[q]);
    } else if constexpr (SHALF) {
      v[0] = __uint_as_float(stg[0] << 16);
    } else {
#pragma unroll
      for (int q = 0; q < SW; ++q) unpack_bf2(stg[q], v[2 * q], v[2 * q + 1]);
    }
    if constexpr (VPT == 4) {
      *reinterpret_cast<float4*>(&sBC[buf][e0]) = make_float4(v[0], v[1], v[2], v[3]);
    } else if constexpr (VPT == 2) {
      *reinterpret_cast<float2*>(&sBC[buf][e0]) = make_float2(v[0], v[1]);
    } else {
#pragma unroll
      for (int q = 0; q < VPT; ++q) sBC[buf][e0 + q] = v[q];
    }
  };
  auto store_tile = [&](int t0, int buf) __attribute__((always_inline)) {
    const uint4 v = *reinterpret_cast<const uint4*>(&sX[buf][0][tid * EPC]);
#ifdef MTTS_DIAG_NOMEM
    if (v.x == 0x12345u && v.y == 0x777u) sX[buf][0][0] = (Tio)0;  // keep the tile alive, never true
    return;
#endif
    // row origin in the vector offset, soffset 0: with a register soffset
    // hipcc drops the store-data wait states (see conv_fwd_tile_kernel)
    if (lvalid)
      __builtin_amdgcn_raw_buffer_store_b128(i32x4{(int)v.x, (int)v.y, (int)v.z, (int)v.w}, ro,
                                             vo + (uint32_t)(t0 * a.out_ls * ES), 0, 0);
  };
  // element (row, local channel) of an array image
  auto at = [&](int row, int ch) __attribute__((always_inline)) {
    return row * (CPR * EPC) + (((ch / EPC) ^ DT::swz(row)) * EPC) + (ch % EPC);
  };

  struct Scal {
    float dt, dtu, ug, gate;
  };
  auto scalar = [&](auto tail, int t0, int buf, int g, Scal& o) __attribute__((always_inline)) {
    constexpr bool TAIL = decltype(tail)::value;
    const int sx = at(g * P + j, cl);
    float dt = fmaf(cvt_raw((raw_t<Tio>)sX[buf][1][sx]), kLog2e, bias2);   // dt / ln2
    if constexpr (SP && !MTTS_DIAG_NOSCALAR) dt = softplus_l2(dt);
    const bool tv = !TAIL || (t0 + g * P + j < t_end);
    o.dt = tv ? dt : 0.f;                             // padded steps: identity map
    o.ug = cvt_raw((raw_t<Tio>)sX[buf][0][sx]);
    o.dtu = tv ? o.dt * o.ug : 0.f;
    if constexpr (MODE == kFull) {
      // branch-free: without z the z image holds u (never used), the gate is 1
      const float zv = cvt_raw((raw_t<Tio>)sX[buf][2][sx]);
      const float gz = MTTS_DIAG_NOSCALAR ? zv : zv * fast_rcp(fmaf(__builtin_amdgcn_exp2f(-zv * kLog2e), kLog2e, kLog2e));
      o.gate = has_z ? gz : kLn2;   // ln2 silu(z): y = ln2 (C.h' + D log2(e) u) silu(z)
    }
  };

  auto compute_tile = [&](auto tail, int t0, int buf, int bb) __attribute__((always_inline)) {
    constexpr bool TAIL = decltype(tail)::value;
#ifdef MTTS_DIAG_NOCOMPUTE
    return;
#endif
    // publish a group's (delta, delta*u) pairs for the lanes of the channel
    // (one ds_write_b64 + two ds_read_b128 per group; the DPP-broadcast form
    // measured equal on bf16 and 2 % slower on fp32)
    auto put = [&](int pb, const Scal& v) __attribute__((always_inline)) {
      *reinterpret_cast<float2*>(&sS[wave][pb][cw][j][0]) = make_float2(v.dt, v.dtu);
    };
    Scal cur;
    scalar(tail, t0, buf, 0, cur);
    put(0, cur);
    static_for<G>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      const int tg = t0 + g * P;
      if constexpr ((TT % kSub) != 0 || (g * P) % kSub == 0) {
        if (nck && cvalid && (tg & (kSub - 1)) == 0 && (!TAIL || tg < t_end)) {
          float hv[NS];
#pragma unroll
          for (int p = 0; p < NP2; ++p) { hv[2 * p] = h[p][0] * kLn2; hv[2 * p + 1] = h[p][1] * kLn2; }
          store_vec<NS>(ck0 + (int64_t)(tg / kSub) * a.dim * kN + lck, hv);
        }
      }
      // (2) first: delta / delta*u of the group's P steps to every lane of the
      // channel, from the LDS exchange (published one group ahead)
      float dts[P], dtus[P];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int q = 0; q < P / 2; ++q) {
        const f4 v = *reinterpret_cast<const f4*>(&sS[wave][g & 1][cw][2 * q][0]);
        dts[2 * q] = v[0]; dtus[2 * q] = v[1]; dts[2 * q + 1] = v[2]; dtus[2 * q + 1] = v[3];
      }
      // (1) this group's B / C rows (their latency hides under the exponentials)
      f4 Bq[P][NS / 4], Cq[P][NS / 4];
#pragma unroll
      for (int s = 0; s < P; ++s) {
        const float* bc = &sBC[bb][(g * P + s) * 2 * kN + j * NS];
#pragma unroll
        for (int q = 0; q < NS / 4; ++q) {
          Bq[s][q] = *reinterpret_cast<const f4*>(bc + 4 * q);
          if constexpr (MODE == kFull) Cq[s][q] = *reinterpret_cast<const f4*>(bc + kN + 4 * q);
        }
      }
      // (3) all exponentials of the group (independent of the recurrence)
      f2 e[P][NP2];
#pragma unroll
      for (int s = 0; s < P; ++s)
#pragma unroll
        for (int p = 0; p < NP2; ++p) {
          const f2 x = f2{dts[s], dts[s]} * A2[p];
          e[s][p] = MTTS_DIAG_NOEXP ? x : f2{__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
        }
      // (4) next group's scalar work, off the chain (kept behind the
      // exponentials so its LDS reads do not wait on this group's B/C reads)
      __builtin_amdgcn_sched_barrier(0);
      Scal nxt;
      if constexpr (g + 1 < G) {
        scalar(tail, t0, buf, g + 1, nxt);
        put((g + 1) & 1, nxt);
      }
      // (5) recurrence + outputs
      float yp[P];
#pragma unroll
      for (int s = 0; s < P; ++s) {
        f2 y2 = {0.f, 0.f};
#pragma unroll
        for (int p = 0; p < NP2; ++p) {
          const f4& bq = Bq[s][p / 2];
          const f2 bv = (p & 1) ? f2{bq[2], bq[3]} : f2{bq[0], bq[1]};
          h[p] = __builtin_elementwise_fma(e[s][p], h[p], f2{dtus[s], dtus[s]} * bv);
          if constexpr (MODE == kFull) {
            const f4& cq = Cq[s][p / 2];
            const f2 cv = (p & 1) ? f2{cq[2], cq[3]} : f2{cq[0], cq[1]};
            y2 = __builtin_elementwise_fma(cv, h[p], y2);
          }
        }
        yp[s] = y2[0] + y2[1];
      }
      if constexpr (MODE == kFull) {
        float y = MTTS_DIAG_NODPP ? yp[0] + yp[1] + yp[P - 1] : group_reduce_scatter<P>(yp, j);
        y = fmaf(Dc2, cur.ug, y) * cur.gate;
        stf(&sX[buf][0][at(g * P + j, cl)], y);     // the output replaces u in the tile image
      } else {
        S += cur.dt;
      }
      if constexpr (g + 1 < G) cur = nxt;
#pragma unroll
      for (int p = 0; p < NP2; ++p) asm volatile("" : "+v"(h[p]));
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  const int nfull = (t_end - t_begin) / TT;
  const int ntiles = (t_end - t_begin + TT - 1) / TT;
  // VMEM order per iteration: [stores of tile it-1] [B/C regs of tile it+1]
  // [DMA of tile it+NB-1]; the end-of-iteration wait leaves only that DMA in
  // flight, so tile it+1 (DMA'd an iteration earlier when NB = 3) is complete.
  load_bc(t_begin);
  dma_tile(t_begin, 0);
  wait_vm<0>(stg);
  stage_bc(0);
  if constexpr (NB == 3)
    if (ntiles > 1) dma_tile(t_begin + TT, 1);
  int buf = 0, prev = NB - 1;
  for (int it = 0; it < ntiles; ++it) {
    const int t0 = __builtin_amdgcn_readfirstlane(t_begin + it * TT);
    block_sync();  // tile it in LDS (every wave's DMA drained); outputs of tile it-1 complete
    if constexpr (MODE == kFull)
      if (it > 0) store_tile(t0 - TT, prev);        // read before this lane's DMA below refills the chunk
    const bool more = it + 1 < ntiles;
    const bool ahead = it + NB - 1 < ntiles;
    if (more) load_bc(t0 + TT);
    if (ahead) dma_tile(t0 + (NB - 1) * TT, prev);  // buffer (it + NB - 1) % NB == (it - 1) % NB
    if (it < nfull) compute_tile(FalseT{}, t0, buf, it & 1);
    else compute_tile(TrueT{}, t0, buf, it & 1);
    if (more) {
      if (NB == 3 && ahead) wait_vm<NA>(stg);
      else wait_vm<0>(stg);
      stage_bc((it + 1) & 1);
    }
    prev = buf;
    buf = buf + 1 == NB ? 0 : buf + 1;
  }
  if constexpr (MODE == kFull) {
    block_sync();
    store_tile(t_begin + (ntiles - 1) * TT, prev);
    if (k == K - 1 && a.last_state && cvalid) {
      float hv[NS];
#pragma unroll
      for (int p = 0; p < NP2; ++p) { hv[2 * p] = h[p][0] * kLn2; hv[2 * p + 1] = h[p][1] * kLn2; }
      store_vec<NS>(a.last_state + ((int64_t)b * a.dim + c) * kN + j * NS, hv);
    }
  } else {
    S = group_allreduce<P>(S);
    if (cvalid) {
      float* sp = seg + (((int64_t)b * K + k) * a.dim + c) * (kN + 1);
#pragma unroll
      for (int p = 0; p < NP2; ++p) { sp[j * NS + 2 * p] = h[p][0]; sp[j * NS + 2 * p + 1] = h[p][1]; }
      if (j == 0) sp[kN] = S;
    }
  }
}

// ------------------------------------------------------------- backward
// P = 4 lanes per channel (NS = 4 states per lane), SUB = 16 steps per chunk
// (4 groups of 4).  Per-lane register history: h and exp(dt*A) for 16 steps.
constexpr int kPB = 4;
constexpr int kNSB = kN / kPB;
constexpr int kGB = kSub / kPB;
constexpr int kChB = kBlock / kPB;   // channels per block (64)
constexpr int kWaves = kBlock / 64;


template <int S>
__device__ __forceinline__ float bcast4(float v) { return dpp<S * 0x55>(v); }

// reduce-scatter stages with the swap instructions (no lane selects):
// lanes 0-31 get a + a[lane+32], lanes 32-63 get b + b[lane-32]
__device__ __forceinline__ float rs_swap32(float a, float b) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// rows 0,2 get a + a[lane+16], rows 1,3 get b + b[lane-16]
__device__ __forceinline__ float rs_swap16(float a, float b) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Reduce 32 values per lane over the 16 channel-lanes of the wave (lane bits
// 2..5), keeping the state-group bits 0..1.  On return lane holds 2 values:
// value index v = (l2<<4)|(l3<<3)|(l4<<2)|(l5<<1)|e  (e = 0, 1).
__device__ __forceinline__ void wave_reduce_scatter32(float (&v)[32], float& o0, float& o1, int lane) {
  // stage xor4: bit 2 of lane <-> bit 4 of v
  float a16[16];
  {
    const bool q = lane & 4;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      float keep = q ? v[16 + k] : v[k];
      float send = q ? v[k] : v[16 + k];
      a16[k] = keep + xor4(send, lane);
    }
  }
  float a8[8];
  {
    const bool q = lane & 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float keep = q ? a16[8 + k] : a16[k];
      float send = q ? a16[k] : a16[8 + k];
      a8[k] = keep + xor8(send);
    }
  }
  float a4[4];
  {
    const bool q = lane & 16;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float keep = q ? a8[4 + k] : a8[k];
      float send = q ? a8[k] : a8[4 + k];
      auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(send), __float_as_uint(send), false, false);
      a4[k] = keep + __uint_as_float(q ? r[0] : r[1]);
    }
  }
  {
    const bool q = lane & 32;
    float k0 = q ? a4[2] : a4[0], k1 = q ? a4[3] : a4[1];
    float s0 = q ? a4[0] : a4[2], s1 = q ? a4[1] : a4[3];
    auto r0 = __builtin_amdgcn_permlane32_swap(__float_as_uint(s0), __float_as_uint(s0), false, false);
    auto r1 = __builtin_amdgcn_permlane32_swap(__float_as_uint(s1), __float_as_uint(s1), false, false);
    o0 = k0 + __uint_as_float(q ? r0[0] : r0[1]);
    o1 = k1 + __uint_as_float(q ? r1[0] : r1[1]);
  }
}

// kPackedHazard (round 6, profiles/r06_race_bg.txt): in the two backward
// kernels, a few packed-f32 ops (v_pk_mul_f32 / v_pk_fma_f32) gave results
// that changed from run to run whenever another kernel's MFMA waves shared
// the SIMD (another process's skinny TN GEMM or attention, or a bare MFMA
// loop: tools/ubench/aggressor.hip) -- the carry pass's adjoint update and its
// exp argument, the main pass's dA accumulation, all with an operand
// broadcast from a value just read from the per-wave dt / dy table.  The
// carry pass does those as plain ops (an empty asm keeps the SLP vectorizer
// from re-packing them); the main pass keeps its packed dA FMA but reads dt
// through one plain v_mov_b32 copy.  0 of 200 mismatching runs under every
// aggressor; C2 backward 0.500 -> 0.514 ms per call (0.524 with the main
// pass's dA as plain ops too).  No packed f32 at all also fixes it, at 3.5x.
// Backward pass 1 (only when L is split into K > 1 segments): for segments
// k = 1..K-1, run the adjoint recurrence  dh_t = dy_t C_t + exp(dt_{t+1} A) dh_{t+1}
// from zero carry-in at the segment end and record the carry leaving the
// segment start, g_k = exp(dt_{t0} A) dh_{t0}, plus S_k = sum(dt).  The carry
// entering segment k is then G_k = sum_{j>k} exp(A (S_{k+1}+..+S_{j-1})) g_j.
template <typename Tio, typename Tbc, bool SP, bool WIDE>
__global__ __launch_bounds__(kBlock, 4) void scan_bwd_carry_kernel(const MttsScanBwdArgs a, const int seg_len,
                                                                   float* __restrict__ seg) {
  constexpr int G = kTileG;          // groups per tile
  constexpr int TT = G * kPB;        // 32 timesteps per tile
  __shared__ __attribute__((aligned(16))) float sC[2][TT * kN];
  // WIDE staging of delta / dout / z tiles (16-byte row chunks through LDS)
  constexpr int ES = (int)sizeof(Tio);
  constexpr int ROWB = kChB * ES;
  constexpr int CPR = ROWB / 16;
  constexpr int EPC = 16 / ES;
  constexpr int PIT = wide_pitch_dw(kPB, ROWB / 4, (64 / kPB) * ES / 4) * 4 / ES;
  constexpr int NCH = 3 * TT * CPR / kBlock;
  __shared__ __attribute__((aligned(16))) Tio sX[WIDE ? 2 : 1][3][WIDE ? TT * PIT : 1];
  // per-wave [dt | dy][channel][step] of the tile (pitch 36 floats: distinct
  // bank groups for the 16 channels' 16-byte reads): one ds_read_b128 per
  // group instead of eight DPP broadcasts (as scan_bwd_kernel)
  constexpr int kBrP = TT + 4;
  __shared__ __attribute__((aligned(16))) float sBr[kWaves][2][16 * kBrP];
  const int cl = threadIdx.x / kPB;
  const MttsScanFwdArgs& f = a.f;
  const int j = threadIdx.x % kPB;
  const int c_raw = blockIdx.x * kChB + threadIdx.x / kPB;
  const bool cvalid = c_raw < f.dim;
  const int c = cvalid ? c_raw : f.dim - 1;
  const int b = blockIdx.y;
  const int k = blockIdx.z + 1;
  const int L = f.seqlen;
  const int K = (L + seg_len - 1) / seg_len;
  const int t_begin = k * seg_len;
  const int t_end = min(L, t_begin + seg_len);
  const Tio* __restrict__ d0 = (const Tio*)f.delta + (int64_t)b * f.delta_bs;
  const bool has_z = f.z != nullptr;
  const Tio* __restrict__ z0 = has_z ? (const Tio*)f.z + (int64_t)b * f.z_bs : d0;  // no z: loads ignored
  const int64_t z_ls = has_z ? f.z_ls : f.delta_ls;
  const Tio* __restrict__ g0 = (const Tio*)a.dout + (int64_t)b * a.dout_bs;
  const uint32_t od = (uint32_t)(j * f.delta_ls + c), oz = (uint32_t)(j * z_ls + c);
  const uint32_t og = (uint32_t)(j * a.dout_ls + c);
  const Tbc* __restrict__ C0 = (const Tbc*)f.Cm + (int64_t)b * f.C_bs;
  const int e0 = threadIdx.x * 2;          // staged C values of this thread: step e0/16, state e0%16
  const int st_s = e0 / kN, st_n = e0 % kN;
  float A2[kNSB];
#pragma unroll
  for (int i = 0; i < kNSB; ++i) A2[i] = ld_A(f, (int64_t)c * kN + j * kNSB + i) * kLog2e;
  const f2 A2v[2] = {f2{A2[0], A2[1]}, f2{A2[2], A2[3]}};
  f2 carry2[2] = {f2{0.f, 0.f}, f2{0.f, 0.f}};
  const float bias = f.delta_bias ? f.delta_bias[c] : 0.f;
  float S = 0.f;
  using R = raw_t<Tio>;
  R cx[G], cg[G], cz[G], nx[G], ng[G], nz[G];
  RawVec<Tbc, 2> st;
  // steps >= t_end load a clamped index; their dy is zeroed at use
  auto load = [&](int t0, R (&xx)[G], R (&gg)[G], R (&zz)[G]) {
    const bool full = t0 + TT <= t_end;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int tg = t0 + g * kPB;
      if (full) {
        xx[g] = ldr(d0 + (int64_t)tg * f.delta_ls + od);
        gg[g] = ldr(g0 + (int64_t)tg * a.dout_ls + og);
        zz[g] = ldr(z0 + (int64_t)tg * z_ls + oz);
      } else {
        const int tc = min(tg + j, L - 1);
        xx[g] = ldr(d0 + (int64_t)tc * f.delta_ls + c);
        gg[g] = ldr(g0 + (int64_t)tc * a.dout_ls + c);
        zz[g] = ldr(z0 + (int64_t)tc * z_ls + c);
      }
    }
    st.load(C0 + (int64_t)min(t0 + st_s, L - 1) * f.C_ls + st_n);
  };
  auto write_stage = [&](int buf) {
    float v[2];
    st.unpack(v);
    *reinterpret_cast<float2*>(&sC[buf][e0]) = make_float2(v[0], v[1]);
  };
  // WIDE: this thread's chunks (array, row, column), loaded as 16-byte pieces
  uint4 wx[WIDE ? NCH : 1];
  const Tio* wsrc[WIDE ? NCH : 1];
  int64_t wls[WIDE ? NCH : 1];
  int wrow[WIDE ? NCH : 1], warr[WIDE ? NCH : 1], wcol[WIDE ? NCH : 1];
  bool wok[WIDE ? NCH : 1];
  if constexpr (WIDE) {
    const int c0 = blockIdx.x * kChB;
#pragma unroll
    for (int q = 0; q < NCH; ++q) {
      const int idx = threadIdx.x + kBlock * q;
      warr[q] = idx / (TT * CPR);
      wrow[q] = (idx % (TT * CPR)) / CPR;
      wcol[q] = (idx % CPR) * EPC;
      wok[q] = c0 + wcol[q] < f.dim;
      const int ar = warr[q];
      wsrc[q] = (ar == 0 ? d0 : ar == 1 ? g0 : z0) + c0 + wcol[q];
      wls[q] = ar == 0 ? f.delta_ls : ar == 1 ? a.dout_ls : z_ls;
    }
  }
  auto load_w = [&](int t0) {
    st.load(C0 + (int64_t)min(t0 + st_s, L - 1) * f.C_ls + st_n);
#pragma unroll
    for (int q = 0; q < NCH; ++q) {
      const int tr = t0 + wrow[q];
      const bool ok = wok[q] && tr < t_end;
      wx[q] = *reinterpret_cast<const uint4*>(wsrc[q] + (int64_t)(ok ? tr : t_begin) * wls[q]);
      if (!ok) wx[q] = make_uint4(0, 0, 0, 0);
    }
  };
  auto write_w = [&](int buf) {
#pragma unroll
    for (int q = 0; q < NCH; ++q) *reinterpret_cast<uint4*>(&sX[buf][warr[q]][wrow[q] * PIT + wcol[q]]) = wx[q];
    write_stage(buf);
  };
  const int ntiles = (t_end - t_begin + TT - 1) / TT;
  if constexpr (WIDE) {
    load_w(t_begin + (ntiles - 1) * TT);
    write_w(0);
  } else {
    load(t_begin + (ntiles - 1) * TT, cx, cg, cz);
    write_stage(0);
  }
  for (int q = 0; q < ntiles; ++q) {
    const int it = ntiles - 1 - q;
    const int t0 = __builtin_amdgcn_readfirstlane(t_begin + it * TT);
    const int buf = q & 1;
    block_sync();
    if (it > 0) {
      if constexpr (WIDE) load_w(t0 - TT);
      else load(t0 - TT, nx, ng, nz);
    }
    // the tile's per-step dt and dy (this lane's steps) into the wave's table
    float* const br = &sBr[threadIdx.x >> 6][0][((threadIdx.x & 63) >> 2) * kBrP];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const bool tv = t0 + g * kPB + j < t_end;
      R rx, rg, rz;
      if constexpr (WIDE) {
        const int sx = (g * kPB + j) * PIT + cl;
        rx = (R)sX[buf][0][sx];
        rg = (R)sX[buf][1][sx];
        rz = (R)sX[buf][2][sx];
      } else {
        rx = cx[g];
        rg = cg[g];
        rz = cz[g];
      }
      float dt = cvt_raw(rx) + bias;
      if constexpr (SP) dt = softplus_f(dt);
      dt = tv ? dt : 0.f;
      float dy = tv ? cvt_raw(rg) : 0.f;
      if (has_z) dy *= silu_f(cvt_raw(rz));
      S += dt;
      br[g * kPB + j] = dt;
      br[16 * kBrP + g * kPB + j] = dy;
    }
    __builtin_amdgcn_wave_barrier();   // the wave's table writes precede the cross-lane f4 reads
    static_for<G>([&](auto gc) {
      constexpr int g = G - 1 - decltype(gc)::value;
      const f4 d4 = *reinterpret_cast<const f4*>(br + g * kPB);
      const f4 y4 = *reinterpret_cast<const f4*>(br + 16 * kBrP + g * kPB);
#pragma unroll
      for (int s = kPB - 1; s >= 0; --s) {
        const float dts = d4[s], dys = y4[s];
        const f4 Cq = *reinterpret_cast<const f4*>(&sC[buf][(g * kPB + s) * kN + j * kNSB]);
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          float x0 = dts * A2v[p][0], x1 = dts * A2v[p][1];
          asm volatile("" : "+v"(x0), "+v"(x1));   // plain ops, not re-packed (kPackedHazard)
          const f2 x = {x0, x1};
          const f2 e = {__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
          const f2 cv = p ? f2{Cq[2], Cq[3]} : f2{Cq[0], Cq[1]};
          float g0 = fmaf(dys, cv[0], carry2[p][0]) * e[0];
          float g1 = fmaf(dys, cv[1], carry2[p][1]) * e[1];
          asm volatile("" : "+v"(g0), "+v"(g1));   // plain ops, not re-packed (kPackedHazard)
          carry2[p] = f2{g0, g1};
        }
      }
#pragma unroll
      for (int p = 0; p < 2; ++p) asm volatile("" : "+v"(carry2[p]));
      __builtin_amdgcn_sched_barrier(0);
    });
    if (it > 0) {
      if constexpr (WIDE) {
        write_w(buf ^ 1);
      } else {
        write_stage(buf ^ 1);
#pragma unroll
        for (int g = 0; g < G; ++g) { cx[g] = nx[g]; cg[g] = ng[g]; cz[g] = nz[g]; }
      }
    }
  }
  S = group_allreduce<kPB>(S);
  if (cvalid) {
    float* sp = seg + (((int64_t)b * K + k) * f.dim + c) * (kN + 1);
#pragma unroll
    for (int i = 0; i < kNSB; ++i) sp[j * kNSB + i] = carry2[i >> 1][i & 1];
    if (j == 0) sp[kN] = S;
  }
}

// WIDE: u / delta / z / dout chunks arrive as 16-byte row pieces through LDS
// and du / ddelta / dz leave the same way (16-byte row chunks).
template <typename Tio, typename Tbc, bool SP, bool WIDE>
__global__ __launch_bounds__(kBlock, 2) void scan_bwd_kernel(const MttsScanBwdArgs a, float* __restrict__ slab,
                                                             float* __restrict__ par, const int seg_len,
                                                             const float* __restrict__ seg) {
  const MttsScanFwdArgs& f = a.f;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int j = threadIdx.x % kPB;
  const int c_raw = blockIdx.x * kChB + threadIdx.x / kPB;
  const bool cvalid = c_raw < f.dim;
  const int c = cvalid ? c_raw : f.dim - 1;
  const int b = blockIdx.y;
  const int L = f.seqlen;
  const int nck = (L + kSub - 1) / kSub;
  const int nblk = gridDim.x;
  const int kseg = blockIdx.z;
  const int K = gridDim.z;
  const int ck_begin = kseg * seg_len / kSub;
  const int ck_end = min(nck, (kseg + 1) * seg_len / kSub);

  __shared__ __attribute__((aligned(16))) float red[kWaves][kSub * 2 * kN];  // per-wave dB/dC of one chunk
  // per-wave [dt | dt*u][channel][step] of the chunk (row pitch 20 floats:
  // the 16 channels' 16-byte reads hit distinct bank groups): a lane reads
  // its channel's 4 steps of a group with one ds_read_b128 instead of four
  // DPP broadcasts (round 4: DPP costs ~2.5 plain VALU ops)
  constexpr int kBrP = 20;
  __shared__ __attribute__((aligned(16))) float sBr[kWaves][2][16 * kBrP];
  __shared__ __attribute__((aligned(16))) float sBC[kSub * 2 * kN];          // B|C of the chunk, fp32
  // WIDE staging: [buffer][u, delta, z, dout][kSub rows of the block's channels]
  constexpr int ES = (int)sizeof(Tio);
  constexpr int ROWB = kChB * ES;
  constexpr int CPR = ROWB / 16;                  // 16-B chunks per row
  constexpr int EPC = 16 / ES;
  constexpr int PIT = wide_pitch_dw(kPB, ROWB / 4, (64 / kPB) * ES / 4) * 4 / ES;
  constexpr int NIN = 4 * kSub * CPR / kBlock;    // input chunks per thread per chunk of steps
  constexpr int NOUT = (3 * kSub * CPR + kBlock - 1) / kBlock;
  __shared__ __attribute__((aligned(16))) Tio sIn[WIDE ? 2 : 1][4][WIDE ? kSub * PIT : 1];
  const int cl = threadIdx.x / kPB;                // local channel
  // exp(dt A) of state pair 1 from the replay, per wave and step (32 KiB per
  // block; with fp32 WIDE staging it would cost the second block per CU, so
  // that form recomputes it)
  constexpr bool kEL = !WIDE || sizeof(Tio) == 2;
  __shared__ __attribute__((aligned(16))) f2 sE[kEL ? kWaves : 1][kEL ? kSub : 1][64];

  // per-batch bases (uniform) + 32-bit per-lane offsets (lane j owns steps 4g+j)
  const Tio* __restrict__ u0 = (const Tio*)f.u + (int64_t)b * f.u_bs;
  const Tio* __restrict__ d0 = (const Tio*)f.delta + (int64_t)b * f.delta_bs;
  const bool has_z = f.z != nullptr;
  const Tio* __restrict__ z0 = has_z ? (const Tio*)f.z + (int64_t)b * f.z_bs : u0;  // no z: loads ignored
  const int64_t z_ls = has_z ? f.z_ls : f.u_ls;
  const Tio* __restrict__ g0 = (const Tio*)a.dout + (int64_t)b * a.dout_bs;
  Tio* __restrict__ du0 = (Tio*)a.du + (int64_t)b * a.du_bs;
  Tio* __restrict__ dd0 = (Tio*)a.ddelta + (int64_t)b * a.ddelta_bs;
  Tio* __restrict__ dz0 = a.dz ? (Tio*)a.dz + (int64_t)b * a.dz_bs : nullptr;
  const uint32_t ou = (uint32_t)(j * f.u_ls + c), od = (uint32_t)(j * f.delta_ls + c);
  const uint32_t oz = (uint32_t)(j * z_ls + c), og = (uint32_t)(j * a.dout_ls + c);
  const uint32_t odu = (uint32_t)(j * a.du_ls + c), odd = (uint32_t)(j * a.ddelta_ls + c);
  const uint32_t odz = (uint32_t)(j * a.dz_ls + c);
  // cooperative B/C staging: 2 values per thread per chunk
  const int e0 = threadIdx.x * 2;
  const int st_s = e0 / (2 * kN), st_col = e0 % (2 * kN);
  const Tbc* __restrict__ st0 = st_col < kN ? (const Tbc*)f.Bm + (int64_t)b * f.B_bs : (const Tbc*)f.Cm + (int64_t)b * f.C_bs;
  const int64_t st_ls = st_col < kN ? f.B_ls : f.C_ls;
  const int st_n = st_col % kN;

  float An[kNSB], A2[kNSB];
#pragma unroll
  for (int i = 0; i < kNSB; ++i) {
    An[i] = ld_A(f, (int64_t)c * kN + j * kNSB + i);
    A2[i] = An[i] * kLog2e;
  }
  const f2 Anv[2] = {f2{An[0], An[1]}, f2{An[2], An[3]}};
  const f2 A2v[2] = {f2{A2[0], A2[1]}, f2{A2[2], A2[3]}};
  const float Dc = f.D ? f.D[c] : 0.f;
  const float bias = f.delta_bias ? f.delta_bias[c] : 0.f;

  float carry[kNSB];
#pragma unroll
  for (int i = 0; i < kNSB; ++i) carry[i] = 0.f;
  for (int kk = K - 1; kk > kseg; --kk) {  // carry entering from later segments (pass 1)
    const float* sp = seg + (((int64_t)b * K + kk) * f.dim + c) * (kN + 1);
    const float Sk = sp[kN];
#pragma unroll
    for (int i = 0; i < kNSB; ++i) carry[i] = fmaf(__builtin_amdgcn_exp2f(A2[i] * Sk), carry[i], sp[j * kNSB + i]);
  }
  if (!cvalid) {
#pragma unroll
    for (int i = 0; i < kNSB; ++i) carry[i] = 0.f;  // with dy = 0 the lane's adjoint stays 0
  }
  f2 carry2[2] = {f2{carry[0], carry[1]}, f2{carry[2], carry[3]}};
  f2 dA2[2] = {f2{0.f, 0.f}, f2{0.f, 0.f}};
  float dD_acc = 0.f, dbias_acc = 0.f;

  // next-chunk prefetch registers (issued one chunk ahead)
  using R = raw_t<Tio>;
  R n_u[kGB], n_x[kGB], n_z[kGB], n_g[kGB];
  RawVec<Tbc, 2> n_st;
  float n_hs[kNSB];
  // WIDE: this thread's input / output chunks (array, row, column) are fixed
  uint4 wx[WIDE ? NIN : 1];
  const Tio* wsrc[WIDE ? NIN : 1];
  int64_t wls[WIDE ? NIN : 1];
  int wrow[WIDE ? NIN : 1], warr[WIDE ? NIN : 1], wcol[WIDE ? NIN : 1];
  bool wok[WIDE ? NIN : 1];
  if constexpr (WIDE) {
    const int c0 = blockIdx.x * kChB;
#pragma unroll
    for (int q = 0; q < NIN; ++q) {
      const int idx = threadIdx.x + kBlock * q;
      warr[q] = idx / (kSub * CPR);
      wrow[q] = (idx % (kSub * CPR)) / CPR;
      wcol[q] = (idx % CPR) * EPC;
      wok[q] = c0 + wcol[q] < f.dim;
      const int ar = warr[q];
      wsrc[q] = ar == 0 ? u0 : ar == 1 ? d0 : ar == 2 ? z0 : g0;
      wsrc[q] += c0 + wcol[q];
      wls[q] = ar == 0 ? f.u_ls : ar == 1 ? f.delta_ls : ar == 2 ? z_ls : a.dout_ls;
    }
  }
  // steps >= L load a clamped index (narrow) or zeros (wide); their dy is zeroed at use
  auto prefetch = [&](int k) {
    const int t_start = __builtin_amdgcn_readfirstlane(k * kSub);
    const bool full = t_start + kSub <= L;
    const int t = full ? t_start + st_s : min(t_start + st_s, L - 1);
    n_st.load(st0 + (int64_t)t * st_ls + st_n);
    load_vec<float, kNSB>(f.ckpt + (((int64_t)b * nck + k) * f.dim + c) * kN + j * kNSB, n_hs);
    if constexpr (WIDE) {
#pragma unroll
      for (int q = 0; q < NIN; ++q) {
        const int tr = t_start + wrow[q];
        const bool ok = wok[q] && tr < L;
        wx[q] = *reinterpret_cast<const uint4*>(wsrc[q] + (int64_t)(ok ? tr : 0) * wls[q]);
        if (!ok) wx[q] = make_uint4(0, 0, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int g = 0; g < kGB; ++g) {
      const int tg = t_start + g * kPB;
      if (full) {
        n_u[g] = ldr(u0 + (int64_t)tg * f.u_ls + ou);
        n_x[g] = ldr(d0 + (int64_t)tg * f.delta_ls + od);
        n_z[g] = ldr(z0 + (int64_t)tg * z_ls + oz);
        n_g[g] = ldr(g0 + (int64_t)tg * a.dout_ls + og);
      } else {
        const int tc = min(tg + j, L - 1);
        n_u[g] = ldr(u0 + (int64_t)tc * f.u_ls + c);
        n_x[g] = ldr(d0 + (int64_t)tc * f.delta_ls + c);
        n_z[g] = ldr(z0 + (int64_t)tc * z_ls + c);
        n_g[g] = ldr(g0 + (int64_t)tc * a.dout_ls + c);
      }
    }
  };
  auto write_in = [&](int buf) {
#pragma unroll
    for (int q = 0; q < NIN; ++q) *reinterpret_cast<uint4*>(&sIn[buf][warr[q]][wrow[q] * PIT + wcol[q]]) = wx[q];
  };
  if (ck_end > ck_begin) {
    prefetch(ck_end - 1);
    if constexpr (WIDE) write_in((ck_end - 1) & 1);
  }

  for (int k = ck_end - 1; k >= ck_begin; --k) {
    const int t_start = __builtin_amdgcn_readfirstlane(k * kSub);
    const bool full = t_start + kSub <= L;
    {
      float v[2];
      n_st.unpack(v);
      *reinterpret_cast<float2*>(&sBC[e0]) = make_float2(v[0], v[1]);
    }
    float uu[kGB], xr[kGB], dt[kGB], zz[kGB], go[kGB], hs[kNSB];
    const int buf = WIDE ? (k & 1) : 0;
    if constexpr (WIDE) {
      block_sync();  // staged inputs + B/C of this chunk visible
#pragma unroll
      for (int g = 0; g < kGB; ++g) {
        const int sx = (g * kPB + j) * PIT + cl;
        uu[g] = cvt_raw((R)sIn[buf][0][sx]);
        xr[g] = cvt_raw((R)sIn[buf][1][sx]) + bias;
        zz[g] = cvt_raw((R)sIn[buf][2][sx]);
        go[g] = (cvalid && (full || t_start + g * kPB + j < L)) ? cvt_raw((R)sIn[buf][3][sx]) : 0.f;
      }
    } else {
#pragma unroll
      for (int g = 0; g < kGB; ++g) {
        uu[g] = cvt_raw(n_u[g]);
        xr[g] = cvt_raw(n_x[g]) + bias;
        zz[g] = cvt_raw(n_z[g]);
        // padded steps (>= L) and lanes past `dim` contribute nothing
        go[g] = (cvalid && (full || t_start + g * kPB + j < L)) ? cvt_raw(n_g[g]) : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < kNSB; ++i) hs[i] = n_hs[i];
    if (k - 1 >= ck_begin) prefetch(k - 1);
#pragma unroll
    for (int g = 0; g < kGB; ++g) {
      float d = xr[g];
      if constexpr (SP) d = softplus_f(d);
      dt[g] = (full || t_start + g * kPB + j < L) ? d : 0.f;
    }
    // the chunk's dt and dt*u into this wave's broadcast table (the previous
    // chunk's reads of it precede these writes in the wave's program order)
    float* const br = &sBr[wave][0][(lane >> 2) * kBrP];
#pragma unroll
    for (int g = 0; g < kGB; ++g) {
      br[g * kPB + j] = dt[g];
      br[16 * kBrP + g * kPB + j] = dt[g] * uu[g];
    }
    __builtin_amdgcn_wave_barrier();   // the wave's table writes precede the cross-lane f4 reads
    auto bcast_dt = [&](int g, f4& d4, f4& u4) __attribute__((always_inline)) {
      d4 = *reinterpret_cast<const f4*>(br + g * kPB);
      u4 = *reinterpret_cast<const f4*>(br + 16 * kBrP + g * kPB);
    };
    if constexpr (!WIDE) block_sync();

    // ---- replay the chunk forward: h history in registers (state pairs, packed f32)
    f2 hh[kSub][2];
    f2 ee[kSub];   // exp(dt A) of state pair 0 (pair 1 is recomputed in the reverse pass)
    const f2 hs2[2] = {f2{hs[0], hs[1]}, f2{hs[2], hs[3]}};
    {
      f2 h2[2] = {hs2[0], hs2[1]};
#pragma unroll
      for (int g = 0; g < kGB; ++g) {
        f4 d4, u4;
        bcast_dt(g, d4, u4);
#pragma unroll
        for (int s = 0; s < kPB; ++s) {
          const float dts = d4[s], dtus = u4[s];
          const f4 Bq = *reinterpret_cast<const f4*>(&sBC[(g * kPB + s) * 2 * kN + j * kNSB]);
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            const f2 x = f2{dts, dts} * A2v[p];
            const f2 e = {__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
            const f2 bv = p ? f2{Bq[2], Bq[3]} : f2{Bq[0], Bq[1]};
            h2[p] = __builtin_elementwise_fma(e, h2[p], f2{dtus, dtus} * bv);
            hh[g * kPB + s][p] = h2[p];
            if (p == 0) ee[g * kPB + s] = e;
            else if constexpr (kEL) sE[wave][g * kPB + s][lane] = e;
          }
        }
      }
    }

    // ---- reverse pass
#pragma unroll
    for (int g = kGB - 1; g >= 0; --g) {
      float yp[kPB];
#pragma unroll
      for (int s = 0; s < kPB; ++s) {
        const f4 Cq = *reinterpret_cast<const f4*>(&sBC[(g * kPB + s) * 2 * kN + kN + j * kNSB]);
        const f2 y2 = __builtin_elementwise_fma(f2{Cq[0], Cq[1]}, hh[g * kPB + s][0], f2{Cq[2], Cq[3]} * hh[g * kPB + s][1]);
        yp[s] = y2[0] + y2[1];
      }
      const float y = fmaf(Dc, uu[g], group_reduce_scatter<kPB>(yp, j));  // pre-gate output, lane j's step
      float dy = go[g], dzv = 0.f;
      if (has_z) {
        const float sg = sigmoid_f(zz[g]);
        dy = go[g] * zz[g] * sg;
        dzv = go[g] * y * sg * (1.f + zz[g] * (1.f - sg));
      }
      dD_acc = fmaf(dy, uu[g], dD_acc);
      f4 d4, u4;
      bcast_dt(g, d4, u4);

      float ddt_p[kPB], du_p[kPB];
#pragma unroll
      for (int s = kPB - 1; s >= 0; --s) {
        float dys = s == 0 ? bcast4<0>(dy) : s == 1 ? bcast4<1>(dy) : s == 2 ? bcast4<2>(dy) : bcast4<3>(dy);
        asm volatile("" : "+v"(dys));
        const float dts = d4[s], dtus = u4[s];
        const f2 dys2 = {dys, dys}, dts2 = {dts, dts}, dtus2 = {dtus, dtus};
        const int tl = g * kPB + s;
        const f4 Bq = *reinterpret_cast<const f4*>(&sBC[tl * 2 * kN + j * kNSB]);
        const f4 Cq = *reinterpret_cast<const f4*>(&sBC[tl * 2 * kN + kN + j * kNSB]);
        f2 ddtA = {0.f, 0.f}, dus = {0.f, 0.f}, vB[2], vC[2];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const f2 bv = p ? f2{Bq[2], Bq[3]} : f2{Bq[0], Bq[1]};
          const f2 cv = p ? f2{Cq[2], Cq[3]} : f2{Cq[0], Cq[1]};
          const f2 dh = __builtin_elementwise_fma(dys2, cv, carry2[p]);
          const f2 hp = tl > 0 ? hh[tl > 0 ? tl - 1 : 0][p] : hs2[p];
          f2 e;
          if (p == 0) {
            e = ee[tl];
          } else if constexpr (kEL) {
            e = sE[wave][tl][lane];
          } else {
            const f2 x = dts2 * A2v[p];
            e = f2{__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
          }
          const f2 t1 = dh * e * hp;
          ddtA = __builtin_elementwise_fma(Anv[p], t1, ddtA);
          dus = __builtin_elementwise_fma(dh, bv, dus);
          {   // packed, but dt through a plain v_mov first (kPackedHazard)
            float dtc;
            asm volatile("v_mov_b32 %0, %1" : "=v"(dtc) : "v"(dts));
            dA2[p] = __builtin_elementwise_fma(t1, f2{dtc, dtc}, dA2[p]);
          }
          vB[p] = dh * dtus2;           // dB contribution (0 on lanes past `dim`)
          vC[p] = dys2 * hh[tl][p];     // dC contribution
          carry2[p] = e * dh;
        }
        ddt_p[s] = ddtA[0] + ddtA[1];   // + u_s * dus_s, added after the reduce (u is per step)
        du_p[s] = dus[0] + dus[1];
        const float vals[8] = {vB[0][0], vB[0][1], vB[1][0], vB[1][1], vC[0][0], vC[0][1], vC[1][0], vC[1][1]};
        // sum the 8 values over the wave's 16 channels (lane bits 2..5):
        // bit5 <- kind (permlane32 swap), bit4 <- i>>1 (permlane16 swap),
        // bit3 <- i&1 (DPP), bit2 all-reduced; no selects in the swap stages
        float a4[4], a2[2];
#pragma unroll
        for (int q = 0; q < 4; ++q) a4[q] = rs_swap32(vals[q], vals[4 + q]);
#pragma unroll
        for (int q = 0; q < 2; ++q) a2[q] = rs_swap16(a4[q], a4[q + 2]);
        const bool q3 = lane & 8;
        float a1 = (q3 ? a2[1] : a2[0]) + xor8(q3 ? a2[0] : a2[1]);
        a1 += xor4(a1, lane);
        // lanes l and l^4 hold the same sum and write it to the same slot
        // (no exec-mask round trip around the store)
        red[wave][(tl * 2 + (lane >> 5)) * kN + j * kNSB + (((lane >> 4) & 1) << 1) + ((lane >> 3) & 1)] = a1;
      }
      // per-channel results for lane j's timestep: ddt = sum_n A t1 + u * sum_n dh B
      const float dus_j = group_reduce_scatter<kPB>(du_p, j);
      const float ddt_j = fmaf(uu[g], dus_j, group_reduce_scatter<kPB>(ddt_p, j));
      const float du_j = fmaf(dus_j, dt[g], Dc * dy);
      const int tg = t_start + g * kPB;
      const bool tv = full || tg + j < L;
      float ddr = ddt_j;
      if constexpr (SP) ddr *= softplus_grad(xr[g]);
      if (tv) dbias_acc += ddr;
      if constexpr (WIDE) {  // into the chunk image (inputs of this step already consumed)
        const int sx = (g * kPB + j) * PIT + cl;
        stf(&sIn[buf][0][sx], du_j);
        stf(&sIn[buf][1][sx], ddr);
        stf(&sIn[buf][2][sx], dzv);
        continue;
      }
      // lanes past `dim` computed zeros for channel dim-1: they must not store
      if (full && cvalid) {
        stf(du0 + (int64_t)tg * a.du_ls + odu, du_j);
        stf(dd0 + (int64_t)tg * a.ddelta_ls + odd, ddr);
        if (has_z) stf(dz0 + (int64_t)tg * a.dz_ls + odz, dzv);
      } else if (tv && cvalid) {
        stf(du0 + (int64_t)(tg + j) * a.du_ls + c, du_j);
        stf(dd0 + (int64_t)(tg + j) * a.ddelta_ls + c, ddr);
        if (has_z) stf(dz0 + (int64_t)(tg + j) * a.dz_ls + c, dzv);
      }
    }
    block_sync();
    // block sum of the chunk's dB/dC -> slab[b][blk][t][2N]
    for (int q = threadIdx.x; q < kSub * 2 * kN; q += kBlock) {
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) sum += red[w][q];
      const int t = t_start + q / (2 * kN);
      if (t < L) slab[(((int64_t)b * nblk + blockIdx.x) * L + t) * (2 * kN) + (q % (2 * kN))] = sum;
    }
    if constexpr (WIDE) {
      // du / ddelta / dz chunks of this chunk of steps -> global
      const int c0 = blockIdx.x * kChB;
#pragma unroll
      for (int q = 0; q < NOUT; ++q) {
        const int idx = threadIdx.x + kBlock * q;
        if (idx < 3 * kSub * CPR) {
          const int ar = idx / (kSub * CPR), row = (idx % (kSub * CPR)) / CPR, col = (idx % CPR) * EPC;
          const int t = t_start + row;
          if (c0 + col < f.dim && t < L && (ar != 2 || has_z)) {
            Tio* dst = ar == 0 ? du0 + (int64_t)t * a.du_ls : ar == 1 ? dd0 + (int64_t)t * a.ddelta_ls
                                                                      : dz0 + (int64_t)t * a.dz_ls;
            *reinterpret_cast<uint4*>(dst + c0 + col) = *reinterpret_cast<const uint4*>(&sIn[buf][ar][row * PIT + col]);
          }
        }
      }
      if (k - 1 >= ck_begin) write_in((k - 1) & 1);
    }
  }

  dD_acc = group_allreduce<kPB>(dD_acc);
  dbias_acc = group_allreduce<kPB>(dbias_acc);
  if (cvalid) {
    float* pp = par + (((int64_t)b * K + kseg) * f.dim + c) * (kN + 2);
#pragma unroll
    for (int i = 0; i < kNSB; ++i) pp[j * kNSB + i] = dA2[i >> 1][i & 1];
    if (j == 0) { pp[kN] = dD_acc; pp[kN + 1] = dbias_acc; }
    if (a.dh0 && kseg == 0) {
#pragma unroll
      for (int i = 0; i < kNSB; ++i) a.dh0[((int64_t)b * f.dim + c) * kN + j * kNSB + i] = carry2[i >> 1][i & 1];
    }
  }
}

// One launch for both fixed-order sums of the backward's partials:
//  * blocks [0, nbc): dB[b,t,n] / dC[b,t,n] = sum over the channel blocks'
//    slabs, one float4 (4 consecutive n of B|C) per thread, the nblk loads
//    issued 8 at a time (sums stay in block order);
//  * blocks [nbc, ..): dA[c,n], dD[c], ddelta_bias[c] = sum over batch x
//    segments of the per-(b, k, c) partials (A_log given: dA_log = dA * A,
//    A = -exp(A_log)).
struct BwdReduceArgs {
  const float* slab;
  const float* par;
  int batch, nblk, L, dim, npar, nbc;
  float *dB, *dC, *dA, *dD, *dbias;
  int64_t dB_bs, dB_ls, dC_bs, dC_ls;
  const float* a_log;
};
__global__ __launch_bounds__(256) void scan_bwd_reduce(const BwdReduceArgs r) {
  if ((int)blockIdx.x < r.nbc) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;   // (b, t, k4)
    const int64_t total = (int64_t)r.batch * r.L * (2 * kN / 4);
    if (idx >= total) return;
    const int k4 = (int)(idx % (2 * kN / 4));
    const int t = (int)((idx / (2 * kN / 4)) % r.L);
    const int b = (int)(idx / ((2 * kN / 4) * (int64_t)r.L));
    const int64_t qs = (int64_t)r.L * 2 * kN;
    const float* p = r.slab + ((int64_t)b * r.nblk * r.L + t) * (2 * kN) + 4 * k4;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    int q = 0;
    for (; q + 8 <= r.nblk; q += 8) {
      f4 v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = *reinterpret_cast<const f4*>(p + (q + i) * qs);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc += v[i];
    }
    for (; q < r.nblk; ++q) acc += *reinterpret_cast<const f4*>(p + q * qs);
    const int k = 4 * k4;
    float* d = k < kN ? r.dB + b * r.dB_bs + t * r.dB_ls + k : r.dC + b * r.dC_bs + t * r.dC_ls + (k - kN);
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] = acc[i];
    return;
  }
  const int idx = ((int)blockIdx.x - r.nbc) * 256 + threadIdx.x;
  if (idx >= r.dim * (kN + 2)) return;
  const int64_t st = (int64_t)r.dim * (kN + 2);
  float s = 0.f;
  int b = 0;
  for (; b + 8 <= r.npar; b += 8) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = r.par[(b + i) * st + idx];
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[i];
  }
  for (; b < r.npar; ++b) s += r.par[b * st + idx];
  const int c = idx / (kN + 2), q = idx % (kN + 2);
  if (q < kN) r.dA[c * kN + q] = r.a_log ? s * -expf(r.a_log[c * kN + q]) : s;
  else if (q == kN) { if (r.dD) r.dD[c] = s; }
  else if (r.dbias) r.dbias[c] = s;
}

// ------------------------------------------------------------- host side
static int check_fwd(const MttsScanFwdArgs* a) {
  MTTS_CHECK(a, "scan: null args");
  MTTS_CHECK(a->batch > 0 && a->dim > 0 && a->seqlen >= 0, "scan: bad sizes b=%d d=%d l=%d", a->batch, a->dim,
             a->seqlen);
  if (a->dstate != kN) {
    set_error("scan: dstate=%d unsupported (fast path needs 16)", a->dstate);
    return MTTS_EUNSUPPORTED;
  }
  MTTS_CHECK(a->dtype_io == MTTS_F32 || a->dtype_io == MTTS_BF16, "scan: bad dtype_io");
  MTTS_CHECK(a->dtype_bc == MTTS_F32 || a->dtype_bc == MTTS_BF16, "scan: bad dtype_bc");
  MTTS_CHECK(a->u && a->delta && a->A && a->Bm && a->Cm && a->out, "scan: null tensor");
  const int esz = a->dtype_bc == MTTS_F32 ? 4 : 2;
  MTTS_CHECK(((uintptr_t)a->Bm % 16 == 0) && ((uintptr_t)a->Cm % 16 == 0) && (a->B_ls * esz) % 16 == 0 &&
                 (a->C_ls * esz) % 16 == 0 && (a->B_bs * esz) % 16 == 0 && (a->C_bs * esz) % 16 == 0,
             "scan: B/C rows must be 16-byte aligned");
  if (a->ckpt) MTTS_CHECK(a->ckpt_chunk == kSub, "scan: ckpt_chunk must be %d", kSub);
  return MTTS_OK;
}

static int pick_p(int batch, int dim) {
  const int p = override_of(MTTS_OVR_SCAN_P);
  if (p == 2 || p == 4) return p;
  const int64_t ch = (int64_t)batch * dim;
  // aim for >= 4 waves per SIMD on 256 CUs (1024 SIMDs * 4 * 64 lanes)
  if (ch >= 131072) return 2;
  return 4;
}

struct FwdPlan {
  int P, K, seg_len;
};

static FwdPlan plan_fwd(int batch, int dim, int seqlen) {
  FwdPlan pl;
  pl.P = pick_p(batch, dim);
  const int64_t lanes = (int64_t)batch * dim * pl.P;
  // >= 1 wave per SIMD on 1024 SIMDs: the LDS-DMA forward keeps its memory
  // pipeline full at one wave per SIMD, so extra state passes only cost
  // (C2, B*D = 16384: one pass 0.181 ms vs K = 4 0.195 ms, tools/scan_segs.py)
  int K = (int)((65536 + lanes - 1) / lanes);
  K = std::max(1, std::min(K, seqlen / 128));
  if (override_of(MTTS_OVR_SCAN_SEGS) >= 1) K = override_of(MTTS_OVR_SCAN_SEGS);
  int seg = (seqlen + K - 1) / K;
  seg = std::max(32, (seg + 31) / 32 * 32);
  pl.seg_len = seg;
  pl.K = std::max(1, (seqlen + seg - 1) / seg);
  return pl;
}

// backward: P = 4 lanes per channel, 2 waves/SIMD resident (<= 256 VGPRs);
// 6 x 64k lanes: C2 runs K = 6 segments (0.496 vs 0.502 ms at K = 4,
// tools/scan_lib_ab.py SWEEP, profiles/r04_scan_ab_bwd_ldsrs.jsonl)
static FwdPlan plan_bwd(int batch, int dim, int seqlen) {
  FwdPlan pl;
  pl.P = kPB;
  const int64_t lanes = (int64_t)batch * dim * kPB;
  int K = (int)((393216 + lanes - 1) / lanes);
  K = std::max(1, std::min(K, seqlen / 128));
  if (override_of(MTTS_OVR_SCAN_BWD_SEGS) >= 1) K = override_of(MTTS_OVR_SCAN_BWD_SEGS);
  int seg = (seqlen + K - 1) / K;
  seg = std::max(kSub, (seg + kSub - 1) / kSub * kSub);
  pl.seg_len = seg;
  pl.K = std::max(1, (seqlen + seg - 1) / seg);
  return pl;
}

// 16-byte chunks of u / delta / z / out rows are addressable (wide kernel)
static bool wide_io_ok(const MttsScanFwdArgs* a) {
  if (override_of(MTTS_OVR_SCAN_PATH) == 3) return false;   // narrow kernels forced
  const int es = a->dtype_io == MTTS_BF16 ? 2 : 4;
  const int64_t epc = 16 / es;
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (a->dim % epc) return false;
  if (!al(a->u) || !al(a->delta) || !al(a->out) || (a->z && !al(a->z))) return false;
  const int64_t st[] = {a->u_bs, a->u_ls, a->delta_bs, a->delta_ls, a->out_bs, a->out_ls,
                        a->z ? a->z_bs : 0, a->z ? a->z_ls : 0};
  for (int64_t v : st)
    if (v % epc) return false;
  return true;
}

// ------------------------------------------------------------- forward, one lane per channel (B*D >= 64k)
// When B*D alone gives every SIMD a wave (north-star: 32 x 2048 channels =
// 1024 waves), a lane owns ALL 16 states of one channel.  The P-lane
// machinery of the kernels above (delta / delta*u exchange, the per-step
// reduce-scatter of y and its lane selects, per-lane B/C slices) disappears:
// B/C are wave-uniform and the per-channel scalar work (softplus, SiLU gate,
// D skip) runs once per channel-step in the lane that uses it.  VALU per
// channel-step: 16 v_exp + 32 packed mul/fma + ~16 scalar.
// One wave per SIMD (the block's LDS makes a block of 4 waves own its CU);
// the waves are independent: each runs its own LDS-DMA ring of u/delta/z
// tiles NB-1 tiles ahead and its own B/C staging, with no workgroup barrier.
// Outputs leave straight from registers: one 4- (2-) byte store per lane and
// step, a wave writing 256 (128) B of one row per instruction.  VMEM issue
// order per tile `it`: [B/C regs of it+1] [DMA of it+NB-1] [checkpoint stores
// of tile it, when any] [TT y stores of tile it]; waiting until at most
// NDMA + TT operations are in flight therefore retires the B/C load and every
// older DMA, i.e. tile it+1 is complete (the checkpoint stores only make the
// wait stricter).
//
// Log2-domain state (round 4): the kernel carries dt' = softplus(x) / ln2 and
// h' = h / ln2.  Then exp(dt A) = exp2(dt' A) (A unscaled), dt' u B = dt u B / ln2
// keeps the recurrence h' = exp2(dt' A) h' + dt' u B exact in form, and
// y = ln2 (C.h' + D log2(e) u): the ln2 rides in the SiLU gate's reciprocal
// (rcp(fma(e, log2e, log2e)) = ln2 / (1 + e)).  softplus in log2 units is
// max(log2(1 + 2^min(xl, 64)), xl) for xl = x log2(e) (torch's x > 20 -> x
// threshold falls out of the max), with log1p's small-argument series below
// e = 1e-3: 10 VALU per step instead of 14.
// (B/C rows as wave-uniform scalar loads into SGPRs were tried: the kernel
// already holds 96 SGPRs, and the 32-64 more spill through v_readlane.)

template <typename Tio, typename Tbc, bool SP, bool HZ>
__global__ __launch_bounds__(256, 1) void scan_fwd_c1_kernel(const MttsScanFwdArgs a) {
  constexpr int ES = (int)sizeof(Tio);
  constexpr int EPC = 16 / ES;            // elements per 16-byte chunk
  constexpr int CPR = 64 / EPC;           // chunks per 64-channel row
  constexpr int RPD = 64 / CPR;           // rows per DMA instruction (1 KiB): 4 fp32, 8 bf16
  constexpr int DPT = ES == 4 ? 4 : 2;    // DMA instructions per array per tile
  constexpr int TT = DPT * RPD;           // steps per tile: 16
  constexpr int NB = ES == 4 ? 3 : 4;     // tile ring: DMA NB-1 tiles ahead (LDS per block: 155 / 112 KiB)
  constexpr int NAR = HZ ? 3 : 2;
  constexpr int IMG = TT * 64;
  constexpr int BCV = TT * 2 * kN / 64;   // B/C values staged per lane per tile
  constexpr int LPS = 2 * kN / BCV;       // lanes per B/C row
  constexpr int BCB = BCV * (int)sizeof(Tbc);  // bytes per lane: 16 or 32
  constexpr int NBCI = BCB > 16 ? 2 : 1;  // B/C load instructions per tile
  constexpr int NDMA = DPT * NAR;         // DMA instructions per tile
  constexpr int EA = 1;                   // exp(dt*A) formed EA steps ahead of its use
  static_assert(kN % BCV == 0 && (BCB == 16 || BCB == 32), "B/C staging");
  __shared__ __attribute__((aligned(16))) Tio sX[4][NB][NAR][IMG];
  // one B/C buffer per wave: staging for tile it+1 follows tile it's last read in program order
  __shared__ __attribute__((aligned(16))) float sBC[4][TT * 2 * kN];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  // XCD-aware: the gridDim.x blocks of one batch row (which share its B/C
  // rows) on one XCD (dispatch assigns linear id % 8 to XCDs round-robin);
  // bf16 north-star 1.993 -> 1.980 ms over three interleaved rounds, fp32 equal
  int bx = blockIdx.x, b = blockIdx.y;
  if ((gridDim.y & 7) == 0) {
    const int id = blockIdx.x + gridDim.x * blockIdx.y, j = id >> 3;
    b = (id & 7) * (gridDim.y >> 3) + j / gridDim.x;
    bx = j % gridDim.x;
  }
  const int c0 = (bx * 4 + wave) * 64;
  if (c0 >= a.dim) return;  // dim % 64 == 0 (host); no barrier anywhere below
  const int c = c0 + lane;
  const int L = a.seqlen;
  const int nt = (L + TT - 1) / TT;

  // u / delta / z / out addressed through buffer descriptors over the wave's
  // 64-channel column of the batch row (host: byte spans below 2 GiB): a
  // lane-constant offset + the row origin in a scalar register
  const int drow = lane / CPR, dcol = (lane % CPR) * EPC;
  auto span = [&](int64_t ls) { return (uint32_t)(((int64_t)(L - 1) * ls + 64) * ES); };
  const i32x4 ru = rsrc4((const Tio*)a.u + (int64_t)b * a.u_bs + c0, span(a.u_ls));
  const i32x4 rd = rsrc4((const Tio*)a.delta + (int64_t)b * a.delta_bs + c0, span(a.delta_ls));
  const i32x4 rz = HZ ? rsrc4((const Tio*)a.z + (int64_t)b * a.z_bs + c0, span(a.z_ls)) : ru;
  const uint32_t vu = (uint32_t)((drow * a.u_ls + dcol) * ES), vd = (uint32_t)((drow * a.delta_ls + dcol) * ES);
  const uint32_t vz = HZ ? (uint32_t)((drow * a.z_ls + dcol) * ES) : vu;
  const uint32_t sx0 = lds_u32(&sX[wave][0][0][0]);   // this wave's tile ring
  const uint64_t op = (uint64_t)(uintptr_t)((Tio*)a.out + (int64_t)b * a.out_bs + c0);
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(   // wave-uniform: no waterfall
      (void*)(uintptr_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(op >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)op)),
      0, __builtin_amdgcn_readfirstlane((int)span(a.out_ls)), 0x00020000);
  // staged B/C: lane -> (step row bs, column bcol of the staged [B | C] row)
  const int bs = lane / LPS, bcol = (lane % LPS) * BCV;
  const Tbc* __restrict__ gbc = bcol < kN ? (const Tbc*)a.Bm + (int64_t)b * a.B_bs + bcol
                                          : (const Tbc*)a.Cm + (int64_t)b * a.C_bs + (bcol - kN);
  const int64_t bc_ls = bcol < kN ? a.B_ls : a.C_ls;

  f2 A2[kN / 2], h[kN / 2];
#pragma unroll
  for (int p = 0; p < kN / 2; ++p) {
    const int64_t ai = (int64_t)c * kN + 2 * p;
    A2[p] = f2{ld_A(a, ai), ld_A(a, ai + 1)};                      // log2 domain: exp2(dt' A)
    const int64_t o = ((int64_t)b * a.dim + c) * kN + 2 * p;
    h[p] = a.h0 ? f2{a.h0[o] * kLog2e, a.h0[o + 1] * kLog2e} : f2{0.f, 0.f};   // h' = h / ln2
  }
  const float Dc2 = a.D ? a.D[c] * kLog2e : 0.f;
  const float bias2 = a.delta_bias ? a.delta_bias[c] * kLog2e : 0.f;
  const int nck = a.ckpt ? (L + kSub - 1) / kSub : 0;
  float* __restrict__ ck = nck ? a.ckpt + (int64_t)b * nck * a.dim * kN + (int64_t)c * kN : nullptr;
  auto store_h = [&](float* dst) __attribute__((always_inline)) {   // h = ln2 h'
#pragma unroll
    for (int q = 0; q < kN / 4; ++q) {
      const f2 lo = h[2 * q] * kLn2, hi = h[2 * q + 1] * kLn2;
      *reinterpret_cast<f4*>(dst + 4 * q) = f4{lo[0], lo[1], hi[0], hi[1]};
    }
  };

  uint32_t stg[BCB / 4];
  auto load_bc = [&](int it) __attribute__((always_inline)) {
    const Tbc* p = gbc + (int64_t)min(it * TT + bs, L - 1) * bc_ls;
#pragma unroll
    for (int q = 0; q < NBCI; ++q) {
      uint32_t w[4];
      ldg_asm<4>(w, reinterpret_cast<const char*>(p) + 16 * q);
#pragma unroll
      for (int i = 0; i < 4; ++i) stg[4 * q + i] = w[i];
    }
  };
  auto stage_bc = [&]() __attribute__((always_inline)) {
    float v[BCV];
    if constexpr (sizeof(Tbc) == 4) {
#pragma unroll
      for (int q = 0; q < BCV; ++q) v[q] = __uint_as_float(stg[q]);
    } else {
#pragma unroll
      for (int q = 0; q < BCV / 2; ++q) unpack_bf2(stg[q], v[2 * q], v[2 * q + 1]);
    }
    float* d = &sBC[wave][bs * 2 * kN + bcol];
#pragma unroll
    for (int q = 0; q < BCV / 4; ++q)
      *reinterpret_cast<f4*>(d + 4 * q) = f4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
  };
  auto dma_tile = [&](int it, int buf) __attribute__((always_inline)) {
#if defined(MTTS_C1_DIAG_NODMA)
    return;   // timing-only builds (tools/diag_build.sh): outputs are wrong; waits below drain to 0
#endif
    const uint32_t lb = sx0 + (uint32_t)(buf * NAR * IMG * ES);
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
      const int t = it * TT + k * RPD;   // rows past L read zeros (never stored)
      const uint32_t lk = lb + (uint32_t)(k * RPD * 64 * ES);
      dma16b(ru, vu, (int)(t * a.u_ls * ES), lk);
      dma16b(rd, vd, (int)(t * a.delta_ls * ES), lk + IMG * ES);
      if constexpr (HZ) dma16b(rz, vz, (int)(t * a.z_ls * ES), lk + 2 * IMG * ES);
    }
  };
  auto compute_tile = [&](auto tail, int it, int buf) __attribute__((always_inline)) {
    constexpr bool TAIL = decltype(tail)::value;
    const int t0 = it * TT;
    // B of step s+1 and C of step s are read (broadcast) during step s;
    // step 0's B goes out first
    f4 bB[2][kN / 4], bC[2][kN / 4];
    auto lds_row = [&](int s, int half, f4 (&o)[kN / 4]) __attribute__((always_inline)) {
      const f4* p = reinterpret_cast<const f4*>(&sBC[wave][s * 2 * kN + half * kN]);
#pragma unroll
      for (int q = 0; q < kN / 4; ++q) o[q] = p[q];
    };
    auto fetch_B = [&](int s) __attribute__((always_inline)) { lds_row(s, 0, bB[s & 1]); };
    auto fetch_C = [&](int s) __attribute__((always_inline)) { lds_row(s, 1, bC[s & 1]); };
    auto Bv = [&](int s, int p) __attribute__((always_inline)) -> f2 {
      const f4& q = bB[s & 1][p / 2];
      return (p & 1) ? f2{q[2], q[3]} : f2{q[0], q[1]};
    };
    auto Cv = [&](int s, int p) __attribute__((always_inline)) -> f2 {
      const f4& q = bC[s & 1][p / 2];
      return (p & 1) ? f2{q[2], q[3]} : f2{q[0], q[1]};
    };
    fetch_B(0);
    // (1) the tile's per-channel scalar work up front: TT independent chains
    float dts[TT], dtus[TT], ugs[TT], gates[TT];
#pragma unroll
    for (int s = 0; s < TT; ++s) {
      const int e = s * 64 + lane;
      const float xl = fmaf(cvt_raw((raw_t<Tio>)sX[wave][buf][1][e]), kLog2e, bias2);
      float dt = SP ? softplus_l2(xl) : xl;                          // dt / ln2
      ugs[s] = cvt_raw((raw_t<Tio>)sX[wave][buf][0][e]);
      const bool tv = !TAIL || t0 + s < L;
      dts[s] = tv ? dt : 0.f;                  // padded steps: identity map
      dtus[s] = tv ? dt * ugs[s] : 0.f;
      if constexpr (HZ) {
        const float zv = cvt_raw((raw_t<Tio>)sX[wave][buf][2][e]);
        gates[s] = zv * fast_rcp(fmaf(__builtin_amdgcn_exp2f(-zv * kLog2e), kLog2e, kLog2e));   // ln2 silu(z)
      } else {
        gates[s] = kLn2;
      }
    }
    // exp(delta*A) of step s+1 also forms during step s (independent of h):
    // the transcendental stream of one step overlaps the FMA chain of the other
    f2 ex[EA + 1][kN / 2];
    auto exps = [&](int s, f2 (&o)[kN / 2]) __attribute__((always_inline)) {
#pragma unroll
      for (int p = 0; p < kN / 2; ++p) {
        const f2 x = f2{dts[s], dts[s]} * A2[p];
        o[p] = f2{__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
      }
    };
#pragma unroll
    for (int k = 0; k < EA && k < TT; ++k) exps(k, ex[k]);
    // y of step s-1 (from h before step s's update) is formed in step s, so
    // no step ends on the dependent y tail (sum, D skip, gate, store)
    auto yout = [&](int s) __attribute__((always_inline)) {
      f2 ya = {0.f, 0.f}, yb = {0.f, 0.f};
#pragma unroll
      for (int q = 0; q < kN / 4; ++q) {
        ya = __builtin_elementwise_fma(Cv(s, 2 * q), h[2 * q], ya);
        yb = __builtin_elementwise_fma(Cv(s, 2 * q + 1), h[2 * q + 1], yb);
      }
      const f2 y2 = ya + yb;
      const float y = fmaf(Dc2, ugs[s], y2[0] + y2[1]) * gates[s];
#if defined(MTTS_C1_DIAG_NOSTORE)
      asm volatile("" ::"v"(y));
#else
      // one 4- (2-) byte store per lane and step; rows past L fall outside the range
      if constexpr (ES == 4)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(y), ro, (uint32_t)(lane * 4), (t0 + s) * (int)a.out_ls * 4, 0);
      else
        __builtin_amdgcn_raw_buffer_store_b16(f2bf(y), ro, (uint32_t)(lane * 2), (t0 + s) * (int)a.out_ls * 2, 0);
#endif
    };
#pragma unroll
    for (int s = 0; s < TT; ++s) {
      if (nck && s % kSub == 0 && ((t0 + s) & (kSub - 1)) == 0 && (!TAIL || t0 + s < L))
        store_h(ck + (int64_t)((t0 + s) / kSub) * a.dim * kN);
      if (s + 1 < TT) fetch_B(s + 1);
      fetch_C(s);
      __builtin_amdgcn_sched_barrier(0);
      if (s + EA < TT) exps(s + EA, ex[(s + EA) % (EA + 1)]);
      if (s >= 1) yout(s - 1);
      const f2 dtu2 = f2{dtus[s], dtus[s]};
#pragma unroll
      for (int p = 0; p < kN / 2; ++p) h[p] = __builtin_elementwise_fma(ex[s % (EA + 1)][p], h[p], dtu2 * Bv(s, p));
      __builtin_amdgcn_sched_barrier(0);
    }
    yout(TT - 1);
  };

  // prologue: B/C of tile 0 and the DMA of tiles 0..NB-2, all complete before tile 0
  load_bc(0);
#pragma unroll
  for (int k = 0; k < NB - 1; ++k)
    if (k < nt) dma_tile(k, k);
  wait_vm<0>(stg);
  stage_bc();
  for (int it = 0; it < nt; ++it) {
    const int buf = it % NB;
    const int prev = (it + NB - 1) % NB;
    const bool more = it + 1 < nt;
    const bool ahead = it + NB - 1 < nt;
    if (more) load_bc(it + 1);
    if (ahead) dma_tile(it + NB - 1, prev);
    if ((it + 1) * TT <= L) compute_tile(FalseT{}, it, buf);
    else compute_tile(TrueT{}, it, buf);
    if (more) {
#if defined(MTTS_C1_DIAG_NODMA) || defined(MTTS_C1_DIAG_NOSTORE)
      // the hand-counted wait below assumes exactly NDMA DMAs and TT stores
      // younger than the B/C load: a build without them must drain instead
      // (an asm load landing in a reallocated VGPR faults the GPU)
      wait_vm<0>(stg);
#else
      if (ahead) wait_vmn<NDMA + TT>(stg);  // stores of a full tile follow the DMA
      else wait_vm<0>(stg);
#endif
      stage_bc();
    }
  }
  if (a.last_state) store_h(a.last_state + ((int64_t)b * a.dim + c) * kN);
}

// the one-lane-per-channel forward applies: whole 64-channel waves, 16-byte
// B/C staging loads, and (unless forced for tests) B*D filling every SIMD
static bool c1_ok(const MttsScanFwdArgs* a) {
  const int path = override_of(MTTS_OVR_SCAN_PATH);
  if (path == 2 || !wide_io_ok(a) || a->dim % 64) return false;
  const int es = a->dtype_io == MTTS_BF16 ? 2 : 4, eb = a->dtype_bc == MTTS_BF16 ? 2 : 4;
  const int bcb = (32 / es) * 2 * kN / 64 * eb;    // B/C bytes per lane per tile
  const int64_t al = std::min(bcb, 16) / eb;       // element alignment of each load
  auto ok = [&](const void* p, int64_t bs, int64_t ls) {
    return ((uintptr_t)p % (al * eb)) == 0 && bs % al == 0 && ls % al == 0;
  };
  if (!ok(a->Bm, a->B_bs, a->B_ls) || !ok(a->Cm, a->C_bs, a->C_ls)) return false;
  // buffer-addressed rows: a batch row's byte span (and the last tile's row origin) below 2 GiB
  auto fits = [&](int64_t ls) { return (int64_t)(a->seqlen + 32) * ls * es < (1ll << 31); };
  if (!fits(a->u_ls) || !fits(a->delta_ls) || !fits(a->out_ls) || (a->z && !fits(a->z_ls))) return false;
  if (path == 1) return true;
  return (int64_t)a->batch * a->dim >= 65536;
}
template <typename Tio, typename Tbc, bool SP, bool HZ>
static void launch_c1(const MttsScanFwdArgs* a, hipStream_t st) {
  hipLaunchKernelGGL((scan_fwd_c1_kernel<Tio, Tbc, SP, HZ>), dim3((a->dim / 64 + 3) / 4, a->batch), dim3(256), 0, st,
                     *a);
}

template <int P, typename Tio, typename Tbc, bool SP>
static void launch_fwd_sp(const MttsScanFwdArgs* a, const FwdPlan& pl, hipStream_t st) {
  const int nbx = (a->dim + kBlock / P - 1) / (kBlock / P);
  float* seg = (float*)a->workspace;
  if (c1_ok(a)) {
    if (a->z) launch_c1<Tio, Tbc, SP, true>(a, st);
    else launch_c1<Tio, Tbc, SP, false>(a, st);
    return;
  }
  // the LDS-DMA kernel addresses rows through buffer descriptors: a batch
  // row's byte span (and the last tile's row origin) below 2 GiB
  const int64_t es = a->dtype_io == MTTS_BF16 ? 2 : 4;
  auto fits = [&](int64_t ls) { return (int64_t)(a->seqlen + 64) * ls * es < (1ll << 31); };
  if (wide_io_ok(a) && fits(a->u_ls) && fits(a->delta_ls) && fits(a->out_ls) && (!a->z || fits(a->z_ls))) {
    if (pl.K > 1)
      hipLaunchKernelGGL((scan_fwd_w2_kernel<P, Tio, Tbc, kState, SP>), dim3(nbx, a->batch, pl.K - 1),
                         dim3(kBlock), 0, st, *a, pl.seg_len, seg);
    hipLaunchKernelGGL((scan_fwd_w2_kernel<P, Tio, Tbc, kFull, SP>), dim3(nbx, a->batch, pl.K), dim3(kBlock), 0,
                       st, *a, pl.seg_len, seg);
    return;
  }
  if (pl.K > 1)
    hipLaunchKernelGGL((scan_fwd_kernel<P, Tio, Tbc, kState, SP>), dim3(nbx, a->batch, pl.K - 1), dim3(kBlock), 0,
                       st, *a, pl.seg_len, seg);
  hipLaunchKernelGGL((scan_fwd_kernel<P, Tio, Tbc, kFull, SP>), dim3(nbx, a->batch, pl.K), dim3(kBlock), 0, st, *a,
                     pl.seg_len, seg);
}
template <int P, typename Tio, typename Tbc>
static void launch_fwd(const MttsScanFwdArgs* a, const FwdPlan& pl, hipStream_t st) {
  if (a->delta_softplus) launch_fwd_sp<P, Tio, Tbc, true>(a, pl, st);
  else launch_fwd_sp<P, Tio, Tbc, false>(a, pl, st);
}

template <int P>
static void launch_fwd_p(const MttsScanFwdArgs* a, const FwdPlan& pl, hipStream_t st) {
  if (a->dtype_io == MTTS_F32) {
    if (a->dtype_bc == MTTS_F32) launch_fwd<P, float, float>(a, pl, st);
    else launch_fwd<P, float, bf16_t>(a, pl, st);
  } else {
    if (a->dtype_bc == MTTS_F32) launch_fwd<P, bf16_t, float>(a, pl, st);
    else launch_fwd<P, bf16_t, bf16_t>(a, pl, st);
  }
}

}  // namespace mtts

using namespace mtts;

extern "C" int64_t mtts_selective_scan_fwd_workspace(int batch, int dim, int seqlen, int dstate) {
  (void)dstate;
  const FwdPlan pl = plan_fwd(batch, dim, seqlen);
  return pl.K > 1 ? (int64_t)batch * pl.K * dim * (kN + 1) * 4 + 256 : 0;
}

extern "C" int mtts_selective_scan_fwd(const MttsScanFwdArgs* a, void* stream) {
  int rc = check_fwd(a);
  if (rc) return rc;
  if (a->seqlen == 0) return MTTS_OK;
  hipStream_t st = (hipStream_t)stream;
  const FwdPlan pl = plan_fwd(a->batch, a->dim, a->seqlen);
  if (pl.K > 1) MTTS_CHECK(a->workspace, "scan: workspace required (mtts_selective_scan_fwd_workspace)");
  if (pl.P == 2) launch_fwd_p<2>(a, pl, st);
  else launch_fwd_p<4>(a, pl, st);
  MTTS_LAUNCH_CHECK("selective_scan_fwd");
  return MTTS_OK;
}

extern "C" int64_t mtts_selective_scan_bwd_workspace(int batch, int dim, int seqlen, int dstate) {
  (void)dstate;
  const FwdPlan pl = plan_bwd(batch, dim, seqlen);
  const int64_t nblk = (dim + kChB - 1) / kChB;
  const int64_t slab = (int64_t)batch * nblk * seqlen * 2 * kN;
  const int64_t par = (int64_t)batch * pl.K * dim * (kN + 2);
  const int64_t segw = pl.K > 1 ? (int64_t)batch * pl.K * dim * (kN + 1) : 0;
  return (slab + par + segw) * 4 + 256;
}

// the backward's activations and gradients are all 16-byte addressable
static bool wide_bwd_ok(const MttsScanBwdArgs* a) {
  if (!wide_io_ok(&a->f)) return false;
  const int64_t epc = a->f.dtype_io == MTTS_BF16 ? 8 : 4;
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (!al(a->dout) || !al(a->du) || !al(a->ddelta) || (a->dz && !al(a->dz))) return false;
  const int64_t st[] = {a->dout_bs, a->dout_ls, a->du_bs, a->du_ls, a->ddelta_bs, a->ddelta_ls,
                        a->dz ? a->dz_bs : 0, a->dz ? a->dz_ls : 0};
  for (int64_t v : st)
    if (v % epc) return false;
  return true;
}

template <typename Tio, typename Tbc>
static void launch_bwd(const MttsScanBwdArgs* a, const FwdPlan& pl, float* slab, float* par, float* segw,
                       hipStream_t st) {
  const int nblk = (a->f.dim + kChB - 1) / kChB;
  const dim3 grid(nblk, a->f.batch, pl.K);
  const bool wide = wide_bwd_ok(a);
  if (pl.K > 1) {
    const dim3 cgrid(nblk, a->f.batch, pl.K - 1);
    if (a->f.delta_softplus) {
      if (wide)
        hipLaunchKernelGGL((scan_bwd_carry_kernel<Tio, Tbc, true, true>), cgrid, dim3(kBlock), 0, st, *a, pl.seg_len,
                           segw);
      else
        hipLaunchKernelGGL((scan_bwd_carry_kernel<Tio, Tbc, true, false>), cgrid, dim3(kBlock), 0, st, *a, pl.seg_len,
                           segw);
    } else {
      if (wide)
        hipLaunchKernelGGL((scan_bwd_carry_kernel<Tio, Tbc, false, true>), cgrid, dim3(kBlock), 0, st, *a, pl.seg_len,
                           segw);
      else
        hipLaunchKernelGGL((scan_bwd_carry_kernel<Tio, Tbc, false, false>), cgrid, dim3(kBlock), 0, st, *a,
                           pl.seg_len, segw);
    }
  }
  if (a->f.delta_softplus) {
    if (wide)
      hipLaunchKernelGGL((scan_bwd_kernel<Tio, Tbc, true, true>), grid, dim3(kBlock), 0, st, *a, slab, par, pl.seg_len,
                         (const float*)segw);
    else
      hipLaunchKernelGGL((scan_bwd_kernel<Tio, Tbc, true, false>), grid, dim3(kBlock), 0, st, *a, slab, par,
                         pl.seg_len, (const float*)segw);
  } else {
    if (wide)
      hipLaunchKernelGGL((scan_bwd_kernel<Tio, Tbc, false, true>), grid, dim3(kBlock), 0, st, *a, slab, par,
                         pl.seg_len, (const float*)segw);
    else
      hipLaunchKernelGGL((scan_bwd_kernel<Tio, Tbc, false, false>), grid, dim3(kBlock), 0, st, *a, slab, par,
                         pl.seg_len, (const float*)segw);
  }
}

extern "C" int mtts_selective_scan_bwd(const MttsScanBwdArgs* a, void* stream) {
  MTTS_CHECK(a, "scan_bwd: null args");
  int rc = check_fwd(&a->f);
  if (rc) return rc;
  MTTS_CHECK(a->f.ckpt && a->f.ckpt_chunk == kSub, "scan_bwd: needs the forward's ckpt with ckpt_chunk=%d", kSub);
  MTTS_CHECK(a->dout && a->du && a->ddelta && a->dB && a->dC && a->dA && a->workspace, "scan_bwd: null tensor");
  MTTS_CHECK(!a->f.z || a->dz, "scan_bwd: dz required when z is given");
  const int L = a->f.seqlen;
  if (L == 0) return MTTS_OK;
  hipStream_t st = (hipStream_t)stream;
  const FwdPlan pl = plan_bwd(a->f.batch, a->f.dim, L);
  const int nblk = (a->f.dim + kChB - 1) / kChB;
  float* slab = (float*)a->workspace;
  float* par = slab + (int64_t)a->f.batch * nblk * L * 2 * kN;
  float* segw = par + (int64_t)a->f.batch * pl.K * a->f.dim * (kN + 2);
  if (a->f.dtype_io == MTTS_F32) {
    if (a->f.dtype_bc == MTTS_F32) launch_bwd<float, float>(a, pl, slab, par, segw, st);
    else launch_bwd<float, bf16_t>(a, pl, slab, par, segw, st);
  } else {
    if (a->f.dtype_bc == MTTS_F32) launch_bwd<bf16_t, float>(a, pl, slab, par, segw, st);
    else launch_bwd<bf16_t, bf16_t>(a, pl, slab, par, segw, st);
  }
  MTTS_LAUNCH_CHECK("selective_scan_bwd");
  BwdReduceArgs r{};
  r.slab = slab; r.par = par;
  r.batch = a->f.batch; r.nblk = nblk; r.L = L; r.dim = a->f.dim; r.npar = a->f.batch * pl.K;
  const int64_t nbc4 = (int64_t)a->f.batch * L * (2 * kN / 4);
  r.nbc = (int)((nbc4 + 255) / 256);
  r.dB = a->dB; r.dB_bs = a->dB_bs; r.dB_ls = a->dB_ls;
  r.dC = a->dC; r.dC_bs = a->dC_bs; r.dC_ls = a->dC_ls;
  r.dA = a->dA; r.dD = a->dD; r.dbias = a->ddelta_bias; r.a_log = a->f.a_is_log ? a->f.A : nullptr;
  const int npb = (a->f.dim * (kN + 2) + 255) / 256;
  hipLaunchKernelGGL(scan_bwd_reduce, dim3(r.nbc + npb), dim3(256), 0, st, r);
  MTTS_LAUNCH_CHECK("selective_scan_bwd_reduce");
  return MTTS_OK;
}
