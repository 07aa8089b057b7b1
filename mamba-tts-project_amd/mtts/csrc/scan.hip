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

namespace mtts {

constexpr int kN = 16;       // d_state
constexpr int kSub = 16;     // checkpoint chunk (timesteps)
constexpr int kBlock = 256;  // threads per block

// ------------------------------------------------------------- helpers
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

// ------------------------------------------------------------- forward
template <int P, typename Tio, typename Tbc>
__global__ __launch_bounds__(kBlock) void scan_fwd_kernel(const MttsScanFwdArgs a) {
  constexpr int NS = kN / P;
  const int j = threadIdx.x % P;
  const int c_raw = blockIdx.x * (kBlock / P) + threadIdx.x / P;
  const bool cvalid = c_raw < a.dim;
  const int c = cvalid ? c_raw : a.dim - 1;
  const int b = blockIdx.y;
  const int L = a.seqlen;

  const Tio* __restrict__ u = (const Tio*)a.u + (int64_t)b * a.u_bs + c;
  const Tio* __restrict__ dl = (const Tio*)a.delta + (int64_t)b * a.delta_bs + c;
  const Tio* __restrict__ zp = a.z ? (const Tio*)a.z + (int64_t)b * a.z_bs + c : nullptr;
  Tio* __restrict__ out = (Tio*)a.out + (int64_t)b * a.out_bs + c;
  const Tbc* __restrict__ Bp = (const Tbc*)a.Bm + (int64_t)b * a.B_bs + j * NS;
  const Tbc* __restrict__ Cp = (const Tbc*)a.Cm + (int64_t)b * a.C_bs + j * NS;

  float A2[NS], h[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    A2[i] = a.A[(int64_t)c * kN + j * NS + i] * kLog2e;
    h[i] = a.h0 ? a.h0[((int64_t)b * a.dim + c) * kN + j * NS + i] : 0.f;
  }
  const float Dc = a.D ? a.D[c] : 0.f;
  const float bias = a.delta_bias ? a.delta_bias[c] : 0.f;
  const bool has_z = zp != nullptr;
  const int nck = a.ckpt ? (L + a.ckpt_chunk - 1) / a.ckpt_chunk : 0;

  // software pipeline: the loads of group g+1 are issued before group g's math
  float nu, nd, nz = 0.f;
  float nB[P][NS], nC[P][NS];
  auto issue = [&](int t0) {
    const int ts = min(t0 + j, L - 1);
    nu = ldf(u + (int64_t)ts * a.u_ls);
    nd = ldf(dl + (int64_t)ts * a.delta_ls);
    if (has_z) nz = ldf(zp + (int64_t)ts * a.z_ls);
#pragma unroll
    for (int s = 0; s < P; ++s) {
      const int tb = min(t0 + s, L - 1);
      load_vec<Tbc, NS>(Bp + (int64_t)tb * a.B_ls, nB[s]);
      load_vec<Tbc, NS>(Cp + (int64_t)tb * a.C_ls, nC[s]);
    }
  };
  if (L > 0) issue(0);

  for (int t0 = 0; t0 < L; t0 += P) {
    if (nck && (t0 % a.ckpt_chunk) == 0 && cvalid)
      store_vec<NS>(a.ckpt + (((int64_t)b * nck + t0 / a.ckpt_chunk) * a.dim + c) * kN + j * NS, h);
    const float uu = nu, dr = nd, zz = nz;
    float Bv[P][NS], Cv[P][NS];
#pragma unroll
    for (int s = 0; s < P; ++s)
#pragma unroll
      for (int i = 0; i < NS; ++i) { Bv[s][i] = nB[s][i]; Cv[s][i] = nC[s][i]; }
    if (t0 + P < L) issue(t0 + P);

    const int ts = t0 + j;
    const bool tv = ts < L;
    float dt = dr + bias;
    if (a.delta_softplus) dt = softplus_f(dt);
    dt = tv ? dt : 0.f;  // padded steps are the identity map
    const float dtu = dt * uu;
    float yp[P];
#pragma unroll
    for (int s = 0; s < P; ++s) {
      float dts, dtus;
      if constexpr (P == 1) { dts = dt; dtus = dtu; }
      else if constexpr (P == 2) {
        dts = s == 0 ? group_bcast<2, 0>(dt) : group_bcast<2, 1>(dt);
        dtus = s == 0 ? group_bcast<2, 0>(dtu) : group_bcast<2, 1>(dtu);
      } else {
        dts = s == 0 ? group_bcast<4, 0>(dt) : s == 1 ? group_bcast<4, 1>(dt)
            : s == 2 ? group_bcast<4, 2>(dt) : group_bcast<4, 3>(dt);
        dtus = s == 0 ? group_bcast<4, 0>(dtu) : s == 1 ? group_bcast<4, 1>(dtu)
             : s == 2 ? group_bcast<4, 2>(dtu) : group_bcast<4, 3>(dtu);
      }
      float y = 0.f;
#pragma unroll
      for (int i = 0; i < NS; ++i) {
        const float dA = __builtin_amdgcn_exp2f(dts * A2[i]);
        h[i] = fmaf(dA, h[i], dtus * Bv[s][i]);
        y = fmaf(Cv[s][i], h[i], y);
      }
      yp[s] = y;
    }
    float y = group_reduce_scatter<P>(yp, j);
    y = fmaf(Dc, uu, y);
    if (has_z) y *= silu_f(zz);
    if (tv && cvalid) stf(out + (int64_t)ts * a.out_ls, y);
  }
  if (a.last_state && cvalid)
    store_vec<NS>(a.last_state + ((int64_t)b * a.dim + c) * kN + j * NS, h);
}

// ------------------------------------------------------------- backward
// P = 4 lanes per channel (NS = 4 states per lane), SUB = 16 steps per chunk
// (4 groups of 4).  Per-lane register history: h and exp(dt*A) for 16 steps.
constexpr int kPB = 4;
constexpr int kNSB = kN / kPB;
constexpr int kGB = kSub / kPB;
constexpr int kChB = kBlock / kPB;   // channels per block (64)
constexpr int kWaves = kBlock / 64;
#ifndef MTTS_BWD_STORE_E
#define MTTS_BWD_STORE_E 0
#endif

template <int S>
__device__ __forceinline__ float bcast4(float v) { return dpp<S * 0x55>(v); }

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

template <typename Tio, typename Tbc>
__global__ __launch_bounds__(kBlock, 2) void scan_bwd_kernel(const MttsScanBwdArgs a, float* __restrict__ slab,
                                                             float* __restrict__ par) {
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

  __shared__ float red[kWaves][kSub * 2 * kN];  // per-wave dB/dC partials of one chunk

  const Tio* __restrict__ u = (const Tio*)f.u + (int64_t)b * f.u_bs + c;
  const Tio* __restrict__ dl = (const Tio*)f.delta + (int64_t)b * f.delta_bs + c;
  const Tio* __restrict__ zp = f.z ? (const Tio*)f.z + (int64_t)b * f.z_bs + c : nullptr;
  const Tio* __restrict__ dop = (const Tio*)a.dout + (int64_t)b * a.dout_bs + c;
  Tio* __restrict__ dup = (Tio*)a.du + (int64_t)b * a.du_bs + c;
  Tio* __restrict__ ddp = (Tio*)a.ddelta + (int64_t)b * a.ddelta_bs + c;
  Tio* __restrict__ dzp = a.dz ? (Tio*)a.dz + (int64_t)b * a.dz_bs + c : nullptr;
  const Tbc* __restrict__ Bp = (const Tbc*)f.Bm + (int64_t)b * f.B_bs + j * kNSB;
  const Tbc* __restrict__ Cp = (const Tbc*)f.Cm + (int64_t)b * f.C_bs + j * kNSB;
  const bool has_z = zp != nullptr;

  float An[kNSB], A2[kNSB];
#pragma unroll
  for (int i = 0; i < kNSB; ++i) {
    An[i] = f.A[(int64_t)c * kN + j * kNSB + i];
    A2[i] = An[i] * kLog2e;
  }
  const float Dc = f.D ? f.D[c] : 0.f;
  const float bias = f.delta_bias ? f.delta_bias[c] : 0.f;

  float carry[kNSB], dA_acc[kNSB];
#pragma unroll
  for (int i = 0; i < kNSB; ++i) { carry[i] = 0.f; dA_acc[i] = 0.f; }
  float dD_acc = 0.f, dbias_acc = 0.f;

  for (int k = nck - 1; k >= 0; --k) {
    const int t_start = k * kSub;
    float hs[kNSB];
    load_vec<float, kNSB>(f.ckpt + (((int64_t)b * nck + k) * f.dim + c) * kN + j * kNSB, hs);

    // ---- per-lane timestep data of the chunk (lane j owns steps g*4+j)
    float uu[kGB], xr[kGB], dt[kGB], zz[kGB], go[kGB];
#pragma unroll
    for (int g = 0; g < kGB; ++g) {
      const int ts = t_start + g * kPB + j;
      const bool tv = ts < L;
      const int tc = tv ? ts : L - 1;
      uu[g] = ldf(u + (int64_t)tc * f.u_ls);
      xr[g] = ldf(dl + (int64_t)tc * f.delta_ls) + bias;
      zz[g] = has_z ? ldf(zp + (int64_t)tc * f.z_ls) : 0.f;
      go[g] = tv ? ldf(dop + (int64_t)tc * a.dout_ls) : 0.f;
      const float d = f.delta_softplus ? softplus_f(xr[g]) : xr[g];
      dt[g] = tv ? d : 0.f;
    }

    // ---- replay the chunk forward: h_t and exp(dt*A) history in registers
    float hh[kSub][kNSB];
#if MTTS_BWD_STORE_E
    float eh[kSub][kNSB];
#endif
    {
      float h[kNSB];
#pragma unroll
      for (int i = 0; i < kNSB; ++i) h[i] = hs[i];
#pragma unroll
      for (int g = 0; g < kGB; ++g) {
        const float dtu = dt[g] * uu[g];
#pragma unroll
        for (int s = 0; s < kPB; ++s) {
          const float dts = s == 0 ? bcast4<0>(dt[g]) : s == 1 ? bcast4<1>(dt[g]) : s == 2 ? bcast4<2>(dt[g]) : bcast4<3>(dt[g]);
          const float dtus = s == 0 ? bcast4<0>(dtu) : s == 1 ? bcast4<1>(dtu) : s == 2 ? bcast4<2>(dtu) : bcast4<3>(dtu);
          const int tb = min(t_start + g * kPB + s, L - 1);
          float Bv[kNSB];
          load_vec<Tbc, kNSB>(Bp + (int64_t)tb * f.B_ls, Bv);
#pragma unroll
          for (int i = 0; i < kNSB; ++i) {
            const float e = __builtin_amdgcn_exp2f(dts * A2[i]);
            h[i] = fmaf(e, h[i], dtus * Bv[i]);
            hh[g * kPB + s][i] = h[i];
#if MTTS_BWD_STORE_E
            eh[g * kPB + s][i] = e;
#endif
          }
        }
      }
    }

    // ---- reverse pass
#pragma unroll
    for (int g = kGB - 1; g >= 0; --g) {
      float Cv[kPB][kNSB], Bv[kPB][kNSB];
      float yp[kPB];
#pragma unroll
      for (int s = 0; s < kPB; ++s) {
        const int tb = min(t_start + g * kPB + s, L - 1);
        load_vec<Tbc, kNSB>(Cp + (int64_t)tb * f.C_ls, Cv[s]);
        load_vec<Tbc, kNSB>(Bp + (int64_t)tb * f.B_ls, Bv[s]);
        float y = 0.f;
#pragma unroll
        for (int i = 0; i < kNSB; ++i) y = fmaf(Cv[s][i], hh[g * kPB + s][i], y);
        yp[s] = y;
      }
      // lane j: gate for its own timestep
      const float y = fmaf(Dc, uu[g], group_reduce_scatter<kPB>(yp, j));
      float dy = go[g], dzv = 0.f;
      if (has_z) {
        const float sg = sigmoid_f(zz[g]);
        const float sl = zz[g] * sg;
        dy = go[g] * sl;
        dzv = go[g] * y * sg * (1.f + zz[g] * (1.f - sg));
      }
      dD_acc = fmaf(dy, uu[g], dD_acc);

      float ddt_p[kPB], du_p[kPB];
      float vals[32];  // [s][kind][i] = s*8 + kind*4 + i
#pragma unroll
      for (int s = kPB - 1; s >= 0; --s) {
        const float dys = s == 0 ? bcast4<0>(dy) : s == 1 ? bcast4<1>(dy) : s == 2 ? bcast4<2>(dy) : bcast4<3>(dy);
        const float dts = s == 0 ? bcast4<0>(dt[g]) : s == 1 ? bcast4<1>(dt[g]) : s == 2 ? bcast4<2>(dt[g]) : bcast4<3>(dt[g]);
        const float us = s == 0 ? bcast4<0>(uu[g]) : s == 1 ? bcast4<1>(uu[g]) : s == 2 ? bcast4<2>(uu[g]) : bcast4<3>(uu[g]);
        const int tl = g * kPB + s;
        float ddt = 0.f, dus = 0.f;
#pragma unroll
        for (int i = 0; i < kNSB; ++i) {
          const float dh = fmaf(dys, Cv[s][i], carry[i]);
          const float hp = tl > 0 ? hh[tl > 0 ? tl - 1 : 0][i] : hs[i];
#if MTTS_BWD_STORE_E
          const float e = eh[tl][i];
#else
          const float e = __builtin_amdgcn_exp2f(dts * A2[i]);
#endif
          const float t1 = dh * e * hp;
          ddt = fmaf(An[i], t1, ddt);
          ddt = fmaf(dh * Bv[s][i], us, ddt);
          dus = fmaf(dh, Bv[s][i], dus);
          dA_acc[i] = fmaf(t1, dts, dA_acc[i]);
          vals[s * 8 + i] = dh * dts * us;           // dB contribution
          vals[s * 8 + 4 + i] = dys * hh[tl][i];     // dC contribution
          carry[i] = e * dh;
        }
        ddt_p[s] = ddt;
        du_p[s] = dus;
      }
      // per-channel results for lane j's timestep
      const float ddt_j = group_reduce_scatter<kPB>(ddt_p, j);
      const float du_j = fmaf(group_reduce_scatter<kPB>(du_p, j), dt[g], Dc * dy);
      const int ts = t_start + g * kPB + j;
      const bool tv = ts < L;
      const float ddr = f.delta_softplus ? ddt_j * softplus_grad(xr[g]) : ddt_j;
      if (tv) dbias_acc += ddr;
      if (tv && cvalid) {
        stf(dup + (int64_t)ts * a.du_ls, du_j);
        stf(ddp + (int64_t)ts * a.ddelta_ls, ddr);
        if (has_z) stf(dzp + (int64_t)ts * a.dz_ls, dzv);
      }
      // dB/dC: sum over the wave's 16 channels, then stash per wave in LDS
      if (!cvalid) {
#pragma unroll
        for (int q = 0; q < 32; ++q) vals[q] = 0.f;
      }
      float o0, o1;
      wave_reduce_scatter32(vals, o0, o1, lane);
      // lane holds v = (l2<<4)|(l3<<3)|(l4<<2)|(l5<<1)|e for state group j;
      // v = s*8 + kind*4 + i.  Lanes l and l^... hold distinct v; write each.
      const int vb = (((lane >> 2) & 1) << 4) | (((lane >> 3) & 1) << 3) | (((lane >> 4) & 1) << 2) |
                     (((lane >> 5) & 1) << 1);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int v = vb | e;
        const int s = v >> 3, kind = (v >> 2) & 1, i = v & 3;
        const int tl = g * kPB + s;
        red[wave][(tl * 2 + kind) * kN + j * kNSB + i] = e ? o1 : o0;
      }
    }
    __syncthreads();
    // block sum of the chunk's dB/dC -> slab[b][blk][t][2N]
    for (int q = threadIdx.x; q < kSub * 2 * kN; q += kBlock) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) s += red[w][q];
      const int tl = q / (2 * kN);
      const int t = t_start + tl;
      if (t < L) slab[(((int64_t)b * nblk + blockIdx.x) * L + t) * (2 * kN) + (q % (2 * kN))] = s;
    }
    __syncthreads();
  }

  // per-(b, c) partials for the parameter grads
  dD_acc = group_allreduce<kPB>(dD_acc);
  dbias_acc = group_allreduce<kPB>(dbias_acc);
  if (cvalid) {
    float* pp = par + ((int64_t)b * f.dim + c) * (kN + 2);
#pragma unroll
    for (int i = 0; i < kNSB; ++i) pp[j * kNSB + i] = dA_acc[i];
    if (j == 0) { pp[kN] = dD_acc; pp[kN + 1] = dbias_acc; }
    if (a.dh0) {
#pragma unroll
      for (int i = 0; i < kNSB; ++i) a.dh0[((int64_t)b * f.dim + c) * kN + j * kNSB + i] = carry[i];
    }
  }
}

// dB[b,t,n] / dC[b,t,n] = sum over channel blocks of the slab
__global__ void scan_bwd_reduce_bc(const float* __restrict__ slab, int batch, int nblk, int L, float* dB,
                                   int64_t dB_bs, int64_t dB_ls, float* dC, int64_t dC_bs, int64_t dC_ls) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)batch * L * 2 * kN;
  if (idx >= total) return;
  const int k = idx % (2 * kN);
  const int t = (idx / (2 * kN)) % L;
  const int b = idx / (2 * kN * (int64_t)L);
  const float* p = slab + ((int64_t)b * nblk * L + t) * (2 * kN) + k;
  float s = 0.f;
  for (int q = 0; q < nblk; ++q) s += p[(int64_t)q * L * 2 * kN];
  if (k < kN) dB[b * dB_bs + t * dB_ls + k] = s;
  else dC[b * dC_bs + t * dC_ls + (k - kN)] = s;
}

// dA[c,n], dD[c], ddelta_bias[c] = sum over batch of the per-(b,c) partials
__global__ void scan_bwd_reduce_par(const float* __restrict__ par, int batch, int dim, float* dA, float* dD,
                                    float* dbias) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= dim * (kN + 2)) return;
  float s = 0.f;
  for (int b = 0; b < batch; ++b) s += par[(int64_t)b * dim * (kN + 2) + idx];
  const int c = idx / (kN + 2), q = idx % (kN + 2);
  if (q < kN) dA[c * kN + q] = s;
  else if (q == kN) { if (dD) dD[c] = s; }
  else if (dbias) dbias[c] = s;
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
  if (a->ckpt) MTTS_CHECK(a->ckpt_chunk > 0 && a->ckpt_chunk % 4 == 0, "scan: ckpt_chunk %% 4 != 0");
  return MTTS_OK;
}

static int pick_p(int batch, int dim) {
  const char* e = getenv("MTTS_SCAN_P");
  if (e) {
    int p = atoi(e);
    if (p == 1 || p == 2 || p == 4) return p;
  }
  const int64_t ch = (int64_t)batch * dim;
  // aim for >= 4 waves per SIMD on 256 CUs (1024 SIMDs * 4 * 64 lanes)
  if (ch >= 262144) return 1;
  if (ch >= 131072) return 2;
  return 4;
}

template <int P, typename Tio, typename Tbc>
static void launch_fwd(const MttsScanFwdArgs* a, hipStream_t st) {
  dim3 grid((a->dim + kBlock / P - 1) / (kBlock / P), a->batch);
  hipLaunchKernelGGL((scan_fwd_kernel<P, Tio, Tbc>), grid, dim3(kBlock), 0, st, *a);
}

template <int P>
static void launch_fwd_p(const MttsScanFwdArgs* a, hipStream_t st) {
  if (a->dtype_io == MTTS_F32) {
    if (a->dtype_bc == MTTS_F32) launch_fwd<P, float, float>(a, st);
    else launch_fwd<P, float, bf16_t>(a, st);
  } else {
    if (a->dtype_bc == MTTS_F32) launch_fwd<P, bf16_t, float>(a, st);
    else launch_fwd<P, bf16_t, bf16_t>(a, st);
  }
}

}  // namespace mtts

using namespace mtts;

extern "C" int mtts_selective_scan_fwd(const MttsScanFwdArgs* a, void* stream) {
  int rc = check_fwd(a);
  if (rc) return rc;
  if (a->seqlen == 0) return MTTS_OK;
  hipStream_t st = (hipStream_t)stream;
  switch (pick_p(a->batch, a->dim)) {
    case 1: launch_fwd_p<1>(a, st); break;
    case 2: launch_fwd_p<2>(a, st); break;
    default: launch_fwd_p<4>(a, st); break;
  }
  MTTS_LAUNCH_CHECK("selective_scan_fwd");
  return MTTS_OK;
}

extern "C" int64_t mtts_selective_scan_bwd_workspace(int batch, int dim, int seqlen, int dstate) {
  (void)dstate;
  const int64_t nblk = (dim + kChB - 1) / kChB;
  const int64_t slab = (int64_t)batch * nblk * seqlen * 2 * kN;
  const int64_t par = (int64_t)batch * dim * (kN + 2);
  return (slab + par) * 4 + 256;
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
  const int nblk = (a->f.dim + kChB - 1) / kChB;
  float* slab = (float*)a->workspace;
  float* par = slab + (int64_t)a->f.batch * nblk * L * 2 * kN;
  dim3 grid(nblk, a->f.batch);
  if (a->f.dtype_io == MTTS_F32) {
    if (a->f.dtype_bc == MTTS_F32) hipLaunchKernelGGL((scan_bwd_kernel<float, float>), grid, dim3(kBlock), 0, st, *a, slab, par);
    else hipLaunchKernelGGL((scan_bwd_kernel<float, bf16_t>), grid, dim3(kBlock), 0, st, *a, slab, par);
  } else {
    if (a->f.dtype_bc == MTTS_F32) hipLaunchKernelGGL((scan_bwd_kernel<bf16_t, float>), grid, dim3(kBlock), 0, st, *a, slab, par);
    else hipLaunchKernelGGL((scan_bwd_kernel<bf16_t, bf16_t>), grid, dim3(kBlock), 0, st, *a, slab, par);
  }
  MTTS_LAUNCH_CHECK("selective_scan_bwd");
  const int64_t tot = (int64_t)a->f.batch * L * 2 * kN;
  hipLaunchKernelGGL(scan_bwd_reduce_bc, dim3((tot + 255) / 256), dim3(256), 0, st, slab, a->f.batch, nblk, L, a->dB,
                     a->dB_bs, a->dB_ls, a->dC, a->dC_bs, a->dC_ls);
  MTTS_LAUNCH_CHECK("selective_scan_bwd_reduce_bc");
  hipLaunchKernelGGL(scan_bwd_reduce_par, dim3((a->f.dim * (kN + 2) + 255) / 256), dim3(256), 0, st, par,
                     a->f.batch, a->f.dim, a->dA, a->dD, a->ddelta_bias);
  MTTS_LAUNCH_CHECK("selective_scan_bwd_reduce_par");
  return MTTS_OK;
}
