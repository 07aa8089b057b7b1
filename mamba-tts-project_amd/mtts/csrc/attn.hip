// Cross-attention core (decoder -> [ref ‖ text], style blocks) on gfx950 MFMA.
//
// Reference: nn.MultiheadAttention(batch_first=True) at mamba_decoder.py:32-36
// called at :72-77, and style_cross_attention.py:91-96/125-131, 237-242/270-276;
// torch computes softmax(q k^T * scale + key_padding_mask(-inf)) v per head,
// and a query whose keys are all masked comes out NaN.  The key side here is
// short (text + reference frames, 10^2 keys) and the query side long (audio
// frames, 10^3-10^4), so:
//
// Forward (one wave = 32 queries, workgroup = up to 4 waves):
//   * S^T = K . Q^T with the QUERY on the MFMA lane and 32 keys in registers:
//     the softmax row max / sum are lane-local plus one permlane32 swap, and
//     the exponentiated tile is directly the B operand of O^T += V^T . P^T
//     (guide §3 "accumulator tile as the next MFMA's operand");
//   * K/V blocks of 64 keys staged in LDS; V^T fragments come from the
//     row-major V image through ds_read_b64_tr_b16 (no transposing copy),
//     with a pitch that makes those reads bank-conflict free;
//   * online softmax across key tiles; l = 0 at the end gives 0/0 = NaN for a
//     fully masked query, exactly torch's result; lse = ln sum exp saved for
//     the backward.
// Backward (workgroup = all keys of one (batch, head) key group of 128, one
// wave per 32 keys; sweeps a chunk of 32-query slices):
//   * S and dP with the KEY on the lane, preloaded with -lse/scale and
//     -delta so that P = exp2(c S) and dS = P dP need no row reductions;
//   * dV += P^T dO and dK += dS^T Q from the accumulators as A operands, the
//     dO / Q B-fragments via transposed LDS reads;  dK/dV stay in registers
//     for the whole sweep;
//   * dS goes through LDS once (transposed image) for dQ = dS K, computed by
//     the wave that owns a 32-column slice of the head dim;
//   * query chunks > 1 write fp32 dK/dV partials that a second pass sums in
//     fixed order (deterministic, no atomics).
// fp32 I/O uses the exact-f32 MFMA (v_mfma_f32_32x32x2_f32) with the same
// structure.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace {
using mtts::bf16_t;
using mtts::block_sync;
using mtts::kLn2;
using mtts::kLog2e;

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// raw buffer resource over `bytes` bytes from p: loads at or past the range read 0
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

constexpr int kKB = 64;  // forward: keys per LDS block

__device__ __forceinline__ f32x16 mfma_bf16(s16x8 a, s16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0,
                                                  0);
}
__device__ __forceinline__ f32x16 mfma_f32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses row q / cols
// 4p..4p+3 of a 4x16 block; lane i receives column i, row q in element q.
__device__ __forceinline__ s16x4 tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
}
__device__ __forceinline__ s16x8 cat(s16x4 lo, s16x4 hi) {
  return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
__device__ __forceinline__ short bfbits(float x) { return __builtin_bit_cast(short, (__bf16)x); }
// registers 8s..8s+7 of a 32x32 accumulator as the bf16 fragment of k-step s:
// element j of lane half h is accumulator row 16s + 8(j>>2) + 4h + (j&3)
__device__ __forceinline__ s16x8 pack8(const f32x16& x, int s) {
  s16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = bfbits(x[8 * s + j]);
  return r;
}
// accumulator row held in register i by lane half h (32x32 C/D layout)
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

__device__ __forceinline__ float exp2_raw(float x) { return __builtin_amdgcn_exp2f(x); }

// XCD-aware block coordinates: dispatch hands linear workgroup id i to XCD
// i % 8, so the workgroups that share a (batch, head)'s K / V (forward, dQ)
// or a query chunk's Q / dO slices (dK / dV) -- consecutive x -- would land on
// all eight L2s.  Re-number so each XCD holds a contiguous 1/8 of the grid
// (x fastest): those workgroups then meet in one L2.  A bijection, so a
// kernel's work set is unchanged.  Off (plain order) for short key sides,
// where there is nothing to share and C2's forward measured 0.8 us slower.
struct Blk { int x, y, z; };
__device__ __forceinline__ Blk xcd_block(bool on = true) {
  if (!on) return {(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
  const int gx = gridDim.x, gy = gridDim.y;
  const int n = gx * gy * gridDim.z;
  const int bid = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int q8 = n / 8, r8 = n % 8, xcd = bid % 8;
  const int id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  return {id % gx, (id / gx) % gy, id / (gx * gy)};
}

// LDS pitch (elements) of a bf16 [rows][hd] image read with tr_read:
// row pitch = 16 or 48 dwords mod 64 makes the 4 rows x 32 columns of a
// 32-lane half hit 64 distinct banks.
constexpr int tr_pitch(int hd) {
  int dw = hd / 2 < 16 ? 16 : hd / 2;
  while (dw % 64 != 16 && dw % 64 != 48) ++dw;
  return dw * 2;
}

// sum over NL consecutive lanes (NL | 64, groups lane-aligned) with DPP /
// permlane stages instead of ds_bpermute shuffles
template <int NL>
__device__ __forceinline__ float lane_group_sum(float v) {
  const int lane = threadIdx.x & 63;
  if constexpr (NL >= 2) v += mtts::dpp<mtts::kQuadXor1>(v);
  if constexpr (NL >= 4) v += mtts::dpp<mtts::kQuadXor2>(v);
  if constexpr (NL >= 8) v += mtts::xor4(v, lane);
  if constexpr (NL >= 16) v += mtts::xor8(v);
  if constexpr (NL >= 32) v = mtts::sum_xor16(v);
  if constexpr (NL >= 64) v = mtts::sum_xor32(v);
  return v;
}

template <int NL>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = 1; o < NL; o <<= 1) v += __shfl_xor(v, o);
  return v;
}

// ============================================================== forward
template <typename T, int HD>
__global__ __launch_bounds__(256) void attn_fwd_kernel(MttsAttnFwdArgs a) {
  constexpr bool BF = sizeof(T) == 2;
  constexpr int KP = BF ? HD + 8 : HD + 4;   // K image: conflict-free row reads
  constexpr int VP = BF ? tr_pitch(HD) : HD;  // V image: conflict-free column reads
  constexpr int ND = (HD + 31) / 32;          // 32-row dim tiles of O^T
  constexpr int CH = 16 / sizeof(T);          // elements per 16-byte chunk
  __shared__ __attribute__((aligned(16))) T sK[kKB * KP];
  __shared__ __attribute__((aligned(16))) T sV[kKB * VP + 32];
  __shared__ uint32_t sMask[kKB / 32];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nthr = blockDim.x;
  const int r = lane & 31, h = lane >> 5;
  const int b = blockIdx.z, hh = blockIdx.y;
  const int q = (blockIdx.x * (nthr >> 6) + wave) * 32 + r;
  const bool qv = q < a.q_len;
  const T* qp = (const T*)a.q + b * a.q_bs + (int64_t)(qv ? q : 0) * a.q_ls + hh * HD;
  const T* kbase = (const T*)a.k + b * a.k_bs + hh * HD;
  const T* vbase = (const T*)a.v + b * a.v_bs + hh * HD;
  const uint8_t* mb = a.key_padding_mask ? a.key_padding_mask + b * a.mask_bs : nullptr;
  const float c = a.scale * kLog2e;

  // Q^T as the B operand (k = head dim)
  constexpr int NQ = BF ? HD / 16 : HD / 2;
  typedef typename std::conditional<BF, s16x8, float>::type QFrag;
  QFrag QF[NQ];
  if constexpr (BF) {
#pragma unroll
    for (int s = 0; s < NQ; ++s) QF[s] = qv ? *(const s16x8*)((const bf16_t*)qp + 16 * s + 8 * h) : s16x8{};
  } else {
    // f32: k-step s, lane half h <-> dim HD/2*h + s
#pragma unroll
    for (int s = 0; s < NQ; s += 4) {
      f32x4 v = qv ? *(const f32x4*)((const float*)qp + HD / 2 * h + s) : f32x4{};
      QF[s] = v[0]; QF[s + 1] = v[1]; QF[s + 2] = v[2]; QF[s + 3] = v[3];
    }
  }

  float m = -INFINITY, l = 0.f;
  f32x16 O[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) O[dt] = f32x16{};

  for (int k0 = 0; k0 < a.kv_len; k0 += kKB) {
    block_sync();
    for (int i = tid; i < kKB * HD / CH; i += nthr) {
      const int row = i / (HD / CH), cc = (i % (HD / CH)) * CH;
      const int key = k0 + row;
      f32x4 kv = {}, vv = {};
      if (key < a.kv_len) {
        kv = *(const f32x4*)(kbase + key * a.k_ls + cc);
        vv = *(const f32x4*)(vbase + key * a.v_ls + cc);
      }
      *(f32x4*)(sK + row * KP + cc) = kv;
      *(f32x4*)(sV + row * VP + cc) = vv;
    }
    if (wave == 0) {
      const int key = k0 + lane;
      const bool ok = key < a.kv_len && !(mb && mb[key]);
      const uint64_t bal = __ballot(ok);
      if (lane == 0) {
        sMask[0] = (uint32_t)bal;
        sMask[1] = (uint32_t)(bal >> 32);
      }
    }
    block_sync();
#pragma unroll
    for (int t = 0; t < kKB / 32; ++t) {
      if (k0 + t * 32 >= a.kv_len) break;
      // S^T tile: rows = 32 keys (registers), cols = 32 queries (lanes)
      f32x16 S = {};
      if constexpr (BF) {
        const bf16_t* kr = (const bf16_t*)sK + (t * 32 + r) * KP + 8 * h;
#pragma unroll
        for (int s = 0; s < NQ; ++s) S = mfma_bf16(*(const s16x8*)(kr + 16 * s), QF[s], S);
      } else {
        const float* kr = (const float*)sK + (t * 32 + r) * KP + HD / 2 * h;
#pragma unroll
        for (int s = 0; s < NQ; ++s) S = mfma_f32(kr[s], QF[s], S);
      }
      const uint32_t w = sMask[t] >> (4 * h);
      float tmax = -INFINITY;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const bool ok = (w >> ((i & 3) + 8 * (i >> 2))) & 1u;
        S[i] = ok ? S[i] * c : -INFINITY;
        tmax = fmaxf(tmax, S[i]);
      }
      tmax = mtts::max_xor32(tmax);
      const float mn = fmaxf(m, tmax);
      const float ms = mn == -INFINITY ? 0.f : mn;
      const float alpha = exp2_raw(m - ms);
      float ps = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        S[i] = exp2_raw(S[i] - ms);
        ps += S[i];
      }
      l = l * alpha + ps;
      m = mn;
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) O[dt][i] *= alpha;
      // O^T += V^T P^T
      if constexpr (BF) {
        const int g = (lane >> 4) & 1, qq = (lane >> 2) & 3, pp = lane & 3;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const s16x8 pb = pack8(S, s);
#pragma unroll
          for (int dt = 0; dt < ND; ++dt) {
            const bf16_t* p0 = (const bf16_t*)sV + (t * 32 + 16 * s + 4 * h + qq) * VP + dt * 32 + 16 * g + 4 * pp;
            O[dt] = mfma_bf16(cat(tr_read(p0), tr_read(p0 + 8 * VP)), pb, O[dt]);
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float* vr = (const float*)sV + (t * 32 + acc_row(i, h)) * VP + r;
#pragma unroll
          for (int dt = 0; dt < ND; ++dt) O[dt] = mfma_f32(vr[dt * 32], S[i], O[dt]);
        }
      }
    }
  }

  const float lt = mtts::sum_xor32(l);
  const float inv = 1.f / lt;  // fully masked: 0 * inf = NaN (torch MHA)
  if (qv) {
    T* op = (T*)a.out + b * a.o_bs + (int64_t)q * a.o_ls + hh * HD;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d0 = dt * 32 + 8 * g4 + 4 * h;
        if (d0 < HD) {
          if constexpr (BF) {
            s16x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = bfbits(O[dt][4 * g4 + e] * inv);
            *(s16x4*)((bf16_t*)op + d0) = v;
          } else {
            f32x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = O[dt][4 * g4 + e] * inv;
            *(f32x4*)((float*)op + d0) = v;
          }
        }
      }
    if (a.lse && h == 0) a.lse[((int64_t)b * a.heads + hh) * a.q_len + q] = (m + __builtin_amdgcn_logf(lt)) * kLn2;
  }
}

// Long key side, bf16, 4 waves (128 queries) per workgroup: attn_fwd_kernel
// with the K / V blocks double-buffered in LDS -- block j+1's rows are loaded
// into registers before block j's MFMAs and written to the other buffer
// after them, one barrier per 64-key block instead of a load -> barrier ->
// compute -> barrier round trip (train.py's 5248-key side: 82 blocks).
constexpr float kDeferMax = 8.f;

// One 32-key step of the online softmax on a swapped S tile (lane = query
// row r, 16 keys of half h): mask, running max, P = exp2(c*S - m) in place,
// l += sum P.  Masking only for tiles that hold padded keys (the mask word
// is wave-uniform: one scalar test per 32 keys).  Deferred max: the running
// max m (log2 units) moves only when some row of the wave grows past it by
// more than kDeferMax, so in the steady state the O accumulators are not
// touched by VALU (P <= 2^8 before its bf16 rounding; lse = m + log l holds
// for any m).
// max of 16 MFMA scores as 8 v_maximum3_f32: __builtin_elementwise_maximum
// (IEEE maximum, NaN-propagating) needs no quieting pass on MFMA results the
// compiler cannot prove canonical (fmaxf got a v_max x, x per operand), and,
// unlike the round-4 inline-asm v_max3_f32, leaves the MFMA -> VALU and
// VALU -> v_permlane32_swap wait states to the compiler: the asm form read
// stale S / t now and then (attention outputs varied by a bf16 ulp from run
// to run, tools/dbg/race_probe.py, round 5)
__device__ __forceinline__ float max3f(float a, float b, float c) {
  return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c);
}
__device__ __forceinline__ float max16_xor32(const f32x16& S) {
  float t = max3f(S[0], S[1], S[2]);
#pragma unroll
  for (int i = 3; i < 16; i += 2) t = max3f(t, S[i], S[i + 1 < 16 ? i + 1 : i]);
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(t), __float_as_uint(t), false, false);
  return __builtin_elementwise_maximum(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

template <int ND>
__device__ __forceinline__ void softmax_step(f32x16& S, uint32_t mask_word, int h, int lane, float c, float& m,
                                             float& l, f32x16 (&O)[ND]) {
  const uint32_t wm = __builtin_amdgcn_readfirstlane(mask_word);
  if (wm != 0xffffffffu) {
    const uint32_t w = wm >> (4 * h);
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (!((w >> ((i & 3) + 8 * (i >> 2))) & 1u)) S[i] = -INFINITY;
  }
  const float tmax = max16_xor32(S) * c;
  if (!__all(tmax <= m + kDeferMax)) {
    const float mn = fmaxf(m, tmax);
    const float alpha = exp2_raw(m - (mn == -INFINITY ? 0.f : mn));
    l *= alpha;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) O[dt][i] *= alpha;
    m = mn;
  }
  const float ms = m == -INFINITY ? 0.f : m;
  float ps0 = 0.f, ps1 = 0.f;
#pragma unroll
  for (int i = 0; i < 16; i += 2) {
    S[i] = exp2_raw(fmaf(S[i], c, -ms));
    S[i + 1] = exp2_raw(fmaf(S[i + 1], c, -ms));
    ps0 += S[i];
    ps1 += S[i + 1];
  }
  l += ps0 + ps1;
}

// One LDS image of a bf16 [rows][HD] tile for BOTH row reads (ds_read_b128
// of 16-byte chunk ch) and transposed reads (ds_read_b64_tr_b16 of 4 rows x
// 16 columns): unpadded rows, 16-byte chunk index XORed with a function of
// the row.  Row reads: the 8 (HD 64: same-parity) rows of a 16-lane phase hit
// distinct chunks; transposed reads: 4 consecutive rows x 4 chunks land on
// 16 distinct 4-bank groups.
template <int HD>
__device__ __forceinline__ int kswz(int row) {
  if constexpr (HD == 128) return ((row & 3) << 2) | ((row >> 2) & 3);
  else return (((row >> 1) & 1) << 2) | ((row >> 2) & 3);
}
template <int HD>
__device__ __forceinline__ int kimg(int row, int ch) { return row * HD + 8 * (ch ^ kswz<HD>(row)); }

// QT = query tiles of 32 per wave: with 2 (hd <= 64) every K / V fragment
// read from LDS feeds two MFMAs, halving the LDS bytes per MFMA.
template <int HD, int QT>
__global__ __launch_bounds__(256, 4) void attn_fwd_db_kernel(MttsAttnFwdArgs a) {
  // hd 64 / 128: K and V in the unpadded swizzled kimg image (row reads of K,
  // transposed reads of V, both conflict-free; 32 KiB per workgroup at hd 64
  // instead of 43, so 4 workgroups fit a CU); other head dims padded pitches
  constexpr bool SWZ = HD == 64 || HD == 128;
  constexpr int KP = SWZ ? HD : HD + 8;
  constexpr int VP = SWZ ? HD : tr_pitch(HD);
  constexpr int ND = (HD + 31) / 32;
  constexpr int CH = 8;
  constexpr int NQ = HD / 16;
  constexpr int NPF = kKB * HD / CH / 256;   // 16-byte K (and V) chunks per thread per block
  static_assert(NPF >= 1 && kKB * HD / CH % 256 == 0, "block staging");
  __shared__ __attribute__((aligned(16))) bf16_t sK[2][kKB * KP];
  __shared__ __attribute__((aligned(16))) bf16_t sV[2][kKB * VP + (SWZ ? 0 : 32)];
  __shared__ uint32_t sMask[2][kKB / 32];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const Blk bk = xcd_block(a.kv_len >= 1024);
  const int b = bk.z, hh = bk.y;
  const int qw = (bk.x * 4 + wave) * 32 * QT + r;   // query of tile u: qw + 32 u
  const bf16_t* kbase = (const bf16_t*)a.k + b * a.k_bs + hh * HD;
  const bf16_t* vbase = (const bf16_t*)a.v + b * a.v_bs + hh * HD;
  const uint8_t* mb = a.key_padding_mask ? a.key_padding_mask + b * a.mask_bs : nullptr;
  const float c = a.scale * kLog2e;

  s16x8 QF[QT][NQ];
#pragma unroll
  for (int u = 0; u < QT; ++u) {
    const int q = qw + 32 * u;
    const bool qv = q < a.q_len;
    const bf16_t* qp = (const bf16_t*)a.q + b * a.q_bs + (int64_t)(qv ? q : 0) * a.q_ls + hh * HD;
#pragma unroll
    for (int s = 0; s < NQ; ++s) QF[u][s] = qv ? *(const s16x8*)(qp + 16 * s + 8 * h) : s16x8{};
  }

  // Loads are issued unconditionally and consumed only in put(): a select or
  // branch on the loaded data in fetch() would make the compiler wait for
  // them before the block's MFMAs, which is exactly what this kernel avoids.
  // K / V rows as buffer loads (round 4): the lane's row / column byte offset
  // is fixed, the block's key origin rides in the scalar offset, and rows at
  // or past kv_len fall outside the buffer's range and read as zeros -- no
  // per-block 64-bit address arithmetic, clamps or selects (host: every
  // range below 2 GiB)
  f32x4 pk[NPF], pv[NPF];
  uint32_t praw = 0;
  int pk0 = 0;
  const __amdgpu_buffer_rsrc_t rk = brsrc(kbase, (uint32_t)(((int64_t)(a.kv_len - 1) * a.k_ls + HD) * 2));
  const __amdgpu_buffer_rsrc_t rv = brsrc(vbase, (uint32_t)(((int64_t)(a.kv_len - 1) * a.k_ls + HD) * 2));
  const __amdgpu_buffer_rsrc_t rm = brsrc(mb ? mb : (const uint8_t*)kbase, mb ? (uint32_t)a.kv_len : 0u);
  // K and V share the row stride (host).  hd 64: chunk i of a thread lies
  // 256 / (HD / CH) rows below chunk 0, so one lane offset serves all chunks
  // and the rest rides in the scalar offset -- one VGPR fewer, which at 4
  // waves per SIMD removes the spill whose in-loop reload made every block
  // wait (vmcnt(0)) for the next block's prefetch (C5m 609 -> 598 us,
  // profiles/r05_attn_ab_fwd_spill.txt; hd 128 measured 0.8 % slower so, keeps
  // per-chunk lane offsets)
  constexpr bool kOneOff = HD == 64;
  uint32_t ok_[kOneOff ? 1 : NPF];
#pragma unroll
  for (int i = 0; i < (kOneOff ? 1 : NPF); ++i) {
    const int idx = tid + 256 * i;
    const int row = idx / (HD / CH), cc = (idx % (HD / CH)) * CH;
    ok_[i] = (uint32_t)((row * a.k_ls + cc) * 2);
  }
  auto fetch = [&](int k0) __attribute__((always_inline)) {
    pk0 = k0;
#pragma unroll
    for (int i = 0; i < NPF; ++i) {
      const int sk = (int)((k0 + (kOneOff ? i * (256 / (HD / CH)) : 0)) * a.k_ls * 2);
      const uint32_t oi = ok_[kOneOff ? 0 : i];
      pk[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rk, oi, sk, 0));
      pv[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rv, oi, sk, 0));
    }
    praw = __builtin_amdgcn_raw_buffer_load_b8(rm, (uint32_t)lane, k0, 0);
  };
  auto put = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NPF; ++i) {
      const int idx = tid + 256 * i;
      const int row = idx / (HD / CH), cc = (idx % (HD / CH)) * CH;
      const int ko = SWZ ? kimg<HD>(row, cc / CH) : row * KP + cc;
      const int vo = SWZ ? kimg<HD>(row, cc / CH) : row * VP + cc;
      *(f32x4*)(sK[buf] + ko) = pk[i];
      *(f32x4*)(sV[buf] + vo) = pv[i];
    }
    const bool ok = pk0 + lane < a.kv_len && !(mb && praw);
    const uint64_t bal = __ballot(ok);
    if (tid == 0) {
      sMask[buf][0] = (uint32_t)bal;
      sMask[buf][1] = (uint32_t)(bal >> 32);
    }
  };

  // lane-constant image offsets: K A-fragment rows (key r, chunk 2s + h) and
  // the V^T transposed reads (keys 4h + qq (+8) of a 16-key step, dims of tile dt)
  const int g = (lane >> 4) & 1, qq = (lane >> 2) & 3, pp = lane & 3;
  int oR[NQ], oT[2][ND];
#pragma unroll
  for (int s = 0; s < NQ; ++s) oR[s] = SWZ ? kimg<HD>(r, 2 * s + h) : r * KP + 16 * s + 8 * h;
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
      oT[u][dt] = SWZ ? kimg<HD>(4 * h + qq + 8 * u, 4 * dt + 2 * g + (pp >> 1)) + 4 * (pp & 1)
                      : (4 * h + qq + 8 * u) * VP + dt * 32 + 16 * g + 4 * pp;
  float m[QT], l[QT];
  f32x16 O[QT][ND];
#pragma unroll
  for (int u = 0; u < QT; ++u) {
    m[u] = -INFINITY;
    l[u] = 0.f;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) O[u][dt] = f32x16{};
  }
  const int nblk = (a.kv_len + kKB - 1) / kKB;
  if (nblk > 0) {
    fetch(0);
    put(0);
  }
  block_sync();
  for (int j = 0; j < nblk; ++j) {
    const int buf = j & 1, k0 = j * kKB;
    fetch(min(k0 + kKB, (nblk - 1) * kKB));   // in flight under this block's math
#pragma unroll
    for (int t = 0; t < kKB / 32; ++t) {
      if (k0 + t * 32 >= a.kv_len) break;
      f32x16 S[QT];
#pragma unroll
      for (int u = 0; u < QT; ++u) S[u] = f32x16{};
      const bf16_t* kt = sK[buf] + t * 32 * KP;
#pragma unroll
      for (int s = 0; s < NQ; ++s) {
        const s16x8 kf = *(const s16x8*)(kt + oR[s]);
#pragma unroll
        for (int u = 0; u < QT; ++u) S[u] = mfma_bf16(kf, QF[u][s], S[u]);
      }
      // V^T fragments of the tile read before the softmax, so their LDS
      // latency hides under its VALU instead of stalling each PV MFMA
      s16x8 vf[2][ND];
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) {
          const bf16_t* vs = sV[buf] + (t * 32 + 16 * s) * VP;
          vf[s][dt] = cat(tr_read(vs + oT[0][dt]), tr_read(vs + oT[1][dt]));
        }
      const uint32_t mw = sMask[buf][t];
#pragma unroll
      for (int u = 0; u < QT; ++u) softmax_step<ND>(S[u], mw, h, lane, c, m[u], l[u], O[u]);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        s16x8 pb[QT];
#pragma unroll
        for (int u = 0; u < QT; ++u) pb[u] = pack8(S[u], s);
#pragma unroll
        for (int dt = 0; dt < ND; ++dt)
#pragma unroll
          for (int u = 0; u < QT; ++u) O[u][dt] = mfma_bf16(vf[s][dt], pb[u], O[u][dt]);
      }
    }
    if (j + 1 < nblk) put(buf ^ 1);
    block_sync();
  }

#pragma unroll
  for (int u = 0; u < QT; ++u) {
    const int q = qw + 32 * u;
    const float lt = mtts::sum_xor32(l[u]);
    const float inv = 1.f / lt;  // fully masked: 0 * inf = NaN (torch MHA)
    if (q < a.q_len) {
      bf16_t* op = (bf16_t*)a.out + b * a.o_bs + (int64_t)q * a.o_ls + hh * HD;
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d0 = dt * 32 + 8 * g4 + 4 * h;
          if (d0 < HD) {
            s16x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = bfbits(O[u][dt][4 * g4 + e] * inv);
            *(s16x4*)(op + d0) = v;
          }
        }
      if (a.lse && h == 0)
        a.lse[((int64_t)b * a.heads + hh) * a.q_len + q] = (m[u] + __builtin_amdgcn_logf(lt)) * kLn2;
    }
  }
}

// Short key side (kv_len <= 128, bf16: C2's 128 text keys): the whole K / V
// of the (batch, head) staged in LDS ONCE per workgroup (one barrier), then
// every wave runs NSL 32-query slices back to back with no further barrier,
// the next slice's Q fragments loaded into registers while the current one
// computes.  Same math per slice as attn_fwd_kernel (all keys in one tile
// sweep, online max / sum across the four 32-key tiles).
constexpr int kShortKV = 128;

template <int HD>
__global__ __launch_bounds__(256, 2) void attn_fwd_short_kernel(MttsAttnFwdArgs a, int nsl) {
  constexpr int KP = HD + 8;         // K image: conflict-free row reads
  constexpr int VP = tr_pitch(HD);   // V image: conflict-free column reads
  constexpr int ND = (HD + 31) / 32;
  constexpr int CH = 8;
  constexpr int NQ = HD / 16;
  __shared__ __attribute__((aligned(16))) bf16_t sK[kShortKV * KP];
  __shared__ __attribute__((aligned(16))) bf16_t sV[kShortKV * VP + 32];
  __shared__ uint32_t sMask[kShortKV / 32];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int b = blockIdx.z, hh = blockIdx.y;
  const bf16_t* kbase = (const bf16_t*)a.k + b * a.k_bs + hh * HD;
  const bf16_t* vbase = (const bf16_t*)a.v + b * a.v_bs + hh * HD;
  const uint8_t* mb = a.key_padding_mask ? a.key_padding_mask + b * a.mask_bs : nullptr;
  const float c = a.scale * kLog2e;
  const int nkt = (a.kv_len + 31) / 32;

  // query slice sl of this wave: 32 queries
  auto qrow = [&](int sl) { return ((blockIdx.x * nsl + sl) * nw + wave) * 32 + r; };
  s16x8 QF[NQ], QN[NQ];
  auto load_q = [&](int sl, s16x8 (&o)[NQ]) {
    const int q = qrow(sl);
    const bool qv = sl < nsl && q < a.q_len;
    const bf16_t* qp = (const bf16_t*)a.q + b * a.q_bs + (int64_t)(qv ? q : 0) * a.q_ls + hh * HD;
#pragma unroll
    for (int s = 0; s < NQ; ++s) o[s] = qv ? *(const s16x8*)(qp + 16 * s + 8 * h) : s16x8{};
  };
  load_q(0, QF);

  for (int i = tid; i < kShortKV * HD / CH; i += blockDim.x) {
    const int row = i / (HD / CH), cc = (i % (HD / CH)) * CH;
    f32x4 kv = {}, vv = {};
    if (row < a.kv_len) {
      kv = *(const f32x4*)(kbase + row * a.k_ls + cc);
      vv = *(const f32x4*)(vbase + row * a.v_ls + cc);
    }
    *(f32x4*)(sK + row * KP + cc) = kv;
    *(f32x4*)(sV + row * VP + cc) = vv;
  }
  if (wave < kShortKV / 64) {
    const int key = 64 * wave + lane;
    const bool ok = key < a.kv_len && !(mb && mb[key]);
    const uint64_t bal = __ballot(ok);
    if (lane == 0) {
      sMask[2 * wave] = (uint32_t)bal;
      sMask[2 * wave + 1] = (uint32_t)(bal >> 32);
    }
  }
  block_sync();

  for (int sl = 0; sl < nsl; ++sl) {
    if (sl + 1 < nsl) load_q(sl + 1, QN);   // in flight under this slice
    const int q = qrow(sl);
    float m = -INFINITY, l = 0.f;
    f32x16 O[ND];
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) O[dt] = f32x16{};
#pragma unroll
    for (int t = 0; t < kShortKV / 32; ++t) {
      if (t >= nkt) break;
      f32x16 S = {};
      const bf16_t* kr = sK + (t * 32 + r) * KP + 8 * h;
#pragma unroll
      for (int s = 0; s < NQ; ++s) S = mfma_bf16(*(const s16x8*)(kr + 16 * s), QF[s], S);
      softmax_step<ND>(S, sMask[t], h, lane, c, m, l, O);
      const int g = (lane >> 4) & 1, qq = (lane >> 2) & 3, pp = lane & 3;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const s16x8 pb = pack8(S, s);
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) {
          const bf16_t* p0 = sV + (t * 32 + 16 * s + 4 * h + qq) * VP + dt * 32 + 16 * g + 4 * pp;
          O[dt] = mfma_bf16(cat(tr_read(p0), tr_read(p0 + 8 * VP)), pb, O[dt]);
        }
      }
    }
    const float lt = mtts::sum_xor32(l);
    const float inv = 1.f / lt;  // fully masked: 0 * inf = NaN (torch MHA)
    if (q < a.q_len) {
      bf16_t* op = (bf16_t*)a.out + b * a.o_bs + (int64_t)q * a.o_ls + hh * HD;
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d0 = dt * 32 + 8 * g4 + 4 * h;
          s16x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = bfbits(O[dt][4 * g4 + e] * inv);
          *(s16x4*)(op + d0) = v;
        }
      if (a.lse && h == 0) a.lse[((int64_t)b * a.heads + hh) * a.q_len + q] = (m + __builtin_amdgcn_logf(lt)) * kLn2;
    }
#pragma unroll
    for (int s = 0; s < NQ; ++s) QF[s] = QN[s];
  }
}

// ============================================================== backward
struct BwdParams {
  MttsAttnBwdArgs a;
  int nchunk, qchunk;  // query chunks (grid.x) and queries per chunk (multiple of 32)
  float* part;         // nchunk > 1: fp32 dK|dV partials [nchunk][B][Tk][2*H*hd]
  float* dq_acc;       // > 1 key group (mode 0): fp32 dq accumulator [B][Tq][H*hd]
  float* delta;        // modes 1/2: -rowsum(dO * O) per (b, h, query) [B][H][Tq]
  int dq_vec;          // dq base / row stride 16-byte aligned: 16-byte dQ row stores
};

// Backward modes.  0: short key side (C2, <= one key group): workgroup =
// (query chunk, head, batch), dK/dV of all keys + dQ.  Long key side (the
// train.py shape, 5k reference keys) splits the work in two launches:
// 2 (first): workgroup = one 32-query slice; loops over all key groups with
//    dQ in registers (no global accumulator); writes -delta per query;
// 1: workgroup = one key group; sweeps all queries with dK/dV in registers
//    (complete: no partials, no reduce pass); delta from mode 2.
constexpr int kBwdShort = 0, kBwdKV = 1, kBwdQ = 2;

template <typename T, int HD>
struct BwdCfg {
  static constexpr bool BF = sizeof(T) == 2;
  static constexpr int KG = (!BF && HD > 64) ? 64 : 128;  // keys per group = 32 x waves
  static constexpr int NW = KG / 32;
  static constexpr int P = BF ? HD + 8 : HD + 4;           // Q / dO / K / V image pitch
  static constexpr int PS = BF ? 32 : 36;                  // dS^T image pitch (queries)
  static constexpr int ND = (HD + 31) / 32;
};

template <typename T, int HD, int MODE>
__global__ __launch_bounds__(256) void attn_bwd_kernel(BwdParams p) {
  using C = BwdCfg<T, HD>;
  constexpr bool BF = C::BF;
  constexpr int KG = C::KG, NW = C::NW, P = C::P, PS = C::PS, ND = C::ND;
  constexpr int CH = 16 / sizeof(T);
  constexpr int NQ = BF ? HD / 16 : HD / 2;
  __shared__ __attribute__((aligned(16))) T sK[KG * P + 32];
  __shared__ __attribute__((aligned(16))) T sV[KG * P + 32];
  __shared__ __attribute__((aligned(16))) T sQ[32 * P + 32];
  __shared__ __attribute__((aligned(16))) T sO[32 * P + 32];  // dO image
  __shared__ __attribute__((aligned(16))) T sS[KG * PS + 32];  // dS^T [key][query]
  __shared__ float sL[32], sD[32];
  __shared__ uint32_t sMask[KG / 32];
  // per wave: its 32x32 dQ tile on the way to 16-byte row stores
  constexpr int DQP = 32 + 16 / sizeof(T);
  __shared__ __attribute__((aligned(16))) T sDq[NW][32 * DQP];

  const MttsAttnBwdArgs& a = p.a;
  const MttsAttnFwdArgs& f = a.f;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int nthr = NW * 64;
  const int r = lane & 31, h = lane >> 5;
  const int g = (lane >> 4) & 1, qq = (lane >> 2) & 3, pp = lane & 3;  // tr_read addressing
  const int b = blockIdx.z, hh = blockIdx.y, chunk = blockIdx.x;
  const int d = f.heads * HD;
  const int nkg = (f.kv_len + KG - 1) / KG;
  // mode 1: grid.x = key group x query chunk (chunk of p.qchunk queries)
  const int kv_kg = chunk % nkg, qc = MODE == kBwdKV ? chunk / nkg : chunk;
  const int qbeg = MODE == kBwdQ ? 32 * chunk : qc * p.qchunk;
  const int qend = min(f.q_len, MODE == kBwdQ ? qbeg + 32 : qbeg + p.qchunk);
  const float c = f.scale * kLog2e;
  const float inv_scale = 1.f / f.scale;
  const uint8_t* mb = f.key_padding_mask ? f.key_padding_mask + b * f.mask_bs : nullptr;
  float* const dbuf = p.delta ? p.delta + ((int64_t)b * f.heads + hh) * f.q_len : nullptr;
  constexpr int NQT = (ND + NW - 1) / NW;   // mode 2: dQ tiles per wave, held across key groups
  f32x16 QA[NQT];
#pragma unroll
  for (int t = 0; t < NQT; ++t) QA[t] = f32x16{};

  for (int kg = MODE == kBwdKV ? kv_kg : 0; kg < (MODE == kBwdKV ? kv_kg + 1 : nkg); ++kg) {
    const int kg0 = kg * KG;
    block_sync();
    {
      const T* kb = (const T*)f.k + b * f.k_bs + hh * HD;
      const T* vb = (const T*)f.v + b * f.v_bs + hh * HD;
      for (int i = tid; i < KG * HD / CH; i += nthr) {
        const int row = i / (HD / CH), cc = (i % (HD / CH)) * CH;
        const int key = kg0 + row;
        f32x4 kv = {}, vv = {};
        if (key < f.kv_len) {
          kv = *(const f32x4*)(kb + key * f.k_ls + cc);
          vv = *(const f32x4*)(vb + key * f.v_ls + cc);
        }
        *(f32x4*)(sK + row * P + cc) = kv;
        *(f32x4*)(sV + row * P + cc) = vv;
      }
      if (wave < KG / 64) {
        const int key = kg0 + 64 * wave + lane;
        const bool ok = key < f.kv_len && !(mb && mb[key]);
        const uint64_t bal = __ballot(ok);
        if (lane == 0) {
          sMask[2 * wave] = (uint32_t)bal;
          sMask[2 * wave + 1] = (uint32_t)(bal >> 32);
        }
      }
    }
    f32x16 dK[ND], dV[ND];
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) dK[dt] = dV[dt] = f32x16{};

    // Q / dO / O of a 32-query slice are loaded into registers ONE SLICE
    // AHEAD (issued right after the current slice is staged), so their
    // global-memory latency hides under the current slice's MFMAs instead of
    // sitting between two barriers of every slice.
    constexpr int NPT = (32 * HD / CH + nthr - 1) / nthr;   // 16-byte chunks per thread per array
    const T* qb = (const T*)f.q + b * f.q_bs + hh * HD;
    const T* ob = (const T*)f.out + b * f.o_bs + hh * HD;
    const T* gb = (const T*)a.dout + b * a.do_bs + hh * HD;
    f32x4 pq[NPT], pg[NPT], po[NPT];
    float plse = 0.f;
    auto load_slice = [&](int q0) {
      if (tid < 32) {
        const int qi = q0 + tid;
        plse = qi < qend ? f.lse[((int64_t)b * f.heads + hh) * f.q_len + qi] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < NPT; ++j) {
        const int i = tid + j * nthr;
        const int row = i / (HD / CH), cc = (i % (HD / CH)) * CH;
        const int qi = q0 + row;
        pq[j] = pg[j] = po[j] = f32x4{};
        if (i < 32 * HD / CH && qi < qend) {
          pq[j] = *(const f32x4*)(qb + qi * f.q_ls + cc);
          pg[j] = *(const f32x4*)(gb + qi * a.do_ls + cc);
          if constexpr (MODE != kBwdKV) po[j] = *(const f32x4*)(ob + qi * f.o_ls + cc);
        }
      }
    };
    if (MODE != kBwdQ || kg == 0) load_slice(qbeg);
    for (int q0 = qbeg; q0 < qend; q0 += 32) {
      block_sync();
      // ---- stage Q, dO images; delta = rowsum(dO * O); -lse/scale
      // (mode 2: its single slice once, kept across key groups)
      if (MODE != kBwdQ || kg == 0) {
#pragma unroll
        for (int j = 0; j < NPT; ++j) {
          const int i = tid + j * nthr;
          if (NPT * nthr != 32 * HD / CH && i >= 32 * HD / CH) break;
          const int row = i / (HD / CH), cc = (i % (HD / CH)) * CH;
          const int qi = q0 + row;
          const f32x4 qv = pq[j], gv = pg[j], ov = po[j];
          *(f32x4*)(sQ + row * P + cc) = qv;
          *(f32x4*)(sO + row * P + cc) = gv;
          float dl = 0.f;
          if constexpr (BF) {
            const s16x8 g8 = __builtin_bit_cast(s16x8, gv), o8 = __builtin_bit_cast(s16x8, ov);
#pragma unroll
            for (int e = 0; e < 8; ++e) dl += mtts::bf2f((bf16_t)g8[e]) * mtts::bf2f((bf16_t)o8[e]);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) dl += gv[e] * ov[e];
          }
          dl = lane_group_sum<HD / CH>(dl);
          if constexpr (MODE != kBwdKV) {
            if (i % (HD / CH) == 0) {
              sD[row] = -dl;
              if (MODE == kBwdQ && qi < qend) dbuf[qi] = -dl;
            }
          }
        }
        if constexpr (MODE == kBwdKV) {
          if (tid < 32) sD[tid] = q0 + tid < qend ? dbuf[q0 + tid] : 0.f;
        }
        if (tid < 32) sL[tid] = q0 + tid < qend ? -plse * inv_scale : 0.f;  // P = exp2(c (S + L))
        if (MODE != kBwdQ && q0 + 32 < qend) load_slice(q0 + 32);   // next slice, in flight under this one
      }
      block_sync();
      // ---- S = Q K^T - lse/scale and dP = dO V^T - delta (key on the lane)
      f32x16 S, D;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        S[i] = sL[acc_row(i, h)];
        D[i] = sD[acc_row(i, h)];
      }
      const int key = wave * 32 + r;  // within the group
      if constexpr (BF) {
        const bf16_t* qr = (const bf16_t*)sQ + r * P + 8 * h;
        const bf16_t* orow = (const bf16_t*)sO + r * P + 8 * h;
        const bf16_t* kr = (const bf16_t*)sK + key * P + 8 * h;
        const bf16_t* vr = (const bf16_t*)sV + key * P + 8 * h;
#pragma unroll
        for (int s = 0; s < NQ; ++s) {
          S = mfma_bf16(*(const s16x8*)(qr + 16 * s), *(const s16x8*)(kr + 16 * s), S);
          D = mfma_bf16(*(const s16x8*)(orow + 16 * s), *(const s16x8*)(vr + 16 * s), D);
        }
      } else {
        const float* qr = (const float*)sQ + r * P + HD / 2 * h;
        const float* orow = (const float*)sO + r * P + HD / 2 * h;
        const float* kr = (const float*)sK + key * P + HD / 2 * h;
        const float* vr = (const float*)sV + key * P + HD / 2 * h;
#pragma unroll
        for (int s = 0; s < NQ; ++s) {
          S = mfma_f32(qr[s], kr[s], S);
          D = mfma_f32(orow[s], vr[s], D);
        }
      }
      const bool kvalid = (sMask[wave] >> r) & 1u;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        S[i] = kvalid ? exp2_raw(c * S[i]) : 0.f;  // P
        D[i] = S[i] * D[i];                         // dS (unscaled)
      }
      // ---- dV += P^T dO, dK += dS^T Q (accumulators as A operands)
      if constexpr (BF) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          if constexpr (MODE == kBwdQ) break;
          const s16x8 pa = pack8(S, s), da = pack8(D, s);
#pragma unroll
          for (int dt = 0; dt < ND; ++dt) {
            const int off = (16 * s + 4 * h + qq) * P + dt * 32 + 16 * g + 4 * pp;
            const bf16_t* po = (const bf16_t*)sO + off;
            const bf16_t* pq = (const bf16_t*)sQ + off;
            dV[dt] = mfma_bf16(pa, cat(tr_read(po), tr_read(po + 8 * P)), dV[dt]);
            dK[dt] = mfma_bf16(da, cat(tr_read(pq), tr_read(pq + 8 * P)), dK[dt]);
          }
        }
        // dS^T image: lane (key) stores query rows 8g4+4h..+3 (read by the dQ
        // product only: not in the dK/dV pass)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          if constexpr (MODE == kBwdKV) break;
          s16x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = bfbits(D[4 * g4 + e]);
          *(s16x4*)((bf16_t*)sS + key * PS + 8 * g4 + 4 * h) = v;
        }
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          if constexpr (MODE == kBwdQ) break;
          const int row = acc_row(i, h);
          const float* po = (const float*)sO + row * P + r;
          const float* pq = (const float*)sQ + row * P + r;
#pragma unroll
          for (int dt = 0; dt < ND; ++dt) {
            dV[dt] = mfma_f32(S[i], po[dt * 32], dV[dt]);
            dK[dt] = mfma_f32(D[i], pq[dt * 32], dK[dt]);
          }
        }
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4)
          if constexpr (MODE != kBwdKV) *(f32x4*)((float*)sS + key * PS + 8 * g4 + 4 * h) =
              f32x4{D[4 * g4], D[4 * g4 + 1], D[4 * g4 + 2], D[4 * g4 + 3]};
      }
      if constexpr (MODE == kBwdKV) continue;   // dQ comes from the mode-2 launch
      block_sync();
      // ---- dQ[q][dims of tile dt] = scale * dS K over the group's keys
      for (int dt = wave; dt < ND; dt += NW) {
        f32x16 Q = MODE == kBwdQ ? QA[(dt - wave) / NW] : f32x16{};
        if constexpr (BF) {
#pragma unroll
          for (int s = 0; s < KG / 16; ++s) {
            const bf16_t* ps = (const bf16_t*)sS + (16 * s + 8 * h + qq) * PS + 16 * g + 4 * pp;
            const bf16_t* pk = (const bf16_t*)sK + (16 * s + 8 * h + qq) * P + dt * 32 + 16 * g + 4 * pp;
            Q = mfma_bf16(cat(tr_read(ps), tr_read(ps + 4 * PS)), cat(tr_read(pk), tr_read(pk + 4 * P)), Q);
          }
        } else {
#pragma unroll 8
          for (int s = 0; s < KG / 2; ++s) {
            const int kk = KG / 2 * h + s;
            Q = mfma_f32(((const float*)sS)[kk * PS + r], ((const float*)sK)[kk * P + dt * 32 + r], Q);
          }
        }
        if constexpr (MODE == kBwdQ) {
          QA[(dt - wave) / NW] = Q;                // summed over all key groups, written after
          continue;
        }
        const int dim = dt * 32 + r;
        if (nkg == 1 && HD % 32 == 0 && p.dq_vec) {
          // one key group: the tile is final.  Through the wave's LDS tile so
          // each lane stores whole 16-byte row pieces (a lane's accumulator
          // holds one column: 16 two-byte stores per lane otherwise, and the
          // store issue, not the MFMAs, set the slice time)
          T* t = sDq[wave];
#pragma unroll
          for (int i = 0; i < 16; ++i) mtts::stf(t + acc_row(i, h) * DQP + r, Q[i] * f.scale);
          __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the wave's own LDS writes, read back below
          __builtin_amdgcn_wave_barrier();
          constexpr int CPRW = 32 * sizeof(T) / 16;   // 16-byte pieces per tile row
#pragma unroll
          for (int j = 0; j < 32 * CPRW / 64; ++j) {
            const int idx = lane + 64 * j, row = idx / CPRW, cc = (idx % CPRW) * (16 / sizeof(T));
            const int qi = q0 + row;
            if (qi < qend)
              *(f32x4*)((T*)a.dq + b * a.dq_bs + (int64_t)qi * a.dq_ls + hh * HD + dt * 32 + cc) =
                  *(const f32x4*)(t + row * DQP + cc);
          }
          __builtin_amdgcn_wave_barrier();
        } else if (dim < HD) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int qi = q0 + acc_row(i, h);
            if (qi < qend) {
              float v = Q[i] * f.scale;
              if (nkg > 1) {
                float* acc = p.dq_acc + ((int64_t)b * f.q_len + qi) * d + hh * HD + dim;
                if (kg > 0) v += *acc;
                if (kg + 1 < nkg) {
                  *acc = v;
                  continue;
                }
              }
              mtts::stf((T*)a.dq + b * a.dq_bs + (int64_t)qi * a.dq_ls + hh * HD + dim, v);
            }
          }
        }
      }
    }
    // ---- dK (scaled), dV of this wave's 32 keys: rows = keys (registers), cols = dims (lanes)
    if constexpr (MODE == kBwdQ) continue;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
      const int dim = dt * 32 + r;
      if (dim >= HD) continue;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int kk = kg0 + wave * 32 + acc_row(i, h);
        if (kk >= f.kv_len) continue;
        const float vk = dK[dt][i] * f.scale, vv = dV[dt][i];
        if (p.nchunk > 1) {
          float* pr = p.part + (((int64_t)qc * f.batch + b) * f.kv_len + kk) * (2 * d) + hh * HD + dim;
          pr[0] = vk;
          pr[d] = vv;
        } else {
          mtts::stf((T*)a.dk + b * a.dk_bs + (int64_t)kk * a.dk_ls + hh * HD + dim, vk);
          mtts::stf((T*)a.dv + b * a.dv_bs + (int64_t)kk * a.dv_ls + hh * HD + dim, vv);
        }
      }
    }
  }
  if constexpr (MODE == kBwdQ) {
#pragma unroll
    for (int t = 0; t < NQT; ++t) {
      const int dt = wave + t * NW;
      const int dim = dt * 32 + r;
      if (dt >= ND || dim >= HD) continue;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qi = qbeg + acc_row(i, h);
        if (qi < qend) mtts::stf((T*)a.dq + b * a.dq_bs + (int64_t)qi * a.dq_ls + hh * HD + dim, QA[t][i] * f.scale);
      }
    }
  }
}

// 16-byte / 4-byte LDS-DMA through a buffer descriptor (round 6, the long-key
// backward passes): lane l's bytes land at lds + 16 * l (4 * l) -- M0 holds the
// wave-uniform LDS base --, the row origin rides in the scalar offset and
// offsets past the descriptor's range read 0.  Inline asm (invisible to the
// compiler's wait insertion): every consumer waits by an explicit counted
// vmcnt + block_sync.  Default cache policy: each slice is re-read by every
// key group of its (batch, head) from L2.
typedef int i32x4a __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4a rsrc4a(const void* p, uint32_t bytes) {   // p, bytes wave-uniform
  const uint64_t q = (uint64_t)(uintptr_t)p;
  return i32x4a{__builtin_amdgcn_readfirstlane((int)(uint32_t)q), __builtin_amdgcn_readfirstlane((int)((q >> 32) & 0xffff)),
                __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000};
}
__device__ __forceinline__ uint32_t lds_addr(const void* lds) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void*)lds);
}
__device__ __forceinline__ void dma16_lds(const i32x4a& rs, uint32_t voff, int soff, uint32_t lds) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, %3 offen lds"
               ::"v"(voff), "s"(lds), "s"(rs), "s"(soff) : "memory", "m0");
#endif
}
__device__ __forceinline__ void dma4_lds(const i32x4a& rs, uint32_t voff, int soff, uint32_t lds) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dword %0, %2, %3 offen lds"
               ::"v"(voff), "s"(lds), "s"(rs), "s"(soff) : "memory", "m0");
#endif
}
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
#if defined(__HIP_DEVICE_COMPILE__)
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
#endif
}

// Long key side, bf16, dQ pass (replaces mode 2 for hd 64 / 128): a
// workgroup owns 128 queries, one 32-query slice per WAVE; Q and dO stay in
// registers as MFMA B fragments for the whole sweep.  Everything is computed
// TRANSPOSED (query on the lane, keys / dims in registers), so dS never
// leaves registers:
//   S^T = K Q^T - lse/scale, dP^T = V dO^T - delta   (key rows, query lane)
//   P = exp2(c S) (masked keys 0), dS^T = P dP^T
//   dQ^T += K^T dS^T  (K^T by transposed LDS reads; dS^T's accumulator
//                      registers are directly the B operand, see pack8)
// K / V blocks of 64 keys are double-buffered in LDS (kimg layout: row and
// transposed reads conflict-free), block j+1 loaded into registers under
// block j's MFMAs, one barrier per block.  delta = rowsum(dO * O) is
// computed once per query and written for the dK/dV pass (mode 1).

template <int HD, bool DMA>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_kernel(BwdParams p) {
  static_assert(HD == 64 || HD == 128, "dq kernel head dims");
  constexpr int KB = 64;
  constexpr int NQ = HD / 16, ND = HD / 32;
  constexpr int NPF = KB * HD / 8 / 256;   // 16-byte K (and V) chunks per thread per block
  // round 6 (kDqDma, hd 64): K / V blocks by LDS-DMA into a 3-deep ring (block
  // j + 2 issued while block j computes; per wave two 1 KiB pieces of K and of
  // V whose per-lane source offsets un-apply the kimg swizzle, wave 0 also the
  // block's 64 key-mask bytes), one counted vmcnt + barrier per block; this
  // frees the 16 staging VGPRs of the register-staged form (kept for hd 128,
  // whose three 32 KiB buffers would not leave room for two workgroups)
  // The key mask arrives as dwords, whose per-dword range check drops the
  // last partial dword of a row: the host takes this form only for
  // kv_len % 4 == 0 (or no mask) with 4-byte aligned mask rows, and only when
  // MTTS_OVR_ATTN_DQ_DMA = 1 (the dK / dV form of this staging measured 3 %
  // slower, profiles/r06_attn_ab_kv_dma.txt; this one: r06_attn_ab_dq_dma.txt)
  constexpr bool kDqDma = DMA && HD == 64;
  constexpr int NBUF = kDqDma ? 3 : 2;
  __shared__ __attribute__((aligned(16))) bf16_t sK[NBUF][KB * HD];
  __shared__ __attribute__((aligned(16))) bf16_t sV[NBUF][KB * HD];
  __shared__ uint32_t sMask[2][KB / 32];
  __shared__ __attribute__((aligned(16))) uint32_t sMraw[NBUF][64];   // kDqDma: mask bytes of the block (16 dwords + zeros)
  const MttsAttnBwdArgs& a = p.a;
  const MttsAttnFwdArgs& f = a.f;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int g = (lane >> 4) & 1, qq = (lane >> 2) & 3, pp = lane & 3;
  const Blk bk = xcd_block(f.kv_len >= 1024);
  const int b = bk.z, hh = bk.y;
  const int q0 = bk.x * 128 + wave * 32;           // this wave's queries
  const float c = f.scale * kLog2e, inv_scale = 1.f / f.scale;
  const uint8_t* mb = f.key_padding_mask ? f.key_padding_mask + b * f.mask_bs : nullptr;
  const bf16_t* qb = (const bf16_t*)f.q + b * f.q_bs + hh * HD;
  const bf16_t* gb = (const bf16_t*)a.dout + b * a.do_bs + hh * HD;
  const bf16_t* ob = (const bf16_t*)f.out + b * f.o_bs + hh * HD;
  const bf16_t* kbase = (const bf16_t*)f.k + b * f.k_bs + hh * HD;
  const bf16_t* vbase = (const bf16_t*)f.v + b * f.v_bs + hh * HD;
  // ---- B fragments of Q^T / dO^T (query r, dims 16s + 8h .. +7), delta, -lse/scale
  const int qi = q0 + r;
  const bool qv = qi < f.q_len;
  s16x8 Qf[NQ], Gf[NQ];
  float dl = 0.f;
#pragma unroll
  for (int s = 0; s < NQ; ++s) {
    Qf[s] = qv ? *(const s16x8*)(qb + (int64_t)qi * f.q_ls + 16 * s + 8 * h) : s16x8{};
    Gf[s] = qv ? *(const s16x8*)(gb + (int64_t)qi * a.do_ls + 16 * s + 8 * h) : s16x8{};
    const s16x8 o8 = qv ? *(const s16x8*)(ob + (int64_t)qi * f.o_ls + 16 * s + 8 * h) : s16x8{};
#pragma unroll
    for (int e = 0; e < 8; ++e) dl += mtts::bf2f((bf16_t)Gf[s][e]) * mtts::bf2f((bf16_t)o8[e]);
  }
  dl += __shfl_xor(dl, 32);
  float Lq = 0.f;
  if (qv) {
    Lq = -f.lse[((int64_t)b * f.heads + hh) * f.q_len + qi] * inv_scale;
    if (h == 0) p.delta[((int64_t)b * f.heads + hh) * f.q_len + qi] = -dl;
  }
  const float Dq = qv ? -dl : 0.f;

  // lane-constant offsets (elements) into the kimg images: A-fragment row
  // reads (key r, chunk 2s + h) and K^T transposed reads (keys 4h + qq
  // (+8) of a 16-key step, dims of tile dt); a tile base that is a multiple
  // of 16 rows leaves the swizzle unchanged
  int oR[NQ], oT[2][ND];
#pragma unroll
  for (int s = 0; s < NQ; ++s) oR[s] = kimg<HD>(r, 2 * s + h);
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) oT[u][dt] = kimg<HD>(4 * h + qq + 8 * u, 4 * dt + 2 * g + (pp >> 1)) + 4 * (pp & 1);

  // block staging: loads issued unconditionally, consumed only in put()
  // buffer loads as attn_fwd_db_kernel: rows past kv_len read zeros (host:
  // K and V share the row stride, 31-bit spans)
  f32x4 pk[NPF], pv[NPF];
  uint32_t praw = 0;
  int pk0 = 0;
  const __amdgpu_buffer_rsrc_t rk = brsrc(kbase, (uint32_t)(((int64_t)(f.kv_len - 1) * f.k_ls + HD) * 2));
  const __amdgpu_buffer_rsrc_t rv = brsrc(vbase, (uint32_t)(((int64_t)(f.kv_len - 1) * f.k_ls + HD) * 2));
  const __amdgpu_buffer_rsrc_t rm = brsrc(mb ? mb : (const uint8_t*)kbase, mb ? (uint32_t)f.kv_len : 0u);
  uint32_t ok_[NPF];
#pragma unroll
  for (int i = 0; i < NPF; ++i) {
    const int idx = tid + 256 * i;
    ok_[i] = (uint32_t)(((idx / (HD / 8)) * f.k_ls + (idx % (HD / 8)) * 8) * 2);
  }
  auto fetch = [&](int k0) __attribute__((always_inline)) {
    pk0 = k0;
    const int sk = (int)(k0 * f.k_ls * 2);
#pragma unroll
    for (int i = 0; i < NPF; ++i) {
      pk[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rk, ok_[i], sk, 0));
      pv[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rv, ok_[i], sk, 0));
    }
    praw = __builtin_amdgcn_raw_buffer_load_b8(rm, (uint32_t)lane, k0, 0);
  };
  auto put = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NPF; ++i) {
      const int idx = tid + 256 * i;
      const int row = idx / (HD / 8), ch = idx % (HD / 8);
      *(f32x4*)(sK[buf] + kimg<HD>(row, ch)) = pk[i];
      *(f32x4*)(sV[buf] + kimg<HD>(row, ch)) = pv[i];
    }
    const bool ok = pk0 + lane < f.kv_len && !(mb && praw);
    const uint64_t bal = __ballot(ok);
    if (tid == 0) {
      sMask[buf][0] = (uint32_t)bal;
      sMask[buf][1] = (uint32_t)(bal >> 32);
    }
  };

  f32x16 QA[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) QA[dt] = f32x16{};
  const int nblk = (f.kv_len + KB - 1) / KB;
  // the math of one 64-key block from LDS buffer `buf` (key mask: the staged
  // 32-bit words, or -- kDqDma -- the raw mask bytes)
  constexpr int kTileUnroll = HD == 64 ? 2 : 1;   // hd 128: no room for two tiles' registers
  auto block = [&](int buf, int k0) __attribute__((always_inline)) {
#pragma unroll kTileUnroll
    for (int t = 0; t < KB / 32; ++t) {
      if (k0 + t * 32 >= f.kv_len) break;
      const bf16_t* kt = sK[buf] + t * 32 * HD;
      const bf16_t* vt = sV[buf] + t * 32 * HD;
      f32x16 S, D;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        S[i] = Lq;
        D[i] = Dq;
      }
#pragma unroll
      for (int s = 0; s < NQ; ++s) {
        S = mfma_bf16(*(const s16x8*)(kt + oR[s]), Qf[s], S);
        D = mfma_bf16(*(const s16x8*)(vt + oR[s]), Gf[s], D);
      }
      uint32_t wm;
      if constexpr (kDqDma) {
        const int kl = t * 32 + r;   // lanes r and r + 32 test the same key
        const uint8_t mbyte = ((const uint8_t*)sMraw[buf])[kl];
        wm = (uint32_t)__ballot(k0 + kl < f.kv_len && mbyte == 0);
      } else {
        wm = __builtin_amdgcn_readfirstlane(sMask[buf][t]);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float pr = exp2_raw(c * S[i]);
        if (wm != 0xffffffffu) pr = ((wm >> acc_row(i, h)) & 1u) ? pr : 0.f;
        S[i] = pr * D[i];   // dS^T (unscaled)
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const s16x8 pb = pack8(S, s);
        const bf16_t* ks = kt + 16 * s * HD;
#pragma unroll
        for (int dt = 0; dt < ND; ++dt)
          QA[dt] = mfma_bf16(cat(tr_read(ks + oT[0][dt]), tr_read(ks + oT[1][dt])), pb, QA[dt]);
      }
    }
  };
  if constexpr (kDqDma) {
    static_assert(NPF == 2, "kDqDma: two 1 KiB pieces per wave and tensor per block");
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    // LDS slot s = 64 * (4 * i + wave) + lane of piece i: image row s / 8,
    // physical chunk s % 8 = logical chunk ^ kswz(row)
    uint32_t vk[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int srow = 8 * (4 * i + wv) + (lane >> 3);
      const int sch = (lane & 7) ^ kswz<HD>(srow);
      vk[i] = (uint32_t)((srow * f.k_ls + 8 * sch) * 2);
    }
    const uint32_t vm = lane < 16 ? (uint32_t)lane * 4 : 0xFFFFFFF0u;   // 16 dwords = 64 mask bytes
    const i32x4a rk4 = rsrc4a(kbase, (uint32_t)(((int64_t)(f.kv_len - 1) * f.k_ls + HD) * 2));
    const i32x4a rv4 = rsrc4a(vbase, (uint32_t)(((int64_t)(f.kv_len - 1) * f.k_ls + HD) * 2));
    const i32x4a rm4 = rsrc4a(mb ? mb : (const uint8_t*)kbase, mb ? (uint32_t)f.kv_len : 0u);
    auto sgpr = [](int v) __attribute__((always_inline)) { return __builtin_amdgcn_readfirstlane(v); };
    auto dma_blk = [&](int k0, int buf) __attribute__((always_inline)) {
      const int sk = sgpr(k0 * f.k_ls * 2);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        dma16_lds(rk4, vk[i], sk, sgpr((int)lds_addr(sK[buf]) + 1024 * (4 * i + wv)));
        dma16_lds(rv4, vk[i], sk, sgpr((int)lds_addr(sV[buf]) + 1024 * (4 * i + wv)));
      }
      if (wv == 0) dma4_lds(rm4, vm, sgpr(k0), lds_addr(sMraw[buf]));
    };
    // VMEM operations one block issues per wave: 5 on wave 0, 4 on the others
    auto wait_blocks = [&](int later) __attribute__((always_inline)) {
      if (wv == 0) {
        if (later >= 1) wait_vmcnt<5>(); else wait_vmcnt<0>();
      } else {
        if (later >= 1) wait_vmcnt<4>(); else wait_vmcnt<0>();
      }
    };
    if (nblk > 0) {
      dma_blk(0, 0);
      if (nblk > 1) dma_blk(KB, 1);
      wait_blocks(nblk > 1 ? 1 : 0);
    }
    block_sync();
    for (int j = 0; j < nblk; ++j) {
      if (j + 2 < nblk) dma_blk((j + 2) * KB, (j + 2) % 3);   // buffer last read in block j - 1
      block(j % 3, j * KB);
      if (j + 1 < nblk) wait_blocks(j + 2 < nblk ? 1 : 0);    // block j + 1 landed
      block_sync();
    }
  } else {
    if (nblk > 0) {
      fetch(0);
      put(0);
    }
    block_sync();
    // hd 128: the next block's 32 staging registers do not fit beside Q / dO /
    // dQ (256 VGPRs); it is loaded after this block's math instead
    constexpr bool kPrefetch = HD == 64;
    for (int j = 0; j < nblk; ++j) {
      const int buf = j & 1, k0 = j * KB;
      if constexpr (kPrefetch) fetch(min(k0 + KB, (nblk - 1) * KB));   // in flight under this block's math
      block(buf, k0);
      if (j + 1 < nblk) {
        if constexpr (!kPrefetch) fetch(k0 + KB);
        put(buf ^ 1);
      }
      block_sync();
    }
  }
  // ---- dQ^T tile dt: lane = query, registers = dims dt*32 + acc_row(i, h)
  if (qv) {
    bf16_t* dqp = (bf16_t*)a.dq + b * a.dq_bs + (int64_t)qi * a.dq_ls + hh * HD;
    const bool vec = ((uintptr_t)dqp & 7) == 0;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d0 = dt * 32 + 8 * g4 + 4 * h;
        s16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = bfbits(QA[dt][4 * g4 + e] * f.scale);
        if (vec) {
          *(s16x4*)(dqp + d0) = v;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) dqp[d0 + e] = (bf16_t)v[e];
        }
      }
  }
}

// Long key side, bf16 hd 64, dK / dV pass (replaces mode 1): a workgroup
// owns 128 keys, 32 per wave, and sweeps the queries of its chunk in 32-query
// slices.  The wave's K / V rows stay in registers as MFMA B fragments (they
// are the same for every slice); a slice's Q / dO rows are staged ONCE per
// workgroup in LDS (kimg layout: A-fragment row reads and the transposed
// reads of the dV / dK products are both conflict-free).
//   S = Q K^T - lse/scale, dP = dO V^T - delta     (query rows, key lane)
//   P = exp2(c S) (masked keys 0), dS = P dP
//   dV += P^T dO, dK += dS^T Q   (the accumulators' registers as A operands)
// Round 6 (kKvDma): the slices arrive by LDS-DMA straight into a 3-deep LDS
// ring (slice j + 2 issued while slice j computes; each wave's 1 KiB piece
// of Q and of dO is ONE buffer_load_dwordx4 ... lds whose per-lane source
// offset un-applies the kimg chunk swizzle, wave 0 also moves the slice's
// lse / delta), one counted vmcnt + barrier per slice.  This frees the 20
// prefetch VGPRs of the register-staged form (round 4/5: two register sets
// of Q / dO / lse / delta, whose 5 spilled VGPRs were reloaded inside the
// slice loop -- and a spill reload's vmcnt wait also waited for the next
// slices' prefetch, the kernel's memory wait).
constexpr bool kKvDma = false;   // measured slower (profiles/r06_attn_ab_kv_dma.txt), kept for reference
template <int HD>
__global__ __launch_bounds__(256, 3) void attn_bwd_kv_kernel(BwdParams p) {
  static_assert(HD == 64, "kv kernel: hd 64 (its K / V / dK / dV registers)");
  constexpr int KG = 128, NQ = HD / 16, ND = HD / 32;
  constexpr int QS = 32;                   // queries per staged slice
  constexpr int NPF = QS * HD / 8 / 256;   // 16-byte Q (and dO) chunks per thread per slice
  static_assert(NPF >= 1, "slice staging");
  static_assert(!kKvDma || NPF == 1, "LDS-DMA staging: one 16-byte piece per thread and tensor per slice");
  constexpr int NB = kKvDma ? 3 : 2;       // slice buffers
  __shared__ __attribute__((aligned(16))) bf16_t sQ[NB][QS * HD];
  __shared__ __attribute__((aligned(16))) bf16_t sG[NB][QS * HD];
  __shared__ __attribute__((aligned(16))) float sL[NB][64], sD[NB][64];
  const MttsAttnBwdArgs& a = p.a;
  const MttsAttnFwdArgs& f = a.f;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int g = (lane >> 4) & 1, qq = (lane >> 2) & 3, pp = lane & 3;
  const Blk bk = xcd_block();
  const int b = bk.z, hh = bk.y;
  const int d = f.heads * HD;
  const int nkg = (f.kv_len + KG - 1) / KG;
  const int kg = bk.x % nkg, qc = bk.x / nkg;
  const int qbeg = qc * p.qchunk, qend = min(f.q_len, qbeg + p.qchunk);
  const float c = f.scale * kLog2e, inv_scale = 1.f / f.scale;
  const uint8_t* mb = f.key_padding_mask ? f.key_padding_mask + b * f.mask_bs : nullptr;
  const float* dbuf = p.delta + ((int64_t)b * f.heads + hh) * f.q_len;
  const float* lbuf = f.lse + ((int64_t)b * f.heads + hh) * f.q_len;
  const bf16_t* qb = (const bf16_t*)f.q + b * f.q_bs + hh * HD;
  const bf16_t* gb = (const bf16_t*)a.dout + b * a.do_bs + hh * HD;

  // ---- this lane's key: B fragments of K / V (dims 16s + 8h .. +7), mask
  const int key = kg * KG + wave * 32 + r;
  const bool kin = key < f.kv_len;
  const bool kvalid = kin && !(mb && mb[key]);
  s16x8 Kf[NQ], Vf[NQ];
  {
    const bf16_t* kr = (const bf16_t*)f.k + b * f.k_bs + (int64_t)(kin ? key : 0) * f.k_ls + hh * HD;
    const bf16_t* vr = (const bf16_t*)f.v + b * f.v_bs + (int64_t)(kin ? key : 0) * f.v_ls + hh * HD;
#pragma unroll
    for (int s = 0; s < NQ; ++s) {
      Kf[s] = kin ? *(const s16x8*)(kr + 16 * s + 8 * h) : s16x8{};
      Vf[s] = kin ? *(const s16x8*)(vr + 16 * s + 8 * h) : s16x8{};
    }
  }
  // lane-constant image offsets: A-fragment rows (query r, chunk 2s + h) and
  // the transposed B reads (queries 4h + qq (+8) of a 16-query step, dims of tile dt)
  int oR[NQ], oT[2][ND];
#pragma unroll
  for (int s = 0; s < NQ; ++s) oR[s] = kimg<HD>(r, 2 * s + h);
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) oT[u][dt] = kimg<HD>(4 * h + qq + 8 * u, 4 * dt + 2 * g + (pp >> 1)) + 4 * (pp & 1);

  f32x16 dK[ND], dV[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) dK[dt] = dV[dt] = f32x16{};
  const int nsl = qend > qbeg ? (qend - qbeg + QS - 1) / QS : 0;

  // one slice of the query sweep from LDS buffer `buf`
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const bf16_t* qs = sQ[buf];
    const bf16_t* gs = sG[buf];
    f32x16 S, D;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if constexpr (kKvDma) {
        S[i] = -sL[buf][acc_row(i, h)] * inv_scale;   // raw lse (0 past the chunk: P = 1 x zero rows)
      } else {
        S[i] = sL[buf][acc_row(i, h)];
      }
      D[i] = sD[buf][acc_row(i, h)];
    }
#pragma unroll
    for (int s = 0; s < NQ; ++s) {
      S = mfma_bf16(*(const s16x8*)(qs + oR[s]), Kf[s], S);
      D = mfma_bf16(*(const s16x8*)(gs + oR[s]), Vf[s], D);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      S[i] = kvalid ? exp2_raw(c * S[i]) : 0.f;  // P
      D[i] = S[i] * D[i];                         // dS (unscaled)
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const s16x8 pa = pack8(S, s), da = pack8(D, s);
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) {
        const int o0 = 16 * s * HD + oT[0][dt], o1 = 16 * s * HD + oT[1][dt];
        dV[dt] = mfma_bf16(pa, cat(tr_read(gs + o0), tr_read(gs + o1)), dV[dt]);
        dK[dt] = mfma_bf16(da, cat(tr_read(qs + o0), tr_read(qs + o1)), dK[dt]);
      }
    }
  };

  if constexpr (kKvDma) {
    // LDS slot s of a slice image (16-byte chunk, s = 64 * wave + lane):
    // image row s / 8, physical chunk s % 8 = logical chunk ^ kswz(row)
    const int srow = 8 * wave + (lane >> 3);
    const int sch = (lane & 7) ^ kswz<HD>(srow);
    const uint32_t vq = (uint32_t)((srow * f.q_ls + 8 * sch) * 2);
    const uint32_t vg = (uint32_t)((srow * a.do_ls + 8 * sch) * 2);
    const uint32_t vl = lane < QS ? (uint32_t)lane * 4 : 0xFFFFFFF0u;   // lanes >= 32: past every range, read 0
    // descriptors over the chunk's rows: rows at or past qend read zeros
    const i32x4a rq = rsrc4a(qb, (uint32_t)(((int64_t)(qend - 1) * f.q_ls + HD) * 2));
    const i32x4a rg = rsrc4a(gb, (uint32_t)(((int64_t)(qend - 1) * a.do_ls + HD) * 2));
    const i32x4a rl = rsrc4a(lbuf, (uint32_t)qend * 4);
    const i32x4a rd = rsrc4a(dbuf, (uint32_t)qend * 4);
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    auto sgpr = [](int v) __attribute__((always_inline)) { return __builtin_amdgcn_readfirstlane(v); };
    auto dma_slice = [&](int q0, int buf) __attribute__((always_inline)) {
      dma16_lds(rq, vq, sgpr(q0 * f.q_ls * 2), sgpr((int)lds_addr(sQ[buf]) + 1024 * wv));
      dma16_lds(rg, vg, sgpr(q0 * a.do_ls * 2), sgpr((int)lds_addr(sG[buf]) + 1024 * wv));
      if (wv == 0) {
        dma4_lds(rl, vl, sgpr(q0 * 4), lds_addr(sL[buf]));
        dma4_lds(rd, vl, sgpr(q0 * 4), lds_addr(sD[buf]));
      }
    };
    // VMEM operations one slice issues per wave: 4 on wave 0, 2 on the others;
    // wait until at most `later` slices' operations are outstanding
    auto wait_slices = [&](int later) __attribute__((always_inline)) {
      if (wv == 0) {
        if (later >= 1) wait_vmcnt<4>(); else wait_vmcnt<0>();
      } else {
        if (later >= 1) wait_vmcnt<2>(); else wait_vmcnt<0>();
      }
    };
    if (nsl > 0) {
      dma_slice(qbeg, 0);
      if (nsl > 1) dma_slice(qbeg + QS, 1);
      wait_slices(nsl > 1 ? 1 : 0);
    }
    block_sync();
    for (int j = 0; j < nsl; ++j) {
      if (j + 2 < nsl) dma_slice(qbeg + QS * (j + 2), (j + 2) % 3);   // buffer last read in slice j - 1
      compute(j % 3);
      if (j + 1 < nsl) wait_slices(j + 2 < nsl ? 1 : 0);              // slice j + 1 landed
      block_sync();
    }
  } else {
    // register-staged slices (round 4/5 form, kept for A/B): slice j + 2 is
    // loaded while slice j computes and slice j + 1 goes to LDS at its end
    f32x4 pq[2][NPF], pg[2][NPF];
    float pl[2] = {0.f, 0.f}, pd[2] = {0.f, 0.f};
    int ps0[2] = {qbeg, qbeg};
    const __amdgpu_buffer_rsrc_t rq = brsrc(qb, (uint32_t)(((int64_t)(qend - 1) * f.q_ls + HD) * 2));
    const __amdgpu_buffer_rsrc_t rg = brsrc(gb, (uint32_t)(((int64_t)(qend - 1) * a.do_ls + HD) * 2));
    const __amdgpu_buffer_rsrc_t rl = brsrc(lbuf, (uint32_t)qend * 4);
    const __amdgpu_buffer_rsrc_t rd = brsrc(dbuf, (uint32_t)qend * 4);
    uint32_t oq_[NPF], og_[NPF];
#pragma unroll
    for (int i = 0; i < NPF; ++i) {
      const int idx = tid + 256 * i;
      const int row = idx / (HD / 8), cc = (idx % (HD / 8)) * 8;
      oq_[i] = (uint32_t)((row * f.q_ls + cc) * 2);
      og_[i] = (uint32_t)((row * a.do_ls + cc) * 2);
    }
    auto fetch = [&](auto set_c, int q0) __attribute__((always_inline)) {
      constexpr int st = decltype(set_c)::value;
      ps0[st] = q0;
      const int sq = (int)(q0 * f.q_ls * 2), sg = (int)(q0 * a.do_ls * 2);
#pragma unroll
      for (int i = 0; i < NPF; ++i) {
        pq[st][i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rq, oq_[i], sq, 0));
        pg[st][i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rg, og_[i], sg, 0));
      }
      const uint32_t ol = (uint32_t)(tid & (QS - 1)) * 4;
      pl[st] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rl, ol, q0 * 4, 0));
      pd[st] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rd, ol, q0 * 4, 0));
    };
    auto put = [&](auto set_c, int buf) __attribute__((always_inline)) {
      constexpr int st = decltype(set_c)::value;
#pragma unroll
      for (int i = 0; i < NPF; ++i) {
        const int idx = tid + 256 * i;
        const int row = idx / (HD / 8), ch = idx % (HD / 8);
        *(f32x4*)(sQ[buf] + kimg<HD>(row, ch)) = pq[st][i];
        *(f32x4*)(sG[buf] + kimg<HD>(row, ch)) = pg[st][i];
      }
      if (tid < QS) {
        const bool in = ps0[st] + tid < qend;
        sL[buf][tid] = in ? -pl[st] * inv_scale : 0.f;   // P = exp2(c (S + L))
        sD[buf][tid] = in ? pd[st] : 0.f;
      }
    };
    const int qlast = qbeg + QS * (nsl - 1);
    using S0_ = std::integral_constant<int, 0>;
    using S1_ = std::integral_constant<int, 1>;
    if (nsl > 0) {
      fetch(S0_{}, qbeg);
      put(S0_{}, 0);
      fetch(S1_{}, min(qbeg + QS, qlast));
    }
    block_sync();
    auto slice = [&](auto par_c, int j) __attribute__((always_inline)) {
      constexpr int par = decltype(par_c)::value;
      const int q0 = qbeg + QS * j;
      fetch(std::integral_constant<int, par>{}, min(q0 + 2 * QS, qlast));   // in flight under two slices' math
      compute(par);
      if (j + 1 < nsl) put(std::integral_constant<int, par ^ 1>{}, par ^ 1);
      block_sync();
    };
    for (int j = 0; j < nsl; j += 2) {
      slice(S0_{}, j);
      if (j + 1 < nsl) slice(S1_{}, j + 1);
    }
  }
  // ---- dK (scaled), dV: rows = keys (registers), cols = dims (lanes)
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) {
    const int dim = dt * 32 + r;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int kk = kg * KG + wave * 32 + acc_row(i, h);
      if (kk >= f.kv_len) continue;
      const float vk = dK[dt][i] * f.scale, vv = dV[dt][i];
      if (p.nchunk > 1) {
        float* pr = p.part + (((int64_t)qc * f.batch + b) * f.kv_len + kk) * (2 * d) + hh * HD + dim;
        pr[0] = vk;
        pr[d] = vv;
      } else {
        mtts::stf((bf16_t*)a.dk + b * a.dk_bs + (int64_t)kk * a.dk_ls + hh * HD + dim, vk);
        mtts::stf((bf16_t*)a.dv + b * a.dv_bs + (int64_t)kk * a.dv_ls + hh * HD + dim, vv);
      }
    }
  }
}

// sum of the query-chunk partials -> dk, dv (fixed order)
template <typename T>
__global__ __launch_bounds__(256) void attn_bwd_reduce_kernel(BwdParams p) {
  const MttsAttnBwdArgs& a = p.a;
  const MttsAttnFwdArgs& f = a.f;
  const int d = f.heads * f.head_dim;
  const int64_t n = (int64_t)f.batch * f.kv_len * 2 * d;
  const int64_t stride = (int64_t)f.batch * f.kv_len * 2 * d;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int cix = 0; cix < p.nchunk; ++cix) s += p.part[cix * stride + e];
    const int col = (int)(e % (2 * d));
    const int64_t bk = e / (2 * d);
    const int b = (int)(bk / f.kv_len), kk = (int)(bk % f.kv_len);
    if (col < d)
      mtts::stf((T*)a.dk + b * a.dk_bs + (int64_t)kk * a.dk_ls + col, s);
    else
      mtts::stf((T*)a.dv + b * a.dv_bs + (int64_t)kk * a.dv_ls + col - d, s);
  }
}

// ============================================================== host side
bool aligned16(const void* ptr) { return ((uintptr_t)ptr & 15) == 0; }

int check_fwd(const MttsAttnFwdArgs* a, const char* who) {
  MTTS_CHECK(a, "%s: null args", who);
  MTTS_CHECK(a->dtype == MTTS_F32 || a->dtype == MTTS_BF16, "%s: dtype must be F32 or BF16", who);
  MTTS_CHECK(a->head_dim == 16 || a->head_dim == 32 || a->head_dim == 64 || a->head_dim == 128,
             "%s: head_dim %d not in {16,32,64,128}", who, a->head_dim);
  MTTS_CHECK(a->batch >= 0 && a->heads > 0 && a->q_len >= 0 && a->kv_len >= 0, "%s: bad sizes", who);
  MTTS_CHECK(a->q && a->k && a->v && a->out, "%s: null tensor", who);
  const int64_t al = a->dtype == MTTS_BF16 ? 8 : 4;
  MTTS_CHECK(aligned16(a->q) && aligned16(a->k) && aligned16(a->v) && aligned16(a->out),
             "%s: q/k/v/out must be 16-byte aligned", who);
  MTTS_CHECK(a->q_bs % al == 0 && a->q_ls % al == 0 && a->k_bs % al == 0 && a->k_ls % al == 0 && a->v_bs % al == 0 &&
                 a->v_ls % al == 0 && a->o_bs % al == 0 && a->o_ls % al == 0,
             "%s: strides must be multiples of 16 bytes", who);
  return MTTS_OK;
}

template <typename T, int HD>
void launch_fwd(const MttsAttnFwdArgs* a, hipStream_t st) {
  if constexpr (sizeof(T) == 2 && HD % 32 == 0) {
    if (a->kv_len <= kShortKV && a->q_len >= 128 && mtts::override_of(MTTS_OVR_ATTN_GENERIC) != 1) {
      // >= 512 workgroups (two per CU), as many query slices per wave as that allows
      const int64_t blocks128 = (int64_t)((a->q_len + 127) / 128) * a->heads * a->batch;
      int nsl = (int)std::max<int64_t>(1, std::min<int64_t>(8, blocks128 / 512));
      dim3 grid((a->q_len + 128 * nsl - 1) / (128 * nsl), a->heads, a->batch);
      attn_fwd_short_kernel<HD><<<grid, 256, 0, st>>>(*a, nsl);
      return;
    }
  }
  const int nw = a->q_len >= 128 ? 4 : (a->q_len + 31) / 32;
  dim3 grid((a->q_len + 32 * nw - 1) / (32 * nw), a->heads, a->batch);
  if constexpr (sizeof(T) == 2 && HD >= 32) {
    // K / V rows by buffer loads: one row stride, 31-bit byte spans
    const bool span_ok = a->k_ls == a->v_ls && (int64_t)(a->kv_len + 64) * a->k_ls * 2 < (1ll << 31);
    if (nw == 4 && span_ok && mtts::override_of(MTTS_OVR_ATTN_GENERIC) != 1) {
      // (two 32-query tiles per wave sharing every K / V fragment read, QT = 2,
      // measured equal to QT = 1 at the C5 shape: 717 vs 680-720 us)
      attn_fwd_db_kernel<HD, 1><<<grid, 256, 0, st>>>(*a);
      return;
    }
  }
  attn_fwd_kernel<T, HD><<<grid, 64 * nw, 0, st>>>(*a);
}

// ---------------------------------------------------------------------------
// Single-query forward (q_len == 1: MambaTTSDecoder.decode_step's
// cross-attention, mamba_decoder.py:222-236).  One workgroup per (batch,
// head), 4 waves; a group of G = HD/8 lanes owns one key at a time (8 dims
// per lane, one 16-byte load of K and of V per lane and key), the key axis
// is strided over the 256/G groups of the workgroup and each group keeps an
// online softmax (m, l, acc[8]); the groups are merged through LDS.  K and V
// of up to 4 keys per group are loaded before any arithmetic.  HBM-bound:
// every K/V byte of the (batch, head) read exactly once.
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void ld8(const T* p, float* v) {
  if constexpr (std::is_same<T, bf16_t>::value) {
    const s16x8 x = *reinterpret_cast<const s16x8*>(p);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = __uint_as_float(((uint32_t)(uint16_t)x[e]) << 16);
  } else {
    const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = a[e], v[4 + e] = b[e];
  }
}

template <typename T, int HD>
__global__ __launch_bounds__(256) void attn_decode_kernel(MttsAttnFwdArgs a) {
  constexpr int G = HD / 8, NG = 256 / G, U = 4;
  __shared__ float sm[NG], sl[NG], sacc[NG][HD + 1];
  const int bh = blockIdx.x, b = bh / a.heads, hh = bh % a.heads;
  const int g = threadIdx.x / G, gl = threadIdx.x % G, d0 = gl * 8;
  const float c = a.scale * kLog2e;
  const uint8_t* mb = a.key_padding_mask ? a.key_padding_mask + b * a.mask_bs : nullptr;
  float q[8];
  ld8((const T*)a.q + b * a.q_bs + hh * HD + d0, q);
#pragma unroll
  for (int e = 0; e < 8; ++e) q[e] *= c;
  const int64_t hs = a.kv_hs ? a.kv_hs : HD;
  const T* kb = (const T*)a.k + b * a.k_bs + hh * hs + d0;
  const T* vb = (const T*)a.v + b * a.v_bs + hh * hs + d0;
  float m = -INFINITY, l = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int j0 = g; j0 < a.kv_len; j0 += NG * U) {
    float kx[U][8], vx[U][8];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = j0 + u * NG;
      ok[u] = j < a.kv_len && !(mb && mb[j]);
      const int jj = j < a.kv_len ? j : j0;
      ld8(kb + (int64_t)jj * a.k_ls, kx[u]);
      ld8(vb + (int64_t)jj * a.v_ls, vx[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) s += q[e] * kx[u][e];
#pragma unroll
      for (int o = 1; o < G; o <<= 1) s += __shfl_xor(s, o);
      if (!ok[u]) continue;
      const float mn = fmaxf(m, s), f = exp2f(m - mn), p = exp2f(s - mn);
      l = l * f + p;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = acc[e] * f + p * vx[u][e];
      m = mn;
    }
  }
  if (gl == 0) sm[g] = m, sl[g] = l;
#pragma unroll
  for (int e = 0; e < 8; ++e) sacc[g][d0 + e] = acc[e];
  block_sync();
  if (threadIdx.x < HD) {
    float M = -INFINITY;
    for (int i = 0; i < NG; ++i) M = fmaxf(M, sm[i]);
    float L = 0.f, o = 0.f;
    for (int i = 0; i < NG; ++i) {
      const float f = sm[i] == -INFINITY ? 0.f : exp2f(sm[i] - M);
      L += sl[i] * f;
      o += sacc[i][threadIdx.x] * f;
    }
    // fully masked: L = 0 -> 0/0 = NaN (torch MHA), lse = -inf
    mtts::stf((T*)a.out + b * a.o_bs + hh * HD + threadIdx.x, o / L);
    if (a.lse && threadIdx.x == 0) a.lse[(int64_t)b * a.heads + hh] = M == -INFINITY ? -INFINITY : (M + log2f(L)) * kLn2;
  }
}

// Short key sides (kv_len <= U * 256 / (HD / 8); C4's 128 text keys): every
// key of the (batch, head) in registers at once, so the softmax needs no
// online rescaling: scores -> block max (wave shuffles + 4 LDS words) ->
// p = exp2(s - max) -> P.V and sum(p) reduced over the wave's groups by
// shuffles and over the 4 waves through LDS (fixed order).  All loads are
// unconditional (clamped key index, masked afterwards).
// wave-level reductions of the single-pass decode kernel with DPP / permlane
// forms instead of ds_bpermute shuffles (no LDS round trip per stage):
// group_sum over the G consecutive lanes of a key group (G | 16), groups_sum /
// groups_max over the 64 / G groups of the wave (lane bits log2 G .. 5)
template <int G>
__device__ __forceinline__ float group_sum(float v, int lane) {
  if constexpr (G >= 2) v += mtts::dpp<mtts::kQuadXor1>(v);
  if constexpr (G >= 4) v += mtts::dpp<mtts::kQuadXor2>(v);
  if constexpr (G >= 8) v += mtts::xor4(v, lane);
  if constexpr (G >= 16) v += mtts::xor8(v);
  return v;
}
template <int G>
__device__ __forceinline__ float groups_sum(float v, int lane) {
  if constexpr (G <= 1) v += mtts::dpp<mtts::kQuadXor1>(v);
  if constexpr (G <= 2) v += mtts::dpp<mtts::kQuadXor2>(v);
  if constexpr (G <= 4) v += mtts::xor4(v, lane);
  if constexpr (G <= 8) v += mtts::xor8(v);
  v = mtts::sum_xor16(v);
  return mtts::sum_xor32(v);
}
template <int G>
__device__ __forceinline__ float groups_max(float v, int lane) {
  if constexpr (G <= 1) v = fmaxf(v, mtts::dpp<mtts::kQuadXor1>(v));
  if constexpr (G <= 2) v = fmaxf(v, mtts::dpp<mtts::kQuadXor2>(v));
  if constexpr (G <= 4) v = fmaxf(v, mtts::xor4(v, lane));
  if constexpr (G <= 8) v = fmaxf(v, mtts::xor8(v));
  v = mtts::max_xor16(v);
  return mtts::max_xor32(v);
}

// The cross-attention's query projection fused into the decode kernel
// (round 5): q = bf16(LN(x) Wq_h^T + bq_h) for the workgroup's (batch, head),
// with LN(x) = bf16(fmaf((x - mean) rstd, w, b)) over the residual row -- the
// values the LayerNorm prologue of the packed projection feeds its MFMAs --
// so the step loses the q-projection launch (mamba_decoder.py:72-77 ->
// nn.MultiheadAttention's q = in_proj(query)[:d]).  Each workgroup reads its
// head's Wq rows (HD x d_model bf16) from L2.
struct QProj {
  const mtts::bf16_t* x;      // (batch, dm) bf16 residual rows
  int64_t x_rs;
  const mtts::bf16_t* w;      // (heads * HD, dm) bf16, row-major
  const mtts::bf16_t* bias;   // (heads * HD) bf16 or null
  const float* lnw;
  const float* lnb;
  float eps;
  int dm;
};
constexpr int kQpMaxDm = 2048;

template <int HD>
__device__ __forceinline__ void qproj_head(const QProj& qp, int b, int hh, float* sx, float* sq, float* sred) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const mtts::bf16_t* xr = qp.x + (int64_t)b * qp.x_rs;
  const int dm = qp.dm;
  // two passes as the LayerNorm prologue: mean, then squared deviations
  float s = 0.f;
  for (int i = tid; i < dm; i += 256) {
    const float v = mtts::bf2f(xr[i]);
    sx[i] = v;
    s += v;
  }
  s = mtts::wave_sum(s);
  if (lane == 0) sred[wave] = s;
  block_sync();
  const float mean = ((sred[0] + sred[1]) + (sred[2] + sred[3])) / dm;
  float s2 = 0.f;
  for (int i = tid; i < dm; i += 256) {
    const float d = sx[i] - mean;
    s2 = fmaf(d, d, s2);
  }
  s2 = mtts::wave_sum(s2);
  block_sync();   // every wave read sred's means
  if (lane == 0) sred[wave] = s2;
  block_sync();
  const float rstd = 1.f / sqrtf(((sred[0] + sred[1]) + (sred[2] + sred[3])) / dm + qp.eps);
  for (int i = tid; i < dm; i += 256) sx[i] = mtts::bf2f(mtts::f2bf(fmaf((sx[i] - mean) * rstd, qp.lnw[i], qp.lnb[i])));
  block_sync();
  // rows of the head: 16 lanes per row (16-byte chunks, stride 256 B), 4 rows per wave and pass
  const int l16 = lane & 15;
#pragma unroll 1
  for (int r0 = 0; r0 < HD; r0 += 16) {
    const int r = r0 + wave * 4 + (lane >> 4);
    const mtts::bf16_t* wr = qp.w + (int64_t)(hh * HD + r) * dm;
    float acc = 0.f;
    for (int c8 = l16; c8 < dm / 8; c8 += 16) {
      const uint4 raw = *reinterpret_cast<const uint4*>(wr + c8 * 8);
      const uint32_t wv[4] = {raw.x, raw.y, raw.z, raw.w};
      const float* xs = sx + c8 * 8;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc = fmaf(__uint_as_float(wv[e] << 16), xs[2 * e], acc);
        acc = fmaf(__uint_as_float(wv[e] & 0xffff0000u), xs[2 * e + 1], acc);
      }
    }
    acc = group_sum<16>(acc, lane);
    if (l16 == 0) sq[r] = mtts::bf2f(mtts::f2bf(acc + (qp.bias ? mtts::bf2f(qp.bias[hh * HD + r]) : 0.f)));
  }
  block_sync();
}

template <typename T, int HD, int U, bool QP = false>
__global__ __launch_bounds__(256) void attn_decode1_kernel(MttsAttnFwdArgs a, QProj qp) {
  constexpr int G = HD / 8, NG = 256 / G;
  __shared__ float swm[4], swl[4], sacc[4][HD];
  __shared__ float sx[QP ? kQpMaxDm : 1], sq[QP ? HD : 1], sred[4];
  const int bh = blockIdx.x, b = bh / a.heads, hh = bh % a.heads;
  const int g = threadIdx.x / G, gl = threadIdx.x % G, d0 = gl * 8, wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const float c = a.scale * kLog2e;
  float q[8];
  if constexpr (QP) {
    qproj_head<HD>(qp, b, hh, sx, sq, sred);
#pragma unroll
    for (int e = 0; e < 8; ++e) q[e] = sq[d0 + e];
  } else {
    ld8((const T*)a.q + b * a.q_bs + hh * HD + d0, q);
  }
  const int64_t hs = a.kv_hs ? a.kv_hs : HD;
  const T* kb = (const T*)a.k + b * a.k_bs + hh * hs + d0;
  const T* vb = (const T*)a.v + b * a.v_bs + hh * hs + d0;
  const uint8_t* mb = a.key_padding_mask ? a.key_padding_mask + b * a.mask_bs : (const uint8_t*)a.q;
  const uint32_t mmask = a.key_padding_mask ? 0xffu : 0u;
  float kx[U][8], vx[U][8];
  bool ok[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int j = g + u * NG;
    const int jj = j < a.kv_len ? j : 0;
    ld8(kb + (int64_t)jj * a.k_ls, kx[u]);
    ld8(vb + (int64_t)jj * a.v_ls, vx[u]);
    ok[u] = j < a.kv_len && ((uint32_t)mb[a.key_padding_mask ? jj : 0] & mmask) == 0;
  }
  float sc[U], m = -INFINITY;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    float sv = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) sv = fmaf(q[e], kx[u][e], sv);
    sv = group_sum<G>(sv, lane);
    sc[u] = ok[u] ? sv * c : -INFINITY;
    m = fmaxf(m, sc[u]);
  }
  m = groups_max<G>(m, lane);
  if ((threadIdx.x & 63) == 0) swm[wave] = m;
  block_sync();
  const float M = fmaxf(fmaxf(swm[0], swm[1]), fmaxf(swm[2], swm[3]));
  float l = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const float p = ok[u] ? exp2f(sc[u] - M) : 0.f;
    l += p;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = fmaf(p, vx[u][e], acc[e]);
  }
  l = groups_sum<G>(l, lane);
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = groups_sum<G>(acc[e], lane);
  if ((threadIdx.x & 63) < G) {
#pragma unroll
    for (int e = 0; e < 8; ++e) sacc[wave][d0 + e] = acc[e];
    if (gl == 0) swl[wave] = l;
  }
  block_sync();
  if (threadIdx.x < HD) {
    const float L = (swl[0] + swl[1]) + (swl[2] + swl[3]);
    const float o = (sacc[0][threadIdx.x] + sacc[1][threadIdx.x]) + (sacc[2][threadIdx.x] + sacc[3][threadIdx.x]);
    // fully masked: L = 0 -> 0/0 = NaN (torch MHA), lse = -inf
    if (a.out) mtts::stf((T*)a.out + b * a.o_bs + hh * HD + threadIdx.x, o / L);
    if constexpr (sizeof(T) == 2) {   // packed activation image for the output projection
      if (a.out_packed) ((mtts::bf16_t*)a.out_packed)[mtts::xpk_index(b, hh * HD + threadIdx.x)] = mtts::f2bf(o / L);
    }
    if (a.lse && threadIdx.x == 0) a.lse[(int64_t)b * a.heads + hh] = M == -INFINITY ? -INFINITY : (M + log2f(L)) * kLn2;
  }
}

template <typename T, int HD>
void launch_decode(const MttsAttnFwdArgs* a, hipStream_t st) {
  constexpr int NG = 256 / (HD / 8);
  const dim3 grid(a->batch * a->heads);
  const QProj none{};
  if (a->kv_len <= 4 * NG) hipLaunchKernelGGL((attn_decode1_kernel<T, HD, 4>), grid, dim3(256), 0, st, *a, none);
  else if (a->kv_len <= 8 * NG) hipLaunchKernelGGL((attn_decode1_kernel<T, HD, 8>), grid, dim3(256), 0, st, *a, none);
  else hipLaunchKernelGGL((attn_decode_kernel<T, HD>), grid, dim3(256), 0, st, *a);
}

template <int HD>
void launch_decode_qp(const MttsAttnFwdArgs* a, const QProj& qp, hipStream_t st) {
  constexpr int NG = 256 / (HD / 8);
  const dim3 grid(a->batch * a->heads);
  if (a->kv_len <= 4 * NG)
    hipLaunchKernelGGL((attn_decode1_kernel<mtts::bf16_t, HD, 4, true>), grid, dim3(256), 0, st, *a, qp);
  else
    hipLaunchKernelGGL((attn_decode1_kernel<mtts::bf16_t, HD, 8, true>), grid, dim3(256), 0, st, *a, qp);
}

template <typename T>
void dispatch_decode(const MttsAttnFwdArgs* a, hipStream_t st) {
  switch (a->head_dim) {
    case 16: launch_decode<T, 16>(a, st); break;
    case 32: launch_decode<T, 32>(a, st); break;
    case 64: launch_decode<T, 64>(a, st); break;
    default: launch_decode<T, 128>(a, st); break;
  }
}

template <typename T>
void dispatch_fwd(const MttsAttnFwdArgs* a, hipStream_t st) {
  switch (a->head_dim) {
    case 16: launch_fwd<T, 16>(a, st); break;
    case 32: launch_fwd<T, 32>(a, st); break;
    case 64: launch_fwd<T, 64>(a, st); break;
    default: launch_fwd<T, 128>(a, st); break;
  }
}

struct BwdPlan {
  int nchunk, qchunk, kg;
  bool split;                  // long key side: modes 2 + 1
  int64_t part_bytes, dq_bytes, delta_bytes;
};

BwdPlan plan_bwd(int batch, int heads, int head_dim, int q_len, int kv_len, int dtype) {
  BwdPlan pl{};
  pl.kg = (dtype == MTTS_F32 && head_dim > 64) ? 64 : 128;
  const int slices = (q_len + 31) / 32;
  const int base = batch * heads;
  int nchunk = base >= 256 ? 1 : (256 + base - 1) / base;
  if (mtts::override_of(MTTS_OVR_ATTN_CHUNKS) >= 1) nchunk = mtts::override_of(MTTS_OVR_ATTN_CHUNKS);
  nchunk = nchunk < 1 ? 1 : (nchunk > slices ? (slices > 0 ? slices : 1) : nchunk);
  const int per = (slices + nchunk - 1) / nchunk;
  pl.qchunk = 32 * (per > 0 ? per : 1);
  pl.nchunk = (q_len + pl.qchunk - 1) / pl.qchunk;
  if (pl.nchunk < 1) pl.nchunk = 1;
  const int64_t d = (int64_t)heads * head_dim;
  // split backward (dQ pass + dK/dV pass) for a key side longer than one key
  // group; the dK/dV pass may be chunked over queries into partials.  (For
  // one key group, C2's 128 text keys, the split form measured 112 us against
  // the fused mode-0 kernel's 106 us per call and is not used.)
  const int force = mtts::override_of(MTTS_OVR_ATTN_BWD);
  pl.split = force == 2 || (kv_len > pl.kg && force != 1);
  if (pl.split) {
    const int nkg = (kv_len + pl.kg - 1) / pl.kg;
    const int wgs = nkg * base;
    int nc = wgs >= 256 ? 1 : (256 + wgs - 1) / wgs;
    if (mtts::override_of(MTTS_OVR_ATTN_CHUNKS) >= 1) nc = mtts::override_of(MTTS_OVR_ATTN_CHUNKS);
    nc = nc < 1 ? 1 : (nc > slices ? (slices > 0 ? slices : 1) : nc);
    const int per2 = (slices + nc - 1) / nc;
    pl.qchunk = 32 * (per2 > 0 ? per2 : 1);
    pl.nchunk = (q_len + pl.qchunk - 1) / pl.qchunk;
    if (pl.nchunk < 1) pl.nchunk = 1;
    pl.part_bytes = pl.nchunk > 1 ? (int64_t)pl.nchunk * batch * kv_len * 2 * d * 4 : 0;
    pl.delta_bytes = ((int64_t)batch * heads * q_len * 4 + 255) / 256 * 256;
    return pl;
  }
  pl.part_bytes = pl.nchunk > 1 ? (int64_t)pl.nchunk * batch * kv_len * 2 * d * 4 : 0;
  pl.dq_bytes = kv_len > pl.kg ? (int64_t)batch * q_len * d * 4 : 0;
  return pl;
}

template <typename T, int HD>
void launch_bwd(const BwdParams& p, bool split, hipStream_t st) {
  constexpr int NT = BwdCfg<T, HD>::NW * 64;
  const MttsAttnFwdArgs& f = p.a.f;
  // the dQ / dK-dV kernels address K / V / Q / dO rows through buffer
  // descriptors: one K / V row stride, 31-bit byte spans
  const bool span_ok = f.k_ls == f.v_ls && (int64_t)(f.kv_len + 64) * f.k_ls * 2 < (1ll << 31) &&
                       (int64_t)(f.q_len + 64) * std::max(f.q_ls, p.a.do_ls) * 2 < (1ll << 31);
  if (split) {
    constexpr int KG = BwdCfg<T, HD>::KG;
    if constexpr (std::is_same<T, bf16_t>::value && (HD == 64 || HD == 128)) {
      const bool dq_dma = HD == 64 && mtts::override_of(MTTS_OVR_ATTN_DQ_DMA) == 1 &&
                          (!f.key_padding_mask || (f.kv_len % 4 == 0 && f.mask_bs % 4 == 0 &&
                                                   (uintptr_t)f.key_padding_mask % 4 == 0));
      if (span_ok && mtts::override_of(MTTS_OVR_ATTN_GENERIC) != 1 && dq_dma)
        attn_bwd_dq_kernel<HD, true><<<dim3((f.q_len + 127) / 128, f.heads, f.batch), 256, 0, st>>>(p);
      else if (span_ok && mtts::override_of(MTTS_OVR_ATTN_GENERIC) != 1)
        attn_bwd_dq_kernel<HD, false><<<dim3((f.q_len + 127) / 128, f.heads, f.batch), 256, 0, st>>>(p);
      else
        attn_bwd_kernel<T, HD, kBwdQ><<<dim3((f.q_len + 31) / 32, f.heads, f.batch), NT, 0, st>>>(p);
    } else {
      attn_bwd_kernel<T, HD, kBwdQ><<<dim3((f.q_len + 31) / 32, f.heads, f.batch), NT, 0, st>>>(p);
    }
    if constexpr (std::is_same<T, bf16_t>::value && HD == 64) {
      if (span_ok && mtts::override_of(MTTS_OVR_ATTN_GENERIC) != 1) {
        attn_bwd_kv_kernel<HD><<<dim3((f.kv_len + 127) / 128 * p.nchunk, f.heads, f.batch), 256, 0, st>>>(p);
        return;
      }
    }
    attn_bwd_kernel<T, HD, kBwdKV><<<dim3((f.kv_len + KG - 1) / KG * p.nchunk, f.heads, f.batch), NT, 0, st>>>(p);
    return;
  }
  attn_bwd_kernel<T, HD, kBwdShort><<<dim3(p.nchunk, f.heads, f.batch), NT, 0, st>>>(p);
}

template <typename T>
void dispatch_bwd(const BwdParams& p, bool split, hipStream_t st) {
  switch (p.a.f.head_dim) {
    case 16: launch_bwd<T, 16>(p, split, st); break;
    case 32: launch_bwd<T, 32>(p, split, st); break;
    case 64: launch_bwd<T, 64>(p, split, st); break;
    default: launch_bwd<T, 128>(p, split, st); break;
  }
  if (p.nchunk > 1) {
    const int64_t n = (int64_t)p.a.f.batch * p.a.f.kv_len * 2 * p.a.f.heads * p.a.f.head_dim;
    int blocks = (int)((n + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    attn_bwd_reduce_kernel<T><<<blocks, 256, 0, st>>>(p);
  }
}

}  // namespace

extern "C" int mtts_attention_fwd(const MttsAttnFwdArgs* a, void* stream) {
  int rc = check_fwd(a, "attention_fwd");
  if (rc) return rc;
  MTTS_CHECK(a->kv_hs == 0 || (a->q_len == 1 && a->kv_hs % 8 == 0 && mtts::override_of(MTTS_OVR_ATTN_GENERIC) != 1),
             "attention_fwd: a k / v head stride is taken by the single-query kernels only (q_len 1)");
  // the packed image is written by the single-pass decode kernel only
  MTTS_CHECK(!a->out_packed || (a->q_len == 1 && a->dtype == MTTS_BF16 && a->batch <= 32 &&
                                (a->heads * a->head_dim) % 32 == 0 && a->kv_len <= 8 * (256 / (a->head_dim / 8)) &&
                                mtts::override_of(MTTS_OVR_ATTN_GENERIC) != 1),
             "attention_fwd: packed output needs q_len 1, bf16, batch <= 32, kv_len <= %d", 8 * (256 / (a->head_dim / 8)));
  if (a->batch == 0 || a->q_len == 0) return MTTS_OK;
  hipStream_t st = (hipStream_t)stream;
  const bool one = a->q_len == 1 && mtts::override_of(MTTS_OVR_ATTN_GENERIC) != 1;   // decode step: single-query kernel
  if (a->dtype == MTTS_BF16)
    one ? dispatch_decode<bf16_t>(a, st) : dispatch_fwd<bf16_t>(a, st);
  else
    one ? dispatch_decode<float>(a, st) : dispatch_fwd<float>(a, st);
  MTTS_LAUNCH_CHECK("attention_fwd");
  return MTTS_OK;
}

extern "C" int mtts_attention_decode_qproj(const MttsAttnQProjArgs* q, void* stream) {
  MTTS_CHECK(q, "attention_decode_qproj: null args");
  MttsAttnFwdArgs a = q->f;
  MTTS_CHECK(a.out || a.out_packed, "attention_decode_qproj: null out and out_packed");
  {   // check_fwd on the k / v / mask side; q is computed in the kernel, out may be packed only
    MttsAttnFwdArgs c = a;
    c.q = q->x;
    c.q_bs = c.q_ls = 0;
    if (!c.out) { c.out = c.out_packed; c.o_bs = c.o_ls = 0; }
    int rc = check_fwd(&c, "attention_decode_qproj");
    if (rc) return rc;
  }
  const int NG = 256 / (a.head_dim / 8);
  MTTS_CHECK(a.q_len == 1 && a.dtype == MTTS_BF16 && a.kv_len <= 8 * NG && a.batch <= 32 &&
                 (a.heads * a.head_dim) % 32 == 0 && (a.head_dim == 64 || a.head_dim == 128),
             "attention_decode_qproj: q_len 1, bf16, head_dim 64 / 128, batch <= 32, kv_len <= %d", 8 * NG);
  MTTS_CHECK(q->x && q->wq && q->ln_w && q->ln_b, "attention_decode_qproj: null x / wq / ln_w / ln_b");
  MTTS_CHECK(q->d_model > 0 && q->d_model <= kQpMaxDm && q->d_model % 8 == 0 && q->x_rs >= q->d_model &&
                 ((uintptr_t)q->wq % 16) == 0,
             "attention_decode_qproj: d_model %d (<= %d, multiple of 8) / 16-byte aligned wq", q->d_model, kQpMaxDm);
  if (a.batch == 0) return MTTS_OK;
  QProj qp{(const bf16_t*)q->x, q->x_rs, (const bf16_t*)q->wq, (const bf16_t*)q->bq, q->ln_w, q->ln_b, q->eps,
           q->d_model};
  hipStream_t st = (hipStream_t)stream;
  if (a.head_dim == 64) launch_decode_qp<64>(&a, qp, st);
  else launch_decode_qp<128>(&a, qp, st);
  MTTS_LAUNCH_CHECK("attention_decode_qproj");
  return MTTS_OK;
}

extern "C" int64_t mtts_attention_bwd_workspace(int batch, int heads, int head_dim, int q_len, int kv_len, int dtype) {
  const BwdPlan pl = plan_bwd(batch, heads, head_dim, q_len, kv_len, dtype);
  return pl.part_bytes + pl.dq_bytes + pl.delta_bytes + 256;
}

extern "C" int mtts_attention_bwd(const MttsAttnBwdArgs* a, void* stream) {
  MTTS_CHECK(a, "attention_bwd: null args");
  int rc = check_fwd(&a->f, "attention_bwd");
  if (rc) return rc;
  const MttsAttnFwdArgs& f = a->f;
  MTTS_CHECK(a->dout && a->dq && a->dk && a->dv && f.lse, "attention_bwd: null tensor (dout/dq/dk/dv/lse)");
  const int64_t al = f.dtype == MTTS_BF16 ? 8 : 4;
  MTTS_CHECK(aligned16(a->dout) && a->do_bs % al == 0 && a->do_ls % al == 0,
             "attention_bwd: dout must be 16-byte aligned with 16-byte strides");
  hipStream_t st = (hipStream_t)stream;
  const int es = f.dtype == MTTS_BF16 ? 2 : 4;
  const int64_t d = (int64_t)f.heads * f.head_dim;
  if (f.batch == 0) return MTTS_OK;
  if (f.q_len == 0 || f.kv_len == 0) {
    // no queries: dk = dv = 0 (dq is empty or has no keys: zero as well)
    for (int b = 0; b < f.batch; ++b) {
      for (int64_t t = 0; t < f.kv_len; ++t) {
        (void)hipMemsetAsync((char*)a->dk + (b * a->dk_bs + t * a->dk_ls) * es, 0, d * es, st);
        (void)hipMemsetAsync((char*)a->dv + (b * a->dv_bs + t * a->dv_ls) * es, 0, d * es, st);
      }
      for (int64_t t = 0; t < f.q_len; ++t)
        (void)hipMemsetAsync((char*)a->dq + (b * a->dq_bs + t * a->dq_ls) * es, 0, d * es, st);
    }
    return MTTS_OK;
  }
  const BwdPlan pl = plan_bwd(f.batch, f.heads, f.head_dim, f.q_len, f.kv_len, f.dtype);
  MTTS_CHECK(a->workspace || (pl.part_bytes + pl.dq_bytes + pl.delta_bytes) == 0,
             "attention_bwd: workspace required");
  BwdParams p;
  p.a = *a;
  p.nchunk = pl.nchunk;
  p.qchunk = pl.qchunk;
  p.part = pl.part_bytes ? (float*)a->workspace : nullptr;
  p.dq_acc = pl.dq_bytes ? (float*)((char*)a->workspace + pl.part_bytes) : nullptr;
  p.delta = pl.delta_bytes ? (float*)((char*)a->workspace + pl.part_bytes + pl.dq_bytes) : nullptr;
  {
    const int es = f.dtype == MTTS_BF16 ? 2 : 4;
    p.dq_vec = ((uintptr_t)a->dq % 16 == 0) && (a->dq_bs * es) % 16 == 0 && (a->dq_ls * es) % 16 == 0;
  }
  if (f.dtype == MTTS_BF16)
    dispatch_bwd<bf16_t>(p, pl.split, st);
  else
    dispatch_bwd<float>(p, pl.split, st);
  MTTS_LAUNCH_CHECK("attention_bwd");
  return MTTS_OK;
}
