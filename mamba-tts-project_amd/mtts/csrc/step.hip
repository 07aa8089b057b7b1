// Decode-step kernels (L = 1) for gfx950: conv-window update and the SSM
// state update.  Replace [upstream] causal_conv1d_update (HF:61-78) and
// selective_state_update (Triton; HF:128-171), i.e. mamba-ssm Mamba.step,
// reached from MambaTTSDecoder.decode_step (mamba_decoder.py:188-256) via
// mamba_decoder.py:63.  States are updated in place (hipGraph-replayable).
// conv update: one thread per (batch, channel); state update: four lanes
// per (batch, channel) over its 64-byte fp32 state row (coalesced KiB rows).
#include "common.h"

namespace mtts {

template <typename T>
__global__ void conv_update_kernel(const MttsConvUpdateArgs a) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)a.batch * a.dim) return;
  const int c = idx % a.dim;
  const int b = idx / a.dim;
  float4* st = reinterpret_cast<float4*>(a.conv_state + idx * 4);
  float4 s = *st;
  const float x = ldf((const T*)a.x + (int64_t)b * a.x_bs + c);
  const float4 w = *reinterpret_cast<const float4*>(a.w + (int64_t)c * 4);
  s = make_float4(s.y, s.z, s.w, x);
  *st = s;
  float v = fmaf(w.x, s.x, fmaf(w.y, s.y, fmaf(w.z, s.z, fmaf(w.w, s.w, a.bias ? a.bias[c] : 0.f))));
  if (a.silu) v = silu_f(v);
  stf((T*)a.out + (int64_t)b * a.out_bs + c, v);
}

// Four lanes per (batch, channel), lane j owning states 4j..4j+3: a wave's
// state / A loads and state stores are 1 KiB contiguous (one 16-byte piece
// per lane), the fused dt_proj dot is split over the quad (a quarter of
// dt_rank each) and dt / y are combined with two quad DPP adds.
template <typename Tio, typename Tbc>
__global__ void state_update_kernel(const MttsStateUpdateArgs a) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t pair = idx >> 2;
  const int j = threadIdx.x & 3;
  const bool ok = pair < (int64_t)a.batch * a.dim;
  const int64_t pc = ok ? pair : 0;   // lanes past the end compute on row 0 and store nothing
  const int c = pc % a.dim;
  const int b = pc / a.dim;
  float4* sp = reinterpret_cast<float4*>(a.state + pc * 16) + j;
  const float4 s = *sp;
  const float4 A = reinterpret_cast<const float4*>(a.A + (int64_t)c * 16)[j];
  const Tbc* Bp = (const Tbc*)a.Bm + (int64_t)b * a.B_bs + 4 * j;
  const Tbc* Cp = (const Tbc*)a.Cm + (int64_t)b * a.C_bs + 4 * j;
  const float Bv[4] = {ldf(Bp), ldf(Bp + 1), ldf(Bp + 2), ldf(Bp + 3)};
  const float Cv[4] = {ldf(Cp), ldf(Cp + 1), ldf(Cp + 2), ldf(Cp + 3)};
  const float x = ldf((const Tio*)a.x + (int64_t)b * a.x_bs + c);
  float dt;
  if (a.dt_rank > 0) {   // fused dt_proj: low-rank input row of batch b . dt_w row c, a quarter per lane
    const int R = a.dt_rank;
    const Tio* xr = (const Tio*)a.dt + (int64_t)b * a.dt_bs;
    const Tio* wr = (const Tio*)a.dt_w + (int64_t)c * R;
    float s0 = 0.f, s1 = 0.f;
    bool done = false;
    if constexpr (sizeof(Tio) == 2) {   // 16-byte pieces when the rows allow it
      if ((R & 31) == 0 && (((uintptr_t)xr | (uintptr_t)wr) & 15) == 0) {
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const int q4 = R >> 2;
        for (int r = j * q4; r < (j + 1) * q4; r += 8) {
          const s16x8 xv = *reinterpret_cast<const s16x8*>(xr + r), wv = *reinterpret_cast<const s16x8*>(wr + r);
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            s0 = fmaf(bf2f((bf16_t)xv[e]), bf2f((bf16_t)wv[e]), s0);
            s1 = fmaf(bf2f((bf16_t)xv[e + 1]), bf2f((bf16_t)wv[e + 1]), s1);
          }
        }
        done = true;
      }
    }
    if (!done) {
      for (int r = j; r < R; r += 8) {
        s0 = fmaf(ldf(xr + r), ldf(wr + r), s0);
        if (r + 4 < R) s1 = fmaf(ldf(xr + r + 4), ldf(wr + r + 4), s1);
      }
    }
    dt = s0 + s1;
    dt += dpp<kQuadXor1>(dt);
    dt += dpp<kQuadXor2>(dt);
  } else {
    dt = ldf((const Tio*)a.dt + (int64_t)b * a.dt_bs + c);
  }
  dt += a.dt_bias ? a.dt_bias[c] : 0.f;
  if (a.dt_softplus) dt = softplus_f(dt);
  const float dtx = dt * x;
  float h[4] = {s.x, s.y, s.z, s.w};
  const float Av[4] = {A.x, A.y, A.z, A.w};
  float y = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float e = __builtin_amdgcn_exp2f(dt * Av[i] * kLog2e);
    h[i] = fmaf(e, h[i], dtx * Bv[i]);
    y = fmaf(Cv[i], h[i], y);
  }
  if (ok) *sp = make_float4(h[0], h[1], h[2], h[3]);
  y += dpp<kQuadXor1>(y);
  y += dpp<kQuadXor2>(y);
  if (!ok || j != 0) return;
  if (a.D) y = fmaf(a.D[c], x, y);
  if (a.z) y *= silu_f(ldf((const Tio*)a.z + (int64_t)b * a.z_bs + c));
  if (a.out) stf((Tio*)a.out + (int64_t)b * a.out_bs + c, y);
  if constexpr (sizeof(Tio) == 2) {   // packed activation image for out_proj (csrc/common.h)
    if (a.out_packed) ((bf16_t*)a.out_packed)[xpk_index(b, c)] = f2bf(y);
  }
}



}  // namespace mtts

using namespace mtts;

extern "C" int mtts_causal_conv1d_update(const MttsConvUpdateArgs* a, void* stream) {
  MTTS_CHECK(a && a->x && a->conv_state && a->w && a->out, "conv_update: null tensor");
  MTTS_CHECK(a->batch > 0 && a->dim > 0, "conv_update: bad sizes");
  if (a->width != 4) {
    set_error("conv_update: width=%d unsupported", a->width);
    return MTTS_EUNSUPPORTED;
  }
  MTTS_CHECK((uintptr_t)a->conv_state % 16 == 0 && (uintptr_t)a->w % 16 == 0, "conv_update: state/w alignment");
  const int64_t n = (int64_t)a->batch * a->dim;
  hipStream_t st = (hipStream_t)stream;
  if (a->dtype == MTTS_F32) hipLaunchKernelGGL(conv_update_kernel<float>, dim3((n + 255) / 256), dim3(256), 0, st, *a);
  else hipLaunchKernelGGL(conv_update_kernel<bf16_t>, dim3((n + 255) / 256), dim3(256), 0, st, *a);
  MTTS_LAUNCH_CHECK("causal_conv1d_update");
  return MTTS_OK;
}

extern "C" int mtts_selective_state_update(const MttsStateUpdateArgs* a, void* stream) {
  MTTS_CHECK(a && a->state && a->x && a->dt && a->A && a->Bm && a->Cm, "state_update: null tensor");
  MTTS_CHECK(a->batch > 0 && a->dim > 0, "state_update: bad sizes");
  MTTS_CHECK(a->dt_rank >= 0 && (a->dt_rank == 0 || a->dt_w), "state_update: dt_rank > 0 needs dt_w");
  if (a->dstate != 16) {
    set_error("state_update: dstate=%d unsupported", a->dstate);
    return MTTS_EUNSUPPORTED;
  }
  MTTS_CHECK((uintptr_t)a->state % 16 == 0 && (uintptr_t)a->A % 16 == 0, "state_update: state/A alignment");
  MTTS_CHECK(a->out || a->out_packed, "state_update: no output");
  MTTS_CHECK(!a->out_packed || (a->dtype_io == MTTS_BF16 && a->batch <= 32 && a->dim % 32 == 0),
             "state_update: packed output needs bf16, batch <= 32, dim %% 32 == 0");
  const int64_t n = (int64_t)a->batch * a->dim * 4;   // four lanes per (batch, channel)
  hipStream_t st = (hipStream_t)stream;
  dim3 g((n + 255) / 256), blk(256);
  if (a->dtype_io == MTTS_F32) {
    if (a->dtype_bc == MTTS_F32) hipLaunchKernelGGL((state_update_kernel<float, float>), g, blk, 0, st, *a);
    else hipLaunchKernelGGL((state_update_kernel<float, bf16_t>), g, blk, 0, st, *a);
  } else {
    if (a->dtype_bc == MTTS_F32) hipLaunchKernelGGL((state_update_kernel<bf16_t, float>), g, blk, 0, st, *a);
    else hipLaunchKernelGGL((state_update_kernel<bf16_t, bf16_t>), g, blk, 0, st, *a);
  }
  MTTS_LAUNCH_CHECK("selective_state_update");
  return MTTS_OK;
}

