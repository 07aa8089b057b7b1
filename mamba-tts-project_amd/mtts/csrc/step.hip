// Decode-step kernels (L = 1) for gfx950: conv-window update and the SSM
// state update.  Replace [upstream] causal_conv1d_update (HF:61-78) and
// selective_state_update (Triton; HF:128-171), i.e. mamba-ssm Mamba.step,
// reached from MambaTTSDecoder.decode_step (mamba_decoder.py:188-256) via
// mamba_decoder.py:63.  States are updated in place (hipGraph-replayable).
// One thread per (batch, channel); the (D, N) fp32 state row of a channel is
// 64 contiguous bytes, so consecutive lanes stream consecutive rows.
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

template <typename Tio, typename Tbc>
__global__ void state_update_kernel(const MttsStateUpdateArgs a) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)a.batch * a.dim) return;
  const int c = idx % a.dim;
  const int b = idx / a.dim;
  const float x = ldf((const Tio*)a.x + (int64_t)b * a.x_bs + c);
  float dt;
  if (a.dt_rank > 0) {   // fused dt_proj: low-rank input row of batch b . dt_w row c
    const Tio* xr = (const Tio*)a.dt + (int64_t)b * a.dt_bs;
    const Tio* wr = (const Tio*)a.dt_w + (int64_t)c * a.dt_rank;
    float s0 = 0.f, s1 = 0.f;
    int r = 0;
    if constexpr (sizeof(Tio) == 2) {   // 16-byte pieces when the rows allow it
      if ((a.dt_rank & 7) == 0 && (((uintptr_t)xr | (uintptr_t)wr) & 15) == 0) {
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        for (; r < a.dt_rank; r += 8) {
          const s16x8 xv = *reinterpret_cast<const s16x8*>(xr + r), wv = *reinterpret_cast<const s16x8*>(wr + r);
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            s0 = fmaf(bf2f((bf16_t)xv[e]), bf2f((bf16_t)wv[e]), s0);
            s1 = fmaf(bf2f((bf16_t)xv[e + 1]), bf2f((bf16_t)wv[e + 1]), s1);
          }
        }
      }
    }
    for (; r + 1 < a.dt_rank; r += 2) {
      s0 = fmaf(ldf(xr + r), ldf(wr + r), s0);
      s1 = fmaf(ldf(xr + r + 1), ldf(wr + r + 1), s1);
    }
    if (r < a.dt_rank) s0 = fmaf(ldf(xr + r), ldf(wr + r), s0);
    dt = s0 + s1;
  } else {
    dt = ldf((const Tio*)a.dt + (int64_t)b * a.dt_bs + c);
  }
  dt += a.dt_bias ? a.dt_bias[c] : 0.f;
  if (a.dt_softplus) dt = softplus_f(dt);
  const float dtx = dt * x;
  float4* sp = reinterpret_cast<float4*>(a.state + idx * 16);
  const float4* Ap = reinterpret_cast<const float4*>(a.A + (int64_t)c * 16);
  const Tbc* Bp = (const Tbc*)a.Bm + (int64_t)b * a.B_bs;
  const Tbc* Cp = (const Tbc*)a.Cm + (int64_t)b * a.C_bs;
  float y = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float4 s = sp[q];
    const float4 A = Ap[q];
    float h[4] = {s.x, s.y, s.z, s.w};
    const float Av[4] = {A.x, A.y, A.z, A.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = 4 * q + i;
      const float e = __builtin_amdgcn_exp2f(dt * Av[i] * kLog2e);
      h[i] = fmaf(e, h[i], dtx * ldf(Bp + n));
      y = fmaf(ldf(Cp + n), h[i], y);
    }
    sp[q] = make_float4(h[0], h[1], h[2], h[3]);
  }
  if (a.D) y = fmaf(a.D[c], x, y);
  if (a.z) y *= silu_f(ldf((const Tio*)a.z + (int64_t)b * a.z_bs + c));
  stf((Tio*)a.out + (int64_t)b * a.out_bs + c, y);
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
  MTTS_CHECK(a && a->state && a->x && a->dt && a->A && a->Bm && a->Cm && a->out, "state_update: null tensor");
  MTTS_CHECK(a->batch > 0 && a->dim > 0, "state_update: bad sizes");
  MTTS_CHECK(a->dt_rank >= 0 && (a->dt_rank == 0 || a->dt_w), "state_update: dt_rank > 0 needs dt_w");
  if (a->dstate != 16) {
    set_error("state_update: dstate=%d unsupported", a->dstate);
    return MTTS_EUNSUPPORTED;
  }
  MTTS_CHECK((uintptr_t)a->state % 16 == 0 && (uintptr_t)a->A % 16 == 0, "state_update: state/A alignment");
  const int64_t n = (int64_t)a->batch * a->dim;
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
