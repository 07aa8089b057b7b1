// Background "aggressor" kernels for tools/dbg/race_probe.py (BG=1,
// ONLY1=ubench:<mode>): which instruction class, running in ANOTHER process's
// workgroups on the same CUs, goes with the scan backward's changing results?
// Each mode holds 64 KiB of LDS per 512-thread workgroup, like the skinny TN
// GEMM (tn_skinny_kernel) that triggers it:
//   0: ds_read_b64_tr_b16 loop      1: MFMA 16x16x32 bf16 loop (no LDS reads)
//   2: ds_read_b128 loop (control)   3: tr reads + MFMA (the skinny kernel's mix)
//   hipcc -O3 -shared -fPIC --offload-arch=gfx950 aggressor.hip -o aggressor.so
#include <hip/hip_runtime.h>

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <int MODE>
__global__ __launch_bounds__(512) void aggress_kernel(int iters, float* out) {
  __shared__ __attribute__((aligned(16))) char s[65536];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < 65536 / 16; i += 512)
    *(uint4*)(s + 16 * i) = make_uint4(i, i * 3, i * 5, i * 7);
  __syncthreads();
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  s16x8 a = {1, 2, 3, 4, 5, 6, 7, (short)lane};
  for (int it = 0; it < iters; ++it) {
    const int base = ((it * 37 + (tid >> 6) * 4096) & 0xFFFF) & ~2047;
    if constexpr (MODE == 0 || MODE == 3) {
      const int off = base + 256 * (lane >> 4) + 16 * ((lane >> 2) & 3) + 8 * (lane & 1);
      s16x4 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(s + off));
      s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(s + off + 1024));
      a = s16x8{r0[0], r0[1], r0[2], r0[3], r1[0], r1[1], r1[2], r1[3]};
      if constexpr (MODE == 0) acc[0] += (float)(a[0] + a[7]);
    }
    if constexpr (MODE == 2) {
      const uint4 v = *(const uint4*)(s + base + 16 * lane);
      acc[0] += (float)(v.x + v.w);
    }
    if constexpr (MODE == 1 || MODE == 3) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, a),
                                                      acc, 0, 0, 0);
    }
  }
  if (acc[0] == 1234.5f) out[blockIdx.x] = acc[1];   // keeps the loop; never true in practice
}

extern "C" int aggress(int mode, int blocks, int iters, float* out, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  switch (mode) {
    case 0: hipLaunchKernelGGL(aggress_kernel<0>, dim3(blocks), dim3(512), 0, st, iters, out); break;
    case 1: hipLaunchKernelGGL(aggress_kernel<1>, dim3(blocks), dim3(512), 0, st, iters, out); break;
    case 2: hipLaunchKernelGGL(aggress_kernel<2>, dim3(blocks), dim3(512), 0, st, iters, out); break;
    case 3: hipLaunchKernelGGL(aggress_kernel<3>, dim3(blocks), dim3(512), 0, st, iters, out); break;
    default: return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
