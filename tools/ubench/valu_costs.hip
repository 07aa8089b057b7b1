// Microbenchmark: SIMD cycles per wave-instruction on gfx950 for the
// instruction kinds of the scan inner loop (fma, packed fma, exp, DPP mul),
// at 1..8 waves per SIMD.  In-kernel s_memtime (shader clock) per wave, so
// DVFS does not enter.  hipcc --offload-arch=gfx950 -O3 valu_costs.hip -o valu_costs
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

enum { K_FMA, K_PKFMA, K_EXP, K_DPPMUL, K_MIX };

template <int KIND>
__global__ __launch_bounds__(256) void bench(float* out, unsigned long long* cyc, int iters, float s) {
  float a[8];
  f2 p[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 1e-3f + i * 0.1f;
#pragma unroll
  for (int i = 0; i < 4; ++i) p[i] = f2{a[2 * i], a[2 * i + 1]};
  __syncthreads();
  const unsigned long long t0 = stamp();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if constexpr (KIND == K_FMA) {
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = fmaf(a[i], s, 0.5f);
      } else if constexpr (KIND == K_PKFMA) {
#pragma unroll
        for (int i = 0; i < 8; ++i) p[i & 3] = __builtin_elementwise_fma(p[i & 3], f2{s, s}, f2{0.5f, 0.25f});
      } else if constexpr (KIND == K_EXP) {
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = __builtin_amdgcn_exp2f(a[i]);
      } else if constexpr (KIND == K_DPPMUL) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float b = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(a[(i + 1) & 7]), 0x55, 0xF, 0xF, true));
          a[i] = a[i] * b;
        }
      } else {  // 1 exp per 3 fma-class ops (state update shape)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float e = __builtin_amdgcn_exp2f(a[i] * s);
          a[i] = fmaf(e, a[i], 0.5f) * s;
        }
      }
    }
  }
  const unsigned long long t1 = stamp();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) t += a[i] + p[i & 3][i & 1];
  out[blockIdx.x * 256 + threadIdx.x] = t;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int KIND>
void run(const char* name, int ninstr_per_rep, float* d, unsigned long long* c, int wpsimd) {
  const int blocks = 256 * wpsimd;  // 4 waves/block; every CU gets wpsimd blocks -> wpsimd waves per SIMD
  const int iters = 1000;
  hipLaunchKernelGGL((bench<KIND>), dim3(blocks), dim3(256), 0, 0, d, c, 10, 0.999f);
  hipLaunchKernelGGL((bench<KIND>), dim3(blocks), dim3(256), 0, 0, d, c, iters, 0.999f);
  hipDeviceSynchronize();
  static unsigned long long h[256 * 8 * 4];
  hipMemcpy(h, c, blocks * 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  double mean = 0;
  for (int i = 0; i < blocks * 4; ++i) mean += (double)h[i];
  mean /= blocks * 4;
  // s_memtime ticks at the shader clock; per SIMD, wpsimd waves share it
  const double per_wave_instr = mean / ((double)iters * 4 * ninstr_per_rep);
  printf("%-10s waves/SIMD=%d  wave-cycles/instr %.2f  -> SIMD cycles/instr %.2f\n", name, wpsimd, per_wave_instr,
         per_wave_instr / wpsimd);
}

int main() {
  float* d;
  unsigned long long* c;
  hipMalloc(&d, 256 * 8 * 256 * 4);
  hipMalloc(&c, 256 * 8 * 4 * sizeof(unsigned long long));
  for (int w : {1, 2, 4, 8}) {
    run<K_FMA>("fma", 8, d, c, w);
    run<K_PKFMA>("pk_fma", 8, d, c, w);
    run<K_EXP>("exp", 8, d, c, w);
    run<K_DPPMUL>("dpp_mul", 8, d, c, w);
    run<K_MIX>("mul+exp+fma+mul", 32, d, c, w);
  }
  return 0;
}
