// Microbenchmark: throughput of v_exp_f32 vs v_fma_f32 and their mix on gfx950.
// hipcc --offload-arch=gfx950 -O3 valu_trans.hip -o valu_trans && ./valu_trans
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int NFMA, int NEXP>
__global__ __launch_bounds__(256) void mix(float* out, int iters, float s) {
  float a[8], e[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x * 1e-3f + i; e[i] = -1e-3f * i; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < NFMA; ++r) {
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = fmaf(a[i], s, 0.5f);
    }
#pragma unroll
    for (int r = 0; r < NEXP; ++r) {
#pragma unroll
      for (int i = 0; i < 8; ++i) e[i] = __builtin_amdgcn_exp2f(e[i]) - 1.0f;  // exp + 1 VALU
    }
  }
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) t += a[i] + e[i];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

template <int NFMA, int NEXP>
void run(const char* name, float* d, int wpsimd) {
  const int blocks = 256 * wpsimd;  // 4 waves per block, 1 block per (CU, wpsimd)
  const int iters = 2000;
  hipLaunchKernelGGL((mix<NFMA, NEXP>), dim3(blocks), dim3(256), 0, 0, d, 10, 0.999f);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((mix<NFMA, NEXP>), dim3(blocks), dim3(256), 0, 0, d, iters, 0.999f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  // per SIMD: waves = wpsimd; instructions per wave = iters * 8 * (NFMA + 2*NEXP)
  double wave_instr = (double)iters * 8 * (NFMA + 2 * NEXP) * wpsimd;
  double cyc = ms * 1e-3 * 2.4e9;  // upper-bound clock
  printf("%-26s waves/SIMD=%d  %.3f ms  -> %.2f cyc/wave-instr @2.4GHz (fma=%d exp=%d)\n", name, wpsimd, ms,
         cyc / wave_instr, NFMA, NEXP);
}

int main() {
  float* d;
  hipMalloc(&d, 256 * 64 * 256 * 4);
  for (int w : {1, 2, 4, 8}) {
    run<4, 0>("fma only", d, w);
    run<0, 4>("exp(+sub) only", d, w);
    run<4, 1>("4 fma : 1 exp(+sub)", d, w);
    run<8, 1>("8 fma : 1 exp(+sub)", d, w);
  }
  return 0;
}
