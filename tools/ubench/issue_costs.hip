// Microbenchmark: SIMD cycles per wave-instruction on gfx950 for the
// instruction kinds of the scan inner loops, at 1/2/4/8 waves per SIMD.
// Cycles come from hipEvent wall time x the in-kernel clock
// (d s_memtime / d s_memrealtime x 100 MHz, median over waves), so the
// number does not depend on what s_memtime counts.
//   hipcc --offload-arch=gfx950 -O3 issue_costs.hip -o issue_costs && ./issue_costs
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));

enum { K_FMA, K_PKFMA, K_PKMUL, K_EXP, K_DPPMOV, K_CNDMASK, K_ADDDPP, K_EXP_PK, K_EXP_FMA, K_LDS128, K_EXP_LDS };
static const char* kNames[] = {"v_fma_f32", "v_pk_fma_f32", "v_pk_mul_f32", "v_exp_f32", "v_mov_b32_dpp",
                               "v_cndmask_b32", "v_add_f32_dpp", "1exp+1pk_fma", "1exp+2fma", "ds_read_b128",
                               "1exp+1ds128"};

__device__ __forceinline__ void stamps(unsigned long long& t, unsigned long long& r) {
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t), "=s"(r)::"memory");
}

template <int KIND>
__global__ __launch_bounds__(256) void bench(float* out, unsigned long long* clk, int iters, float s) {
  __shared__ float4 lds[1024];
  lds[threadIdx.x] = make_float4(threadIdx.x, 1.f, 2.f, 3.f);
  float a[8];
  f2 p[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 1e-3f + i * 0.1f;
#pragma unroll
  for (int i = 0; i < 8; ++i) p[i] = f2{a[i], a[(i + 1) & 7]};
  float4 acc = make_float4(0, 0, 0, 0);
  float b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) b[i] = a[i] * 0.5f;
  const f2 sv = f2{s, 0.999f}, cv = f2{0.5f, 0.25f};
  const unsigned long long mask = 0x5555555555555555ull;
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4 q[8];
  const unsigned laddr = (threadIdx.x & 63) * 16;
  __syncthreads();
  unsigned long long t0, r0, t1, r1;
  stamps(t0, r0);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      // inline asm: exactly one instruction of the named kind (no SLP packing)
      if constexpr (KIND == K_FMA) {
        asm volatile("v_fma_f32 %0, %0, %1, 0.5" : "+v"(a[i]) : "v"(s));
      } else if constexpr (KIND == K_PKFMA) {
        asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[i]) : "v"(sv), "v"(cv));
      } else if constexpr (KIND == K_PKMUL) {
        asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p[i]) : "v"(sv));
      } else if constexpr (KIND == K_EXP) {
        asm volatile("v_exp_f32 %0, %0" : "+v"(a[i]));
      } else if constexpr (KIND == K_DPPMOV) {
        asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf" : "=v"(a[i]) : "v"(a[(i + 3) & 7]));
      } else if constexpr (KIND == K_CNDMASK) {
        asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(a[(i + 5) & 7]), "s"(mask));
      } else if constexpr (KIND == K_ADDDPP) {
        asm volatile("v_add_f32_dpp %0, %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(a[i]) : "v"(a[(i + 3) & 7]));
      } else if constexpr (KIND == K_EXP_PK) {
        asm volatile("v_exp_f32 %0, %0" : "+v"(a[i]));
        asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[i]) : "v"(sv), "v"(cv));
      } else if constexpr (KIND == K_EXP_FMA) {
        asm volatile("v_exp_f32 %0, %0" : "+v"(a[i]));
        asm volatile("v_fma_f32 %0, %0, %1, 0.5" : "+v"(b[i]) : "v"(s));
        asm volatile("v_fma_f32 %0, %0, %1, 0.5" : "+v"(b[(i + 4) & 7]) : "v"(s));
      } else if constexpr (KIND == K_LDS128) {
        asm volatile("ds_read_b128 %0, %1" : "=v"(q[i]) : "v"(laddr));
      } else {
        asm volatile("v_exp_f32 %0, %0" : "+v"(a[i]));
        asm volatile("ds_read_b128 %0, %1" : "=v"(q[i]) : "v"(laddr));
      }
    }
    if constexpr (KIND == K_LDS128 || KIND == K_EXP_LDS) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(q[i]));
    }
    asm volatile("" ::: "memory");
  }
  stamps(t1, r1);
  float t = acc.x;
#pragma unroll
  for (int i = 0; i < 8; ++i) t += a[i] + p[i][0] + p[i][1] + b[i] + q[i][0];
  out[blockIdx.x * 256 + threadIdx.x] = t;
  if ((threadIdx.x & 63) == 0) {
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
    clk[2 * w] = t1 - t0;
    clk[2 * w + 1] = r1 - r0;
  }
}

template <int KIND>
void run(float* d, unsigned long long* c, int wpsimd) {
  const int blocks = 256 * wpsimd;  // 4 waves per block, wpsimd blocks per CU
  const int iters = 4000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((bench<KIND>), dim3(blocks), dim3(256), 0, 0, d, c, 200, 0.999f);
  hipEventRecord(e0);
  hipLaunchKernelGGL((bench<KIND>), dim3(blocks), dim3(256), 0, 0, d, c, iters, 0.999f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(blocks * 8);
  hipMemcpy(h.data(), c, blocks * 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  std::vector<double> mhz, cyc;
  for (int w = 0; w < blocks * 4; ++w) {
    mhz.push_back((double)h[2 * w] / (double)h[2 * w + 1] * 100.0);
    cyc.push_back((double)h[2 * w]);
  }
  std::sort(mhz.begin(), mhz.end());
  std::sort(cyc.begin(), cyc.end());
  const double clock_mhz = mhz[mhz.size() / 2];
  const double n = (double)iters * 8;  // wave-instructions (or pairs) per wave
  const double simd_cyc_wall = ms * 1e-3 * clock_mhz * 1e6 / (n * wpsimd);
  const double simd_cyc_stamp = cyc[cyc.size() / 2] / (n * wpsimd);
  printf("%-14s waves/SIMD=%d clock=%.0f MHz  SIMD cycles per wave-instr: wall %.2f  stamp %.2f\n", kNames[KIND],
         wpsimd, clock_mhz, simd_cyc_wall, simd_cyc_stamp);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  float* d;
  unsigned long long* c;
  hipMalloc(&d, 256 * 8 * 256 * 4);
  hipMalloc(&c, 256 * 8 * 4 * 2 * sizeof(unsigned long long));
  for (int w : {1, 2, 4, 8}) {
    run<K_FMA>(d, c, w);
    run<K_PKFMA>(d, c, w);
    run<K_PKMUL>(d, c, w);
    run<K_EXP>(d, c, w);
    run<K_DPPMOV>(d, c, w);
    run<K_CNDMASK>(d, c, w);
    run<K_ADDDPP>(d, c, w);
    run<K_EXP_PK>(d, c, w);
    run<K_EXP_FMA>(d, c, w);
    run<K_LDS128>(d, c, w);
    run<K_EXP_LDS>(d, c, w);
  }
  return 0;
}
