// Streaming floor of the forward scan's HBM pattern (timing only).
// out = u + delta + z over (B, L, D) fp32 channel-last tensors, each block
// owning CPB channels of one batch row and an L/K slice of timesteps, walking
// the slice in row order like scan_fwd_w2_kernel.  Reports GB/s per
// (CPB, threads, K) so the channel width of a block's row chunk can be chosen
// by measurement.   hipcc -O3 --offload-arch=gfx950 stream_pattern.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int CPB, int T, int U>
__global__ __launch_bounds__(T) void stream_rows(const float4* __restrict__ u, const float4* __restrict__ d,
                                                 const float4* __restrict__ z, float4* __restrict__ o, int L, int D,
                                                 int seg) {
  constexpr int CPR = CPB / 4;       // float4 chunks per row
  constexpr int R = T / CPR;         // rows per pass
  const int tid = threadIdx.x;
  const int row = tid / CPR, col = tid % CPR;
  const int b = blockIdx.y;
  const int t0 = blockIdx.z * seg;
  const int64_t D4 = D / 4;
  const int64_t base = (int64_t)b * L * D4 + blockIdx.x * CPR + col;
  for (int t = t0; t < t0 + seg; t += R * U) {
    float4 a[U], bb[U], c[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int64_t i = base + (int64_t)(t + q * R + row) * D4;
      a[q] = u[i]; bb[q] = d[i]; c[q] = z[i];
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int64_t i = base + (int64_t)(t + q * R + row) * D4;
      o[i] = make_float4(a[q].x + bb[q].x + c[q].x, a[q].y + bb[q].y + c[q].y, a[q].z + bb[q].z + c[q].z,
                         a[q].w + bb[q].w + c[q].w);
    }
  }
}

template <int CPB, int T, int U>
int run(float4* u, float4* d, float4* z, float4* o, int B, int L, int D, int K) {
  dim3 grid(D / CPB, B, K);
  const int seg = L / K;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) stream_rows<CPB, T, U><<<grid, T>>>(u, d, z, o, L, D, seg);
  std::vector<float> ms;
  CK(hipEventRecord(e0));
  const int it = 20;
  for (int w = 0; w < it; ++w) stream_rows<CPB, T, U><<<grid, T>>>(u, d, z, o, L, D, seg);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float t;
  CK(hipEventElapsedTime(&t, e0, e1));
  t /= it;
  const double bytes = 16.0 * B * L * D;
  printf("CPB=%4d T=%3d U=%d K=%2d blocks=%6d  %.3f ms  %.0f GB/s\n", CPB, T, U, K, grid.x * grid.y * grid.z, t,
         bytes / t / 1e6);
  return 0;
}

int main() {
  const int B = 32, L = 8192, D = 2048;
  const size_t n = (size_t)B * L * D;
  float4 *u, *d, *z, *o;
  CK(hipMalloc(&u, n * 4));
  CK(hipMalloc(&d, n * 4));
  CK(hipMalloc(&z, n * 4));
  CK(hipMalloc(&o, n * 4));
  CK(hipMemset(u, 0, n * 4));
  CK(hipMemset(d, 0, n * 4));
  CK(hipMemset(z, 0, n * 4));
  for (int r = 0; r < 2; ++r) {
    run<64, 256, 4>(u, d, z, o, B, L, D, 1);
    run<64, 256, 2>(u, d, z, o, B, L, D, 1);
    run<64, 256, 4>(u, d, z, o, B, L, D, 2);
    run<128, 256, 4>(u, d, z, o, B, L, D, 1);
    run<128, 256, 4>(u, d, z, o, B, L, D, 2);
    run<128, 512, 4>(u, d, z, o, B, L, D, 1);
    run<256, 256, 4>(u, d, z, o, B, L, D, 4);
    run<256, 512, 4>(u, d, z, o, B, L, D, 2);
    run<512, 512, 4>(u, d, z, o, B, L, D, 4);
    run<2048, 256, 4>(u, d, z, o, B, L, D, 32);
  }
  return 0;
}
