// Deterministic column sums over per-block partial slabs (LN / conv1d / ...
// parameter gradients).  out[g][c] = sum_{p in group g} part[p][c].
// One 256-thread block per 64 columns and group: the 4 waves stride over
// the partials with 8 independent loads in flight per lane, then combine in
// LDS in a fixed order (bitwise reproducible).
#include "common.h"

namespace mtts {

__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ part, int nparts, int ppg,
                                                     int64_t pstride, int ncols, float* __restrict__ out,
                                                     int64_t out_gstride) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int g = blockIdx.y;
  const int p0 = g * ppg, p1 = min(nparts, p0 + ppg);
  float acc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] = 0.f;
  if (c < ncols) {
    int p = p0 + w;
    for (; p + 28 < p1; p += 32) {
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += part[(int64_t)(p + 4 * q) * pstride + c];
    }
    for (; p < p1; p += 4) acc[0] += part[(int64_t)p * pstride + c];
  }
  float s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && c < ncols) out[(int64_t)g * out_gstride + c] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

void colsum(const float* part, int nparts, int ppg, int64_t pstride, int ncols, float* out, int64_t out_gstride,
            hipStream_t st) {
  const int ngroups = (nparts + ppg - 1) / ppg;
  hipLaunchKernelGGL(colsum_kernel, dim3((ncols + 63) / 64, ngroups), dim3(256), 0, st, part, nparts, ppg, pstride,
                     ncols, out, out_gstride);
}

}  // namespace mtts
