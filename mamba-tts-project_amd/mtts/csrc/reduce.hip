// Deterministic column sums over per-block partial slabs (LN / conv1d / ...
// parameter gradients).  out[g][c] = sum_{p in group g} part[p][c].
// One 256-thread block per 64 columns and group: the 4 waves stride over
// the partials with 8 independent loads in flight per lane, then combine in
// LDS in a fixed order (bitwise reproducible).
#include "common.h"

namespace mtts {

template <typename T>
__global__ __launch_bounds__(256) void colsum_kernel(const T* __restrict__ part, int nparts, int ppg,
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
      for (int q = 0; q < 8; ++q) acc[q] += ldf(part + (int64_t)(p + 4 * q) * pstride + c);
    }
    for (; p < p1; p += 4) acc[0] += ldf(part + (int64_t)p * pstride + c);
  }
  float s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && c < ncols) out[(int64_t)g * out_gstride + c] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

void colsum(const float* part, int nparts, int ppg, int64_t pstride, int ncols, float* out, int64_t out_gstride,
            hipStream_t st) {
  const int ngroups = (nparts + ppg - 1) / ppg;
  hipLaunchKernelGGL(colsum_kernel<float>, dim3((ncols + 63) / 64, ngroups), dim3(256), 0, st, part, nparts, ppg,
                     pstride, ncols, out, out_gstride);
}

}  // namespace mtts

extern "C" int64_t mtts_colsum_workspace(int rows, int cols, int rows_per_group) {
  if (rows_per_group <= 1024) return 0;
  const int64_t chunks = (int64_t)(rows + 255) / 256;
  return chunks * cols * 4 + 256;
}

extern "C" int mtts_colsum(const void* in, int dtype, int rows, int cols, int64_t row_stride, int rows_per_group,
                           float* out, int64_t out_gstride, void* workspace, void* stream) {
  using namespace mtts;
  MTTS_CHECK(in && out && rows >= 0 && cols > 0 && rows_per_group > 0, "colsum: bad args");
  MTTS_CHECK(dtype == MTTS_F32 || dtype == MTTS_BF16, "colsum: bad dtype");
  hipStream_t st = (hipStream_t)stream;
  if (rows == 0) {
    (void)hipMemsetAsync(out, 0, (size_t)cols * 4, st);
    return MTTS_OK;
  }
  if (rows_per_group > 1024) {
    // two stages: 256-row chunks -> fp32 partial slab -> per-group sum of chunks
    MTTS_CHECK(workspace, "colsum: workspace required (mtts_colsum_workspace)");
    MTTS_CHECK(rows_per_group % 256 == 0 || rows_per_group >= rows, "colsum: rows_per_group %% 256 != 0");
    const int chunks = (rows + 255) / 256;
    float* part = (float*)workspace;
    dim3 g1((cols + 63) / 64, chunks);
    if (dtype == MTTS_F32)
      hipLaunchKernelGGL(colsum_kernel<float>, g1, dim3(256), 0, st, (const float*)in, rows, 256, row_stride, cols,
                         part, (int64_t)cols);
    else
      hipLaunchKernelGGL(colsum_kernel<bf16_t>, g1, dim3(256), 0, st, (const bf16_t*)in, rows, 256, row_stride,
                         cols, part, (int64_t)cols);
    MTTS_LAUNCH_CHECK("colsum stage 1");
    const int cpg = rows_per_group >= rows ? chunks : rows_per_group / 256;
    colsum(part, chunks, cpg, cols, cols, out, out_gstride, st);
    MTTS_LAUNCH_CHECK("colsum stage 2");
    return MTTS_OK;
  }
  const int ngroups = (rows + rows_per_group - 1) / rows_per_group;
  dim3 grid((cols + 63) / 64, ngroups);
  if (dtype == MTTS_F32)
    hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(256), 0, st, (const float*)in, rows, rows_per_group,
                       row_stride, cols, out, out_gstride);
  else
    hipLaunchKernelGGL(colsum_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)in, rows, rows_per_group,
                       row_stride, cols, out, out_gstride);
  MTTS_LAUNCH_CHECK("colsum");
  return MTTS_OK;
}

namespace mtts {

}  // namespace mtts
