// Deterministic column sums over per-block partial slabs (LN / conv1d / ...
// parameter gradients).  out[g][c] = sum_{p in group g} part[p][c].
// One 256-thread block per 64 columns and group: the 4 waves stride over
// the partials with 8 independent loads in flight per lane, then combine in
// LDS in a fixed order (bitwise reproducible).
#include "common.h"

namespace mtts {

template <typename T, int W = 4>
__global__ __launch_bounds__(64 * W) void colsum_kernel(const T* __restrict__ part, int nparts, int ppg,
                                                        int64_t pstride, int ncols, float* __restrict__ out,
                                                        int64_t out_gstride, int outer = 0) {
  __shared__ float red[W][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int g = blockIdx.y;
  int p0 = g * ppg, p1 = min(nparts, p0 + ppg);
  if (outer > 0) {   // chunks of ppg rows within groups of `outer` rows (the last chunk of a group ragged)
    const int cpg = (outer + ppg - 1) / ppg;
    const int og = g / cpg;
    p0 = og * outer + (g % cpg) * ppg;
    p1 = min(min(nparts, p0 + ppg), (og + 1) * outer);
  }
  float acc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] = 0.f;
  if (c < ncols) {
    int p = p0 + w;
    for (; p + 7 * W < p1; p += 8 * W) {
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += ldf(part + (int64_t)(p + W * q) * pstride + c);
    }
    for (; p < p1; p += W) acc[0] += ldf(part + (int64_t)p * pstride + c);
  }
  float s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  red[w][lane] = s;
  block_sync();
  if (w == 0 && c < ncols) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < W; i += 4) t += (red[i][lane] + red[i + 1][lane]) + (red[i + 2][lane] + red[i + 3][lane]);
    out[(int64_t)g * out_gstride + c] = t;
  }
}

void colsum(const float* part, int nparts, int ppg, int64_t pstride, int ncols, float* out, int64_t out_gstride,
            hipStream_t st) {
  const int ngroups = (nparts + ppg - 1) / ppg;
  if (ngroups * ((ncols + 63) / 64) < 128 && ppg >= 64) {
    // few blocks over many partials (a chunked column sum's second stage: 16
    // blocks x 128 partials took ~11 us on 4 waves): 16 waves, one batch of
    // 8 loads each
    hipLaunchKernelGGL((colsum_kernel<float, 16>), dim3((ncols + 63) / 64, ngroups), dim3(1024), 0, st, part, nparts,
                       ppg, pstride, ncols, out, out_gstride);
    return;
  }
  hipLaunchKernelGGL((colsum_kernel<float, 4>), dim3((ncols + 63) / 64, ngroups), dim3(256), 0, st, part, nparts, ppg,
                     pstride, ncols, out, out_gstride);
}

// Up to 5 column-sum jobs over slabs of the same width in ONE launch
// (blockIdx.z = job): the LayerNorm backward's dw / db / dgamma / dbeta / dx sums.
struct ColsumJobs {
  ColsumJob j[5];
  int ncols;
  int64_t pstride;
};
template <int W>
__global__ __launch_bounds__(64 * W) void colsum_multi_kernel(const ColsumJobs J) {
  const ColsumJob& jb = J.j[blockIdx.z];
  const int g = blockIdx.y;
  const int p0 = g * jb.ppg;
  if (p0 >= jb.nparts) return;   // block-uniform: before any barrier
  __shared__ float red[W][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int p1 = min(jb.nparts, p0 + jb.ppg);
  float acc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] = 0.f;
  if (c < J.ncols) {
    int p = p0 + w;
    for (; p + 7 * W < p1; p += 8 * W) {
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += jb.part[(int64_t)(p + W * q) * J.pstride + c];
    }
    for (; p < p1; p += W) acc[0] += jb.part[(int64_t)p * J.pstride + c];
  }
  const float s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  red[w][lane] = s;
  block_sync();
  if (w == 0 && c < J.ncols) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < W; i += 4) t += (red[i][lane] + red[i + 1][lane]) + (red[i + 2][lane] + red[i + 3][lane]);
    jb.out[(int64_t)g * jb.out_gstride + c] = t;
  }
}

void colsum_multi(const ColsumJob* jobs, int n, int ncols, int64_t pstride, hipStream_t st) {
  ColsumJobs J{};
  int gmax = 1, pmax = 0;
  for (int i = 0; i < n; ++i) {
    J.j[i] = jobs[i];
    gmax = std::max(gmax, (jobs[i].nparts + jobs[i].ppg - 1) / jobs[i].ppg);
    pmax = std::max(pmax, std::min(jobs[i].ppg, jobs[i].nparts));
  }
  J.ncols = ncols;
  J.pstride = pstride;
  const dim3 grid((ncols + 63) / 64, gmax, n);
  if ((int)(grid.x * grid.y * grid.z) < 128 && pmax >= 64)   // few blocks over many partials: 16 waves
    hipLaunchKernelGGL(colsum_multi_kernel<16>, grid, dim3(1024), 0, st, J);
  else
    hipLaunchKernelGGL(colsum_multi_kernel<4>, grid, dim3(256), 0, st, J);
}

// Stage 1 of a long column sum (bias gradients: rows = tokens): a block owns
// 512 bf16 (256 fp32) columns as 16-byte row pieces, one per lane (a wave
// reads 1 KiB of a row per instruction), 4 waves striding a 128-row chunk
// with 4 rows in flight per lane; fixed-order combine of the waves in LDS.
template <typename T>
__global__ __launch_bounds__(256) void colsum_rows_kernel(const T* __restrict__ in, int rows, int cols,
                                                          int64_t ld, int rchunk, float* __restrict__ part) {
  constexpr int EPL = 16 / (int)sizeof(T);   // columns per lane
  constexpr int CB = 64 * EPL;               // columns per block
  __shared__ float red[4][CB];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * CB + lane * EPL;
  const int r0 = blockIdx.y * rchunk, r1 = min(rows, r0 + rchunk);
  float acc[EPL];
#pragma unroll
  for (int e = 0; e < EPL; ++e) acc[e] = 0.f;
  auto add = [&](const uint4 v) {
    if constexpr (sizeof(T) == 2) {
      const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[2 * q] += __uint_as_float(x[q] << 16);
        acc[2 * q + 1] += __uint_as_float(x[q] & 0xffff0000u);
      }
    } else {
      acc[0] += __uint_as_float(v.x); acc[1] += __uint_as_float(v.y);
      acc[2] += __uint_as_float(v.z); acc[3] += __uint_as_float(v.w);
    }
  };
  if (c < cols) {
    int r = r0 + w;
    // 16 rows in flight per lane (a 64-row chunk is one batch of loads)
    for (; r + 60 < r1; r += 64) {
      uint4 v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = *reinterpret_cast<const uint4*>(in + (int64_t)(r + 4 * q) * ld + c);
#pragma unroll
      for (int q = 0; q < 16; ++q) add(v[q]);
    }
    for (; r + 12 < r1; r += 16) {
      uint4 v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = *reinterpret_cast<const uint4*>(in + (int64_t)(r + 4 * q) * ld + c);
#pragma unroll
      for (int q = 0; q < 4; ++q) add(v[q]);
    }
    for (; r < r1; r += 4) add(*reinterpret_cast<const uint4*>(in + (int64_t)r * ld + c));
  }
#pragma unroll
  for (int e = 0; e < EPL; ++e) red[w][lane * EPL + e] = acc[e];
  block_sync();
  for (int q = threadIdx.x; q < CB; q += 256) {
    const int cc = blockIdx.x * CB + q;
    if (cc < cols) part[(int64_t)blockIdx.y * cols + cc] = (red[0][q] + red[1][q]) + (red[2][q] + red[3][q]);
  }
}

}  // namespace mtts

extern "C" int64_t mtts_colsum_workspace(int rows, int cols, int rows_per_group) {
  if (rows_per_group <= 1024 && !(rows_per_group >= rows && rows >= 256)) return 0;
  const int64_t chunks = (int64_t)(rows + 15) / 16;     // the single-group path's chunks (>= 16 rows each)
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
  const int es = dtype == MTTS_F32 ? 4 : 2;
  if (rows_per_group >= rows && rows >= 256 && cols % (16 / es) == 0 && row_stride % (16 / es) == 0 &&
      (uintptr_t)in % 16 == 0) {
    // one group over many rows (bias gradients): 16-byte row pieces, 128-row
    // chunks -> fp32 partial slab -> sum of the chunks
    MTTS_CHECK(workspace, "colsum: workspace required (mtts_colsum_workspace)");
    // 128-row chunks (tools/bench_colsum.py: 64 / 32 measured equal at 1024 columns, slower at 2048+);
    // up to 1024 rows (the text encoder's 1024 x 1024 fp32 bias gradients: 16
    // blocks took 13 us) the chunks shrink to 16 rows until ~256 blocks run
    int rchunk = 128;
    if (rows <= 1024) {
      const int cblocks = (cols + 64 * (16 / es) - 1) / (64 * (16 / es));
      const int want = (256 + cblocks - 1) / cblocks;
      rchunk = std::min(128, std::max(16, ((rows + want - 1) / want + 15) / 16 * 16));
    }
    const int chunks = (rows + rchunk - 1) / rchunk;
    float* part = (float*)workspace;
    if (dtype == MTTS_F32)
      hipLaunchKernelGGL(colsum_rows_kernel<float>, dim3((cols + 255) / 256, chunks), dim3(256), 0, st,
                         (const float*)in, rows, cols, row_stride, rchunk, part);
    else
      hipLaunchKernelGGL(colsum_rows_kernel<bf16_t>, dim3((cols + 511) / 512, chunks), dim3(256), 0, st,
                         (const bf16_t*)in, rows, cols, row_stride, rchunk, part);
    MTTS_LAUNCH_CHECK("colsum rows");
    colsum(part, chunks, chunks, cols, cols, out, out_gstride, st);
    MTTS_LAUNCH_CHECK("colsum chunks");
    return MTTS_OK;
  }
  if (rows_per_group > 1024) {
    // two stages: 256-row chunks -> fp32 partial slab -> per-group sum of chunks
    // (a group of rows_per_group % 256 != 0 rows ends in a ragged chunk)
    MTTS_CHECK(workspace, "colsum: workspace required (mtts_colsum_workspace)");
    const int rpg = std::min(rows_per_group, rows);
    const bool ragged = rpg % 256 != 0 && rpg < rows;
    const int cpg = (rpg + 255) / 256;
    const int chunks = ragged ? ((rows + rpg - 1) / rpg) * cpg : (rows + 255) / 256;
    float* part = (float*)workspace;
    dim3 g1((cols + 63) / 64, chunks);
    if (dtype == MTTS_F32)
      hipLaunchKernelGGL((colsum_kernel<float, 4>), g1, dim3(256), 0, st, (const float*)in, rows, 256, row_stride, cols,
                         part, (int64_t)cols, ragged ? rpg : 0);
    else
      hipLaunchKernelGGL((colsum_kernel<bf16_t, 4>), g1, dim3(256), 0, st, (const bf16_t*)in, rows, 256, row_stride,
                         cols, part, (int64_t)cols, ragged ? rpg : 0);
    MTTS_LAUNCH_CHECK("colsum stage 1");
    colsum(part, chunks, rows_per_group >= rows ? chunks : cpg, cols, cols, out, out_gstride, st);
    MTTS_LAUNCH_CHECK("colsum stage 2");
    return MTTS_OK;
  }
  const int ngroups = (rows + rows_per_group - 1) / rows_per_group;
  dim3 grid((cols + 63) / 64, ngroups);
  if (dtype == MTTS_F32)
    hipLaunchKernelGGL((colsum_kernel<float, 4>), grid, dim3(256), 0, st, (const float*)in, rows, rows_per_group,
                       row_stride, cols, out, out_gstride);
  else
    hipLaunchKernelGGL((colsum_kernel<bf16_t, 4>), grid, dim3(256), 0, st, (const bf16_t*)in, rows, rows_per_group,
                       row_stride, cols, out, out_gstride);
  MTTS_LAUNCH_CHECK("colsum");
  return MTTS_OK;
}

namespace mtts {

}  // namespace mtts
