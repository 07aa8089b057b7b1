// Per-step compute-dtype weight copies for the GEMMs (mtts/linear.py
// cast_scope): every fp32 master W (rows x cols) becomes a bf16 W and,
// for 2-D weights, a bf16 W^T (cols x rows), in ONE launch over the whole
// parameter list.  The transposed copy lets every data-gradient GEMM run as
// dy @ (W^T)^T, the operand layout hipBLASLt is fastest at on these shapes
// (tools/bench_gemm.py: "dgrad_nt" 1.1-1.4 PF/s vs "dgrad_nn" 0.9-1.2).
// A block owns a 64x64 tile of one tensor: coalesced fp32 row reads, bf16
// row writes, and the transposed write through a padded LDS tile.
#include "common.h"

namespace mtts {

constexpr int kCT = 64;

__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

__global__ __launch_bounds__(256) void cast_multi_kernel(const MttsCastDesc* __restrict__ descs, int n) {
  __shared__ float tile[kCT][kCT + 1];
  const int64_t blk = blockIdx.x;
  int lo = 0, hi = n - 1;  // last descriptor with tile0 <= blk
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (descs[mid].tile0 <= blk) lo = mid;
    else hi = mid - 1;
  }
  const MttsCastDesc d = descs[lo];
  const int tcols = (d.cols + kCT - 1) / kCT;
  const int64_t t = blk - d.tile0;
  const int r0 = (int)(t / tcols) * kCT, c0 = (int)(t % tcols) * kCT;
  const int tid = threadIdx.x;
  const bool full = r0 + kCT <= d.rows && c0 + kCT <= d.cols && (d.cols % 4) == 0 && (d.rows % 4) == 0;
  bf16_t* __restrict__ dst = (bf16_t*)d.dst;
  bf16_t* __restrict__ dstT = (bf16_t*)d.dstT;
  if (full) {
    const int cq = (tid % 16) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = i * 16 + tid / 16;
      const float4 v = *reinterpret_cast<const float4*>(d.src + (int64_t)(r0 + r) * d.cols + c0 + cq);
      *reinterpret_cast<uint2*>(dst + (int64_t)(r0 + r) * d.cols + c0 + cq) =
          make_uint2(pack_bf2(v.x, v.y), pack_bf2(v.z, v.w));
      tile[r][cq] = v.x; tile[r][cq + 1] = v.y; tile[r][cq + 2] = v.z; tile[r][cq + 3] = v.w;
    }
    if (!dstT) return;
    block_sync();
    const int rq = (tid % 16) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = i * 16 + tid / 16;
      *reinterpret_cast<uint2*>(dstT + (int64_t)(c0 + c) * d.rows + r0 + rq) =
          make_uint2(pack_bf2(tile[rq][c], tile[rq + 1][c]), pack_bf2(tile[rq + 2][c], tile[rq + 3][c]));
    }
  } else {
    for (int i = 0; i < 16; ++i) {
      const int r = i * 4 + tid / 64, c = tid % 64;
      if (r0 + r < d.rows && c0 + c < d.cols) {
        const float v = d.src[(int64_t)(r0 + r) * d.cols + c0 + c];
        dst[(int64_t)(r0 + r) * d.cols + c0 + c] = f2bf(v);
        tile[r][c] = v;
      }
    }
    if (!dstT) return;
    block_sync();
    for (int i = 0; i < 16; ++i) {
      const int c = i * 4 + tid / 64, r = tid % 64;
      if (r0 + r < d.rows && c0 + c < d.cols) dstT[(int64_t)(c0 + c) * d.rows + r0 + r] = f2bf(tile[r][c]);
    }
  }
}

}  // namespace mtts

using namespace mtts;

extern "C" int64_t mtts_cast_tiles(int rows, int cols) {
  if (rows <= 0 || cols <= 0) return 0;
  return (int64_t)((rows + kCT - 1) / kCT) * ((cols + kCT - 1) / kCT);
}

extern "C" int mtts_cast_bf16_multi(const MttsCastDesc* descs, int n, int64_t total_tiles, void* stream) {
  MTTS_CHECK(descs && n > 0 && total_tiles > 0, "cast_bf16_multi: bad args");
  MTTS_CHECK(total_tiles < (1ll << 31), "cast_bf16_multi: too many tiles");
  hipLaunchKernelGGL(cast_multi_kernel, dim3((unsigned)total_tiles), dim3(256), 0, (hipStream_t)stream, descs, n);
  MTTS_LAUNCH_CHECK("cast_bf16_multi");
  return MTTS_OK;
}
