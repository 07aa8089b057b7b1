// Compile probe: global_load_lds_dwordx4 (LDS-DMA) from HIP on gfx950.
// hipcc -O3 --offload-arch=gfx950 -S --cuda-device-only dma_probe.hip -o dma_probe.s
#include <hip/hip_runtime.h>
__global__ void k(const uint4* __restrict__ g, float* out) {
  __shared__ __attribute__((aligned(16))) uint4 s[64 * 4];
  const int w = threadIdx.x / 64;
  __builtin_amdgcn_global_load_lds((const void*)(g + blockIdx.x * 256 + threadIdx.x),
                                   (__attribute__((address_space(3))) void*)&s[w * 64], 16, 0, 0);
  __builtin_amdgcn_s_waitcnt(0x3F70);  // vmcnt(0)
  __syncthreads();
  out[threadIdx.x] = __uint_as_float(s[(threadIdx.x * 7) & 255].x);
}
