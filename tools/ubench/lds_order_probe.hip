// Probe: is a plain ds_write_b128 by one wave visible to another wave's
// ds_read after a bare s_barrier (no s_waitcnt lgkmcnt(0) in between)?
// hipcc's __syncthreads() on gfx950 emits a bare s_barrier (LLVM assumes LDS
// operations of all waves are observed in one global order).  Each
// workgroup runs ITER rounds: every wave writes a tile of round-dependent
// values to its own LDS region with ds_write_b128, s_barrier, then reads its
// NEIGHBOUR wave's region with ds_read_u16 / b32 and counts stale values.
//   hipcc -O3 --offload-arch=gfx950 lds_order_probe.hip -o lds_order_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s\n", hipGetErrorString(e)); return 1; } } while (0)

template <bool WAIT>
__global__ __launch_bounds__(256) void probe(int iters, unsigned* bad) {
  __shared__ __attribute__((aligned(16))) unsigned sm[2][4][64 * 4 * 4];   // [buf][wave][16 dwords per lane]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  unsigned nbad = 0;
  for (int it = 0; it < iters; ++it) {
    const int buf = it & 1;
    const unsigned tag = (unsigned)(it * 131071 + blockIdx.x * 7 + wave);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint4 v = make_uint4(tag + q, tag ^ 0x55555555u, tag + 3 * q, ~tag);
      *reinterpret_cast<uint4*>(&sm[buf][wave][(q * 64 + lane) * 4]) = v;   // ds_write_b128
    }
    if (WAIT) __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int nb = (wave + 1) & 3;
    const unsigned ntag = (unsigned)(it * 131071 + blockIdx.x * 7 + nb);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const unsigned short lo = *reinterpret_cast<const unsigned short*>(&sm[buf][nb][(q * 64 + lane) * 4]);   // ds_read_u16
      const unsigned w = sm[buf][nb][(q * 64 + lane) * 4 + 3];
      nbad += (lo != (unsigned short)(ntag + q)) + (w != ~ntag);
    }
    // a little VALU work so waves drift apart
    float x = (float)lane;
#pragma unroll
    for (int k = 0; k < 16 * (wave + 1); ++k) x = __builtin_fmaf(x, 1.0001f, 0.5f);
    if (x == 12345.f) nbad += 1000000;
  }
  if (nbad) atomicAdd(bad, nbad);
}

int main() {
  unsigned* d;
  CK(hipMalloc(&d, 8));
  for (int wait = 0; wait < 2; ++wait) {
    unsigned total = 0;
    for (int rep = 0; rep < 20; ++rep) {
      CK(hipMemset(d, 0, 4));
      if (wait) hipLaunchKernelGGL(probe<true>, dim3(2048), dim3(256), 0, 0, 2000, d);
      else hipLaunchKernelGGL(probe<false>, dim3(2048), dim3(256), 0, 0, 2000, d);
      CK(hipDeviceSynchronize());
      unsigned h;
      CK(hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost));
      total += h;
    }
    printf("%s s_barrier: %u stale neighbour-wave LDS reads in 20 x 2048 workgroups x 2000 rounds x 4 waves\n",
           wait ? "lgkmcnt(0) +" : "bare", total);
  }
  return 0;
}
