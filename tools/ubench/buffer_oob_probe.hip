// Probe: what does the gfx950 buffer range check cover?  (round-5 verdict item 1)
//
// The buffer-addressed kernels (scan fwd c1/w2, conv bwd tile, attention K/V
// rows) put a tile's row origin in the SCALAR offset (soffset) of a raw
// buffer access (stride 0) and rely on rows outside [0, num_records) reading
// 0 / stores being dropped.  This program answers, for loads (b32, b128),
// LDS-DMA loads (buffer_load_dwordx4 ... offen lds) and stores (b32, b128):
//   * is soffset part of the range check at all?
//   * is voffset + soffset summed in 32 bits (wrapping) or wider?
//   * what address does an unchecked access actually touch?
//
// Safety: the descriptor base sits 1 MiB into an 8 GiB + 2 MiB allocation, so
// every address base + voff + soff (unsigned 32-bit offsets, summed in 64 or
// 32 bits, sign-extended or not) stays inside memory this process owns.  The
// allocation is a ramp (dword i holds i + 1), so a loaded value names the
// exact dword it came from; stores write markers that a search kernel finds.
//
//   hipcc -O3 --offload-arch=gfx950 buffer_oob_probe.hip -o buffer_oob_probe && ./buffer_oob_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr uint64_t kPad = 1ull << 20;                   // bytes before the descriptor base
constexpr uint64_t kBytes = (8ull << 30) + 2 * kPad;    // whole allocation
constexpr uint32_t kRecords = 4096;                     // descriptor num_records (bytes)

struct Case { uint32_t voff, soff; const char* what; };
static const Case kCases[] = {
    {0, 0, "voff 0, soff 0 (in range)"},
    {kRecords - 4, 0, "voff R-4 (last dword, in range)"},
    {kRecords, 0, "voff R (first byte past range)"},
    {0, kRecords - 4, "soff R-4 only (sum in range)"},
    {0, kRecords, "soff R only (sum = R, past range)"},
    {kRecords - 4, 4, "voff R-4 + soff 4 (sum = R)"},
    {0, 2 * kRecords, "soff 2R (far past range)"},
    {0, 0xFFFFFFF0u, "soff -16 (negative row origin, as a wrapped int)"},
    {32, 0xFFFFFFF0u, "voff 32 + soff -16 (32-bit sum 16, in range)"},
    {0xFFFFFFF0u, 0, "voff 0xFFFFFFF0 (invalid-lane sentinel)"},
    {0xFFFFFFF0u, 32, "voff 0xFFFFFFF0 + soff 32 (32-bit sum 16, in range)"},
    {0, 0xFFFFF000u, "soff -4096 (row -1 of a 4 KiB row)"},
};
constexpr int kNC = sizeof(kCases) / sizeof(kCases[0]);

__global__ void fill_ramp(uint32_t* p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = (uint32_t)(i + 1);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(void* base) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  return __builtin_amdgcn_make_buffer_rsrc(
      (void*)(uintptr_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(a >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a)),
      0, (int)kRecords, 0x00020000);
}

// lane i < n runs case i with the builtin b32 / b128 loads (soff must be an
// SGPR: every lane of a launch uses one case, the case index is a kernel arg)
__global__ void probe_load(void* base, uint32_t voff, uint32_t soff, uint32_t* out) {
  const __amdgpu_buffer_rsrc_t r = rsrc(base);
  const uint32_t so = __builtin_amdgcn_readfirstlane(soff);
  const uint32_t vo = voff;   // same for every lane
  const uint32_t v1 = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, vo, (int)so, 0);
  const i32x4 v4 = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(r, vo, (int)so, 0));
  if (threadIdx.x == 0) {
    out[0] = v1;
    out[1] = (uint32_t)v4[0]; out[2] = (uint32_t)v4[1]; out[3] = (uint32_t)v4[2]; out[4] = (uint32_t)v4[3];
  }
}

// the product's LDS-DMA form (scan.hip dma16b): buffer_load_dwordx4 ... offen lds
__global__ void probe_dma(void* base, uint32_t voff, uint32_t soff, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint32_t s[64 * 4];
  for (int i = threadIdx.x; i < 64 * 4; i += 64) s[i] = 0xCAFEBABEu;
  __syncthreads();
  const uint64_t a = (uint64_t)(uintptr_t)base;
  const i32x4 rs = i32x4{__builtin_amdgcn_readfirstlane((int)(uint32_t)a), __builtin_amdgcn_readfirstlane((int)((a >> 32) & 0xffff)),
                         __builtin_amdgcn_readfirstlane((int)kRecords), 0x00020000};
  const uint32_t lds = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)&s[0]);
  const int so = (int)__builtin_amdgcn_readfirstlane(soff);
  const uint32_t vo = voff;
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, %3 offen lds" ::"v"(vo), "s"(lds), "s"(rs), "s"(so)
               : "memory", "m0");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) { out[0] = s[0]; out[1] = s[1]; out[2] = s[2]; out[3] = s[3]; }
}

__global__ void probe_store(void* base, uint32_t voff, uint32_t soff, uint32_t marker, int wide) {
  const __amdgpu_buffer_rsrc_t r = rsrc(base);
  const uint32_t so = __builtin_amdgcn_readfirstlane(soff);
  if (threadIdx.x == 0) {
    if (wide) __builtin_amdgcn_raw_buffer_store_b128(i32x4{(int)marker, (int)marker, (int)marker, (int)marker}, r, voff, (int)so, 0);
    else __builtin_amdgcn_raw_buffer_store_b32((int)marker, r, voff, (int)so, 0);
  }
}

// find every dword equal to marker; restore it to its ramp value
__global__ void find_marker(uint32_t* p, uint64_t n, uint32_t marker, unsigned long long* hits, int* nh) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (p[i] == marker) {
      const int k = atomicAdd(nh, 1);
      if (k < 16) hits[k] = i;
      p[i] = (uint32_t)(i + 1);
    }
}

static void describe(uint32_t v, uint64_t base_dw) {
  if (v == 0) { printf("0"); return; }
  if (v == 0xCAFEBABEu) { printf("untouched"); return; }
  const int64_t rel = ((int64_t)v - 1 - (int64_t)base_dw) * 4;
  printf("mem[base%+lld]", (long long)rel);
}

int main() {
  uint32_t* buf;
  CK(hipMalloc(&buf, kBytes));
  const uint64_t ndw = kBytes / 4;
  hipLaunchKernelGGL(fill_ramp, dim3(4096), dim3(256), 0, 0, buf, ndw);
  CK(hipDeviceSynchronize());
  char* base = (char*)buf + kPad;
  const uint64_t base_dw = kPad / 4;
  uint32_t *dout, hout[8];
  unsigned long long* dhits;
  int* dnh;
  CK(hipMalloc(&dout, 64));
  CK(hipMalloc(&dhits, 16 * 8));
  CK(hipMalloc(&dnh, 4));
  printf("# gfx950 raw buffer range check probe: num_records = %u bytes, stride 0, flags 0x00020000\n", kRecords);
  printf("# a value mem[base+X] = the access read the dword at byte X from the descriptor base (no range check)\n");
  for (int c = 0; c < kNC; ++c) {
    const Case& k = kCases[c];
    printf("case %2d  voff=0x%08x soff=0x%08x  %s\n", c, k.voff, k.soff, k.what);
    hipLaunchKernelGGL(probe_load, dim3(1), dim3(64), 0, 0, base, k.voff, k.soff, dout);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hout, dout, 20, hipMemcpyDeviceToHost));
    printf("   load_b32: "); describe(hout[0], base_dw);
    printf("\n   load_b128:");
    for (int q = 0; q < 4; ++q) { printf(" "); describe(hout[1 + q], base_dw); }
    hipLaunchKernelGGL(probe_dma, dim3(1), dim3(64), 0, 0, base, k.voff, k.soff, dout);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hout, dout, 16, hipMemcpyDeviceToHost));
    printf("\n   lds_dma_x4:");
    for (int q = 0; q < 4; ++q) { printf(" "); describe(hout[q], base_dw); }
    for (int wide = 0; wide < 2; ++wide) {
      const uint32_t marker = 0xDEAD0000u | (uint32_t)(c * 2 + wide);
      CK(hipMemset(dnh, 0, 4));
      hipLaunchKernelGGL(probe_store, dim3(1), dim3(64), 0, 0, base, k.voff, k.soff, marker, wide);
      hipLaunchKernelGGL(find_marker, dim3(8192), dim3(256), 0, 0, buf, ndw, marker, dhits, dnh);
      CK(hipDeviceSynchronize());
      int nh;
      unsigned long long hits[16];
      CK(hipMemcpy(&nh, dnh, 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hits, dhits, sizeof(hits), hipMemcpyDeviceToHost));
      printf("\n   store_%s: %s", wide ? "b128" : "b32", nh ? "wrote" : "dropped");
      for (int i = 0; i < nh && i < 16; ++i) printf(" base%+lld", (long long)(((int64_t)hits[i] - (int64_t)base_dw) * 4));
    }
    printf("\n");
  }
  CK(hipFree(buf));
  printf("# done\n");
  return 0;
}
