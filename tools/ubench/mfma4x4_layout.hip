// Probe: operand/result lane layout of v_mfma_f32_4x4x1f32 (16 blocks) on gfx950.
// Prints, for lanes 0..7, D[r] given A = lane+1, B = 100*(lane+1).
//   hipcc --offload-arch=gfx950 -O3 mfma4x4_layout.hip -o mfma4x4_layout
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void probe(float* out) {
  const int l = threadIdx.x;
  const float a = (float)(l + 1), b = 100.f * (float)(l + 1);
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = acc[r];
}

int main() {
  float* d;
  hipMalloc(&d, 64 * 4 * sizeof(float));
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  float h[256];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 12; ++l)
    printf("lane %2d: D = %8.0f %8.0f %8.0f %8.0f\n", l, h[l * 4], h[l * 4 + 1], h[l * 4 + 2], h[l * 4 + 3]);
  printf("lane 63: D = %8.0f %8.0f %8.0f %8.0f\n", h[252], h[253], h[254], h[255]);
  return 0;
}
