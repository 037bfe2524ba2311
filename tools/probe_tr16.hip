// Probe of ds_read_b64_tr_b16 lane semantics (tools only): LDS holds a [16 rows][64 cols] int16 tile with
// value row*64 + col; lane l of the wave supplies the address of row (l & 15) >> 2, columns 4 * (l & 3)
// (+ 16 * (l >> 4) rows offset per group), and prints the 4 values it receives.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((ext_vector_type(4))) short i16x4;

__global__ void probe(int* out) {
  __shared__ short t[16 * 64];
  for (int i = threadIdx.x; i < 16 * 64; i += 64) t[i] = (short)i;
  __syncthreads();
  const int l = threadIdx.x, g = l >> 4, gi = l & 15;
  const int row = 4 * g + (gi >> 2), col = 4 * (gi & 3);
  const i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(t + row * 64 + col));
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = v[e];
}

int main() {
  int* d;
  if (hipMalloc(&d, 256 * 4) != hipSuccess) { std::printf("malloc failed\n"); return 1; }
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  int h[256];
  hipError_t e = hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost); std::printf("status %s\n", hipGetErrorString(e)); fflush(stdout);
  for (int l = 0; l < 64; ++l) {
    std::printf("lane %2d:", l);
    for (int e = 0; e < 4; ++e) std::printf("  (r%2d,c%2d)", h[l * 4 + e] / 64, h[l * 4 + e] % 64);
    std::printf("\n");
  }
  return 0;
}
