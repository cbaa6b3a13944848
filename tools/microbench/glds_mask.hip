// Probe: LDS destination of global_load_lds_dwordx4 when some lanes are masked off.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k(const uint32_t* g, uint32_t* out, int mode) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[64 * 4 + 64];
  for (int i = threadIdx.x; i < 64 * 4 + 64; i += 64) lds[i] = 0xFFFFFFFF;
  __syncthreads();
  int lane = threadIdx.x;
  bool active = mode == 0 ? true : (mode == 1 ? (lane & 1) == 0 : (lane >= 8 && lane < 12) || lane == 40);
  if (active)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + lane * 4),
                                     (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 4; i += 64) out[i] = lds[i];
}
int main() {
  uint32_t h[256], *d, *o, r[256];
  for (int i = 0; i < 256; i++) h[i] = i / 4;  // lane id in each dword of its 16-byte chunk
  hipMalloc(&d, 1024); hipMalloc(&o, 1024);
  hipMemcpy(d, h, 1024, hipMemcpyHostToDevice);
  for (int mode = 0; mode < 3; mode++) {
    hipLaunchKernelGGL(k, 1, 64, 0, 0, d, o, mode);
    hipMemcpy(r, o, 1024, hipMemcpyDeviceToHost);
    printf("mode %d: chunk->lane:", mode);
    for (int c = 0; c < 64; c++) printf(" %d", (int)(r[c * 4] == 0xFFFFFFFF ? -1 : (int)r[c * 4]));
    printf("\n");
  }
  return 0;
}
