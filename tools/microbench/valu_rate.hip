// Probe: VALU issue rate per SIMD on gfx950 for the integer ops the pre-process kernel uses,
// against v_fma_f32 and v_pk_fma_f32. 8 independent chains per lane, 8 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define N_ITER 4096
template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  float f[8];
  for (int i = 0; i < 8; i++) { a[i] = seed + threadIdx.x * 7 + i; f[i] = (float)a[i]; }
  for (int it = 0; it < N_ITER; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if constexpr (OP == 0) a[i] = __umul24(a[i], 0x1234u) + 77u;                 // v_mad_u32_u24
      else if constexpr (OP == 1) { asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(a[(i+1)&7]), "v"(a[(i+2)&7])); }
      else if constexpr (OP == 2) { asm volatile("v_med3_i32 %0, %0, 0, %1" : "+v"(a[i]) : "v"(a[(i+3)&7])); }
      else if constexpr (OP == 3) f[i] = __builtin_fmaf(f[i], 1.0001f, 0.5f);          // v_fma_f32
      else if constexpr (OP == 4) { asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i+5)&7])); }
      else if constexpr (OP == 5) { asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(a[i])); }
      else { asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(*(double*)&f[i & 6]) : "v"(*(double*)&f[(i+2)&6]), "v"(*(double*)&f[(i+4)&6])); }
    }
  }
  uint32_t s = 0;
  for (int i = 0; i < 8; i++) s += a[i] + (uint32_t)f[i];
  if (s == 0x12345678) out[threadIdx.x] = s;
}
template <int OP>
void run(const char* name, uint32_t* d) {
  int ncu = 0; hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  int grid = ncu * 8;  // 8 WGs x 4 waves = 32 waves per CU = 8 per SIMD
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(256), 0, 0, d, 1u);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(256), 0, 0, d, 1u);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double instr_per_simd = (double)N_ITER * 8 * 8;  // per wave 8 instrs/iter, 8 waves per SIMD
  double cyc = ms * 1e-3 * 2.4e9;
  printf("%-16s %.3f ms  -> %.2f cycles per wave-instruction per SIMD (at 2.4 GHz)\n", name, ms, cyc / instr_per_simd);
}
int main() {
  uint32_t* d; hipMalloc(&d, 4096);
  run<0>("v_mad_u32_u24", d); run<1>("v_add3_u32", d); run<2>("v_med3_i32", d); run<3>("v_fma_f32", d);
  run<4>("v_mul_hi_u32_u24", d); run<5>("v_lshrrev_b32", d); run<6>("v_pk_fma_f32", d);
  return 0;
}
