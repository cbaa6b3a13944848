// rec_hostwrite.hip — can the host write per-call ROI records straight into device memory? (diagnostic
// microbenchmark, not product code)
//
// 1,600 workgroups (the C3 batch) each read one 64-byte record with one scalar load and write one dword. Per
// launch: the host rewrites every record (a new value each time), then launches; the kernel's sums are checked, so
// a stale or torn read shows up as a mismatch. Records in:
//   (a) pinned coherent host memory (the product layout: read over PCIe),
//   (b) fine-grained device memory written by the host through its mapping (hipExtMallocWithFlags),
// kernel time with HIP events and the host time of the record writes.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/rec_hostwrite tools/microbench/rec_hostwrite.hip && /tmp/rec_hostwrite
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

struct alignas(64) Rec { uint32_t w[16]; };

__global__ __launch_bounds__(256) void from_ptr(const Rec* __restrict__ recs, uint32_t* out) {
    typedef unsigned int u32x16 __attribute__((ext_vector_type(16)));
    const u32x16 r = *((const __attribute__((address_space(4))) u32x16*)recs + blockIdx.x);
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) v += r[i];
    if (threadIdx.x == 0) out[blockIdx.x] = v;
}

int main() {
    const int n = 1600, iters = 200;
    uint32_t *out, *hout;
    CK(hipMalloc(&out, n * 4));
    CK(hipHostMalloc((void**)&hout, n * 4, 0));
    Rec* hc;
    CK(hipHostMalloc((void**)&hc, n * sizeof(Rec), hipHostMallocMapped | hipHostMallocCoherent));
    Rec* hcd;
    CK(hipHostGetDevicePointer((void**)&hcd, hc, 0));
    Rec* fg = nullptr;
    hipError_t e = hipExtMallocWithFlags((void**)&fg, n * sizeof(Rec), hipDeviceMallocFinegrained);
    printf("hipExtMallocWithFlags(fine-grained): %s\n", hipGetErrorString(e));
    hipPointerAttribute_t pa{};
    if (e == hipSuccess && hipPointerGetAttributes(&pa, fg) == hipSuccess)
        printf("  type %d device %d devicePointer %p hostPointer %p\n", (int)pa.type, pa.device, pa.devicePointer, pa.hostPointer);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto fill = [&](Rec* dst, uint32_t it, bool stream) {
        for (int i = 0; i < n; i++) {
            Rec r;
            for (int k = 0; k < 16; k++) r.w[k] = it * 7 + i + k;
            if (stream) {
                const __m256i* s = reinterpret_cast<const __m256i*>(&r);
                __m256i* d = reinterpret_cast<__m256i*>(&dst[i]);
                _mm256_stream_si256(d, _mm256_loadu_si256(s));
                _mm256_stream_si256(d + 1, _mm256_loadu_si256(s + 1));
            } else {
                dst[i] = r;
            }
        }
        _mm_sfence();
    };
    auto run = [&](const char* name, Rec* host_view, Rec* dev_view, bool stream) {
        double host_us = 0;
        float total = 0;
        int bad = 0;
        for (int it = 0; it < iters + 20; it++) {
            auto t0 = std::chrono::steady_clock::now();
            fill(host_view, (uint32_t)it, stream);
            auto t1 = std::chrono::steady_clock::now();
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(from_ptr, dim3(n), dim3(256), 0, 0, dev_view, out);
            CK(hipEventRecord(e1));
            CK(hipMemcpyAsync(hout, out, n * 4, hipMemcpyDeviceToHost, 0));
            CK(hipStreamSynchronize(0));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            for (int i = 0; i < n; i++) {
                uint32_t want = 0;
                for (int k = 0; k < 16; k++) want += (uint32_t)it * 7 + i + k;
                bad += hout[i] != want;
            }
            if (it >= 20) { total += ms; host_us += std::chrono::duration<double, std::micro>(t1 - t0).count(); }
        }
        printf("%-52s kernel %7.2f us  host write %7.2f us  mismatches %d\n", name, total * 1e3 / iters, host_us / iters, bad);
    };
    run("records in pinned coherent host memory", hc, hcd, false);
    if (e == hipSuccess) {
        fflush(stdout);
        run("records in fine-grained device memory (host stores)", fg, fg, false);
        run("records in fine-grained device memory (streaming)", fg, fg, true);
    }
    return 0;
}
