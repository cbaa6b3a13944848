// rec_latency.hip — where should per-call ROI records live? (diagnostic microbenchmark, not product code)
//
// 1,600 workgroups (the C3 batch) each read one 16-byte record and write one dword; kernel time with
// HIP events, averaged over 200 launches, for records in:
//   (a) pinned coherent host memory (read over PCIe, the round-2 layout),
//   (b) pinned non-coherent host memory,
//   (c) device memory,
//   (d) the kernel arguments (3,200 B: 200 records, indexed blockIdx % 200),
//   (e) a large kernel-argument block (25,600 B: all 1,600 records), if the runtime accepts it.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/rec_latency tools/microbench/rec_latency.hip && /tmp/rec_latency
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

struct Rec { uint32_t a, b, c, d; };
template <int N> struct RecArgs { Rec r[N]; };

__global__ __launch_bounds__(256) void from_ptr(const Rec* __restrict__ recs, uint32_t* out) {
    const __attribute__((address_space(4))) Rec* r = (const __attribute__((address_space(4))) Rec*)recs + blockIdx.x;
    const uint32_t v = r->a + r->b + r->c + r->d;
    if (threadIdx.x == 0) out[blockIdx.x] = v;
}
template <int N>
__global__ __launch_bounds__(256) void from_args(const RecArgs<N> P, uint32_t* out) {
    const Rec& r = P.r[blockIdx.x % N];
    const uint32_t v = r.a + r.b + r.c + r.d;
    if (threadIdx.x == 0) out[blockIdx.x] = v;
}
__global__ __launch_bounds__(256) void empty_k(uint32_t* out) {
    if (threadIdx.x == 0) out[blockIdx.x] = blockIdx.x;
}

int main() {
    const int n = 1600, iters = 200;
    uint32_t* out;
    CK(hipMalloc(&out, n * 4));
    Rec *hc, *hn, *dv;
    CK(hipHostMalloc((void**)&hc, n * sizeof(Rec), hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostMalloc((void**)&hn, n * sizeof(Rec), hipHostMallocMapped | hipHostMallocNonCoherent));
    CK(hipMalloc(&dv, n * sizeof(Rec)));
    for (int i = 0; i < n; i++) hc[i] = hn[i] = Rec{(uint32_t)i, 1, 2, 3};
    CK(hipMemcpy(dv, hc, n * sizeof(Rec), hipMemcpyHostToDevice));
    Rec *hcd, *hnd;
    CK(hipHostGetDevicePointer((void**)&hcd, hc, 0));
    CK(hipHostGetDevicePointer((void**)&hnd, hn, 0));
    static RecArgs<200> a200;
    static RecArgs<1600> a1600;
    for (int i = 0; i < 200; i++) a200.r[i] = Rec{(uint32_t)i, 1, 2, 3};
    for (int i = 0; i < 1600; i++) a1600.r[i] = Rec{(uint32_t)i, 1, 2, 3};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) {
        for (int i = 0; i < 20; i++) launch();
        if (hipDeviceSynchronize() != hipSuccess || hipGetLastError() != hipSuccess) { printf("%-40s failed\n", name); return; }
        float total = 0;
        for (int i = 0; i < iters; i++) {  // one launch per event pair: kernel time, not back-to-back overlap
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            total += ms;
        }
        printf("%-40s %8.2f us\n", name, total * 1e3 / iters);
    };
    run("empty kernel (1600 WGs)", [&] { hipLaunchKernelGGL(empty_k, dim3(n), dim3(256), 0, 0, out); });
    run("records in pinned coherent host memory", [&] { hipLaunchKernelGGL(from_ptr, dim3(n), dim3(256), 0, 0, hcd, out); });
    run("records in pinned non-coherent host mem", [&] { hipLaunchKernelGGL(from_ptr, dim3(n), dim3(256), 0, 0, hnd, out); });
    run("records in device memory", [&] { hipLaunchKernelGGL(from_ptr, dim3(n), dim3(256), 0, 0, dv, out); });
    run("records in kernel args (3.2 KB)", [&] { hipLaunchKernelGGL((from_args<200>), dim3(n), dim3(256), 0, 0, a200, out); });
    run("records in kernel args (25.6 KB)", [&] { hipLaunchKernelGGL((from_args<1600>), dim3(n), dim3(256), 0, 0, a1600, out); });
    // host cost of a launch with a 25.6 KB argument block vs 3.2 KB (back-to-back, host clock)
    return 0;
}
