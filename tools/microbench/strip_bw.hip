// strip_bw.hip — the C2 data movement (32 x 1080p NV12 frames -> 32 x 3 x 512 x 512 fp32) in the access
// patterns of the strip kernel and of its alternatives, with no pixel arithmetic (diagnostic microbenchmark,
// not product code). Every variant moves the bytes one C2 launch moves: for each output row, its two luma
// source rows and its chroma row(s) (the OpenCV 1080 -> 512 row table), each read as the column window of
// the variant's strip, into LDS by LDS-DMA; and three fp32 output planes written with non-temporal dword
// stores (one pixel per lane). The loop per wave is the strip kernel's: a ring of D rows in flight, a
// counted vmcnt wait per row, stores, then the DMA of row i + D into the freed entry. Frame / output sets
// cycle over a pool >= 3x the Infinity Cache.
//
// Variants (template): SP = output columns per wave strip (64 / 128 / 256 / 512; a lane owns SP / 64 pixels),
// D = ring depth, W = waves per workgroup, TH = rows per tile, XCD = XCD-contiguous tile order.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/strip_bw tools/microbench/strip_bw.hip && /tmp/strip_bw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int kW = 1920, kH = 1080, kN = 32, kDW = 512, kDH = 512, kSets = 5;
constexpr size_t kFrame = (size_t)kW * kH * 3 / 2;
constexpr size_t kPlane = (size_t)kDW * kDH;
constexpr size_t kOut = kPlane * 3 * 4;

__device__ inline int xcd_tile(int b, int grid) {
    const int q = grid >> 3, r = grid & 7, x = b & 7, i = b >> 3;
    return x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}

__device__ __forceinline__ void vm_wait(int n) {
    n = __builtin_amdgcn_readfirstlane(n);
#define V(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    switch (n) { V(0) V(1) V(2) V(3) V(4) V(5) V(6) V(7) V(8) V(9) V(10) V(11) V(12) V(13) V(14) V(15) V(16)
                 V(17) V(18) V(19) V(20) V(21) V(22) V(23) V(24) V(25) V(26) V(27) V(28) V(29) V(30) V(31)
                 V(32) V(33) V(34) V(35) V(36) V(37) V(38) V(39) V(40) V(41) V(42) V(43) V(44) V(45) V(46)
                 V(47) V(48) V(49) V(50) V(51) V(52) V(53) V(54) V(55) V(56) V(57) V(58) V(59) V(60) V(61) V(62)
                 default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break; }
#undef V
}

template <int SP, int D, int W, int TH, bool XCD>
__global__ __launch_bounds__(512) void strip(const uint8_t* __restrict__ src, float* __restrict__ dst) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int PXL = SP / 64;                     // pixels per lane
    constexpr int SEG = ((SP * 15 / 4 + 31) / 16) * 16;  // staged bytes of a strip's source window (+ alignment)
    constexpr int NCK = SEG / 16;                    // 16-B chunks
    constexpr int NI = (NCK + 63) / 64;              // DMA instructions per segment
    constexpr int GRP = 4 * SEG;                     // Y0, Y1, C0, C1
    constexpr int STRIPS = kDW / SP;
    constexpr int TX = (STRIPS + W - 1) / W;
    constexpr int TPI = TX * (kDH / TH);
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int t = XCD ? xcd_tile(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int frame = t / TPI, tile = t % TPI, ty = tile / TX, s = (tile % TX) * W + wave;
    if (s >= STRIPS) return;
    const int Y0 = ty * TH;
    const uint8_t* Yp = src + (size_t)frame * kFrame;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)Yp, (short)0, 0x7FFFFFFF, 0x00020000);
    const int fs = (s * SP * 15 / 4) & ~15;  // window start in a source row
    uint8_t* ring = smem + wave * D * GRP;
    auto rows = [&](int y, int& a, int& b) {
        a = min(max((int)((y + 0.5) * (1080.0 / 512) - 0.5), 0), kH - 1);
        b = min(a + 1, kH - 1);
    };
    auto seg = [&](uint8_t* e, int off) {
#pragma unroll
        for (int k = 0; k < NI; k++)
            if (lane + 64 * k < NCK)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(e + 1024 * k), 16,
                                                         (lane + 64 * k) * 16, off + fs, 0, 0);
    };
    auto issue = [&](int i) -> int {
        int a, b;
        rows(Y0 + i, a, b);
        uint8_t* e = ring + (i % D) * GRP;
        seg(e, a * kW);
        seg(e + SEG, b * kW);
        seg(e + 2 * SEG, kW * kH + (a >> 1) * kW);
        if ((a >> 1) != (b >> 1)) { seg(e + 3 * SEG, kW * kH + (b >> 1) * kW); return 4 * NI; }
        return 3 * NI;
    };
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)(dst + (size_t)frame * kPlane * 3), (short)0, 0x7FFFFFFF, 0x00020000);
    for (int i = 0; i < D; i++) issue(i);
    constexpr int NMIN = 3 * NI, NST = 3 * PXL;
    for (int i = 0; i < TH; i++) {
        vm_wait(NMIN * (min(i + D - 1, TH - 1) - i) + NST * min(i, D - 1));
        const uint8_t* e = ring + (i % D) * GRP;
        const uint32_t v = e[lane] + e[SEG + lane];  // consume the row (one LDS read per source row)
        const int so = ((Y0 + i) * kDW + s * SP) * 4;
#pragma unroll
        for (int p = 0; p < 3; p++)
#pragma unroll
            for (int j = 0; j < PXL; j++)
                __builtin_amdgcn_raw_buffer_store_b32(v + p + j, ro, (lane + 64 * j) * 4, so + p * (int)kPlane * 4, 2);
        asm volatile("" ::: "memory");
        if (i + D < TH) issue(i + D);
        asm volatile("" ::: "memory");
    }
}

int main() {
    std::vector<uint8_t*> src(kSets);
    std::vector<float*> dst(kSets);
    for (int k = 0; k < kSets; k++) {
        CK(hipMalloc(&src[k], kFrame * kN));
        CK(hipMalloc(&dst[k], kOut * kN));
        CK(hipMemset(src[k], k, kFrame * kN));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double alg = 97.1e6 + 100.66e6;
    auto run = [&](const char* name, auto launch) {
        for (int i = 0; i < 30; i++) launch(i % kSets);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        const int iters = 300;
        for (int i = 0; i < iters; i++) launch(i % kSets);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / iters;
        printf("%-44s %8.2f us  %6.3f TB/s\n", name, us, alg / us / 1e6);
    };
#define RUN(SP, D, W, TH, XCD)                                                                                  \
    {                                                                                                        \
        constexpr int SEG = ((SP * 15 / 4 + 31) / 16) * 16, STRIPS = kDW / SP, TX = (STRIPS + W - 1) / W;     \
        const int grid = kN * TX * (kDH / TH), lds = W * D * 4 * SEG;                                        \
        CK(hipFuncSetAttribute((const void*)strip<SP, D, W, TH, XCD>, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
        run("strip SP " #SP " D " #D " W " #W " TH " #TH " XCD " #XCD, [&](int k) {                        \
            hipLaunchKernelGGL((strip<SP, D, W, TH, XCD>), dim3(grid), dim3(64 * W), lds, 0, src[k], dst[k]); }); \
    }
    // the strip kernel's own shape (C2: 64-column strips, D 4, 4 waves, 16-row tiles, XCD order), then
    // wider strips (fewer, longer DMA segments per row), deeper / shallower rings, taller tiles
    RUN(64, 4, 4, 16, true) RUN(64, 4, 4, 16, false) RUN(64, 2, 4, 16, false) RUN(64, 4, 8, 16, false)
    RUN(64, 4, 4, 32, false) RUN(128, 4, 4, 16, false) RUN(128, 2, 4, 16, false) RUN(128, 3, 4, 32, false)
    RUN(128, 2, 4, 8, false) RUN(256, 2, 2, 16, false) RUN(256, 2, 2, 32, false) RUN(256, 3, 2, 32, false)
    RUN(256, 2, 2, 8, false) RUN(256, 2, 4, 8, false) RUN(512, 2, 1, 8, false) RUN(512, 2, 1, 4, false)
    RUN(512, 3, 1, 8, false) RUN(512, 2, 2, 4, false)
    RUN(64, 4, 4, 16, true) RUN(128, 2, 4, 16, false) RUN(256, 2, 2, 16, false)
    return 0;
}
