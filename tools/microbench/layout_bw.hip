// layout_bw.hip — HBM ceiling of the C2 byte layout (diagnostic microbenchmark, not product code).
//
// Moves exactly the bytes one C2 launch moves (32 x 1080p NV12 frames: the 1,024 luma rows and 540
// chroma rows the 1080 -> 512 row table touches, each read in two 960-byte half-row segments; 32 x 3 x
// 512 x 512 fp32 output planes written) with no arithmetic, in several access shapes, cycling 5 frame /
// output sets (>= 3x the 256 MiB Infinity Cache) so every launch streams from HBM. Prints us/launch and
// TB/s per shape next to a plain float4 copy of the same byte count.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/layout_bw tools/microbench/layout_bw.hip && /tmp/layout_bw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int kW = 1920, kH = 1080, kN = 32, kDW = 512, kDH = 512, kSets = 5;
constexpr size_t kFrame = (size_t)kW * kH * 3 / 2;     // NV12
constexpr size_t kOut = (size_t)kDW * kDH * 3 * 4;     // fp32 planar

__global__ void copy4(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

__global__ void read4(const uint4* __restrict__ a, uint32_t* __restrict__ out, size_t n) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) out[0] = acc;
}
__global__ void write4(float4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

// One workgroup per (frame, 256-column half, 16-row band): reads the band's touched source row segments
// (2 luma rows per output row, 1 chroma row per 2 output rows; 960 B each) with 16 B per lane, then
// writes 16 rows x 256 px x 3 planes. STORE4: float4 stores (lanes own 4 adjacent px) vs dword stores.
template <bool STORE4, bool LDS>
__global__ __launch_bounds__(256) void layout(const uint8_t* __restrict__ src, float* __restrict__ dst) {
    __shared__ uint4 stage[4][64];
    const int b = blockIdx.x;
    const int frame = b / 64, rest = b % 64, half = rest & 1, band = rest >> 1;
    const uint8_t* Y = src + (size_t)frame * kFrame;
    const uint8_t* UV = Y + (size_t)kW * kH;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t acc = 0;
    // all 16 rows' loads first (LDS: written to LDS, nothing waits on them; registers: folded into acc
    // once all are issued), then all stores
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int oy = band * 16 + r;
        const int sy = (int)((oy + 0.5) * (1080.0 / 512) - 0.5);
        const int rowY = wave < 2 ? min(max(sy + wave, 0), kH - 1) : 0;
        const uint8_t* p = wave < 2 ? Y + (size_t)rowY * kW : UV + (size_t)(min(max(sy, 0), kH - 1) >> 1) * kW;
        if (lane < 60 && (wave < 3)) {
            const uint4 v = *reinterpret_cast<const uint4*>(p + half * 960 + lane * 16);
            if (LDS) stage[wave][lane] = v; else acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int oy = band * 16 + r;
        float* o = dst + (size_t)frame * kDW * kDH * 3 + (size_t)oy * kDW + half * 256;
        if (STORE4) {
            if (wave < 3) {
                float4 f = make_float4(acc, r, lane, wave);
                *reinterpret_cast<float4*>(o + (size_t)wave * kDW * kDH + lane * 4) = f;
            }
        } else {
            for (int pl = 0; pl < 3; pl++) o[(size_t)pl * kDW * kDH + tid] = (float)(acc + pl);
        }
    }
    if (acc == 0x12345678u) dst[0] = 1.f;
}


// Generalised shape: a workgroup covers WCOLS output columns (256 = half row, 512 = full row) x BAND output
// rows; it reads the band's touched source row segments (WCOLS * 3.75 bytes each, 16 B per lane), then
// writes BAND x WCOLS x 3 planes with dword stores (lane = pixel). Loads land in LDS (nothing waits on
// them), so loads and stores overlap freely: this is the access shape alone.
template <int WCOLS, int BAND, int MODE>  // MODE 0: loads + stores, 1: loads only, 2: stores only, 3: per-row interleaved (4-8: below)
__global__ __launch_bounds__(256) void shape(const uint8_t* __restrict__ src, float* __restrict__ dst) {
    __shared__ uint4 stage[4][128];
    constexpr int tiles_x = 512 / WCOLS, bands = 512 / BAND, seg = WCOLS * 15 / 4;  // bytes per source segment
    constexpr int chunks = seg / 16;
    const int b = blockIdx.x;
    const int frame = b / (tiles_x * bands), rest = b % (tiles_x * bands), tx = rest % tiles_x, band = rest / tiles_x;
    const uint8_t* Y = src + (size_t)frame * kFrame;
    const uint8_t* UV = Y + (size_t)kW * kH;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    auto loads = [&](int r) {
        const int oy = band * BAND + r;
        const int sy = (int)((oy + 0.5) * (1080.0 / 512) - 0.5);
        // waves 0, 1: luma taps; wave 2: chroma row (shared by both taps for half the rows)
        if (wave < 3) {
            const uint8_t* p = wave < 2 ? Y + (size_t)min(max(sy + wave, 0), kH - 1) * kW
                                        : UV + (size_t)(min(max(sy, 0), kH - 1) >> 1) * kW;
            for (int c = lane; c < chunks; c += 64)
                stage[wave][c & 127] = *reinterpret_cast<const uint4*>(p + tx * seg + c * 16);
        }
    };
    auto stores = [&](int r) {
        const int oy = band * BAND + r;
        float* o = dst + (size_t)frame * kDW * kDH * 3 + (size_t)oy * kDW + tx * WCOLS;
        for (int x = tid; x < WCOLS; x += 256)
            for (int pl = 0; pl < 3; pl++) o[(size_t)pl * kDW * kDH + x] = (float)(r + pl);
    };
    if (MODE == 3) {
        for (int r = 0; r < BAND; r++) { loads(r); stores(r); }
        return;
    }
    if (MODE == 4 || MODE == 5) {
        // stores of row r carry a value derived from row r's loads (read back from LDS after a barrier):
        // the staged kernel's dependency, with MODE 5 prefetching one row ahead (double buffer)
        auto stores_dep = [&](int r, uint32_t v) {
            const int oy = band * BAND + r;
            float* o = dst + (size_t)frame * kDW * kDH * 3 + (size_t)oy * kDW + tx * WCOLS;
            for (int x = tid; x < WCOLS; x += 256)
                for (int pl = 0; pl < 3; pl++) o[(size_t)pl * kDW * kDH + x] = (float)(v + pl);
        };
        if (MODE == 4) {
            for (int r = 0; r < BAND; r++) {
                loads(r);
                __syncthreads();
                stores_dep(r, stage[tid >> 6][tid & 63].x);
                __syncthreads();
            }
        } else {
            loads(0);
            for (int r = 0; r < BAND; r++) {
                __syncthreads();
                const uint32_t v = stage[tid >> 6][tid & 63].x;
                __syncthreads();
                if (r + 1 < BAND) loads(r + 1);
                stores_dep(r, v);
            }
        }
        return;
    }
    if (MODE >= 6 && MODE <= 11) {
        // 9 / 10 / 11: MODE 8 plus a dependent integer chain of 32 / 64 / 112 VALU per pixel between the
        // staged value and its stores (the conversion arithmetic's issue slots and latency, no extra bytes)
        // MODE 5's double-buffered row loop with the staged kernel's two memory choices: 6 = LDS-DMA loads
        // (buffer_load ... lds, 16 B per lane), 7 = non-temporal stores, 8 = both
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 0x7FFFFFFF, 0x00020000);
        auto loads_dma = [&](int r) {
            const int oy = band * BAND + r;
            const int sy = (int)((oy + 0.5) * (1080.0 / 512) - 0.5);
            if (wave < 3) {
                const size_t base = (size_t)frame * kFrame +
                                    (wave < 2 ? (size_t)min(max(sy + wave, 0), kH - 1) * kW
                                              : (size_t)kW * kH + (size_t)(min(max(sy, 0), kH - 1) >> 1) * kW) +
                                    (size_t)tx * seg;
                for (int c0 = 0; c0 < chunks; c0 += 64)
                    if (c0 + lane < chunks)
                        __builtin_amdgcn_raw_ptr_buffer_load_lds(
                            rs, (__attribute__((address_space(3))) void*)&stage[wave][c0 & 127], 16, (c0 + lane) * 16,
                            (int)base, 0, 0);
            }
        };
        auto stores_nt = [&](int r, uint32_t v) {
            const int oy = band * BAND + r;
            float* o = dst + (size_t)frame * kDW * kDH * 3 + (size_t)oy * kDW + tx * WCOLS;
            for (int x = tid; x < WCOLS; x += 256)
                for (int pl = 0; pl < 3; pl++) {
                    if (MODE == 6) o[(size_t)pl * kDW * kDH + x] = (float)(v + pl);
                    else if (MODE >= 9) __builtin_nontemporal_store(__uint_as_float(v + pl), &o[(size_t)pl * kDW * kDH + x]);
                    else __builtin_nontemporal_store((float)(v + pl), &o[(size_t)pl * kDW * kDH + x]);
                }
        };
        constexpr int CHAIN = MODE == 9 ? 32 : (MODE == 10 ? 64 : (MODE == 11 ? 112 : 0));
        if (MODE == 7) loads(0); else loads_dma(0);
        for (int r = 0; r < BAND; r++) {
            if (MODE != 7) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            uint32_t v = stage[tid >> 6][tid & 63].x;
            __syncthreads();
            if (r + 1 < BAND) { if (MODE == 7) loads(r + 1); else loads_dma(r + 1); }
#pragma unroll
            for (int k = 0; k < CHAIN; k++) {  // one v_mad_u32_u24 per step, each depending on the previous
                v = __umul24(v, 0x9E37u) + (uint32_t)k;
                asm volatile("" : "+v"(v));
            }
            stores_nt(r, v);
        }
        return;
    }
    if (MODE != 2) for (int r = 0; r < BAND; r++) loads(r);
    if (MODE != 1) for (int r = 0; r < BAND; r++) stores(r);
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
    const int iters = 300;
    auto run = [&](const char* name, auto launch, double bytes) {
        for (int i = 0; i < 20; i++) launch(i % kSets);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int i = 0; i < iters; i++) launch(i % kSets);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / iters;
        printf("%-34s %8.2f us  %6.3f TB/s\n", name, us, bytes / us / 1e6);
    };
    const double alg = 96.1e6 + 100.66e6;  // C2 algorithmic bytes per launch (reads, writes)
    const size_t n4 = (size_t)(alg / 2 / 16);
    run("copy float4 (same bytes)", [&](int k) {
        hipLaunchKernelGGL(copy4, dim3(4096), dim3(256), 0, 0, (const float4*)src[k], (float4*)dst[k], n4);
    }, 2.0 * n4 * 16);
    run("read-only uint4 (96 MB)", [&](int k) {
        hipLaunchKernelGGL(read4, dim3(4096), dim3(256), 0, 0, (const uint4*)src[k], (uint32_t*)dst[k], (size_t)(96.1e6 / 16));
    }, 96.1e6);
    run("write-only float4 (100.7 MB)", [&](int k) {
        hipLaunchKernelGGL(write4, dim3(4096), dim3(256), 0, 0, (float4*)dst[k], (size_t)(100.66e6 / 16));
    }, 100.66e6);
    const int grid = kN * 64;
    run("C2 layout, dword stores", [&](int k) {
        hipLaunchKernelGGL((layout<false, false>), dim3(grid), dim3(256), 0, 0, src[k], dst[k]);
    }, alg);
    run("C2 layout, float4 stores", [&](int k) {
        hipLaunchKernelGGL((layout<true, false>), dim3(grid), dim3(256), 0, 0, src[k], dst[k]);
    }, alg);
    run("C2 layout, LDS staging, dword st", [&](int k) {
        hipLaunchKernelGGL((layout<false, true>), dim3(grid), dim3(256), 0, 0, src[k], dst[k]);
    }, alg);
#define SHAPE(WC, BD, M, B) run("shape " #WC " cols x " #BD " rows mode " #M, [&](int k) { \
        hipLaunchKernelGGL((shape<WC, BD, M>), dim3(kN * (512 / WC) * (512 / BD)), dim3(256), 0, 0, src[k], dst[k]); }, B);
    SHAPE(256, 16, 0, alg) SHAPE(256, 16, 1, 96.1e6) SHAPE(256, 16, 2, 100.66e6) SHAPE(256, 16, 3, alg)
    SHAPE(512, 4, 0, alg) SHAPE(512, 4, 1, 96.1e6) SHAPE(512, 4, 2, 100.66e6) SHAPE(512, 4, 3, alg)
    SHAPE(512, 2, 0, alg) SHAPE(512, 2, 3, alg)
    SHAPE(256, 16, 4, alg) SHAPE(256, 16, 5, alg) SHAPE(512, 8, 4, alg) SHAPE(512, 8, 5, alg)
    SHAPE(256, 16, 6, alg) SHAPE(256, 16, 7, alg) SHAPE(256, 16, 8, alg) SHAPE(256, 16, 5, alg)
    SHAPE(256, 16, 6, alg) SHAPE(256, 16, 7, alg) SHAPE(256, 16, 8, alg)
    SHAPE(256, 16, 9, alg) SHAPE(256, 16, 10, alg) SHAPE(256, 16, 11, alg) SHAPE(256, 16, 8, alg)
    SHAPE(256, 16, 9, alg) SHAPE(256, 16, 10, alg) SHAPE(256, 16, 11, alg)
    // the same shapes held to 6 resident workgroups per CU (the staged kernel's SGPR-bound occupancy) by
    // 16 KB of unused dynamic LDS (8 KB static + 16 KB = 24 KB: 160 / 24 -> 6)
#define SHAPE6(WC, BD, M, B) run("shape " #WC " cols x " #BD " rows mode " #M " @6/CU", [&](int k) { \
        hipLaunchKernelGGL((shape<WC, BD, M>), dim3(kN * (512 / WC) * (512 / BD)), dim3(256), 16384, 0, src[k], dst[k]); }, B);
    SHAPE6(256, 16, 8, alg) SHAPE6(256, 16, 11, alg) SHAPE(256, 16, 8, alg) SHAPE(256, 16, 11, alg)
    SHAPE6(256, 16, 8, alg) SHAPE6(256, 16, 11, alg)
    return 0;
}
