// Store-shape probe for the Winograd input transforms (HISTORY.md 6b, "Transform stores"):
// the V2 write of winograd_first (4096 images x 169 points x 512 channels, hi + lo fp16,
// 1.42 GB) as one wave per (image, 64 channels), each lane one channel, written
//   mode 0: as today, [hi(512) | lo(512)] rows: two 2-byte stores per point (128 B per
//           wave-instruction each)
//   mode 1: [hi0 lo0 hi1 lo1 ...] rows: one 4-byte store per point (256 B per instruction)
//   mode 2: 32-channel blocks [hi(32) | lo(32)] (AZG_WINO_SPLIT2): two 2-byte stores per
//           point, each two 64-B pieces
// Same bytes, same grid; prints TB/s per mode.  Build and run:
//   hipcc --offload-arch=gfx950 -O3 -o tools/store_probe tools/store_probe.hip && tools/store_probe
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int IMAGES = 4096, POINTS = 169, C = 512;

template <int MODE>
__global__ __launch_bounds__(64) void store_kernel(_Float16* V, float seed) {
    const int cb = blockIdx.x % (C / 64), b = blockIdx.x / (C / 64);
    const int c = cb * 64 + threadIdx.x;
    float v = seed * (float)(c + 1) + (float)b;
    for (int e = 0; e < POINTS; ++e) {
        v = v * 1.0001f + 0.5f;  // a value per point, as a transform would produce
        const _Float16 hi = (_Float16)v, lo = (_Float16)(v - (float)hi);
        _Float16* row = V + ((size_t)e * IMAGES + b) * 2 * C;
        if constexpr (MODE == 0) {
            row[c] = hi;
            row[C + c] = lo;
        } else if constexpr (MODE == 2) {
            const int o = 64 * (c >> 5) + (c & 31);
            row[o] = hi;
            row[o + 32] = lo;
        } else {
            union {
                _Float16 h[2];
                unsigned u;
            } p;
            p.h[0] = hi;
            p.h[1] = lo;
            ((unsigned*)row)[c] = p.u;
        }
    }
}

int main() {
    const size_t bytes = (size_t)IMAGES * POINTS * 2 * C * sizeof(_Float16);
    _Float16* V = nullptr;
    if (hipMalloc(&V, bytes) != hipSuccess) return 1;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const dim3 grid(IMAGES * (C / 64)), block(64);
    for (int round = 0; round < 3; ++round)
        for (int mode = 0; mode < 3; ++mode) {
            auto launch = [&]() {
                if (mode == 0) hipLaunchKernelGGL(store_kernel<0>, grid, block, 0, 0, V, 0.37f);
                else if (mode == 1) hipLaunchKernelGGL(store_kernel<1>, grid, block, 0, 0, V, 0.37f);
                else hipLaunchKernelGGL(store_kernel<2>, grid, block, 0, 0, V, 0.37f);
            };
            for (int w = 0; w < 3; ++w) launch();
            hipEventRecord(a);
            const int reps = 20;
            for (int r = 0; r < reps; ++r) launch();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            const double us = 1000.0 * ms / reps;
            printf("{\"round\": %d, \"mode\": %d, \"us\": %.1f, \"TB_per_s\": %.2f}\n", round, mode, us,
                   bytes / (us * 1e-6) / 1e12);
            fflush(stdout);
        }
    if (hipGetLastError() != hipSuccess) return 2;
    hipFree(V);
    return 0;
}
