// dma_probe.hip -- how fast can LDS-DMA (buffer_load_dwordx4 ... lds) fill LDS on gfx950,
// as a function of where the bytes come from (L2-resident, Infinity-Cache-resident, HBM)?
// The split GEMM (azg_split_gemm.hip) moves 64 KB per 256x256x32 stage per CU this way;
// its stage time follows those bytes (HISTORY.md 4.1).  This probe keeps the GEMM's stage
// structure -- 512-thread workgroups, one per CU, double-buffered 64 KB stages, every
// wave issuing its pieces then vmcnt(0) + barrier -- with no MFMAs and no LDS reads.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/dma_probe tools/dma_probe.hip && tools/dma_probe
//
// Prints one JSON line per (source size, pieces per wave per stage).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                 \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

template <int PIECES>
__global__ __launch_bounds__(512, 1) void dma_kernel(const char* src, long long src_bytes, int stages, int* sink) {
    __shared__ __attribute__((aligned(16))) char smem[2 * 8 * PIECES * 1024];
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, 0x7FFFFFFF, 0x00020000);
    // each CU streams its own region, 8 * PIECES KB per stage, wrapping inside src
    const long long per_stage = 8LL * PIECES * 1024;
    const long long regions = src_bytes / per_stage;
    long long slot = blockIdx.x % regions;
    for (int s = 0; s < stages; ++s) {
        const long long base = (slot * per_stage) % (src_bytes - per_stage + 1);
        char* lbase = smem + (s & 1) * 8 * PIECES * 1024 + wid * PIECES * 1024;
#pragma unroll
        for (int p = 0; p < PIECES; ++p) {
            // byte offset within the 2 GB window of the descriptor: base + piece
            const long long off = base + (long long)(wid * PIECES + p) * 1024;
            const int voff = (int)((off & 0x3FFFFFFF)) + lane * 16;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(lbase + p * 1024),
                                                     16, voff, 0, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        slot += gridDim.x;
        if (slot >= regions) slot -= regions;
    }
    if (tid == 0 && smem[(stages & 1) * 64] == 123) sink[blockIdx.x] = 1;
}

template <int P>
double run(const char* src, long long bytes, int stages, int* sink, int blocks) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(dma_kernel<P>, dim3(blocks), dim3(512), 0, 0, src, bytes, stages, sink);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(dma_kernel<P>, dim3(blocks), dim3(512), 0, 0, src, bytes, stages, sink);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms / 5;
}

int main() {
    const long long maxb = 1LL << 30;  // 1 GiB (descriptor offsets stay below 2^30)
    char* src;
    int* sink;
    CHECK(hipMalloc(&src, maxb));
    CHECK(hipMalloc(&sink, 4096 * 4));
    CHECK(hipMemset(src, 1, maxb));
    const int blocks = 256, stages = 2000;
    const long long sizes[] = {1LL << 20, 2LL << 20, 16LL << 20, 128LL << 20, maxb};
    for (long long s : sizes) {
        double ms4 = run<4>(src, s, stages, sink, blocks);
        double ms8 = run<8>(src, s, stages, sink, blocks);
        double ms16 = run<10>(src, s, stages, sink, blocks);
        const double b4 = 8.0 * 4 * 1024 * stages * blocks, b8 = 2 * b4, b16 = 2.5 * b4;
        printf("{\"src_bytes\": %lld, \"tbps_32KB_stage\": %.3f, \"tbps_64KB_stage\": %.3f, \"tbps_80KB_stage\": %.3f, "
               "\"us_per_stage_64KB\": %.3f}\n",
               s, b4 / ms4 / 1e9, b8 / ms8 / 1e9, b16 / ms16 / 1e9, ms8 * 1e3 / stages);
        fflush(stdout);
    }
    return 0;
}
