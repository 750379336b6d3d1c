// azg_winograd_first.hip -- the fused conv1 + conv2 input transform's entry point
// (kernel: azg_winograd_kern.h, winograd_first_kernel).
#include "azg_winograd_kern.h"

extern "C" int azg_winograd_first_nchw(const float* planes, const float* w1, const float* b1, void* V, int32_t batch,
                                       int32_t depth, int32_t n, int32_t c, int32_t vfmt, int32_t* overflow,
                                       void* stream) {
    if (!planes || !w1 || !b1 || !V || batch <= 0 || depth < 1 || depth > 4 || n < 3 || n > 9 || c <= 0 ||
        c % 64 || bad_fmt(vfmt, overflow))
        return AZG_ERR_ARG;
    const dim3 grid((unsigned)(batch * (c / 64)));
    // the boards' sides (6-8) have two tile rows for conv2 (pad 1): two waves per item
    static_assert(WSeq(7).p == 2 && WSeq(8).p == 2 && WSeq(6).p == 2, "two tile rows");
    const dim3 grid2((unsigned)(2 * batch * (c / 64)));
    const size_t lds_reg = 0, lds = (4 * 81 + (size_t)n * n * 64) * sizeof(float);
    hipStream_t st = (hipStream_t)stream;
    const long long B = batch;
#define AZG_FIRST(N, SP, L)                                                                                       \
    {                                                                                                             \
        hipLaunchKernelGGL((winograd_first_kernel<N, SP, (N > 0 ? 2 : 1)>), N > 0 ? grid2 : grid, dim3(64), L, st, \
                           planes, w1, b1, V, depth, n, c, B, overflow);                                          \
        return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;                                                 \
    }
#define AZG_FIRST_FMT(N, L)                                          \
    {                                                                \
        if (vfmt == AZG_WINO_SPLIT2) AZG_FIRST(N, AZG_WINO_SPLIT2, L) \
        if (vfmt == AZG_WINO_SPLIT) AZG_FIRST(N, AZG_WINO_SPLIT, L)   \
        AZG_FIRST(N, AZG_WINO_F32, L)                                 \
    }
#define AZG_FIRST_REG(N) \
    if (n == N) AZG_FIRST_FMT(N, lds_reg)
    AZG_FIRST_REG(7)
    AZG_FIRST_REG(8)
    AZG_FIRST_REG(6)
#undef AZG_FIRST_REG
    AZG_FIRST_FMT(0, lds)
#undef AZG_FIRST_FMT
#undef AZG_FIRST
}
