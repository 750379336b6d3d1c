// azg_winograd_mid.hip -- the fused output + next-input transform's entry point
// (kernel: azg_winograd_kern.h, winograd_mid_kernel).
#include "azg_winograd_kern.h"

extern "C" int azg_winograd_mid_nhwc(const float* M, const float* bias, void* V, int32_t batch, int32_t h, int32_t c,
                                     float mscale, int32_t vfmt, int32_t* overflow, void* stream) {
    if (!M || !bias || !V || batch <= 0 || h < 3 || h > 9 || c <= 0 || c % 64 || bad_fmt(vfmt, overflow))
        return AZG_ERR_ARG;
    const dim3 grid((unsigned)(batch * (c / 64)));
    const size_t lds = (size_t)h * h * 64 * sizeof(float);
    hipStream_t st = (hipStream_t)stream;
    const long long B = batch;
// mid<5> (conv3 -> conv4) as four items per 256-thread block: +0.3% at C4 alternating on one box
// (transforms 599-602 -> 594-598 us per forward; profiles/r04_ab_mid5_wpb4); mid<7> stays one wave
// per block (four per block spilled it, 40% slower, HISTORY.md 4.1)
#define AZG_MID(H, SP, L)                                                                                          \
    {                                                                                                              \
        if (H == 5 && grid.x % 32 == 0)                                                                            \
            hipLaunchKernelGGL((winograd_mid_kernel<H, SP, (H == 5 ? 4 : 1)>), dim3(grid.x / 4), dim3(256), L, st, \
                               M, bias, V, h, c, B, mscale, overflow);                                             \
        else                                                                                                       \
            hipLaunchKernelGGL((winograd_mid_kernel<H, SP>), grid, dim3(64), L, st, M, bias, V, h, c, B, mscale,    \
                               overflow);                                                                          \
        return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;                                                  \
    }
    // the board sides of the supported games get register-resident planes
#define AZG_MID_FMT(H, L)                       \
    {                                           \
        if (vfmt == AZG_WINO_SPLIT2) AZG_MID(H, AZG_WINO_SPLIT2, L) \
        if (vfmt == AZG_WINO_SPLIT) AZG_MID(H, AZG_WINO_SPLIT, L)   \
        AZG_MID(H, AZG_WINO_F32, L)                                 \
    }
#define AZG_MID_REG(H) \
    if (h == H) AZG_MID_FMT(H, 0)
    AZG_MID_REG(7)
    AZG_MID_REG(5)
    AZG_MID_REG(8)
    AZG_MID_REG(6)
    AZG_MID_REG(4)
#undef AZG_MID_REG
    AZG_MID_FMT(0, lds)
#undef AZG_MID_FMT
#undef AZG_MID
}
