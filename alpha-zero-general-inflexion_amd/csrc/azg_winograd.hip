// azg_winograd.hip -- the Winograd layout / table queries and the input and output
// transforms' entry points (kernels: azg_winograd_kern.h).
#include "azg_winograd_kern.h"


extern "C" int azg_winograd_layout(int32_t h_out, int32_t* seq, int32_t* groups) {
    if (h_out < 1 || h_out > 64) return AZG_ERR_ARG;
    const WSeq S(h_out);
    if (seq)
        for (int i = 0; i < S.p; ++i) seq[i] = S.m(i);
    if (groups)  // tiles per image of each group (big,big) (big,small) (small,big) (small,small)
        for (int g = 0; g < 4; ++g) groups[g] = S.cnt(g < 2 ? S.big : S.small()) * S.cnt((g & 1) ? S.small() : S.big);
    return S.p;
}

extern "C" int azg_winograd_tables(int32_t m, float* bt, float* at) {
    if (m < 2 || m > 5 || !bt || !at) return AZG_ERR_ARG;
    const int n = m + 2;
    auto copy = [&](const auto& BT, const auto& AT) {
        for (int i = 0; i < n * n; ++i) bt[i] = BT[i / n][i % n];
        for (int i = 0; i < m * n; ++i) at[i] = AT[i / n][i % n];
    };
    if (m == 2) copy(WinoT<2>::BT, WinoT<2>::AT);
    if (m == 3) copy(WinoT<3>::BT, WinoT<3>::AT);
    if (m == 4) copy(WinoT<4>::BT, WinoT<4>::AT);
    if (m == 5) copy(WinoT<5>::BT, WinoT<5>::AT);
    return 0;
}

extern "C" int azg_winograd_in_nhwc(const float* x, const float* in_bias, void* V, int32_t batch, int32_t h_in,
                                    int32_t pad, int32_t c, int32_t vfmt, int32_t* overflow, void* stream) {
    const int h_out = h_in + 2 * pad - 2;
    if (!x || !V || batch <= 0 || h_out <= 0 || h_out > 64 || c <= 0 || c % 4 || ((uintptr_t)x & 15) ||
        ((uintptr_t)V & 15) || ((uintptr_t)in_bias & 15) || bad_fmt(vfmt, overflow) ||
        (vfmt == AZG_WINO_SPLIT2 && c % 32) ||
        (long long)batch * h_out * h_out * (c / 4) > (1ll << 38))
        return AZG_ERR_ARG;
    const WSeq S(h_out);
    const dim3 grid(grid_for((long long)batch * S.p * S.p * (c / 4)));
    hipStream_t st = (hipStream_t)stream;
    auto launch = [&](auto F_, auto H_) {
        hipLaunchKernelGGL((winograd_in_kernel<decltype(F_)::value, decltype(H_)::value>), grid, dim3(256), 0, st,
                           (const float4*)x, (const float4*)in_bias, V, h_in, pad, c / 4, (long long)batch,
                           overflow);
    };
    auto by_side = [&](auto F_) {  // the output sides of the supported boards get their own build
        switch (h_out) {
            case 3: launch(F_, IC<3>{}); break;
            case 4: launch(F_, IC<4>{}); break;
            case 5: launch(F_, IC<5>{}); break;
            case 6: launch(F_, IC<6>{}); break;
            case 7: launch(F_, IC<7>{}); break;
            case 8: launch(F_, IC<8>{}); break;
            default: launch(F_, IC<0>{});
        }
    };
    if (vfmt == AZG_WINO_F32) by_side(IC<AZG_WINO_F32>{});
    if (vfmt == AZG_WINO_SPLIT) by_side(IC<AZG_WINO_SPLIT>{});
    if (vfmt == AZG_WINO_SPLIT2) by_side(IC<AZG_WINO_SPLIT2>{});
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_winograd_out_nhwc(const float* M, const float* bias, float* y, int32_t batch, int32_t h_out,
                                     int32_t k, int32_t relu, float mscale, void* stream) {
    if (!M || !bias || !y || batch <= 0 || h_out <= 0 || h_out > 64 || k <= 0 || k % 4 || ((uintptr_t)M & 15) ||
        ((uintptr_t)bias & 15) || ((uintptr_t)y & 15) || (long long)batch * h_out * h_out * (k / 4) > (1ll << 38))
        return AZG_ERR_ARG;
    return launch_out(AZG_WINO_F32, M, bias, y, batch, h_out, k, relu, mscale, nullptr, 1, stream);
}

extern "C" int azg_winograd_out_split(const float* M, const float* bias, void* y, int32_t batch, int32_t h_out,
                                      int32_t k, int32_t relu, float mscale, int32_t vfmt, int32_t kparts,
                                      int32_t* overflow, void* stream) {
    const long long width = (long long)h_out * h_out * k;
    if (!M || !bias || !y || batch <= 0 || h_out <= 0 || h_out > 64 || k <= 0 || k % 4 || ((uintptr_t)M & 15) ||
        ((uintptr_t)bias & 15) || ((uintptr_t)y & 15) || vfmt == AZG_WINO_F32 || bad_fmt(vfmt, overflow) ||
        kparts < 1 || width % kparts || (width / kparts) % (vfmt == AZG_WINO_SPLIT2 ? 32 : 4) ||
        width > (1ll << 28) || (long long)batch * h_out * h_out * (k / 4) > (1ll << 38))
        return AZG_ERR_ARG;
    return launch_out(vfmt, M, bias, y, batch, h_out, k, relu, mscale, overflow, kparts, stream);
}
