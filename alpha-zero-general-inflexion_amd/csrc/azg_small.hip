// azg_small.hip -- the leaf network at a few leaves (C1: one game, one leaf per
// simulation; anything below the Winograd path's 64 leaves): conv1-4 (3x3, BN folded,
// bias + ReLU, InflexionNNet.py:39-45) and fc1 / fc2 / [fc3 | fc4] (:47-54) as one
// small f32 GEMM each,
//     out[px][co] = sum_k W[co][k] * X[k][px],   k = tap * Cin + ci,
// px = (leaf, y, x) output pixels (taps = 9; the FC layers are taps = 1, one pixel per
// leaf), W the folded weights as [co][ky][kx][ci] (a channels_last conv weight; an FC
// weight [co][ci]).  At one leaf a layer
// is 49 pixels x 512 channels x 4608 products (231 MFLOP) against 9.4 MB of weights: a
// weight stream, so the K dimension is what spreads it over the chip.
//
//  * small_gemm_partial: block (co tile of 128, px tile of 64, K-split z) accumulates its
//    K range slab by slab (kc <= 64 consecutive k of one tap, a power of two): the slab's
//    weights and the matching im2col values (zero padding, any input strides: NCHW leaf
//    planes or the NHWC activations this file writes) go through LDS, each thread keeps
//    4 x 4 outputs, f32 fmaf in k order.  Partial sums to part[z][px][co].
//  * small_gemm_reduce: out[px][co] = sum_z part[z][px][co] in z order, + bias, ReLU,
//    written NHWC (the next layer's input, or the FC rows).  Deterministic.
// Two launches per layer, no library: this path replaces MIOpen and hipBLASLt below
// the batched forward's sizes.
#include <hip/hip_runtime.h>

#include "../../include/azg.h"

namespace {

constexpr int SM_CO = 128;    // co tile (512 threads: 32 rows of 4 co)
constexpr int SM_T = 64;      // px tile (16 columns of 4 px)
constexpr int SM_KMAX = 64;   // slab of K in LDS (a power of two, within one tap)
constexpr int SM_PW = SM_CO + 4, SM_PX = SM_T + 4;  // LDS row pitches: 16-B aligned float4 reads
constexpr int SM_PERW = SM_CO * SM_KMAX / 512, SM_PERX = SM_T * SM_KMAX / 512;  // loads in flight per thread

// Block (co tile of 128, px tile of 64, K-split z), 512 threads of 4 x 4 outputs, over its
// slabs: each slab (KC = 2^kc_shift consecutive k of one tap, KC | Cin) is staged in two
// phases -- every thread issues all its weight and im2col loads into registers, then
// stores them to LDS -- and the next slab's loads are issued before this slab's
// multiply-adds (software pipeline); the pixel decomposition is computed once.
__global__ __launch_bounds__(512) void small_gemm_partial_kernel(const float* __restrict__ x, long long sB, int sY,
                                                                 int sX, int sC, int H, int W, int pad, int taps,
                                                                 int Ho, int Wo, int npx,
                                                                 const float* __restrict__ w, int Cin, int Cout,
                                                                 int kc_shift, int slabs_per_split,
                                                                 float* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) float sw[SM_KMAX * SM_PW];  // [kk][co]
    __shared__ __attribute__((aligned(16))) float sx[SM_KMAX * SM_PX];  // [kk][px]
    __shared__ long long s_base[SM_T];      // input offset of the pixel's leaf
    __shared__ int s_oy[SM_T], s_ox[SM_T];   // its output position (-1 past npx)
    const int tid = threadIdx.x, KC = 1 << kc_shift;
    const int co0 = blockIdx.x * SM_CO, px0 = blockIdx.y * SM_T, z = blockIdx.z;
    const int ty = tid >> 4, tx = tid & 15;  // outputs co0 + 4 ty .., px0 + 4 tx ..
    const int K = Cin * taps;
    if (tid < SM_T) {
        const int px = px0 + tid, hw = Ho * Wo;
        const int b = px / hw, r = px - b * hw;
        s_base[tid] = (long long)b * sB;
        s_oy[tid] = px < npx ? r / Wo : -1;
        s_ox[tid] = r % Wo;
    }
    float acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
    __syncthreads();

    const int nw = SM_CO << kc_shift, nx = SM_T << kc_shift;
    // slab sl's weights and im2col values into registers (all loads issued together)
    float tw[SM_PERW], tv[SM_PERX];
    auto load = [&](int sl) {
        const int k0 = (z * slabs_per_split + sl) << kc_shift;
        const int tap = k0 / Cin, ci0 = k0 - tap * Cin;
        const int dy = taps == 9 ? tap / 3 - pad : 0, dx = taps == 9 ? tap % 3 - pad : 0;
#pragma unroll
        for (int r = 0; r < SM_PERW; ++r) {
            const int i = tid + 512 * r;
            tw[r] = 0.f;
            if (i < nw) {
                const int row = i >> kc_shift, kk = i & (KC - 1);
                if (co0 + row < Cout) tw[r] = w[(long long)(co0 + row) * K + k0 + kk];
            }
        }
#pragma unroll
        for (int r = 0; r < SM_PERX; ++r) {
            const int i = tid + 512 * r;
            tv[r] = 0.f;
            if (i < nx) {
                const int row = i >> kc_shift, kk = i & (KC - 1);
                const int oy = s_oy[row];
                const int iy = oy + dy, ix = s_ox[row] + dx;
                if (oy >= 0 && iy >= 0 && iy < H && ix >= 0 && ix < W)
                    tv[r] = x[s_base[row] + (long long)iy * sY + (long long)ix * sX + (long long)(ci0 + kk) * sC];
            }
        }
    };
    load(0);
    for (int sl = 0; sl < slabs_per_split; ++sl) {
#pragma unroll
        for (int r = 0; r < SM_PERW; ++r) {
            const int i = tid + 512 * r;
            if (i < nw) sw[(i & (KC - 1)) * SM_PW + (i >> kc_shift)] = tw[r];
        }
#pragma unroll
        for (int r = 0; r < SM_PERX; ++r) {
            const int i = tid + 512 * r;
            if (i < nx) sx[(i & (KC - 1)) * SM_PX + (i >> kc_shift)] = tv[r];
        }
        __syncthreads();
        if (sl + 1 < slabs_per_split) load(sl + 1);
        for (int kk = 0; kk < KC; ++kk) {
            const float4 a = *(const float4*)(sw + kk * SM_PW + 4 * ty);
            const float4 c = *(const float4*)(sx + kk * SM_PX + 4 * tx);
            const float av[4] = {a.x, a.y, a.z, a.w}, cv[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], cv[j], acc[i][j]);
        }
        __syncthreads();
    }
    float* pz = part + (long long)z * npx * Cout;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int px = px0 + 4 * tx + j;
        if (px >= npx) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int co = co0 + 4 * ty + i;
            if (co < Cout) pz[(long long)px * Cout + co] = acc[i][j];
        }
    }
}

__global__ __launch_bounds__(256) void small_gemm_reduce_kernel(const float* __restrict__ part, int ksplit, int npx,
                                                                int Cout, const float* __restrict__ bias, int relu,
                                                                float* __restrict__ y, int ldy) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)npx * Cout) return;
    const int px = (int)(i / Cout), co = (int)(i - (long long)px * Cout);
    // in split order; the loads 8 at a time (independent), the adds in sequence
    const long long stride = (long long)npx * Cout;
    float s = part[i];
    int z = 1;
    for (; z + 8 <= ksplit; z += 8) {
        float t[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) t[j] = part[(z + j) * stride + i];
#pragma unroll
        for (int j = 0; j < 8; ++j) s += t[j];
    }
    for (; z < ksplit; ++z) s += part[z * stride + i];
    if (bias) s += bias[co];
    if (relu) s = fmaxf(s, 0.f);
    y[(long long)px * ldy + co] = s;
}

}  // namespace

extern "C" int azg_small_gemm_partial(const float* x, int64_t sB, int32_t sY, int32_t sX, int32_t sC, int32_t batch,
                                      int32_t H, int32_t W, int32_t pad, int32_t taps, const float* w, int32_t Cin,
                                      int32_t Cout, int32_t kc, int32_t ksplit, float* part, void* stream) {
    if (!x || !w || !part || batch <= 0 || H <= 0 || W <= 0 || (taps != 1 && taps != 9) || Cin <= 0 || Cout <= 0 ||
        kc <= 0 || kc > SM_KMAX || (kc & (kc - 1)) || Cin % kc || ksplit <= 0 || pad < 0 || (taps == 1 && pad))
        return AZG_ERR_ARG;
    int kc_shift = 0;
    while ((1 << kc_shift) < kc) ++kc_shift;
    const int Ho = taps == 9 ? H + 2 * pad - 2 : H, Wo = taps == 9 ? W + 2 * pad - 2 : W;
    if (Ho <= 0 || Wo <= 0) return AZG_ERR_ARG;
    const long long npx = (long long)batch * Ho * Wo;
    const int slabs = taps * Cin / kc;
    if (npx > (1 << 24) || ksplit > slabs || slabs % ksplit) return AZG_ERR_ARG;
    const dim3 grid((unsigned)((Cout + SM_CO - 1) / SM_CO), (unsigned)((npx + SM_T - 1) / SM_T), (unsigned)ksplit);
    hipLaunchKernelGGL(small_gemm_partial_kernel, grid, dim3(512), 0, (hipStream_t)stream, x, (long long)sB, sY, sX,
                       sC, H, W, pad, taps, Ho, Wo, (int)npx, w, Cin, Cout, kc_shift, slabs / ksplit, part);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_small_gemm_reduce(const float* part, int32_t ksplit, int32_t npx, int32_t Cout, const float* bias,
                                     int32_t relu, float* y, int32_t ldy, void* stream) {
    if (!part || !y || ksplit <= 0 || npx <= 0 || Cout <= 0 || ldy < Cout) return AZG_ERR_ARG;
    const long long n = (long long)npx * Cout;
    hipLaunchKernelGGL(small_gemm_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, part, ksplit, npx, Cout, bias, relu, y, ldy);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}
