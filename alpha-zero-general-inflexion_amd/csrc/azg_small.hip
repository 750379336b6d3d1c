// azg_small.hip -- the leaf network at one to four leaves (C1: one game, one leaf per
// simulation; the drop-in MCTS; small arenas): conv1-4 (3x3, BN folded, bias + ReLU,
// InflexionNNet.py:39-45) and fc1 / fc2 / [fc3 | fc4] (:47-54), one launch per layer, meant
// to be replayed from a HIP graph (the drop-in captures each call's simulations).
//
// At one leaf a layer is a weight stream with little reuse: conv2 is 49 pixels x 512
// channels x 4608 products against 9.4 MB of weights, fc1 1024 x 4608 against 18.9 MB.
// The cost that matters is latency -- dependent memory round trips and the serial chain of
// multiply-adds in one lane -- so both kernels spread every layer over the whole chip and
// keep each lane's chain short:
//
//  * small_conv_kernel<PXL, CO_PB, VEC, WLDS>: block = CO_PB output channels x the output
//    pixels of one leaf at a time, 512 threads = PXL pixels x (512 / PXL) K-slices.  The leaf's
//    input plane (one burst of loads, rows padded so a ds_read_b128 phase is conflict-free) and
//    the block's weight rows (WLDS, when both fit the CU's 160 KB) are staged in LDS, so the
//    multiply-adds wait on one memory round trip, not on one per step.  Thread (p, s) sums,
//    for its pixel p, the products of its contiguous slice of k = tap * Cin + ci (float4 steps
//    along ci for NHWC inputs: VEC), then the slices' partial sums are added through LDS in
//    slice order, + bias, ReLU, written as NHWC rows.  PXL is the smallest of 16 / 32 / 64 /
//    128 / 256 that holds one leaf's output pixels, so conv3 / conv4's 25 / 9 pixels cut K
//    into 16 / 32 slices and the lanes stay busy; each leaf is summed in the same order
//    whatever the batch (batch-invariant).  A lane's chain is CO_PB x 9 Cin / slices
//    multiply-adds (conv2: 1152).
//  * small_fc_kernel<NPB, BMAX>: block = NPB output rows, 256 threads split K in float4
//    steps (lane-contiguous: 1 KB of weights per wave-instruction), each thread holding
//    NPB x B sums; a wave butterfly then an LDS step across the 4 waves, in a fixed order.
//
// Everything is f32 with a fixed summation order (deterministic; per leaf the same whatever the batch);
// P and v stay within the north_star's 1e-5 of the reference module
// (tests/test_gpu_nn.py::test_small_forward_matches_reference).  The softmax / tanh heads are
// azg_policy_value (azg_heads.hip).  Replaces round 3's split-K partial / reduce GEMMs and
// one-launch layer (3.4-3.7 ms per 25-simulation drop-in call against the library form's
// 3.0).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "../../include/azg.h"

namespace {

constexpr int SC_T = 512;  // small_conv threads
constexpr size_t SC_LDS_MAX = 160 * 1024;  // the CU's whole LDS: one block per CU
constexpr int SC_UNR = 16;   // input staging loads in flight per thread
constexpr int SC_UNRW = 6;   // weight staging loads per thread (2 x 4608 floats: 4.5)
constexpr int SF_T = 256;  // small_fc threads

// LDS row pitch (floats) of a staged input pixel: channels rounded up to float4, + 4 so that
// the 16 lanes of a ds_read_b128 phase (16 neighbouring pixels) start on 16 different
// 4-bank groups (pitch % 64 == 4 for Cin % 64 == 0)
__host__ __device__ constexpr int sc_pitch(int cin) { return ((cin + 3) & ~3) + 4; }

template <int PXL, int CO_PB, bool VEC, bool WLDS>
__global__ __launch_bounds__(SC_T) void small_conv_kernel(const float* __restrict__ x, long long sB, int sY, int sX,
                                                          int sC, int B, int H, int pad,
                                                          const float* __restrict__ w, int Cin, int Cout,
                                                          const float* __restrict__ bias, int relu,
                                                          float* __restrict__ y, int ldy) {
    constexpr int KSL = SC_T / PXL;  // K slices
    __shared__ __attribute__((aligned(16))) float lds[SC_LDS_MAX / 4];
    const int tid = threadIdx.x;
    const int p = tid % PXL, s = tid / PXL;
    const int co0 = blockIdx.x * CO_PB;
    const int Ho = H + 2 * pad - 2, hw = Ho * Ho;
    const int K = 9 * Cin, P = sc_pitch(Cin);
    float* xs = lds;                          // [H * H][P] one leaf's input
    float* ws = xs + H * H * P;               // [CO_PB][K] the block's weights (WLDS)
    float* red = ws + (WLDS ? CO_PB * K : 0);  // [KSL][PXL][CO_PB]
    constexpr int STEP = VEC ? 4 : 1;
    const int KS = K / STEP;
    const int per = (KS + KSL - 1) / KSL;
    const int k0 = s * per, k1 = min(KS, k0 + per);
    // staging: every thread's loads are issued together (SC_UNR float4 in flight per thread,
    // one memory round trip per SC_UNR x 8 KB), then stored to LDS
    const int nw4 = WLDS ? CO_PB * K / 4 : 0;  // the block's weights: CO_PB contiguous rows
    const float4* __restrict__ w4 = (const float4*)(w + (long long)co0 * K);
    int oy = 0, ox = 0;
    if (p < hw) oy = p / Ho, ox = p - (p / Ho) * Ho;
    for (int b = 0; b < B; ++b) {
        // stage leaf b's input plane into LDS (NHWC float4 rows, or any strides element-wise);
        // with the weights on the first leaf
        const float* __restrict__ xb = x + b * sB;
        if constexpr (VEC) {
            const int c4 = Cin / 4, nx4 = H * H * c4;
            // one batch of input vectors from `base` (and with WW the block's weights: their loads
            // issued first, their stores after the batch's loads are in flight)
            auto batch = [&](int base, auto WW) {
                constexpr bool WITHW = decltype(WW)::value;
                float4 rw[WITHW ? SC_UNRW : 1];
                if constexpr (WITHW) {
#pragma unroll
                    for (int u = 0; u < SC_UNRW; ++u) rw[u] = w4[min(tid + u * SC_T, nw4 - 1)];
                }
                float4 r[SC_UNR];
#pragma unroll
                for (int u = 0; u < SC_UNR; ++u) {  // past the end: a duplicate load, not stored
                    const int i = min(base + u * SC_T, nx4 - 1);
                    const int pix = i / c4, c = (i - pix * c4) * 4, iy = pix / H, ix = pix - iy * H;
                    r[u] = *(const float4*)(xb + (long long)iy * sY + (long long)ix * sX + c);
                }
                if constexpr (WITHW) {
#pragma unroll
                    for (int u = 0; u < SC_UNRW; ++u)  // past the end: rewrites the last vector with its own value
                        ((float4*)ws)[min(tid + u * SC_T, nw4 - 1)] = rw[u];
                    for (int i = tid + SC_UNRW * SC_T; i < nw4; i += SC_T) ((float4*)ws)[i] = w4[i];
                }
#pragma unroll
                for (int u = 0; u < SC_UNR; ++u) {
                    const int i = base + u * SC_T;
                    if (i < nx4) {
                        const int pix = i / c4, c = (i - pix * c4) * 4;
                        *(float4*)(xs + pix * P + c) = r[u];
                    }
                }
            };
            if (WLDS && b == 0) batch(tid, std::true_type{});
            else batch(tid, std::false_type{});
            for (int base = tid + SC_T * SC_UNR; base < nx4; base += SC_T * SC_UNR) batch(base, std::false_type{});
        } else {
            if (b == 0)
                for (int i = tid; i < nw4; i += SC_T) ((float4*)ws)[i] = w4[i];
            const int n = H * H * Cin;
            for (int i = tid; i < n; i += SC_T) {
                const int pix = i / Cin, c = i - pix * Cin, iy = pix / H, ix = pix - iy * H;
                xs[pix * P + c] = xb[(long long)iy * sY + (long long)ix * sX + (long long)c * sC];
            }
        }
        __syncthreads();
        float acc[CO_PB];
#pragma unroll
        for (int c = 0; c < CO_PB; ++c) acc[c] = 0.f;
        if (p < hw) {
            int kk = k0;
            while (kk < k1) {  // k runs tap-major: a slice is a few runs of one tap each
                const int k = kk * STEP;
                const int tap = k / Cin, ci0 = k - tap * Cin;
                const int run = min(k1 - kk, (Cin - ci0) / STEP);
                const int iy = oy + tap / 3 - pad, ix = ox + tap % 3 - pad;
                if (iy >= 0 && iy < H && ix >= 0 && ix < H) {
                    const float* xp = xs + (iy * H + ix) * P + ci0;
                    if constexpr (VEC) {
#pragma unroll 4
                        for (int j = 0; j < run; ++j) {
                            const float4 xv = *(const float4*)(xp + 4 * j);
#pragma unroll
                            for (int c = 0; c < CO_PB; ++c) {
                                const float4 wv = WLDS ? *(const float4*)(ws + c * K + k + 4 * j)
                                                       : *(const float4*)(w + (long long)(co0 + c) * K + k + 4 * j);
                                float a = acc[c];
                                a = fmaf(wv.x, xv.x, a);
                                a = fmaf(wv.y, xv.y, a);
                                a = fmaf(wv.z, xv.z, a);
                                a = fmaf(wv.w, xv.w, a);
                                acc[c] = a;
                            }
                        }
                    } else {
                        for (int j = 0; j < run; ++j) {
                            const float xv = xp[j];
#pragma unroll
                            for (int c = 0; c < CO_PB; ++c)
                                acc[c] = fmaf(WLDS ? ws[c * K + k + j] : w[(long long)(co0 + c) * K + k + j], xv, acc[c]);
                        }
                    }
                }
                kk += run;
            }
        }
#pragma unroll
        for (int c = 0; c < CO_PB; ++c) red[(s * PXL + p) * CO_PB + c] = acc[c];
        __syncthreads();
        for (int t = tid; t < hw * CO_PB; t += SC_T) {
            const int pp = t / CO_PB, c = t - pp * CO_PB;
            float sum = 0.f;
            for (int q = 0; q < KSL; ++q) sum += red[(q * PXL + pp) * CO_PB + c];  // slice order
            float o = sum + (bias ? bias[co0 + c] : 0.f);
            if (relu) o = fmaxf(o, 0.f);
            y[(long long)(b * hw + pp) * ldy + co0 + c] = o;
        }
        __syncthreads();  // xs and red are rewritten for the next leaf
    }
}

template <int NPB, int BMAX>
__global__ __launch_bounds__(SF_T) void small_fc_kernel(const float* __restrict__ x, int ldx, int B,
                                                        const float* __restrict__ w, int K, int N,
                                                        const float* __restrict__ bias, int relu,
                                                        float* __restrict__ y, int ldy) {
    __shared__ float red[SF_T / 64][NPB * BMAX];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n0 = blockIdx.x * NPB;
    const int K4 = K / 4;
    float acc[NPB][BMAX];
#pragma unroll
    for (int r = 0; r < NPB; ++r)
#pragma unroll
        for (int b = 0; b < BMAX; ++b) acc[r][b] = 0.f;
#pragma unroll 8
    for (int k4 = tid; k4 < K4; k4 += SF_T) {
        float4 xv[BMAX];
#pragma unroll
        for (int b = 0; b < BMAX; ++b)
            xv[b] = b < B ? *(const float4*)(x + (long long)b * ldx + 4 * k4) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int r = 0; r < NPB; ++r) {
            if (n0 + r >= N) break;
            const float4 wr = *(const float4*)(w + (long long)(n0 + r) * K + 4 * k4);
#pragma unroll
            for (int b = 0; b < BMAX; ++b) {
                float a = acc[r][b];
                a = fmaf(wr.x, xv[b].x, a);
                a = fmaf(wr.y, xv[b].y, a);
                a = fmaf(wr.z, xv[b].z, a);
                a = fmaf(wr.w, xv[b].w, a);
                acc[r][b] = a;
            }
        }
    }
    // wave butterfly, then the 4 waves' sums in wave order (fixed: deterministic)
#pragma unroll
    for (int r = 0; r < NPB; ++r)
#pragma unroll
        for (int b = 0; b < BMAX; ++b) {
            float v = acc[r][b];
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
            if (lane == 0) red[wv][r * BMAX + b] = v;
        }
    __syncthreads();
    if (tid < NPB * BMAX) {
        const int r = tid / BMAX, b = tid - r * BMAX;
        if (n0 + r < N && b < B) {
            float sum = 0.f;
#pragma unroll
            for (int q = 0; q < SF_T / 64; ++q) sum += red[q][tid];
            float o = sum + (bias ? bias[n0 + r] : 0.f);
            if (relu) o = fmaxf(o, 0.f);
            y[(long long)b * ldy + n0 + r] = o;
        }
    }
}

template <int PXL, bool VEC>
int launch_conv(dim3 grid, hipStream_t st, const float* x, long long sB, int sY, int sX, int sC, int B, int H,
                int pad, const float* w, int Cin, int Cout, const float* bias, int relu, float* y, int ldy) {
    constexpr int CO_PB = 2;
    const size_t xs = (size_t)H * H * sc_pitch(Cin) * 4, red = (size_t)SC_T * CO_PB * 4, wb = (size_t)CO_PB * 9 * Cin * 4;
    if (xs + red > SC_LDS_MAX) return AZG_ERR_ARG;
    if (xs + red + wb <= SC_LDS_MAX && ((uintptr_t)w & 15) == 0 && Cin % 4 == 0)
        hipLaunchKernelGGL((small_conv_kernel<PXL, CO_PB, VEC, true>), grid, dim3(SC_T), 0, st, x, sB, sY, sX, sC, B,
                           H, pad, w, Cin, Cout, bias, relu, y, ldy);
    else
        hipLaunchKernelGGL((small_conv_kernel<PXL, CO_PB, VEC, false>), grid, dim3(SC_T), 0, st, x, sB, sY, sX, sC, B,
                           H, pad, w, Cin, Cout, bias, relu, y, ldy);
    return 0;
}

}  // namespace

extern "C" int azg_small_conv3x3(const float* x, int64_t sB, int32_t sY, int32_t sX, int32_t sC, int32_t batch,
                                 int32_t H, int32_t pad, const float* w, int32_t Cin, int32_t Cout,
                                 const float* bias, int32_t relu, float* y, int32_t ldy, void* stream) {
    const int Ho = H + 2 * pad - 2;
    if (!x || !w || !y || batch <= 0 || batch > 4 || H <= 0 || H > 16 || Ho <= 0 || pad < 0 || pad > 1 || Cin <= 0 ||
        Cout <= 0 || Cout % 2 || ldy < Cout || Ho * Ho > 256 || sB < 0 || sY < 0 || sX < 0 || sC < 0)
        return AZG_ERR_ARG;
    // NHWC input with float4 along the channels (aligned rows), else element-wise staging
    const bool vec = sC == 1 && Cin % 4 == 0 && sX % 4 == 0 && sY % 4 == 0 && sB % 4 == 0 &&
                     ((uintptr_t)x & 15) == 0 && ((uintptr_t)w & 15) == 0;
    const dim3 grid((unsigned)(Cout / 2));
    hipStream_t st = (hipStream_t)stream;
    const int n = Ho * Ho;  // output pixels of one leaf: the leaves run one after another
    int rc = 0;
    auto go = [&](auto V_) {
        constexpr bool V = decltype(V_)::value;
        if (n <= 16) rc = launch_conv<16, V>(grid, st, x, sB, sY, sX, sC, batch, H, pad, w, Cin, Cout, bias, relu, y, ldy);
        else if (n <= 32) rc = launch_conv<32, V>(grid, st, x, sB, sY, sX, sC, batch, H, pad, w, Cin, Cout, bias, relu, y, ldy);
        else if (n <= 64) rc = launch_conv<64, V>(grid, st, x, sB, sY, sX, sC, batch, H, pad, w, Cin, Cout, bias, relu, y, ldy);
        else if (n <= 128) rc = launch_conv<128, V>(grid, st, x, sB, sY, sX, sC, batch, H, pad, w, Cin, Cout, bias, relu, y, ldy);
        else rc = launch_conv<256, V>(grid, st, x, sB, sY, sX, sC, batch, H, pad, w, Cin, Cout, bias, relu, y, ldy);
    };
    if (vec) go(std::true_type{});
    else go(std::false_type{});
    if (rc) return rc;
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_small_fc(const float* x, int32_t ldx, int32_t batch, const float* w, int32_t K, int32_t N,
                            const float* bias, int32_t relu, float* y, int32_t ldy, void* stream) {
    if (!x || !w || !y || batch <= 0 || batch > 4 || K <= 0 || K % 4 || N <= 0 || ldx % 4 || ldx < K ||
        ldy < N || ((uintptr_t)x & 15) || ((uintptr_t)w & 15))
        return AZG_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (batch == 1)
        hipLaunchKernelGGL((small_fc_kernel<4, 1>), dim3((unsigned)((N + 3) / 4)), dim3(SF_T), 0, st, x, ldx, batch, w,
                           K, N, bias, relu, y, ldy);
    else
        hipLaunchKernelGGL((small_fc_kernel<4, 4>), dim3((unsigned)((N + 3) / 4)), dim3(SF_T), 0, st, x, ldx, batch, w,
                           K, N, bias, relu, y, ldy);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}
