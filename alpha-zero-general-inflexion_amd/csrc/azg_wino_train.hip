// azg_wino_train.hip -- the trainer's 3x3 convolutions (NNetWrapper.train, NNet.py:36-76:
// conv2-4 of InflexionNNet.py:39-45 forward and backward) on the Winograd transforms and
// libazg's split-fp16 GEMM (azg_split_gemm.hip), f32-accurate like the inference form.
//
// Per layer, with V = B^T d B the input transform (azg_winograd_in_nhwc, AZG_WINO_SPLIT2),
// U_e = G_a g G_b^T the weights' transform and M_e = V_e U_e per transformed point e:
//
//   forward   y  = A^T M A + b                       (wt_out: M -> NHWC y, no ReLU: BN follows)
//   backward  dM = A dy A^T                          (wt_dout: the output transform's adjoint)
//             dV_e = dM_e U_e^T                      (split GEMM, B operand U rows [c][k])
//             dx = sum over tiles of B dV B^T        (wt_din: the input transform's adjoint,
//                                                     overlapping windows gathered per pixel)
//             dU_e = V_e^T dM_e                      (split GEMM over the tiles: both operands
//                                                     transposed by wt_split2_transpose)
//             dg = sum_e G_a^T dU_e G_b              (the caller, torch)
//
// Every split operand is scaled by a power of two chosen on the device from a max|.| the
// kernels here reduce (no host synchronisation): U by 2^ku with max |U| 2^ku in (512, 1024]
// (as nnet._split_u), dM by 2^kd with max |dy| 2^kd in (16, 32] (gradients are far below
// fp16's normal range); the consumers undo them exactly (powers of two).
#include <algorithm>

#include "azg_winograd_kern.h"

namespace {

// nnet.WINOGRAD_G in f64 (F(m,3) weight transforms G [m+2][3])
template <int M>
struct WinoG;
template <>
struct WinoG<2> {
    static constexpr double G[4][3] = {{1.0, 0.0, 0.0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0.0, 0.0, 1.0}};
};
template <>
struct WinoG<3> {
    static constexpr double G[5][3] = {
        {0.5, 0.0, 0.0}, {-0.5, -0.5, -0.5}, {-1.0 / 6, 1.0 / 6, -1.0 / 6}, {1.0 / 6, 1.0 / 3, 2.0 / 3}, {0.0, 0.0, 1.0}};
};
template <>
struct WinoG<4> {
    static constexpr double G[6][3] = {{0.5, 0.0, 0.0},
                                       {-1.0 / 6, -1.0 / 6, -1.0 / 6},
                                       {1.0 / 6, -1.0 / 6, 1.0 / 6},
                                       {1.0 / 30, 1.0 / 15, 2.0 / 15},
                                       {-16.0 / 15, 8.0 / 15, -4.0 / 15},
                                       {0.0, 0.0, 0.5}};
};
template <>
struct WinoG<5> {
    static constexpr double G[7][3] = {{1.0 / 6, 0.0, 0.0},           {-1.0 / 18, -1.0 / 18, -1.0 / 18},
                                       {1.0 / 10, -1.0 / 10, 1.0 / 10}, {-4.0 / 9, 2.0 / 9, -1.0 / 9},
                                       {-1.0 / 126, 1.0 / 63, -2.0 / 63}, {4.0 / 105, 2.0 / 35, 3.0 / 35},
                                       {0.0, 0.0, 0.25}};
};

// 2^floor(log2(target / amax)) (1 for amax 0 or not finite): the power of two that puts the
// largest magnitude in (target / 2, target]; every kernel of a step computes it from the same
// amax, so producer and consumer agree bit for bit
__device__ __forceinline__ float pow2_scale(unsigned amax_bits, float target) {
    const float a = __uint_as_float(amax_bits);
    if (!(a > 0.f) || !(a < 3.0e38f)) return 1.f;
    int e;
    (void)frexpf(target / a, &e);  // target / a = f 2^e, f in [0.5, 1)
    return ldexpf(1.f, e - 1);
}

// U of one (c, k) pair for every point of the groups of an h_out-side layer, in the
// order of nnet._winograd_u (groups (big,big) (big,small) (small,big) (small,small), point
// e = a (mb + 2) + b within a group): f(point index, U value rounded to f32)
template <class F>
__device__ __forceinline__ void u_points(const float* __restrict__ w9, int h_out, F&& f) {
    double g[3][3];
#pragma unroll
    for (int i = 0; i < 9; ++i) g[i / 3][i % 3] = (double)w9[i];
    const WSeq S(h_out);
    int e0 = 0;
    for (int q = 0; q < 4; ++q) {
        const int ma = q < 2 ? S.big : S.small(), mb = (q & 1) ? S.small() : S.big;
        if (S.cnt(ma) * S.cnt(mb) == 0) continue;  // absent tile type
        with_types(ma, mb, [&](auto A_, auto B_) {
            constexpr int MA = decltype(A_)::value, MB = decltype(B_)::value;
            double s[MA + 2][3];
#pragma unroll
            for (int a = 0; a < MA + 2; ++a)
#pragma unroll
                for (int c = 0; c < 3; ++c)
                    s[a][c] = WinoG<MA>::G[a][0] * g[0][c] + WinoG<MA>::G[a][1] * g[1][c] + WinoG<MA>::G[a][2] * g[2][c];
#pragma unroll
            for (int a = 0; a < MA + 2; ++a)
#pragma unroll
                for (int b = 0; b < MB + 2; ++b)
                    f(e0 + a * (MB + 2) + b,
                      (float)(s[a][0] * WinoG<MB>::G[b][0] + s[a][1] * WinoG<MB>::G[b][1] + s[a][2] * WinoG<MB>::G[b][2]));
        });
        e0 += (ma + 2) * (mb + 2);
    }
}

// the block's max of m (non-negative) -> one atomicMax on the bit pattern (non-negative floats order as
// their bits); one atomic per block, not per wave: 8192 waves' atomics on one word held wt_absmax at
// 97 us for conv2's 51 MB gradient (profiles/r05_prof_train_probe_wino.md)
template <int T>
__device__ __forceinline__ void block_max_atomic(float m, unsigned* out) {
    __shared__ float wm[T / 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float b = wm[0];
#pragma unroll
        for (int q = 1; q < T / 64; ++q) b = fmaxf(b, wm[q]);
        atomicMax(out, __float_as_uint(b));
    }
}

// max |x| of n floats (x % 4 == 0 handled by the caller); *out must be 0 before the launch
__global__ __launch_bounds__(256) void wt_absmax_kernel(const float4* __restrict__ x, long long n4,
                                                        unsigned* __restrict__ out) {
    float m = 0.f;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
        const float4 v = x[i];
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    block_max_atomic<256>(m, out);
}

// ---- U built without an f32 intermediate (round 6) --------------------------------------------------
// Round 5's build wrote U in f32 (P K C floats) and read it back to split it (conv2: 127 MB each way;
// 219 us of a 2.5 ms training step, profiles/r06_prof_train_probe*.md).  Here pass 1 computes
// every U value only for its maximum (a per-block max, no stores, no memset / atomic), and pass 2
// recomputes U per 32 x 32 (k, c) tile from the tile's staged weights -- the same f64 expressions as
// u_points, so the same f32 values -- scales it by the power of two of the maximum it reduces from
// pass 1's block maxima, and writes both split layouts.
// max |U| in f32 (it only picks the power of two 2^ku: pass 2's f64-exact U then has max |U| 2^ku within
// one part in 10^6 of (512, 1024], far inside fp16's range); the f64 form held 2 waves per SIMD at 24 us
template <int MA, int MB>
__device__ __forceinline__ float u_max_type(const float (&g)[3][3]) {
    float s[MA + 2][3];
#pragma unroll
    for (int a = 0; a < MA + 2; ++a)
#pragma unroll
        for (int c = 0; c < 3; ++c)
            s[a][c] = (float)WinoG<MA>::G[a][0] * g[0][c] + (float)WinoG<MA>::G[a][1] * g[1][c] +
                      (float)WinoG<MA>::G[a][2] * g[2][c];
    float m = 0.f;
#pragma unroll
    for (int a = 0; a < MA + 2; ++a)
#pragma unroll
        for (int b = 0; b < MB + 2; ++b)
            m = fmaxf(m, fabsf(s[a][0] * (float)WinoG<MB>::G[b][0] + s[a][1] * (float)WinoG<MB>::G[b][1] +
                               s[a][2] * (float)WinoG<MB>::G[b][2]));
    return m;
}

__global__ __launch_bounds__(256) void wt_u_max_kernel(const float* __restrict__ w, int C, int K, int h_out,
                                                       float* __restrict__ pmax) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x, CK = (long long)C * K;
    float m = 0.f;
    if (i < CK) {
        float g[3][3];
#pragma unroll
        for (int j = 0; j < 9; ++j) g[j / 3][j % 3] = w[i * 9 + j];
        const WSeq S(h_out);
        for (int q = 0; q < 4; ++q) {
            const int ma = q < 2 ? S.big : S.small(), mb = (q & 1) ? S.small() : S.big;
            if (S.cnt(ma) * S.cnt(mb) == 0) continue;
            with_types(ma, mb, [&](auto A_, auto B_) {
                m = fmaxf(m, u_max_type<decltype(A_)::value, decltype(B_)::value>(g));
            });
        }
    }
    __shared__ float wm[4];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) pmax[blockIdx.x] = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
}

// block (32-channel c tile, 32-channel k tile, tile type q): U of the type's points for the tile,
// 2^ku-scaled and split into UT [P][K][2C] and UN [P][C][2K] (32-channel [hi | lo] blocks = one
// 128-B row segment per row).  Thread t owns pairs (k, c) = (t / 8 + 32 i / 8 ..): 4 per thread.
__global__ __launch_bounds__(256) void wt_u_direct_kernel(const float* __restrict__ w, int C, int K, int h_out,
                                                          const float* __restrict__ pmax, int npm,
                                                          unsigned* __restrict__ uamax, unsigned* __restrict__ ut,
                                                          unsigned* __restrict__ un) {
    __shared__ float tl[7][32][33];  // [point b of the row][k][c], scaled
    __shared__ float red[4];
    const int t = threadIdx.x, c0 = blockIdx.x * 32, k0 = blockIdx.y * 32, q = blockIdx.z;
    const WSeq S(h_out);
    const int ma = q < 2 ? S.big : S.small(), mb = (q & 1) ? S.small() : S.big;
    if (S.cnt(ma) * S.cnt(mb) == 0) return;  // absent tile type (block-uniform)
    // the global max |U| from pass 1's block maxima -> the scale (every block reduces the same values)
    float m = 0.f;
    for (int i = t; i < npm; i += 256) m = fmaxf(m, pmax[i]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((t & 63) == 0) red[t >> 6] = m;
    __syncthreads();
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (t == 0 && blockIdx.x == 0 && blockIdx.y == 0 && q == 0) *uamax = __float_as_uint(m);  // for the consumers
    const float sc = pow2_scale(__float_as_uint(m), 1024.f);
    // the type's first point index (u_points' order: the groups before it)
    int e0 = 0;
    for (int g2 = 0; g2 < q; ++g2) {
        const int qa = g2 < 2 ? S.big : S.small(), qb = (g2 & 1) ? S.small() : S.big;
        if (S.cnt(qa) * S.cnt(qb)) e0 += (qa + 2) * (qb + 2);
    }
    // this thread's 4 pairs: (kl, cl) = (t / 32 + 8 i, t % 32), weights in f64
    const int cl = t & 31;
    double g[4][3][3];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int kl = (t >> 5) + 8 * i;
        const float* w9 = w + ((long long)(k0 + kl) * C + c0 + cl) * 9;
#pragma unroll
        for (int j = 0; j < 9; ++j) g[i][j / 3][j % 3] = (double)w9[j];
    }
    auto word = [&](float a, float b, bool lo) {
        const _Float16 ha = (_Float16)a, hb = (_Float16)b;
        unsigned short xa = __builtin_bit_cast(unsigned short, ha), xb = __builtin_bit_cast(unsigned short, hb);
        if (lo) {
            xa = __builtin_bit_cast(unsigned short, (_Float16)(a - (float)ha));
            xb = __builtin_bit_cast(unsigned short, (_Float16)(b - (float)hb));
        }
        return (unsigned)xa | ((unsigned)xb << 16);
    };
    with_types(ma, mb, [&](auto A_, auto B_) {
        constexpr int MA = decltype(A_)::value, MB = decltype(B_)::value;
        for (int a = 0; a < MA + 2; ++a) {
            double sa[4][3];  // u_points' s[a][c] for the thread's pairs
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int c = 0; c < 3; ++c)
                    sa[i][c] = WinoG<MA>::G[a][0] * g[i][0][c] + WinoG<MA>::G[a][1] * g[i][1][c] +
                               WinoG<MA>::G[a][2] * g[i][2][c];
            for (int b = 0; b < MB + 2; ++b)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float u = (float)(sa[i][0] * WinoG<MB>::G[b][0] + sa[i][1] * WinoG<MB>::G[b][1] +
                                            sa[i][2] * WinoG<MB>::G[b][2]);
                    tl[b][(t >> 5) + 8 * i][cl] = u * sc;  // exact (a power of two)
                }
            __syncthreads();
            // per point, 32 rows x 32 words per layout: thread t writes words t % 32 of rows t / 32 + 8 i
            const int wd = t & 31, ch = 2 * (wd & 15);
            const bool lo = wd >= 16;
            for (int b = 0; b < MB + 2; ++b) {
                const int e = e0 + a * (MB + 2) + b;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int r = (t >> 5) + 8 * i;
                    if (ut) ut[(((long long)e * K + k0 + r) * 2 * C + 2 * c0) / 2 + wd] = word(tl[b][r][ch], tl[b][r][ch + 1], lo);
                    if (un) un[(((long long)e * C + c0 + r) * 2 * K + 2 * k0) / 2 + wd] = word(tl[b][ch][r], tl[b][ch + 1][r], lo);
                }
            }
            __syncthreads();
        }
    });
}

// Forward output transform without ReLU (BatchNorm follows): y = bias + 2^-ku A^T M A,
// NHWC f32, one thread per (tile, 4 channels) (winograd_out_kernel with the scale read on
// the device)
template <int HC>
__global__ __launch_bounds__(256) void wt_out_kernel(const float4* __restrict__ Min, const float4* __restrict__ bias,
                                                     float4* __restrict__ y, int Ho, int K4, long long B,
                                                     const unsigned* __restrict__ uamax) {
    const WSeq S(HC > 0 ? HC : Ho);
    if (HC > 0) Ho = HC;
    const long long item = xcd_item();
    if (item >= B * S.p * S.p * K4) return;
    const int k4 = (int)(item % K4);
    const long long t = item / K4;
    const int j = (int)(t % S.p);
    const long long r = t / S.p;
    const int i = (int)(r % S.p);
    const long long b = r / S.p;
    const float mscale = 1.f / pow2_scale(*uamax, 1024.f);
    const long long row = S.row0(i, j, b, B), ps = S.pstride(i, j, B);
    const float4 bb = bias[k4];
    with_types_of<HC>(S.m(i), S.m(j), [&](auto A_, auto B_) {
        constexpr int MA = decltype(A_)::value, MB = decltype(B_)::value;
        float4 m[MA + 2][MB + 2];
#pragma unroll
        for (int e = 0; e < (MA + 2) * (MB + 2); ++e)
            m[e / (MB + 2)][e % (MB + 2)] = vmul(mscale, Min[(row + e * ps) * K4 + k4]);
        float4 yt[MA][MB];
        out_tile<MA, MB>(m, yt);
#pragma unroll
        for (int a = 0; a < MA; ++a)
#pragma unroll
            for (int q = 0; q < MB; ++q) {
                const int oy = S.off(i) + a, ox = S.off(j) + q;
                if (oy >= Ho || ox >= Ho) continue;
                y[((b * Ho + oy) * Ho + ox) * K4 + k4] = vadd(yt[a][q], bb);
            }
    });
}

// dM = 2^kd A dy A^T (the adjoint of Y = A^T M A), AZG_WINO_SPLIT2 rows [P][T][2K] in the
// layout of M; one thread per (tile, 4 channels).  |dM| > 65504 sets *overflow.
template <int HC>
__global__ __launch_bounds__(256) void wt_dout_kernel(const float4* __restrict__ dy, void* __restrict__ dM, int Ho,
                                                      int K4, long long B, const unsigned* __restrict__ dyamax,
                                                      int* overflow) {
    const WSeq S(HC > 0 ? HC : Ho);
    if (HC > 0) Ho = HC;
    const long long item = xcd_item();
    if (item >= B * S.p * S.p * K4) return;
    const int k4 = (int)(item % K4);
    const long long t = item / K4;
    const int j = (int)(t % S.p);
    const long long r = t / S.p;
    const int i = (int)(r % S.p);
    const long long b = r / S.p;
    const float sd = pow2_scale(*dyamax, 32.f);
    const long long row = S.row0(i, j, b, B), ps = S.pstride(i, j, B);
    with_types_of<HC>(S.m(i), S.m(j), [&](auto A_, auto B_) {
        constexpr int MA = decltype(A_)::value, MB = decltype(B_)::value;
        float4 g[MA][MB];
#pragma unroll
        for (int a = 0; a < MA; ++a)
#pragma unroll
            for (int q = 0; q < MB; ++q) {
                const int oy = S.off(i) + a, ox = S.off(j) + q;
                g[a][q] = (oy < Ho && ox < Ho) ? vmul(sd, dy[((b * Ho + oy) * Ho + ox) * K4 + k4])
                                               : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        // s[a][v] = sum_q AT_b[q][v] g[a][q]; dM[u][v] = sum_a AT_a[a][u] s[a][v]
        float4 s[MA][MB + 2];
#pragma unroll
        for (int a = 0; a < MA; ++a)
#pragma unroll
            for (int v = 0; v < MB + 2; ++v) {
                float cf[MB];
#pragma unroll
                for (int q = 0; q < MB; ++q) cf[q] = WinoT<MB>::AT[q][v];
                s[a][v] = combine<MB, float4>(cf, [&](int q) { return g[a][q]; });
            }
#pragma unroll
        for (int u = 0; u < MA + 2; ++u)
#pragma unroll
            for (int v = 0; v < MB + 2; ++v) {
                float cf[MA];
#pragma unroll
                for (int a = 0; a < MA; ++a) cf[a] = WinoT<MA>::AT[a][u];
                const float4 d = combine<MA, float4>(cf, [&](int a) { return s[a][v]; });
                store_v<AZG_WINO_SPLIT2>(dM, row + (u * (MB + 2) + v) * ps, K4, k4, d, overflow);
            }
    });
}

// dx = 2^-(kd + ku) sum over the tiles whose input window holds the pixel of B dV B^T
// (the adjoint of V = B^T d B with zero padding PAD); dV f32 [P][T][C] in the layout of
// V.  One wave per (image, 64 channels), one channel per lane, the lane's H x H gradient
// plane in registers, tiles accumulated in a fixed order (deterministic).
template <int H, int PAD>
__global__ __launch_bounds__(64) void wt_din_kernel(const float* __restrict__ dV, float* __restrict__ dx, int C,
                                                    long long B, const unsigned* __restrict__ uamax,
                                                    const unsigned* __restrict__ dyamax) {
    constexpr int HO = H + 2 * PAD - 2;
    const unsigned lane = threadIdx.x;
    const int cblocks = C / 64;
    const long long b = blockIdx.x / cblocks;
    const int c0 = (blockIdx.x % cblocks) * 64;
    const float inv = 1.f / (pow2_scale(*uamax, 1024.f) * pow2_scale(*dyamax, 32.f));
    const WSeq S(HO);
    float pl[H * H];
#pragma unroll
    for (int q = 0; q < H * H; ++q) pl[q] = 0.f;
    for_tiles<HO>(S, [&](auto A_, auto B_, int i, int j) {
        constexpr int MA = decltype(A_)::value, MB = decltype(B_)::value;
        const long long row = S.row0(i, j, b, B), ps = S.pstride(i, j, B);
        const int y0 = S.off(i) - PAD, x0 = S.off(j) - PAD;
        float v[MA + 2][MB + 2];
#pragma unroll
        for (int e = 0; e < (MA + 2) * (MB + 2); ++e) v[e / (MB + 2)][e % (MB + 2)] = dV[(row + e * ps) * C + c0 + lane];
        // s[a][x] = sum_b BT_b[b][x] v[a][b]; d[u][x] = sum_a BT_a[a][u] s[a][x]
        float s[MA + 2][MB + 2];
#pragma unroll
        for (int a = 0; a < MA + 2; ++a)
#pragma unroll
            for (int xx = 0; xx < MB + 2; ++xx) {
                float cf[MB + 2];
#pragma unroll
                for (int bb = 0; bb < MB + 2; ++bb) cf[bb] = WinoT<MB>::BT[bb][xx];
                s[a][xx] = combine<MB + 2, float>(cf, [&](int bb) { return v[a][bb]; });
            }
#pragma unroll
        for (int u = 0; u < MA + 2; ++u)
#pragma unroll
            for (int xx = 0; xx < MB + 2; ++xx) {
                const int iy = y0 + u, ix = x0 + xx;
                if (iy < 0 || iy >= H || ix < 0 || ix >= H) continue;  // compile-time with HO > 0
                float cf[MA + 2];
#pragma unroll
                for (int a = 0; a < MA + 2; ++a) cf[a] = WinoT<MA>::BT[a][u];
                pl[iy * H + ix] += combine<MA + 2, float>(cf, [&](int a) { return s[a][xx]; });
            }
    });
#pragma unroll
    for (int q = 0; q < H * H; ++q) dx[(b * H * H + q) * C + c0 + lane] = pl[q] * inv;
}

// AZG_WINO_SPLIT2 [P][T][2C] -> [P][C][2T]: 64 x 64 (t, c) tiles through LDS, 256 threads
__global__ __launch_bounds__(256) void wt_split2_transpose_kernel(const unsigned short* __restrict__ src,
                                                                  unsigned short* __restrict__ dst, int T, int C) {
    __shared__ unsigned short hi[64][65], lo[64][65];
    const int tt = blockIdx.x, ct = blockIdx.y, e = blockIdx.z;
    const int t0 = tt * 64, c0 = ct * 64;
    const unsigned short* s = src + (long long)e * T * 2 * C;
    unsigned short* d = dst + (long long)e * C * 2 * T;
    // read: 64 rows t, each 128 halves (two 32-channel blocks [hi | lo])
    for (int q = threadIdx.x; q < 64 * 128; q += 256) {
        const int r = q >> 7, x = q & 127;  // x: 64 (block) + 32 (lo) + lane
        const unsigned short v = s[(long long)(t0 + r) * 2 * C + 2 * c0 + x];
        const int c = ((x >> 6) << 5) + (x & 31);
        if (x & 32) lo[r][c] = v;
        else hi[r][c] = v;
    }
    __syncthreads();
    for (int q = threadIdx.x; q < 64 * 128; q += 256) {
        const int r = q >> 7, x = q & 127;  // r: channel, x: t in the same block layout
        const int t = ((x >> 6) << 5) + (x & 31);
        d[(long long)(c0 + r) * 2 * T + 2 * t0 + x] = (x & 32) ? lo[t][r] : hi[t][r];
    }
}

// The same transpose with 16-B global accesses and a conflict-free LDS tile.  A (t, c) element's hi and lo
// halves (64 B apart in both layouts) are paired into one dword, so the tile is a 64 x 64 dword transpose
// (word (c, t) at c * 65 + t: bank (c + t) mod 64).  Read: lane (channel group cg of 8, row tl) loads the
// hi and the lo 16 B of its 8 channels of row t (a wave covers 8 whole 256-B rows) and writes 8 dwords
// whose banks (8 cg + t + k) are distinct across the wave; write: lane (channel, t-group of 8) reads 8
// consecutive t of one channel (banks c + 8 tg + k, distinct) and stores their hi and lo 16 B (64-B runs
// per row).  The element-wise kernel above moved ~3.7 TB/s over the trainer's 408 MB per step.
__global__ __launch_bounds__(256) void wt_split2_transpose_v_kernel(const uint4* __restrict__ src,
                                                                    uint4* __restrict__ dst, int T, int C) {
    __shared__ unsigned tile[64 * 65];
    const int tt = blockIdx.x, ct = blockIdx.y, e = blockIdx.z, tid = threadIdx.x;
    const int t0 = tt * 64, c0 = ct * 64;
    const unsigned short* s = reinterpret_cast<const unsigned short*>(src) + (long long)e * T * 2 * C;
    unsigned short* d = reinterpret_cast<unsigned short*>(dst) + (long long)e * C * 2 * T;
    const int lane = tid & 63, wv = tid >> 6;
    {
        const int cg = lane & 7, tl = lane >> 3;   // 8 channel groups x 8 rows per wave
        const int cb = cg * 8;                     // the group's first channel in the tile
        const int hoff = 64 * (cb >> 5) + (cb & 31);  // its hi halves within the row's two 32-channel blocks
        uint4 hv[2], lv[2];
#pragma unroll
        for (int p = 0; p < 2; ++p) {  // rows wv * 8 + tl and 32 further: all loads in flight first
            const int t = p * 32 + wv * 8 + tl;
            const unsigned short* row = s + (long long)(t0 + t) * 2 * C + 2 * c0;
            hv[p] = *reinterpret_cast<const uint4*>(row + hoff);
            lv[p] = *reinterpret_cast<const uint4*>(row + hoff + 32);
        }
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int t = p * 32 + wv * 8 + tl;
            const unsigned h[4] = {hv[p].x, hv[p].y, hv[p].z, hv[p].w}, l[4] = {lv[p].x, lv[p].y, lv[p].z, lv[p].w};
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const unsigned hk = (h[k >> 1] >> (16 * (k & 1))) & 0xffffu, lk = (l[k >> 1] >> (16 * (k & 1))) & 0xffffu;
                tile[(cb + k) * 65 + t] = hk | (lk << 16);
            }
        }
    }
    __syncthreads();
    {
        const int tg = lane & 7, cl = lane >> 3;  // 8 t-groups x 8 channels per wave
        const int tb = tg * 8;                    // the group's first t in the tile
        const int toff = 64 * (tb >> 5) + (tb & 31);
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int c = p * 32 + wv * 8 + cl;
            unsigned w[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) w[k] = tile[c * 65 + tb + k];
            uint4 hv, lv;
            hv.x = (w[0] & 0xffffu) | (w[1] << 16);
            hv.y = (w[2] & 0xffffu) | (w[3] << 16);
            hv.z = (w[4] & 0xffffu) | (w[5] << 16);
            hv.w = (w[6] & 0xffffu) | (w[7] << 16);
            lv.x = (w[0] >> 16) | (w[1] & 0xffff0000u);
            lv.y = (w[2] >> 16) | (w[3] & 0xffff0000u);
            lv.z = (w[4] >> 16) | (w[5] & 0xffff0000u);
            lv.w = (w[6] >> 16) | (w[7] & 0xffff0000u);
            unsigned short* row = d + (long long)(c0 + c) * 2 * T + 2 * t0;
            *reinterpret_cast<uint4*>(row + toff) = hv;
            *reinterpret_cast<uint4*>(row + toff + 32) = lv;
        }
    }
}

template <class F>
int by_side(int h, F&& f) {
    switch (h) {
        case 3: f(IC<3>{}); break;
        case 5: f(IC<5>{}); break;
        case 7: f(IC<7>{}); break;
        default: return AZG_ERR_ARG;
    }
    return 0;
}

}  // namespace

extern "C" int azg_absmax(const float* x, int64_t n, uint32_t* out, void* stream) {
    if (!x || !out || n <= 0 || n % 4 || ((uintptr_t)x & 15)) return AZG_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(out, 0, 4, st) != hipSuccess) return AZG_ERR_HIP;
    const long long n4 = n / 4;
    const unsigned grid = (unsigned)std::min<long long>((n4 + 255) / 256, 1024);
    hipLaunchKernelGGL(wt_absmax_kernel, dim3(grid), dim3(256), 0, st, (const float4*)x, n4, out);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_wt_u_build(const float* w, int32_t c, int32_t k, int32_t h_out, uint32_t* uamax, void* ut,
                              void* un, float* work, void* stream) {
    if (!w || !uamax || !work || (!ut && !un) || c <= 0 || k <= 0 || c % 64 || k % 64 || h_out < 2 || h_out > 9 ||
        ((uintptr_t)ut & 3) || ((uintptr_t)un & 3))
        return AZG_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    const WSeq S(h_out);
    int P = 0;  // transformed points: sum over the tile types of (ma + 2)(mb + 2)
    for (int i = 0; i < S.p; ++i)
        for (int j = 0; j < S.p; ++j)
            if (S.idx(i) == 0 && S.idx(j) == 0) P += (S.m(i) + 2) * (S.m(j) + 2);
    (void)P;
    // pass 1: the block maxima of |U| (work: >= ceil(c k / 256) floats); pass 2: U per tile, scaled, split
    const int npm = (int)(((long long)c * k + 255) / 256);
    hipLaunchKernelGGL(wt_u_max_kernel, dim3((unsigned)npm), dim3(256), 0, st, w, c, k, h_out, work);
    hipLaunchKernelGGL(wt_u_direct_kernel, dim3((unsigned)(c / 32), (unsigned)(k / 32), 4u), dim3(256), 0, st, w, c,
                       k, h_out, work, npm, uamax, (unsigned*)ut, (unsigned*)un);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_wt_out(const float* M, const float* bias, float* y, int32_t batch, int32_t h_out, int32_t k,
                          const uint32_t* uamax, void* stream) {
    if (!M || !bias || !y || !uamax || batch <= 0 || k <= 0 || k % 4 || ((uintptr_t)M & 15) || ((uintptr_t)bias & 15) ||
        ((uintptr_t)y & 15))
        return AZG_ERR_ARG;
    const WSeq S(h_out);
    const dim3 grid(grid_for((long long)batch * S.p * S.p * (k / 4)));
    const int rc = by_side(h_out, [&](auto H_) {
        hipLaunchKernelGGL((wt_out_kernel<decltype(H_)::value>), grid, dim3(256), 0, (hipStream_t)stream,
                           (const float4*)M, (const float4*)bias, (float4*)y, h_out, k / 4, (long long)batch, uamax);
    });
    return rc ? rc : (hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP);
}

extern "C" int azg_wt_dout(const float* dy, void* dM, int32_t batch, int32_t h_out, int32_t k, const uint32_t* dyamax,
                           int32_t* overflow, void* stream) {
    if (!dy || !dM || !dyamax || batch <= 0 || k <= 0 || k % 32 || ((uintptr_t)dy & 15) || ((uintptr_t)dM & 15) ||
        !azg_device_writable(overflow))
        return AZG_ERR_ARG;
    const WSeq S(h_out);
    const dim3 grid(grid_for((long long)batch * S.p * S.p * (k / 4)));
    const int rc = by_side(h_out, [&](auto H_) {
        hipLaunchKernelGGL((wt_dout_kernel<decltype(H_)::value>), grid, dim3(256), 0, (hipStream_t)stream,
                           (const float4*)dy, dM, h_out, k / 4, (long long)batch, dyamax, overflow);
    });
    return rc ? rc : (hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP);
}

extern "C" int azg_wt_din(const float* dV, float* dx, int32_t batch, int32_t h_in, int32_t pad, int32_t c,
                          const uint32_t* uamax, const uint32_t* dyamax, void* stream) {
    if (!dV || !dx || !uamax || !dyamax || batch <= 0 || c <= 0 || c % 64) return AZG_ERR_ARG;
    const dim3 grid((unsigned)(batch * (c / 64)));
    hipStream_t st = (hipStream_t)stream;
    if (h_in == 7 && pad == 1)
        hipLaunchKernelGGL((wt_din_kernel<7, 1>), grid, dim3(64), 0, st, dV, dx, c, (long long)batch, uamax, dyamax);
    else if (h_in == 7 && pad == 0)
        hipLaunchKernelGGL((wt_din_kernel<7, 0>), grid, dim3(64), 0, st, dV, dx, c, (long long)batch, uamax, dyamax);
    else if (h_in == 5 && pad == 0)
        hipLaunchKernelGGL((wt_din_kernel<5, 0>), grid, dim3(64), 0, st, dV, dx, c, (long long)batch, uamax, dyamax);
    else
        return AZG_ERR_ARG;
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_wt_split2_transpose(const void* src, void* dst, int32_t points, int32_t t, int32_t c,
                                       void* stream) {
    if (!src || !dst || points <= 0 || t <= 0 || c <= 0 || t % 64 || c % 64) return AZG_ERR_ARG;
    if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0)  // (every caller's operands: 16-B aligned)
        hipLaunchKernelGGL(wt_split2_transpose_v_kernel, dim3(t / 64, c / 64, points), dim3(256), 0,
                           (hipStream_t)stream, (const uint4*)src, (uint4*)dst, t, c);
    else
        hipLaunchKernelGGL(wt_split2_transpose_kernel, dim3(t / 64, c / 64, points), dim3(256), 0,
                           (hipStream_t)stream, (const unsigned short*)src, (unsigned short*)dst, t, c);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

namespace {
// dw[k][c][r][s] = 2^-kd sum over the groups of sum_{a,b} G_a[a][r] G_b[b][s] dU_e[c][k] (e = the
// group's point (a, b)): the adjoint of U = G g G^T, one thread per (c, k) with k fastest (the dU
// reads coalesced), f32
__global__ __launch_bounds__(256) void wt_dw_kernel(const float* __restrict__ dU, int C, int K, int h_out,
                                                    const unsigned* __restrict__ dyamax, float* __restrict__ dw) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long long)C * K) return;
    const int k = (int)(i % K), c = (int)(i / K);
    const long long CK = (long long)C * K;
    const float* u = dU + (long long)c * K + k;
    float acc[3][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
    const WSeq S(h_out);
    int e0 = 0;
    for (int q = 0; q < 4; ++q) {
        const int ma = q < 2 ? S.big : S.small(), mb = (q & 1) ? S.small() : S.big;
        if (S.cnt(ma) * S.cnt(mb) == 0) continue;
        with_types(ma, mb, [&](auto A_, auto B_) {
            constexpr int MA = decltype(A_)::value, MB = decltype(B_)::value;
            float t[MA + 2][3];  // t[a][s] = sum_b G_b[b][s] dU[(a, b)]
#pragma unroll
            for (int a = 0; a < MA + 2; ++a) {
                float v[MB + 2];
#pragma unroll
                for (int b = 0; b < MB + 2; ++b) v[b] = u[(long long)(e0 + a * (MB + 2) + b) * CK];
#pragma unroll
                for (int s2 = 0; s2 < 3; ++s2) {
                    float x = 0.f;
#pragma unroll
                    for (int b = 0; b < MB + 2; ++b) x = fmaf((float)WinoG<MB>::G[b][s2], v[b], x);
                    t[a][s2] = x;
                }
            }
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int s2 = 0; s2 < 3; ++s2) {
                    float x = acc[r][s2];
#pragma unroll
                    for (int a = 0; a < MA + 2; ++a) x = fmaf((float)WinoG<MA>::G[a][r], t[a][s2], x);
                    acc[r][s2] = x;
                }
        });
        e0 += (ma + 2) * (mb + 2);
    }
    const float inv = 1.f / pow2_scale(*dyamax, 32.f);
    float* o = dw + ((long long)k * C + c) * 9;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s2 = 0; s2 < 3; ++s2) o[r * 3 + s2] = acc[r][s2] * inv;
}

__global__ void wt_pow2_scale_kernel(const unsigned* amax, float target, float* out) {
    if (threadIdx.x == 0) out[0] = pow2_scale(*amax, target);
}
}  // namespace

// *out = the power of two the kernels above scale by for this amax and target (1024 for U,
// 32 for the output gradients): the host side (torch) undoes it from the same device value
extern "C" int azg_wt_pow2_scale(const uint32_t* amax, float target, float* out, void* stream) {
    if (!amax || !out || !(target > 0.f)) return AZG_ERR_ARG;
    hipLaunchKernelGGL(wt_pow2_scale_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, amax, target, out);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

// dw [k][c][3][3] from dU [P][c][k] (the weight gradient's adjoint transform, scale undone)
extern "C" int azg_wt_dw(const float* dU, int32_t c, int32_t k, int32_t h_out, const uint32_t* dyamax, float* dw,
                         void* stream) {
    if (!dU || !dyamax || !dw || c <= 0 || k <= 0 || h_out < 2 || h_out > 9) return AZG_ERR_ARG;
    hipLaunchKernelGGL(wt_dw_kernel, dim3((unsigned)(((long long)c * k + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, dU, c, k, h_out, dyamax, dw);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}
