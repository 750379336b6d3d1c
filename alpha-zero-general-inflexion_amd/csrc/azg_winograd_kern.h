// azg_winograd.hip -- the leaf network's 3x3 convolutions as Winograd convolutions
// over mixed F(5,3) / F(4,3) / F(3,3) / F(2,3) tiles.
//
// conv2-4 of InflexionNNet.forward (InflexionNNet.py:39-45, BN folded) are
// y = relu(bias + conv3x3(x, w)).  Winograd F(m,3) along one axis turns m outputs
// into n = m + 2 transformed points; the 2-D transform is separable, so a tile may
// use F(ma,3) down its rows and F(mb,3) across its columns:
//     Y = A_ma^T [ U (.) V ] A_mb,  U = G_ma g G_mb^T (per (c, k)),  V = B_ma^T d B_mb.
// An h-long output axis is cut into the fewest tiles of side <= 5, sides as equal as
// possible (at most two per axis; h = 7: 4+3; 5: 5; 3: 3; 8: 4+4; 6: 3+3; 4: 4), the
// fewest transformed points that cover it exactly with F(m <= 5, 3): 11^2 instead of
// 13^2 (3+2+2) for a 7x7 output, 7^2 instead of 9^2 (3+2) for 5x5.
//
// Summed over input channels c, each transformed point e of a tile type
// g = (ma, mb) is one GEMM  M_e[T_g x K] = V_e[T_g x C] x U_e[C x K].  Layout of V
// (and M, with K for C): the groups (big,big), (big,small), (small,big), (small,small)
// (small = big - 1, per layer: WSeq) one after another
// (absent types skipped), group g as [P_g][batch * n_g][row] with P_g = (ma+2)(mb+2)
// points and n_g tiles of that type per image, tiles row-major within the image.
// The GEMMs (hipBLASLt through torch.bmm) are the caller's; these kernels are the
// transforms, HBM-bound, consecutive lanes on consecutive channels:
//   * winograd_in   : NHWC input (zero padding; optionally the previous layer's
//                     bias + ReLU applied on load) -> V
//   * winograd_out  : M -> NHWC output, bias + ReLU fused, tiles cropped; or (split
//                     formats) the flattened activation as one split row per image,
//                     fc1's A operand
//   * winograd_mid  : layer i's output transform + layer i+1's input transform in
//                     one pass (the activation stays on chip)
//   * winograd_first: conv1 + bias + ReLU from the NCHW planes + conv2's input
//                     transform in one pass
// B and A have small entries (B^T integers up to 17; A^T powers of the points, exact
// in f32); U is formed in f64 by the caller (G entries like 1/6, 1/15).
//
// V is written in one of three formats (vfmt):
//   AZG_WINO_F32  : f32 rows of C;
//   AZG_WINO_SPLIT2: fp16 rows of 2C = [hi | lo], the A operand of libazg's split
//                   GEMM (azg_split_gemm.hip), which forms the three products itself;
//   AZG_WINO_SPLIT: fp16 rows of 3C = [hi | lo | hi], hi = fp16(v), lo = fp16(v - hi),
//                   for the error-compensated GEMM M = [hi|lo|hi] x [Uh; Uh; Ul] =
//                   hi Uh + lo Uh + hi Ul on the fp16 MFMA with f32 accumulation.
//                   hi + lo holds v to 2^-22 relative (2^-25 absolute below
//                   |v| = 2^-3), the dropped lo Ul term is ~2^-22, so the products
//                   are f32-accurate; U is pre-scaled by a power of
//                   two that mscale undoes exactly in the output transforms.
//                   |v| > 65504 or NaN sets *overflow.
#pragma once
// (azg_winograd_kern.h: the kernels and helpers, shared by azg_winograd.hip, _mid.hip and
// _first.hip, which each instantiate only the kernels they launch: three translation
// units that compile in parallel)
#include <hip/hip_runtime.h>

#include <utility>

#include "../../include/azg.h"
#include "azg_conv1.h"
#include "azg_ptr.h"

namespace {

template <int V>
struct IC {
    static constexpr int value = V;
};

// Tile sequence of an h-long output axis: the fewest tiles of side <= 5, p = ceil(h / 5),
// with sides as equal as possible -- big = ceil(h / p) for the first nbig tiles,
// big - 1 for the rest (h = 7: 4+3; 5: 5; 3: 3; 8: 4+4; 6: 3+3; 4: 4; 9: 5+4).
// h = 1: one 2-tile, cropped.
struct WSeq {
    int h, p, big, nbig;
    __host__ __device__ static constexpr int tiles(int h_) { return h_ <= 5 ? 1 : (h_ + 4) / 5; }
    __host__ __device__ static constexpr int side(int h_) {
        return h_ < 2 ? 2 : (h_ + tiles(h_) - 1) / tiles(h_);
    }
    __host__ __device__ constexpr explicit WSeq(int h_)
        : h(h_), p(tiles(h_)), big(side(h_)), nbig(h_ < 2 ? 1 : h_ - tiles(h_) * (side(h_) - 1)) {}
    __host__ __device__ constexpr int small() const { return big - 1; }
    __host__ __device__ constexpr int m(int i) const { return i < nbig ? big : big - 1; }
    __host__ __device__ constexpr int off(int i) const {
        return i < nbig ? big * i : big * nbig + (big - 1) * (i - nbig);
    }
    __host__ __device__ constexpr int cnt(int mm) const { return mm == big ? nbig : p - nbig; }
    __host__ __device__ constexpr int idx(int i) const { return i < nbig ? i : i - nbig; }  // index among its type
    // rows of V (or M) before group (ma, mb); group order (big,big) (big,small) (small,big) (small,small)
    __host__ __device__ constexpr long long base(int ma, int mb, long long B) const {
        const int g = (ma == big ? 0 : 2) + (mb == big ? 0 : 1);
        long long r = 0;
        for (int q = 0; q < g; ++q) {
            const int qa = q < 2 ? big : big - 1, qb = (q & 1) ? big - 1 : big;
            r += (long long)(qa + 2) * (qb + 2) * B * cnt(qa) * cnt(qb);
        }
        return r;
    }
    // row of point 0 of tile (i, j) of image b, and the row stride between points
    __host__ __device__ constexpr long long row0(int i, int j, long long b, long long B) const {
        const int ma = m(i), mb = m(j), ng = cnt(ma) * cnt(mb);
        return base(ma, mb, B) + b * ng + (long long)idx(i) * cnt(mb) + idx(j);
    }
    __host__ __device__ constexpr long long pstride(int i, int j, long long B) const {
        return B * cnt(m(i)) * cnt(m(j));
    }
};

// run f(IC<ma>, IC<mb>): the tile bodies are compiled per type; with constant
// ma, mb (unrolled compile-time sequences) the branches fold away
template <class F>
__device__ __forceinline__ void with_type(int m, F&& f) {
    if (m == 5) f(IC<5>{});
    else if (m == 4) f(IC<4>{});
    else if (m == 3) f(IC<3>{});
    else f(IC<2>{});
}
template <class F>
__device__ __forceinline__ void with_types(int ma, int mb, F&& f) {
    with_type(ma, [&](auto A_) { with_type(mb, [&](auto B_) { f(A_, B_); }); });
}

// with_types restricted to the sides a compile-time output side HC has (HC > 0): the
// per-thread kernels then instantiate only the tile types that occur
template <int HC, class F>
__device__ __forceinline__ void with_types_of(int ma, int mb, F&& f) {
    if constexpr (HC > 0) {
        constexpr WSeq SC(HC);
        constexpr int BG = SC.big, SM = SC.nbig == SC.p ? SC.big : SC.big - 1;
        if (ma == BG) {
            if (mb == BG) f(IC<BG>{}, IC<BG>{});
            else f(IC<BG>{}, IC<SM>{});
        } else {
            if (mb == BG) f(IC<SM>{}, IC<BG>{});
            else f(IC<SM>{}, IC<SM>{});
        }
    } else {
        with_types(ma, mb, f);
    }
}

template <int... Is, class F>
__device__ __forceinline__ void static_for_impl(std::integer_sequence<int, Is...>, F&& f) {
    (f(IC<Is>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(std::make_integer_sequence<int, N>{}, f);
}

// f(IC<ma>, IC<mb>, i, j) for every tile (i, j) of an axis sequence S, row-major.
// With a compile-time side HC (S == WSeq(HC)) the tiles are expanded at compile time,
// so every index into a lane's register plane is a constant (no scratch);
// otherwise a runtime loop over the types.
template <int HC, class F>
__device__ __forceinline__ void for_tiles(const WSeq& S, F&& f) {
    if constexpr (HC > 0) {
        constexpr WSeq SC(HC);
        static_for<SC.p>([&](auto I) {
            static_for<SC.p>([&](auto J) {
                constexpr int i = decltype(I)::value, j = decltype(J)::value;
                f(IC<SC.m(i)>{}, IC<SC.m(j)>{}, i, j);
            });
        });
    } else {
        for (int i = 0; i < S.p; ++i)
            for (int j = 0; j < S.p; ++j) with_types(S.m(i), S.m(j), [&](auto A_, auto B_) { f(A_, B_, i, j); });
    }
}

// transform tables: B^T [n][n] (input), A^T [m][n] (output)
template <int M>
struct WinoT;
template <>
struct WinoT<2> {
    static constexpr float BT[4][4] = {{1, 0, -1, 0}, {0, 1, 1, 0}, {0, -1, 1, 0}, {0, 1, 0, -1}};
    static constexpr float AT[2][4] = {{1, 1, 1, 0}, {0, 1, -1, -1}};
};
template <>
struct WinoT<3> {
    // F(3,3): interpolation points 0, 1, -1, 2, inf
    static constexpr float BT[5][5] = {
        {2, -1, -2, 1, 0}, {0, -2, -1, 1, 0}, {0, 2, -3, 1, 0}, {0, -1, 0, 1, 0}, {0, 2, -1, -2, 1}};
    static constexpr float AT[3][5] = {{1, 1, 1, 1, 0}, {0, 1, -1, 2, 0}, {0, 1, 1, 4, 1}};
};
template <>
struct WinoT<4> {
    // F(4,3): interpolation points 0, 1, -1, 2, -1/2, inf (-1/2 rather than -2 keeps the
    // error at F(3,3)'s); B^T's rows scaled to small integers, their inverse scales in G
    // (nnet.WINOGRAD_G, applied to the weights in f64)
    static constexpr float BT[6][6] = {{2, 3, -4, -3, 2, 0},  {0, -2, -5, -1, 2, 0}, {0, 2, 1, -5, 2, 0},
                                       {0, -1, -2, 1, 2, 0}, {0, 2, -1, -2, 1, 0},  {0, 2, 3, -4, -3, 2}};
    static constexpr float AT[4][6] = {
        {1, 1, 1, 1, 1, 0}, {0, 1, -1, 2, -0.5f, 0}, {0, 1, 1, 4, 0.25f, 0}, {0, 1, -1, 8, -0.125f, 1}};
};
template <>
struct WinoT<5> {
    // F(5,3): interpolation points 0, 1, -1, -1/2, -2, 3/2, inf (A^T's powers exact in
    // f32; the set with the smallest error among dyadic ones, tools/wino_error_sim.py);
    // B^T's rows scaled to integers, their inverse scales in G
    static constexpr float BT[7][7] = {{6, 11, -10, -15, 4, 4, 0}, {0, -6, -17, -7, 8, 4, 0},
                                       {0, 6, 5, -15, 0, 4, 0},    {0, 6, -1, -8, 1, 2, 0},
                                       {0, 3, 4, -7, -4, 4, 0},    {0, -2, -5, 0, 5, 2, 0},
                                       {0, 6, 11, -10, -15, 4, 4}};
    static constexpr float AT[5][7] = {{1, 1, 1, 1, 1, 1, 0},
                                       {0, 1, -1, -0.5f, -2, 1.5f, 0},
                                       {0, 1, 1, 0.25f, 4, 2.25f, 0},
                                       {0, 1, -1, -0.125f, -8, 3.375f, 0},
                                       {0, 1, 1, 0.0625f, 16, 5.0625f, 1}};
};

// a float4 read once (non-temporal: it neither stays in nor evicts from the caches)
__device__ __forceinline__ float4 nt_load4(const float4* p) {
    using v4 = __attribute__((ext_vector_type(4))) float;
    const v4 x = __builtin_nontemporal_load((const v4*)p);
    return make_float4(x[0], x[1], x[2], x[3]);
}

__device__ __forceinline__ float vadd(float a, float b) { return a + b; }
__device__ __forceinline__ float vmul(float c, float a) { return c * a; }
__device__ __forceinline__ float4 vadd(float4 a, float4 b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 vmul(float c, float4 a) { return make_float4(c * a.x, c * a.y, c * a.z, c * a.w); }
__device__ __forceinline__ float4 vrelu(float4 a) {
    return make_float4(fmaxf(a.x, 0.f), fmaxf(a.y, 0.f), fmaxf(a.z, 0.f), fmaxf(a.w, 0.f));
}

// sum_j coef[j] * x(j), skipping zero coefficients at compile time (x1 folds)
template <int L, class T, class X>
__device__ __forceinline__ T combine(const float (&coef)[L], X&& x) {
    T acc{};
    bool first = true;
#pragma unroll
    for (int j = 0; j < L; ++j) {
        if (coef[j] == 0.f) continue;
        const T term = coef[j] == 1.f ? x(j) : vmul(coef[j], x(j));
        acc = first ? term : vadd(acc, term);
        first = false;
    }
    return acc;
}

// V = B_ma^T d B_mb  (d, V: (ma+2) x (mb+2))
template <int MA, int MB, class T>
__device__ __forceinline__ void in_tile(const T (&d)[MA + 2][MB + 2], T (&V)[MA + 2][MB + 2]) {
    constexpr int NA = MA + 2, NB = MB + 2;
    T s[NA][NB];
#pragma unroll
    for (int v = 0; v < NB; ++v)
#pragma unroll
        for (int a = 0; a < NA; ++a) s[a][v] = combine<NA, T>(WinoT<MA>::BT[a], [&](int u) { return d[u][v]; });
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) V[a][bb] = combine<NB, T>(WinoT<MB>::BT[bb], [&](int v) { return s[a][v]; });
}

// Y = A_ma^T M A_mb  (M: (ma+2) x (mb+2), Y: ma x mb)
template <int MA, int MB, class T>
__device__ __forceinline__ void out_tile(const T (&mm)[MA + 2][MB + 2], T (&y)[MA][MB]) {
    constexpr int NA = MA + 2, NB = MB + 2;
    T s[MA][NB];
#pragma unroll
    for (int v = 0; v < NB; ++v)
#pragma unroll
        for (int a = 0; a < MA; ++a) s[a][v] = combine<NA, T>(WinoT<MA>::AT[a], [&](int u) { return mm[u][v]; });
#pragma unroll
    for (int a = 0; a < MA; ++a)
#pragma unroll
        for (int q = 0; q < MB; ++q) y[a][q] = combine<NB, T>(WinoT<MB>::AT[q], [&](int v) { return s[a][v]; });
}

// One V element: f32 (FMT 0); its fp16 (hi, lo, hi) at columns c, C + c, 2C + c of
// a 3C-wide row (FMT 1, AZG_WINO_SPLIT); or (hi, lo) in a 2C-wide row of 32-channel
// blocks [hi(32) | lo(32)], at 64 (c / 32) + c % 32 and 32 further (FMT 2,
// AZG_WINO_SPLIT2: a split-GEMM stage of 32 channels is one 128-B line per row).
template <int FMT>
__device__ __forceinline__ void store_v(void* V, long long row, int C, int c, float v, int* overflow) {
    if constexpr (FMT == AZG_WINO_F32) {
        ((float*)V)[row * C + c] = v;
    } else {
        const _Float16 hi = (_Float16)v;  // round to nearest even
        const _Float16 lo = (_Float16)(v - (float)hi);
        _Float16* r = (_Float16*)V + row * (FMT == AZG_WINO_SPLIT ? 3 : 2) * C;
        if constexpr (FMT == AZG_WINO_SPLIT) {
            r[c] = hi;
            r[C + c] = lo;
            r[2 * C + c] = hi;
        } else {
            const int o = 64 * (c >> 5) + (c & 31);
            r[o] = hi;
            r[o + 32] = lo;
        }
        if (!(fabsf(v) <= 65504.f)) atomicOr(overflow, 1);
    }
}

// One V element per lane of a full wave whose lanes hold 64 consecutive channels
// c0 + lane (c0 % 64 == 0), in AZG_WINO_SPLIT2: one v_permlane32_swap turns (hi, lo)
// into the two 32-channel blocks [hi(32) | lo(32)] as they lie in the row, so each of
// the two stores writes one whole 128-B line (per-lane stores would write each line
// in two 64-B halves from two instructions).  rowp = the row's halves at channel c0,
// wave-uniform, so the stores take a scalar base and a 32-bit lane offset.  Returns
// whether v is out of fp16 range (the caller raises the flag once).
template <bool NT = false>
__device__ __forceinline__ bool store_v2_wave(unsigned short* rowp, unsigned lane, float v) {
    const _Float16 hi = (_Float16)v;  // round to nearest even
    const _Float16 lo = (_Float16)(v - (float)hi);
    const auto sw = __builtin_amdgcn_permlane32_swap((unsigned)__builtin_bit_cast(unsigned short, hi),
                                                     (unsigned)__builtin_bit_cast(unsigned short, lo), false, false);
    if constexpr (NT) {
        __builtin_nontemporal_store((unsigned short)sw[0], rowp + lane);
        __builtin_nontemporal_store((unsigned short)sw[1], rowp + 64 + lane);
    } else {
        rowp[lane] = (unsigned short)sw[0];       // lanes 0-31: hi of c0 + lane; 32-63: lo of c0 + lane - 32
        rowp[64 + lane] = (unsigned short)sw[1];  // the same for channels c0 + 32 ..
    }
    return !(fabsf(v) <= 65504.f);
}

// Four consecutive channels (c4 = c / 4) of one V row.
template <int FMT>
__device__ __forceinline__ void store_v(void* V, long long row, int C4, int c4, float4 v, int* overflow) {
    if constexpr (FMT == AZG_WINO_F32) {
        ((float4*)V)[row * C4 + c4] = v;
    } else {
        const float x[4] = {v.x, v.y, v.z, v.w};
        union {
            _Float16 h[4];
            uint2 u;
        } hi, lo;
        bool bad = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            hi.h[j] = (_Float16)x[j];
            lo.h[j] = (_Float16)(x[j] - (float)hi.h[j]);
            bad |= !(fabsf(x[j]) <= 65504.f);
        }
        uint2* r = (uint2*)V + row * (FMT == AZG_WINO_SPLIT ? 3 : 2) * C4;
        if constexpr (FMT == AZG_WINO_SPLIT) {
            r[c4] = hi.u;
            r[C4 + c4] = lo.u;
            r[2 * C4 + c4] = hi.u;
        } else {  // 32-channel blocks: 8 uint2 of hi, then 8 of lo
            const int o = 16 * (c4 >> 3) + (c4 & 7);
            r[o] = hi.u;
            r[o + 8] = lo.u;
        }
        if (bad) atomicOr(overflow, 1);
    }
}

// Work item of a thread: block ids are dealt round-robin to the 8 XCDs, so the
// block -> work mapping gives each XCD one contiguous eighth of the work:
// neighbouring tiles, which share input halo pixels, then hit the same L2.
__device__ __forceinline__ long long xcd_item() {
    const unsigned per = gridDim.x / 8;  // the grid is a multiple of 8 blocks
    const unsigned vb = (blockIdx.x % 8) * per + blockIdx.x / 8;
    return (long long)vb * blockDim.x + threadIdx.x;
}

// Work item of a one-wave block (grids of one wave per (image, 64 channels)): the
// items of each XCD are one contiguous range (blocks are dealt to the 8 XCDs
// round-robin), so an image's channel blocks run side by side on one XCD and its
// V / M rows are read and written there together; the identity when the grid is not
// a multiple of 8.
__device__ __forceinline__ unsigned xcd_block() {
    if (gridDim.x % 8) return blockIdx.x;
    return (blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8;
}

// One thread per (tile, 4 channels); tiles image-major, row-major in the image.
// in_bias != null: x is the previous layer's raw output and relu(x + in_bias) is
// applied on load (that layer's bias + ReLU fused here; padding stays 0).
template <int FMT, int HC>
__global__ __launch_bounds__(256) void winograd_in_kernel(const float4* __restrict__ x,
                                                          const float4* __restrict__ in_bias, void* __restrict__ V,
                                                          int H, int pad, int C4, long long B, int* overflow) {
    const WSeq S(HC > 0 ? HC : H + 2 * pad - 2);
    const long long item = xcd_item();
    if (item >= B * S.p * S.p * C4) return;
    const int c4 = (int)(item % C4);
    const long long t = item / C4;
    const int j = (int)(t % S.p);
    const long long r = t / S.p;
    const int i = (int)(r % S.p);
    const long long b = r / S.p;
    const float4 ib = in_bias ? in_bias[c4] : make_float4(0.f, 0.f, 0.f, 0.f);
    const long long row = S.row0(i, j, b, B), ps = S.pstride(i, j, B);
    const int y0 = S.off(i) - pad, x0 = S.off(j) - pad;
    with_types_of<HC>(S.m(i), S.m(j), [&](auto A_, auto B_) {
        constexpr int MA = decltype(A_)::value, MB = decltype(B_)::value;
        float4 d[MA + 2][MB + 2];
#pragma unroll
        for (int u = 0; u < MA + 2; ++u)
#pragma unroll
            for (int v = 0; v < MB + 2; ++v) {
                const int iy = y0 + u, ix = x0 + v;
                float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
                if (iy >= 0 && iy < H && ix >= 0 && ix < H) {
                    z = x[((b * H + iy) * H + ix) * C4 + c4];
                    if (in_bias) z = vrelu(vadd(z, ib));
                }
                d[u][v] = z;
            }
        float4 Vt[MA + 2][MB + 2];
        in_tile<MA, MB>(d, Vt);
#pragma unroll
        for (int e = 0; e < (MA + 2) * (MB + 2); ++e)
            store_v<FMT>(V, row + e * ps, C4, c4, Vt[e / (MB + 2)][e % (MB + 2)], overflow);
    });
}

// FMT = AZG_WINO_F32: y is the NHWC f32 activation.  Otherwise y is one fp16 row
// per image in V format FMT over the image's flattened NHWC activation (width
// Ho * Ho * K): the A operand of a split GEMM over it (the network's fc1).
// With kparts > 1 (split formats) the row is cut into kparts equal chunks stored as
// kparts matrices one after another, [kparts][B][chunk]: the A operands of a split-K
// GEMM whose parts are the split GEMM's "points".
template <int FMT, int HC>
__global__ __launch_bounds__(256) void winograd_out_kernel(const float4* __restrict__ Min,
                                                           const float4* __restrict__ bias, void* __restrict__ y,
                                                           int Ho, int K4, long long B, int relu, float mscale,
                                                           int* overflow, int kparts) {
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
    const long long row = S.row0(i, j, b, B), ps = S.pstride(i, j, B);
    const float4 bb = bias[k4];
    with_types_of<HC>(S.m(i), S.m(j), [&](auto A_, auto B_) {
        constexpr int MA = decltype(A_)::value, MB = decltype(B_)::value;
        float4 m[MA + 2][MB + 2];
#pragma unroll
        for (int e = 0; e < (MA + 2) * (MB + 2); ++e)  // M is read once: nt
            m[e / (MB + 2)][e % (MB + 2)] = vmul(mscale, nt_load4(Min + (row + e * ps) * K4 + k4));
        float4 yt[MA][MB];
        out_tile<MA, MB>(m, yt);
#pragma unroll
        for (int a = 0; a < MA; ++a)
#pragma unroll
            for (int q = 0; q < MB; ++q) {
                const int oy = S.off(i) + a, ox = S.off(j) + q;
                if (oy >= Ho || ox >= Ho) continue;  // h = 1: one 2-tile, cropped
                float4 z = vadd(yt[a][q], bb);
                if (relu) z = vrelu(z);
                if constexpr (FMT == AZG_WINO_F32) {
                    ((float4*)y)[((b * Ho + oy) * Ho + ox) * K4 + k4] = z;
                } else {
                    const int wc4 = Ho * Ho * K4 / kparts, j4 = (oy * Ho + ox) * K4 + k4, e = j4 / wc4;
                    store_v<FMT>(y, e * B + b, wc4, j4 - e * wc4, z, overflow);
                }
            }
    });
}

// A lane's private h x h plane: in registers when the side is a compile-time
// HC (loops fully unrolled, every index constant), else in its own LDS column.
template <int HC>
struct Plane {
    float r[HC > 0 ? HC * HC : 1];
    float* lds;
    int lane;
    __device__ __forceinline__ void put(int i, float v) {
        if constexpr (HC > 0) r[i] = v;
        else lds[i * 64 + lane] = v;
    }
    __device__ __forceinline__ float get(int i) const {
        if constexpr (HC > 0) return r[i];
        else return lds[i * 64 + lane];
    }
};

// The next layer's input transform (pad PAD) of the lane's h x h plane: V out.  The
// wave's lanes hold channels c0 + lane (c0 wave-uniform, a multiple of 64).  only_row >= 0:
// only the tiles of that tile row (wave-uniform; the caller's waves split the rows).
template <int HC, int FMT, int PAD, bool NT = false, class P>
__device__ __forceinline__ void plane_to_V(const P& ys, int h_rt, long long b, int c0, unsigned lane, int C,
                                           long long B, void* __restrict__ Vout, int* overflow,
                                           int only_row = -1) {
    const int h = HC > 0 ? HC : h_rt;
    const int c = c0 + (int)lane;
    const WSeq S(h + 2 * PAD - 2);
    constexpr int HO = HC > 0 ? HC + 2 * PAD - 2 : 0;
    bool bad = false;
    for_tiles<HO>(S, [&](auto A_, auto B_, int i, int j) {
        constexpr int MA = decltype(A_)::value, MB = decltype(B_)::value;
        if (only_row >= 0 && i != only_row) return;
        const long long row = S.row0(i, j, b, B), ps = S.pstride(i, j, B);
        const int y0 = S.off(i) - PAD, x0 = S.off(j) - PAD;
        float d[MA + 2][MB + 2];
#pragma unroll
        for (int u = 0; u < MA + 2; ++u)
#pragma unroll
            for (int v = 0; v < MB + 2; ++v) {
                const int iy = y0 + u, ix = x0 + v;
                d[u][v] = (iy >= 0 && iy < h && ix >= 0 && ix < h) ? ys.get(iy * h + ix) : 0.f;
            }
        float Vt[MA + 2][MB + 2];
        in_tile<MA, MB>(d, Vt);
#pragma unroll
        for (int e = 0; e < (MA + 2) * (MB + 2); ++e) {
            if constexpr (FMT == AZG_WINO_SPLIT2)
                bad |= store_v2_wave<NT>((unsigned short*)Vout + (row + e * ps) * 2 * C + 2 * c0, lane,
                                     Vt[e / (MB + 2)][e % (MB + 2)]);
            else
                store_v<FMT>(Vout, row + e * ps, C, c, Vt[e / (MB + 2)][e % (MB + 2)], overflow);
        }
    });
    if (bad) atomicOr(overflow, 1);
}

// Layer i's output transform fused with layer i+1's input transform (pad 0
// between them, as conv2->conv3->conv4): one wave per (image, 64 channels),
// each lane owning one channel.  The lane's h x h output plane of layer i
// (bias + ReLU applied) is kept in registers (compile-time side HC) or its own
// LDS column -- only that lane reads it back, so no barrier -- and the next
// layer's tiles are transformed from it: layer i's activation never goes to HBM.
template <int HC, int FMT, int WPB = 1>
__global__ __launch_bounds__(64 * WPB) void winograd_mid_kernel(const float* __restrict__ Min,
                                                                const float* __restrict__ bias,
                                                                void* __restrict__ Vout, int h_rt, int C, long long B,
                                                                float mscale, int* overflow) {
    extern __shared__ float ys_raw[];  // [h * h][64] when HC == 0
    static_assert(WPB == 1 || HC > 0, "several items per block: register planes only");
    const int h = HC > 0 ? HC : h_rt;
    const unsigned lane = threadIdx.x & 63u;
    const int cblocks = C / 64;
    // WPB waves per block, one (image, 64 channels) item each, adjacent items
    const unsigned blk = xcd_block() * WPB + (WPB > 1 ? (unsigned)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0u);
    const long long b = blk / cblocks;
    const int c0 = (blk % cblocks) * 64, c = c0 + (int)lane;
    const float bc = bias[c];
    const WSeq S(h);
    Plane<HC> ys;
    ys.lds = ys_raw;
    ys.lane = lane;
    for_tiles<HC>(S, [&](auto A_, auto B_, int i, int j) {
        constexpr int MA = decltype(A_)::value, MB = decltype(B_)::value;
        const long long row = S.row0(i, j, b, B), ps = S.pstride(i, j, B);
        const int y0 = S.off(i), x0 = S.off(j);
        float mm[MA + 2][MB + 2];
#pragma unroll
        for (int e = 0; e < (MA + 2) * (MB + 2); ++e)  // uniform row base + lane; M is read once: nt
            mm[e / (MB + 2)][e % (MB + 2)] = mscale * __builtin_nontemporal_load(Min + (row + e * ps) * C + c0 + lane);
        float y[MA][MB];
        out_tile<MA, MB>(mm, y);
#pragma unroll
        for (int a = 0; a < MA; ++a)
#pragma unroll
            for (int q = 0; q < MB; ++q)
                if (y0 + a < h && x0 + q < h) ys.put((y0 + a) * h + x0 + q, fmaxf(y[a][q] + bc, 0.f));
    });
    plane_to_V<HC, FMT, 0>(ys, h, b, c0, lane, C, B, Vout, overflow);
}

// The network's first two layers' front end in one pass: conv1 (depth -> C
// channels, 3x3, pad 1) + bias + ReLU computed directly from the NCHW leaf
// planes, then conv2's Winograd input transform (pad 1) -- conv1's activation
// never leaves the chip.  One wave per (image, 64 output channels of conv1,
// tile row part of ROWS), one channel per lane: with a compile-time side NC the
// planes are read as wave-uniform scalars and conv1 runs as conv1_sparse, the
// lane's output plane in registers; otherwise the image's planes are shared
// through LDS and each output is gathered, the plane in the lane's own LDS column.
// ROWS = 2 (the boards' two tile rows): two waves per (image, channels), each
// computing conv1 whole and storing one tile row's V: twice the (cheap, sparse)
// conv1 work for half the stores per wave, measured 204 -> 175 us at 4096 leaves
// and 18.8 -> 17.7 us at 256 (tools/first_probe.py, HISTORY.md 6b).
template <int NC, int FMT, int ROWS = 1>
__global__ __launch_bounds__(64) void winograd_first_kernel(const float* __restrict__ planes,
                                                            const float* __restrict__ w1,
                                                            const float* __restrict__ b1, void* __restrict__ Vout,
                                                            int depth, int n_rt, int C, long long B, int* overflow) {
    constexpr int DMAX = 4;
    extern __shared__ float lds[];
    const int n = NC > 0 ? NC : n_rt;
    const unsigned lane = threadIdx.x;
    const int cblocks = C / 64;
    // (blocks in dispatch order: the XCD-contiguous mapping of the mid kernels measured
    // 7% slower here, where nothing is read back; a (image, channels) item's ROWS waves adjacent)
    const unsigned item = blockIdx.x / ROWS;
    const int part = ROWS > 1 ? (int)(blockIdx.x % ROWS) : -1;
    const long long b = item / cblocks;
    const int k0 = (item % cblocks) * 64, k = k0 + (int)lane;
    const float bk = b1[k];
    Plane<NC> ys;
    if constexpr (NC > 0) {
        float acc[NC * NC];
        conv1_sparse<NC>(planes + b * depth * NC * NC, w1 + (size_t)k * depth * 9, depth, lane, acc);
#pragma unroll
        for (int q = 0; q < NC * NC; ++q) ys.put(q, fmaxf(acc[q] + bk, 0.f));
    } else {
        float* xs = lds;  // [depth][n][n], then the lanes' planes [n * n][64]
        for (int i = lane; i < depth * n * n; i += 64) xs[i] = planes[b * depth * n * n + i];
        float w[DMAX * 9];
#pragma unroll
        for (int j = 0; j < DMAX * 9; ++j) w[j] = j < depth * 9 ? w1[(size_t)k * depth * 9 + j] : 0.f;
        __syncthreads();
        ys.lds = lds + DMAX * 81;
        ys.lane = lane;
        for (int y = 0; y < n; ++y)
            for (int x = 0; x < n; ++x) {
                float acc = 0.f;
#pragma unroll
                for (int c = 0; c < DMAX; ++c) {
                    if (c >= depth) break;
#pragma unroll
                    for (int dy = 0; dy < 3; ++dy) {
                        const int iy = y + dy - 1;
                        if (iy < 0 || iy >= n) continue;
#pragma unroll
                        for (int dx = 0; dx < 3; ++dx) {
                            const int ix = x + dx - 1;
                            if (ix < 0 || ix >= n) continue;
                            acc = fmaf(w[c * 9 + dy * 3 + dx], xs[(c * n + iy) * n + ix], acc);
                        }
                    }
                }
                ys.put(y * n + x, fmaxf(acc + bk, 0.f));
            }
    }
    // V2 goes out with non-temporal stores: nothing here reads it back, and the GEMM
    // reads it only after the whole grid (241 -> 209 us at 4096 leaves, HISTORY.md 6b,
    // profiles/r02_nt_store_probe)
    plane_to_V<NC, FMT, 1, true>(ys, n, b, k0, lane, C, B, Vout, overflow, part);
}

// one thread per work item, rounded up to whole groups of 8 blocks (xcd_item)
inline unsigned grid_for(long long n) {
    const long long blocks = (n + 255) / 256;
    return (unsigned)(((blocks + 7) / 8) * 8);
}

// winograd_out_kernel for the output sides of the supported boards (compile-time
// tile types) or any side (all types)
inline int launch_out(int vfmt, const float* M, const float* bias, void* y, int batch, int h_out, int k, int relu,
               float mscale, int* overflow, int kparts, void* stream) {
    const WSeq S(h_out);
    const dim3 grid(grid_for((long long)batch * S.p * S.p * (k / 4)));
    hipStream_t st = (hipStream_t)stream;
    auto launch = [&](auto F_, auto H_) {
        hipLaunchKernelGGL((winograd_out_kernel<decltype(F_)::value, decltype(H_)::value>), grid, dim3(256), 0, st,
                           (const float4*)M, (const float4*)bias, y, h_out, k / 4, (long long)batch, relu, mscale,
                           overflow, kparts);
    };
    auto by_side = [&](auto F_) {
        switch (h_out) {
            case 2: launch(F_, IC<2>{}); break;
            case 3: launch(F_, IC<3>{}); break;
            case 4: launch(F_, IC<4>{}); break;
            case 5: launch(F_, IC<5>{}); break;
            default: launch(F_, IC<0>{});
        }
    };
    if (vfmt == AZG_WINO_F32) by_side(IC<AZG_WINO_F32>{});
    if (vfmt == AZG_WINO_SPLIT) by_side(IC<AZG_WINO_SPLIT>{});
    if (vfmt == AZG_WINO_SPLIT2) by_side(IC<AZG_WINO_SPLIT2>{});
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

inline bool bad_fmt(int vfmt, const int* overflow) {
    return !(vfmt == AZG_WINO_F32 ||
             ((vfmt == AZG_WINO_SPLIT || vfmt == AZG_WINO_SPLIT2) && azg_device_writable(overflow)));
}
}  // namespace
