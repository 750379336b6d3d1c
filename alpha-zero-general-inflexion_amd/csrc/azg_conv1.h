// azg_conv1.h -- the leaf network's conv1 for one image and one output channel per lane,
// shared by winograd_first_kernel (azg_winograd_kern.h) and the small-batch conv12 kernel
// (azg_small.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace {

// conv1 of one image for the lane's output channel k into acc[NC * NC] (no bias),
// compile-time side NC, the image's planes read as wave-uniform scalars (every lane
// reads the same cells).  Exact restructuring of the 3x3 zero-padded convolution
// (InflexionNNet.py:39, conv1) for leaf planes, which are mostly constant planes and
// sparse 0/1 planes (InflexionGame.py:84-91: turn and can_spawn planes are constant,
// own/opponent planes disjoint): per input plane c,
//   * constant value x (all cells equal): out(y, x') += x * S_c(class(y), class(x')),
//     S_c the sum of the taps that stay inside the board for that border class
//     (first / inner / last row and column) -- one multiply-add per output;
//   * otherwise: each nonzero input cell adds w[dy][dx] * x to the <= 9 outputs it
//     reaches (a zero cell contributes exactly nothing: skipped on a uniform branch).
// Any plane values are handled; only the work depends on them (at most 361 multiply-
// adds per plane, as the gather).  The sums are in a different order than the gather.
// Weight of plane c, tap t: wk[c * wsc + t * wst] (NCHW weights: 9, 1; channels_last: 1, depth).
template <int NC>
__device__ __forceinline__ void conv1_sparse(const float* __restrict__ pb, const float* __restrict__ wk, int depth,
                                             unsigned lane, float (&acc)[NC * NC], int wsc = 9, int wst = 1) {
    constexpr int DMAX = 4, NN = NC * NC;
#pragma unroll
    for (int q = 0; q < NN; ++q) acc[q] = 0.f;
#pragma unroll
    for (int c = 0; c < DMAX; ++c) {
        if (c >= depth) break;
        const float* __restrict__ pc = pb + c * NN;
        float w[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) w[t] = wk[c * wsc + t * wst];
        const float x0 = pc[0];
        const bool cst = __all(pc[lane < NN ? lane : 0] == x0);
        if (cst) {
            if (x0 != 0.f) {
                // row sums of the taps valid in each column class, then the 3x3 classes
                float rs[3][3];  // [dy][column class]
#pragma unroll
                for (int dy = 0; dy < 3; ++dy) {
                    rs[dy][0] = w[dy * 3 + 1] + w[dy * 3 + 2];  // first column: dx = 0 falls outside
                    rs[dy][1] = w[dy * 3 + 0] + w[dy * 3 + 1] + w[dy * 3 + 2];
                    rs[dy][2] = w[dy * 3 + 0] + w[dy * 3 + 1];  // last column
                }
                float S[3][3];  // [row class][column class]
#pragma unroll
                for (int cx = 0; cx < 3; ++cx) {
                    S[0][cx] = rs[1][cx] + rs[2][cx];
                    S[1][cx] = rs[0][cx] + rs[1][cx] + rs[2][cx];
                    S[2][cx] = rs[0][cx] + rs[1][cx];
                }
#pragma unroll
                for (int y = 0; y < NC; ++y)
#pragma unroll
                    for (int x = 0; x < NC; ++x) {
                        const int cy = y == 0 ? 0 : (y == NC - 1 ? 2 : 1), cx = x == 0 ? 0 : (x == NC - 1 ? 2 : 1);
                        acc[y * NC + x] = fmaf(x0, S[cy][cx], acc[y * NC + x]);
                    }
            }
        } else {
            unsigned xb[NN];  // the plane's bits, wave-uniform (scalar loads, issued together)
#pragma unroll
            for (int q = 0; q < NN; ++q) xb[q] = __builtin_amdgcn_readfirstlane(__float_as_uint(pc[q]));
#pragma unroll
            for (int q = 0; q < NN; ++q) {
                const float xq = __uint_as_float(xb[q]);
                if (xb[q] << 1) {  // nonzero (either zero skips)
                    asm volatile("");  // a real (uniform) branch, not a select over the multiply-adds
                    const int iy = q / NC, ix = q % NC;
#pragma unroll
                    for (int dy = 0; dy < 3; ++dy) {
                        const int oy = iy - dy + 1;
                        if (oy < 0 || oy >= NC) continue;
#pragma unroll
                        for (int dx = 0; dx < 3; ++dx) {
                            const int ox = ix - dx + 1;
                            if (ox < 0 || ox >= NC) continue;
                            acc[oy * NC + ox] = fmaf(w[dy * 3 + dx], xq, acc[oy * NC + ox]);
                        }
                    }
                }
            }
        }
    }
}

}  // namespace
