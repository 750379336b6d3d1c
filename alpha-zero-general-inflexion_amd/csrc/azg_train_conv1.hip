// azg_train_conv1.hip -- conv1 of the trainer (InflexionNNet.py:39, nn.Conv2d(depth, C, 3, stride 1,
// padding 1) on the board planes) forward and weight / bias gradients, so no training step reaches
// MIOpen: its conv1 kernels were compiled on a fresh process's first step (2.2 s of the first
// train_examples call, tools/train_first_use.py; bench.py's learn iteration measured 14.8 s as a
// box's first process against 12.3 s as its second) and took ~70 us per step after that.
//
// Shapes: x NHWC [B][n][n][D] (the planes in channels_last), w [K][D][3][3] (torch's layout),
// y NHWC [B][n][n][K]; D <= 8, n <= 8, K % 64 == 0.  The planes never need a gradient, so
// the backward is dw and db only.
//
//  * c1_fwd_kernel<D>: block = 64 output channels (one per lane, its 9 D weights in registers)
//    x C1_IMG images (staged zero-padded in LDS), 4 waves dealing the images' pixels; each
//    output is bias + the 9 D products (taps in (c, r, s) order), written as one 256-B row
//    segment per wave instruction.  HBM-bound on y (B x n^2 x K x 4 B).
//  * c1_wgrad_kernel<D>: block = 64 channels x one chunk of images; each lane accumulates its
//    channel's 9 D + 1 sums (weights, bias) in f32 over its wave's pixels (dy read once,
//    coalesced; ~100 terms a lane at B = 512), the 4 waves' partials are added in f64 in wave
//    order into work[chunk][K][9 D + 1]; c1_wgrad_finish_kernel sums the chunks in order in f64.
//    Fixed summation order (deterministic).
#include <hip/hip_runtime.h>

#include "../../include/azg.h"

namespace {

constexpr int C1_T = 256;       // threads (4 waves)
constexpr int C1_IMG = 4;       // images per forward block
constexpr int C1_CHUNKS = 64;   // image chunks of the weight gradient (work rows)
constexpr int C1_NMAX = 8;      // board side
constexpr int C1_DMAX = 8;      // input planes
constexpr int C1_PADN = C1_NMAX + 2;

// stage images [b0, b0 + nimg) zero-padded: xs[img][(iy + 1) * (n + 2) + ix + 1][D]
template <int D>
__device__ __forceinline__ void c1_stage(const float* __restrict__ x, float* xs, long long b0, int nimg, int n) {
    const int pn = n + 2, per = pn * pn * D;
    for (int i = threadIdx.x; i < nimg * per; i += C1_T) {
        const int img = i / per, r = i - img * per, pix = r / D, c = r - pix * D;
        const int py = pix / pn, px = pix - py * pn, iy = py - 1, ix = px - 1;
        xs[i] = (iy >= 0 && iy < n && ix >= 0 && ix < n) ? x[(((b0 + img) * n + iy) * n + ix) * D + c] : 0.f;
    }
}

template <int D>
__global__ __launch_bounds__(C1_T) void c1_fwd_kernel(const float* __restrict__ x, long long B, int n,
                                                      const float* __restrict__ w, const float* __restrict__ bias,
                                                      int K, float* __restrict__ y) {
    __shared__ __attribute__((aligned(16))) float xs[C1_IMG * C1_PADN * C1_PADN * D];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int k = blockIdx.x * 64 + lane;
    const long long b0 = (long long)blockIdx.y * C1_IMG;
    const int nimg = (int)min((long long)C1_IMG, B - b0);
    float wr[9 * D];
#pragma unroll
    for (int j = 0; j < 9 * D; ++j) wr[j] = w[(long long)k * 9 * D + j];  // [c][r][s]
    const float bk = bias ? bias[k] : 0.f;
    c1_stage<D>(x, xs, b0, nimg, n);
    __syncthreads();
    const int pn = n + 2, hw = n * n;
    for (int it = wv; it < nimg * hw; it += C1_T / 64) {
        const int img = it / hw, p = it - img * hw, oy = p / n, ox = p - oy * n;
        const float* xb = xs + img * pn * pn * D;
        float acc = 0.f;
#pragma unroll
        for (int c = 0; c < D; ++c)
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int s = 0; s < 3; ++s) acc = fmaf(wr[c * 9 + r * 3 + s], xb[((oy + r) * pn + ox + s) * D + c], acc);
        y[((b0 + img) * hw + p) * K + k] = acc + bk;
    }
}

template <int D>
__global__ __launch_bounds__(C1_T) void c1_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                        long long B, int n, int K, long long per_chunk,
                                                        double* __restrict__ work) {
    constexpr int J = 9 * D + 1;
    __shared__ __attribute__((aligned(16))) float xs[C1_IMG * 2 * C1_PADN * C1_PADN * D];  // 8 images at a time
    __shared__ float red[4][J][64];
    constexpr int SIMG = C1_IMG * 2;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int k = blockIdx.x * 64 + lane;
    const long long c0 = (long long)blockIdx.y * per_chunk, c1 = min(B, c0 + per_chunk);
    float acc[J];
#pragma unroll
    for (int j = 0; j < J; ++j) acc[j] = 0.f;
    const int pn = n + 2, hw = n * n;
    for (long long b0 = c0; b0 < c1; b0 += SIMG) {
        const int nimg = (int)min((long long)SIMG, c1 - b0);
        __syncthreads();  // (the previous group's reads of xs are done)
        c1_stage<D>(x, xs, b0, nimg, n);
        __syncthreads();
        for (int it = wv; it < nimg * hw; it += C1_T / 64) {
            const int img = it / hw, p = it - img * hw, oy = p / n, ox = p - oy * n;
            const float g = dy[((b0 + img) * hw + p) * K + k];
            const float* xb = xs + img * pn * pn * D;
#pragma unroll
            for (int c = 0; c < D; ++c)
#pragma unroll
                for (int r = 0; r < 3; ++r)
#pragma unroll
                    for (int s = 0; s < 3; ++s)
                        acc[c * 9 + r * 3 + s] = fmaf(g, xb[((oy + r) * pn + ox + s) * D + c], acc[c * 9 + r * 3 + s]);
            acc[J - 1] += g;
        }
    }
#pragma unroll
    for (int j = 0; j < J; ++j) red[wv][j][lane] = acc[j];
    __syncthreads();
    for (int i = threadIdx.x; i < J * 64; i += C1_T) {
        const int j = i / 64, l = i - j * 64;
        const double s = (((double)red[0][j][l] + red[1][j][l]) + red[2][j][l]) + red[3][j][l];  // wave order
        work[((long long)blockIdx.y * K + blockIdx.x * 64 + l) * J + j] = s;
    }
}

// dw[k][j] / db[k] = the chunks' partials summed in chunk order (f64), one thread per (k, j)
__global__ __launch_bounds__(256) void c1_wgrad_finish_kernel(const double* __restrict__ work, int chunks, int K,
                                                              int J, float* __restrict__ dw, float* __restrict__ db) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= K * J) return;
    const int k = i / J, j = i - k * J;
    double s = 0.0;
    for (int q = 0; q < chunks; ++q) s += work[((long long)q * K + k) * J + j];
    if (j < J - 1)
        dw[(long long)k * (J - 1) + j] = (float)s;
    else if (db)
        db[k] = (float)s;
}

template <template <int> class F, class... A>
bool c1_dispatch(int D, A... a) {
    switch (D) {
        case 1: F<1>::run(a...); return true;
        case 2: F<2>::run(a...); return true;
        case 3: F<3>::run(a...); return true;
        case 4: F<4>::run(a...); return true;
        case 5: F<5>::run(a...); return true;
        case 6: F<6>::run(a...); return true;
        case 7: F<7>::run(a...); return true;
        case 8: F<8>::run(a...); return true;
        default: return false;
    }
}

template <int D>
struct Fwd {
    static void run(const float* x, long long B, int n, const float* w, const float* b, int K, float* y,
                    hipStream_t st) {
        hipLaunchKernelGGL(c1_fwd_kernel<D>, dim3(K / 64, (unsigned)((B + C1_IMG - 1) / C1_IMG)), dim3(C1_T), 0, st,
                           x, B, n, w, b, K, y);
    }
};

template <int D>
struct Wgrad {
    static void run(const float* x, const float* dy, long long B, int n, int K, long long per, int chunks,
                    double* work, hipStream_t st) {
        hipLaunchKernelGGL(c1_wgrad_kernel<D>, dim3(K / 64, chunks), dim3(C1_T), 0, st, x, dy, B, n, K, per, work);
    }
};

bool c1_args_ok(const float* x, int64_t batch, int32_t depth, int32_t n, int32_t K) {
    // (the forward's grid.y = batch / C1_IMG stays within the 65535 a launch dimension allows)
    return x && batch > 0 && depth >= 1 && depth <= C1_DMAX && n >= 1 && n <= C1_NMAX && K > 0 && K % 64 == 0 &&
           batch <= (int64_t)65535 * C1_IMG;
}

}  // namespace

extern "C" int azg_conv1_train_fwd(const float* x, int64_t batch, int32_t depth, int32_t n, const float* w,
                                   const float* bias, int32_t K, float* y, void* stream) {
    if (!c1_args_ok(x, batch, depth, n, K) || !w || !y) return AZG_ERR_ARG;
    if (!c1_dispatch<Fwd>(depth, x, (long long)batch, (int)n, w, bias, (int)K, y, (hipStream_t)stream))
        return AZG_ERR_ARG;
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_conv1_train_wgrad(const float* x, const float* dy, int64_t batch, int32_t depth, int32_t n,
                                     int32_t K, float* dw, float* db, double* work, void* stream) {
    if (!c1_args_ok(x, batch, depth, n, K) || !dy || !dw || !work) return AZG_ERR_ARG;
    const int chunks = (int)(batch < C1_CHUNKS ? batch : C1_CHUNKS);
    const long long per = (batch + chunks - 1) / chunks;
    const int used = (int)((batch + per - 1) / per);  // chunks with at least one image
    if (!c1_dispatch<Wgrad>(depth, x, dy, (long long)batch, (int)n, (int)K, per, used, work, (hipStream_t)stream))
        return AZG_ERR_ARG;
    const int J = 9 * depth + 1;
    hipLaunchKernelGGL(c1_wgrad_finish_kernel, dim3((unsigned)((K * J + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, work, used, (int)K, J, dw, db);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}
