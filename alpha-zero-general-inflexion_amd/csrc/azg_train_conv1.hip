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
//  * c1_fwd_row_kernel<D, N> / c1_wgrad_row_kernel<D, N> (round 6; the boards' D in {2, 4} and
//    N in {6, 7, 8}): the same block decomposition, but a wave takes whole output rows: the row's
//    3 x (N + 2) x D inputs are read from LDS once (D-wide vector reads of one broadcast address)
//    into registers and feed all N outputs of the row, instead of 9 D LDS reads per output -- the
//    per-pixel kernels were LDS-issue-bound (62 / 58 us per step at B = 512, 0.8 TB/s on y / dy;
//    profiles/r06_prof_train_probe*.md).  The forward keeps the per-pixel kernel's summation order
//    (taps in (c, r, s) order, then the bias): bit-identical y.
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

// the padded input rows oy .. oy + 2 of one staged image into registers (uniform across lanes)
template <int D, int N>
__device__ __forceinline__ void c1_row_inputs(const float* xb, int oy, float (&xr)[3][N + 2][D]) {
    constexpr int PN = N + 2;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int cx = 0; cx < PN; ++cx) {
            const float* src = xb + ((oy + r) * PN + cx) * D;
            if constexpr (D == 4) {
                const float4 v = *reinterpret_cast<const float4*>(src);
                xr[r][cx][0] = v.x, xr[r][cx][1] = v.y, xr[r][cx][2] = v.z, xr[r][cx][3] = v.w;
            } else if constexpr (D == 2) {
                const float2 v = *reinterpret_cast<const float2*>(src);
                xr[r][cx][0] = v.x, xr[r][cx][1] = v.y;
            } else {
#pragma unroll
                for (int c = 0; c < D; ++c) xr[r][cx][c] = src[c];
            }
        }
}

constexpr int C1_RIMG = 8;  // images per block of the row kernels

template <int D, int N>
__global__ __launch_bounds__(C1_T) void c1_fwd_row_kernel(const float* __restrict__ x, long long B,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ bias, int K,
                                                          float* __restrict__ y) {
    constexpr int PN = N + 2, HW = N * N;
    __shared__ __attribute__((aligned(16))) float xs[C1_RIMG * PN * PN * D];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int k = blockIdx.x * 64 + lane;
    const long long b0 = (long long)blockIdx.y * C1_RIMG;
    const int nimg = (int)min((long long)C1_RIMG, B - b0);
    float wr[9 * D];
#pragma unroll
    for (int j = 0; j < 9 * D; ++j) wr[j] = w[(long long)k * 9 * D + j];  // [c][r][s]
    const float bk = bias ? bias[k] : 0.f;
    c1_stage<D>(x, xs, b0, nimg, N);
    __syncthreads();
    for (int it = wv; it < nimg * N; it += C1_T / 64) {
        const int img = it / N, oy = it - img * N;
        float xr[3][PN][D];
        c1_row_inputs<D, N>(xs + img * PN * PN * D, oy, xr);
        float acc[N];
#pragma unroll
        for (int ox = 0; ox < N; ++ox) acc[ox] = 0.f;
#pragma unroll
        for (int c = 0; c < D; ++c)
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int s = 0; s < 3; ++s)
#pragma unroll
                    for (int ox = 0; ox < N; ++ox) acc[ox] = fmaf(wr[c * 9 + r * 3 + s], xr[r][ox + s][c], acc[ox]);
        float* yr = y + ((b0 + img) * HW + (long long)oy * N) * K + k;
#pragma unroll
        for (int ox = 0; ox < N; ++ox) yr[(long long)ox * K] = acc[ox] + bk;
    }
}

template <int D, int N>
__global__ __launch_bounds__(C1_T) void c1_wgrad_row_kernel(const float* __restrict__ x,
                                                            const float* __restrict__ dy, long long B, int K,
                                                            long long per_chunk, double* __restrict__ work) {
    constexpr int J = 9 * D + 1, PN = N + 2, HW = N * N;
    __shared__ __attribute__((aligned(16))) float xs[C1_RIMG * PN * PN * D];
    __shared__ float red[4][J][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int k = blockIdx.x * 64 + lane;
    const long long c0 = (long long)blockIdx.y * per_chunk, c1 = min(B, c0 + per_chunk);
    float acc[J];
#pragma unroll
    for (int j = 0; j < J; ++j) acc[j] = 0.f;
    for (long long b0 = c0; b0 < c1; b0 += C1_RIMG) {
        const int nimg = (int)min((long long)C1_RIMG, c1 - b0);
        __syncthreads();  // (the previous group's reads of xs are done)
        c1_stage<D>(x, xs, b0, nimg, N);
        __syncthreads();
        for (int it = wv; it < nimg * N; it += C1_T / 64) {
            const int img = it / N, oy = it - img * N;
            const float* gr = dy + ((b0 + img) * HW + (long long)oy * N) * K + k;
            float g[N];
#pragma unroll
            for (int ox = 0; ox < N; ++ox) g[ox] = gr[(long long)ox * K];
            float xr[3][PN][D];
            c1_row_inputs<D, N>(xs + img * PN * PN * D, oy, xr);
#pragma unroll
            for (int c = 0; c < D; ++c)
#pragma unroll
                for (int r = 0; r < 3; ++r)
#pragma unroll
                    for (int s = 0; s < 3; ++s)
#pragma unroll
                        for (int ox = 0; ox < N; ++ox)
                            acc[c * 9 + r * 3 + s] = fmaf(g[ox], xr[r][ox + s][c], acc[c * 9 + r * 3 + s]);
#pragma unroll
            for (int ox = 0; ox < N; ++ox) acc[J - 1] += g[ox];
        }
    }
#pragma unroll
    for (int j = 0; j < J; ++j) red[wv][j][lane] = acc[j];
    __syncthreads();
    for (int i = threadIdx.x; i < J * 64; i += C1_T) {
        const int j = i / 64, l = i - j * 64;
        const double sum = (((double)red[0][j][l] + red[1][j][l]) + red[2][j][l]) + red[3][j][l];  // wave order
        work[((long long)blockIdx.y * K + blockIdx.x * 64 + l) * J + j] = sum;
    }
}

// the row kernels for the boards' shapes; false: use the per-pixel kernels
template <int D>
bool c1_row_fwd(int n, const float* x, long long B, const float* w, const float* b, int K, float* y, hipStream_t st) {
    const dim3 grid(K / 64, (unsigned)((B + C1_RIMG - 1) / C1_RIMG));
    switch (n) {
        case 6: hipLaunchKernelGGL((c1_fwd_row_kernel<D, 6>), grid, dim3(C1_T), 0, st, x, B, w, b, K, y); return true;
        case 7: hipLaunchKernelGGL((c1_fwd_row_kernel<D, 7>), grid, dim3(C1_T), 0, st, x, B, w, b, K, y); return true;
        case 8: hipLaunchKernelGGL((c1_fwd_row_kernel<D, 8>), grid, dim3(C1_T), 0, st, x, B, w, b, K, y); return true;
        default: return false;
    }
}

template <int D>
bool c1_row_wgrad(int n, const float* x, const float* dy, long long B, int K, long long per, int chunks,
                  double* work, hipStream_t st) {
    const dim3 grid(K / 64, chunks);
    switch (n) {
        case 6: hipLaunchKernelGGL((c1_wgrad_row_kernel<D, 6>), grid, dim3(C1_T), 0, st, x, dy, B, K, per, work); return true;
        case 7: hipLaunchKernelGGL((c1_wgrad_row_kernel<D, 7>), grid, dim3(C1_T), 0, st, x, dy, B, K, per, work); return true;
        case 8: hipLaunchKernelGGL((c1_wgrad_row_kernel<D, 8>), grid, dim3(C1_T), 0, st, x, dy, B, K, per, work); return true;
        default: return false;
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
    hipStream_t st = (hipStream_t)stream;
    const bool row = depth == 4   ? c1_row_fwd<4>(n, x, (long long)batch, w, bias, (int)K, y, st)
                     : depth == 2 ? c1_row_fwd<2>(n, x, (long long)batch, w, bias, (int)K, y, st)
                                  : false;
    if (!row && !c1_dispatch<Fwd>(depth, x, (long long)batch, (int)n, w, bias, (int)K, y, st)) return AZG_ERR_ARG;
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_conv1_train_wgrad(const float* x, const float* dy, int64_t batch, int32_t depth, int32_t n,
                                     int32_t K, float* dw, float* db, double* work, void* stream) {
    if (!c1_args_ok(x, batch, depth, n, K) || !dy || !dw || !work) return AZG_ERR_ARG;
    const int chunks = (int)(batch < C1_CHUNKS ? batch : C1_CHUNKS);
    const long long per = (batch + chunks - 1) / chunks;
    const int used = (int)((batch + per - 1) / per);  // chunks with at least one image
    hipStream_t st = (hipStream_t)stream;
    const bool row = depth == 4   ? c1_row_wgrad<4>(n, x, dy, (long long)batch, (int)K, per, used, work, st)
                     : depth == 2 ? c1_row_wgrad<2>(n, x, dy, (long long)batch, (int)K, per, used, work, st)
                                  : false;
    if (!row && !c1_dispatch<Wgrad>(depth, x, dy, (long long)batch, (int)n, (int)K, per, used, work, st))
        return AZG_ERR_ARG;
    const int J = 9 * depth + 1;
    hipLaunchKernelGGL(c1_wgrad_finish_kernel, dim3((unsigned)((K * J + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, work, used, (int)K, J, dw, db);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}
