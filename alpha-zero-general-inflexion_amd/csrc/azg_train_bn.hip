// azg_train_bn.hip -- the trainer's BatchNorm2d + ReLU (InflexionNNet.py:39-45:
// relu(bn_i(conv_i(x))), training mode) on channels-last activations, forward and backward.
//
// torch hands channels-last BatchNorm to MIOpen's NHWC kernels, which ran at ~1.3 TB/s on the
// trainer's 512 x 512 x 7 x 7 activations (BwdSpatialDX + BwdSpatialDScaleDBias 116 + 115 us,
// FwdTrainSpatialNorm 84 us per layer and step; profiles/r05_prof_train_probe_wino.md).  Here x is
// [rows][C] (rows = batch x H x W, the channels contiguous) and every pass streams it with float4
// loads:
//
//   forward   stats  : per channel sum x, sum x^2 over the rows (f64, block partials reduced in a
//                      fixed order), mean, biased var, invstd = 1/sqrt(var + eps); scale = gamma
//                      invstd; running stats (momentum, unbiased var)
//             apply  : y = max((x - mean) scale + beta, 0)
//   backward  reduce : g = dy where (x - mean) scale + beta > 0 (the forward's own f32 expression, so the
//                      same mask), per channel sum g and sum g xhat, xhat = (x - mean) invstd (f64)
//             apply  : dx = scale (g - sum g / n - xhat sum(g xhat) / n); dgamma = sum g xhat,
//                      dbeta = sum g
//
// Deterministic (fixed partial and butterfly order).  Tolerance-equal to torch's f32 BatchNorm (the sums are
// f64 here); the trainer's tests bound the whole step against the reference trainer.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/azg.h"

namespace {

constexpr int BN_T = 256;       // threads per block
constexpr int BN_PARTS = 512;   // row ranges (blocks) of the reductions

// per block: channel quad q = t % C4 of rows r = row0 + t / C4 + k (T / C4) for k >= 0
template <class F>
__device__ __forceinline__ void rows_of_block(long long rows, int C4, F&& f) {
    const int lanes = BN_T / C4;  // row lanes per block (C4 <= BN_T)
    const int q = threadIdx.x % C4, l = threadIdx.x / C4;
    if (l >= lanes) return;
    const long long per = (rows + gridDim.x - 1) / gridDim.x;
    const long long r0 = (long long)blockIdx.x * per, r1 = r0 + per < rows ? r0 + per : rows;
#pragma unroll 4
    for (long long r = r0 + l; r < r1; r += lanes) f(r, q);
}

// the block's row lanes' f64 quads summed in lane order -> part[blockIdx][which][4 q .. 4 q + 3]
__device__ __forceinline__ void block_sum_store(double (&a)[8], int C4, double* __restrict__ part) {
    __shared__ double red[BN_T][9];  // (padded: 9 doubles per thread)
    const int lanes = BN_T / C4, q = threadIdx.x % C4, l = threadIdx.x / C4;
#pragma unroll
    for (int i = 0; i < 8; ++i) red[threadIdx.x][i] = a[i];
    __syncthreads();
    if (l == 0) {
        for (int k = 1; k < lanes; ++k)
#pragma unroll
            for (int i = 0; i < 8; ++i) a[i] += red[k * C4 + q][i];
        double* p = part + (long long)blockIdx.x * 8 * C4;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            p[4 * q + i] = a[i];           // [0, C): first sums
            p[4 * C4 + 4 * q + i] = a[4 + i];  // [C, 2C): second sums
        }
    }
}

__global__ __launch_bounds__(BN_T) void bn_stats_kernel(const float4* __restrict__ x, long long rows, int C4,
                                                        double* __restrict__ part) {
    double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    rows_of_block(rows, C4, [&](long long r, int q) {
        const float4 v = x[r * C4 + q];
        const double d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            a[i] += d[i];
            a[4 + i] += d[i] * d[i];
        }
    });
    block_sum_store(a, C4, part);
}

// the nparts partial (sum, second sum) pairs of channel c: one 64-lane wave per channel, lane l summing
// parts l, l + 64, ... in order, then a fixed butterfly (deterministic); every lane returns the totals.
// (One thread per channel summing the 512 parts serially took 36 us per call: a dependent f64 chain.)
__device__ __forceinline__ void channel_sums(const double* __restrict__ part, int nparts, int C, int c, double& s,
                                             double& s2) {
    const int lane = threadIdx.x & 63;
    s = 0, s2 = 0;
    for (int p = lane; p < nparts; p += 64) {
        s += part[(long long)p * 2 * C + c];
        s2 += part[(long long)p * 2 * C + C + c];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o);
        s2 += __shfl_xor(s2, o);
    }
}

// per channel: the parts -> sums [2C] f64 (the first sums, then the second); one wave per channel
__global__ __launch_bounds__(BN_T) void bn_sums_kernel(const double* __restrict__ part, int nparts, int C,
                                                       double* __restrict__ sums) {
    const int c = blockIdx.x * (BN_T / 64) + (int)(threadIdx.x >> 6);
    if (c >= C) return;  // wave-uniform
    double s, s2;
    channel_sums(part, nparts, C, c, s, s2);
    if ((threadIdx.x & 63) != 0) return;
    sums[c] = s;
    sums[C + c] = s2;
}

// The convolution backward's dy statistics in one read of dy [rows][C] (wino_train.WinogradConv3x3.backward):
// per block the per-channel partial sums (f64, the second half of the part row zero) and max |dy|;
// dy_finish_kernel sums the parts in order (db = dy.sum over batch, h, w: the conv bias's gradient)
// and max-reduces the block maxima into *amax (the bits of max |dy|, the dM scale's input).  Replaces a
// memset + azg_absmax's pass + torch's reduction (38.7 us per layer and step at conv2's 51 MB,
// profiles/r06_prof_train_probe_adam.md).
__global__ __launch_bounds__(BN_T) void dy_part_kernel(const float4* __restrict__ dy, long long rows, int C4,
                                                       double* __restrict__ part, float* __restrict__ pmax) {
    double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    float m = 0.f;
    rows_of_block(rows, C4, [&](long long r, int q) {
        const float4 v = dy[r * C4 + q];
        a[0] += (double)v.x;
        a[1] += (double)v.y;
        a[2] += (double)v.z;
        a[3] += (double)v.w;
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    });
    block_sum_store(a, C4, part);
    __shared__ float wm[BN_T / 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float b = wm[0];
#pragma unroll
        for (int q = 1; q < BN_T / 64; ++q) b = fmaxf(b, wm[q]);
        pmax[blockIdx.x] = b;
    }
}

// one wave per channel: db[c] = the parts' sums in order (f32); the wave of channel 0 also writes
// *amax = bits of the largest block maximum (non-negative floats order as their bits)
__global__ __launch_bounds__(BN_T) void dy_finish_kernel(const double* __restrict__ part, const float* __restrict__ pmax,
                                                         int nparts, int C, float* __restrict__ db,
                                                         unsigned* __restrict__ amax) {
    const int c = blockIdx.x * (BN_T / 64) + (int)(threadIdx.x >> 6);
    if (c >= C) return;  // wave-uniform
    double s, s2;
    channel_sums(part, nparts, C, c, s, s2);
    const int lane = threadIdx.x & 63;
    if (lane == 0 && db) db[c] = (float)s;
    if (c == 0) {
        float m = 0.f;
        for (int p = lane; p < nparts; p += 64) m = fmaxf(m, pmax[p]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
        if (lane == 0) *amax = __float_as_uint(m);
    }
}

// per channel, from (sum x, sum x^2) over n rows (every rank's, data-parallel): mean, var, scale (f32),
// running stats
__global__ __launch_bounds__(BN_T) void bn_finalize_kernel(const double* __restrict__ sums, int C, long long n,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float eps, float momentum,
                                                           float* __restrict__ run_mean, float* __restrict__ run_var,
                                                           float* __restrict__ sv) {
    const int c = blockIdx.x * BN_T + threadIdx.x;
    if (c >= C) return;
    const double s = sums[c], s2 = sums[C + c];
    const double mean = s / (double)n;
    double var = s2 / (double)n - mean * mean;
    if (var < 0) var = 0;
    const double invstd = 1.0 / sqrt(var + (double)eps);
    const float scale = (float)((double)gamma[c] * invstd);
    sv[c] = scale;                  // scale
    sv[C + c] = beta[c];            // beta
    sv[2 * C + c] = (float)mean;    // mean
    sv[3 * C + c] = (float)invstd;  // invstd
    if (run_mean) run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mean;
    if (run_var) run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)(var * (double)n / (double)(n - 1));
}

// relu(bn(x)) = max((x - mean) scale + beta, 0) in f32: x - mean first (no cancellation against a
// large mean, as x scale + (beta - mean scale) would have: conv3's weight gradient 4.5% off, r05f)
__device__ __forceinline__ float bn_pre(float x, float mean, float scale, float beta) {
    return (x - mean) * scale + beta;
}
__device__ __forceinline__ float bn_out(float x, float mean, float scale, float beta) {
    return fmaxf(bn_pre(x, mean, scale, beta), 0.f);
}

__global__ __launch_bounds__(BN_T) void bn_apply_relu_kernel(const float4* __restrict__ x,
                                                             const float4* __restrict__ sv, long long n4, int C4,
                                                             float4* __restrict__ y) {
    for (long long i = (long long)blockIdx.x * BN_T + threadIdx.x; i < n4; i += (long long)gridDim.x * BN_T) {
        const int q = (int)(i % C4);
        const float4 v = x[i], sc = sv[q], be = sv[C4 + q], mu = sv[2 * C4 + q];
        y[i] = make_float4(bn_out(v.x, mu.x, sc.x, be.x), bn_out(v.y, mu.y, sc.y, be.y),
                           bn_out(v.z, mu.z, sc.z, be.z), bn_out(v.w, mu.w, sc.w, be.w));
    }
}

// the ReLU's mask from the forward's own expression, then g and xhat
__device__ __forceinline__ void bwd_terms(float4 v, float4 d, float4 sc, float4 sh, float4 mu, float4 is,
                                          double (&g)[4], double (&xh)[4]) {
    const float vv[4] = {v.x, v.y, v.z, v.w}, dd[4] = {d.x, d.y, d.z, d.w}, s[4] = {sc.x, sc.y, sc.z, sc.w},
                h[4] = {sh.x, sh.y, sh.z, sh.w}, m[4] = {mu.x, mu.y, mu.z, mu.w}, iv[4] = {is.x, is.y, is.z, is.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        g[i] = bn_pre(vv[i], m[i], s[i], h[i]) > 0.f ? (double)dd[i] : 0.0;
        xh[i] = ((double)vv[i] - (double)m[i]) * (double)iv[i];
    }
}

__global__ __launch_bounds__(BN_T) void bn_bwd_reduce_kernel(const float4* __restrict__ x,
                                                             const float4* __restrict__ dy,
                                                             const float4* __restrict__ sv, long long rows, int C4,
                                                             double* __restrict__ part) {
    double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    rows_of_block(rows, C4, [&](long long r, int q) {
        double g[4], xh[4];
        bwd_terms(x[r * C4 + q], dy[r * C4 + q], sv[q], sv[C4 + q], sv[2 * C4 + q], sv[3 * C4 + q], g, xh);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            a[i] += g[i];
            a[4 + i] += g[i] * xh[i];
        }
    });
    block_sum_store(a, C4, part);
}

// per channel, from (sum g, sum g xhat) over n rows (every rank's, data-parallel): the apply's
// coefficients c1 = sum g / n, c2 = sum g xhat / n (f32), and -- when dgamma is given -- dbeta = sum g,
// dgamma = sum g xhat
__global__ __launch_bounds__(BN_T) void bn_bwd_coef_kernel(const double* __restrict__ sums, int C, long long n,
                                                           float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                           float* __restrict__ co) {
    const int c = blockIdx.x * BN_T + threadIdx.x;
    if (c >= C) return;
    const double s = sums[c], s2 = sums[C + c];
    if (dgamma) {
        dbeta[c] = (float)s;
        dgamma[c] = (float)s2;
    }
    co[c] = (float)(s / (double)n);
    co[C + c] = (float)(s2 / (double)n);
}

// dx = scale (g - c1 - xhat c2)
__global__ __launch_bounds__(BN_T) void bn_bwd_apply_kernel(const float4* __restrict__ x, const float4* __restrict__ dy,
                                                            const float4* __restrict__ sv,
                                                            const float4* __restrict__ co, long long n4, int C4,
                                                            float4* __restrict__ dx) {
    for (long long i = (long long)blockIdx.x * BN_T + threadIdx.x; i < n4; i += (long long)gridDim.x * BN_T) {
        const int q = (int)(i % C4);
        const float4 sc = sv[q];
        double g[4], xh[4];
        bwd_terms(x[i], dy[i], sc, sv[C4 + q], sv[2 * C4 + q], sv[3 * C4 + q], g, xh);
        const float4 c1 = co[q], c2 = co[C4 + q];
        const float s[4] = {sc.x, sc.y, sc.z, sc.w}, a1[4] = {c1.x, c1.y, c1.z, c1.w}, a2[4] = {c2.x, c2.y, c2.z, c2.w};
        float o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = s[k] * (float)(g[k] - (double)a1[k] - xh[k] * (double)a2[k]);
        dx[i] = make_float4(o[0], o[1], o[2], o[3]);
    }
}

unsigned stream_grid(long long n4) {
    const long long b = (n4 + BN_T - 1) / BN_T;
    return (unsigned)(b < 2048 ? b : 2048);
}

}  // namespace

static bool bn_args_ok(const float* x, int64_t rows, int32_t C) {
    return x && rows >= 2 && C > 0 && C % 4 == 0 && C / 4 <= BN_T && ((uintptr_t)x & 15) == 0;
}

// sums [2C] f64 = per channel (sum x, sum x^2) over the rows of x [rows][C]; work >= 2 * 512 * C doubles
extern "C" int azg_bn_sums(const float* x, int64_t rows, int32_t C, double* sums, double* work, void* stream) {
    if (!bn_args_ok(x, rows, C) || !sums || !work) return AZG_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(bn_stats_kernel, dim3(BN_PARTS), dim3(BN_T), 0, st, (const float4*)x, (long long)rows, C / 4,
                       work);
    hipLaunchKernelGGL(bn_sums_kernel, dim3((C + BN_T / 64 - 1) / (BN_T / 64)), dim3(BN_T), 0, st, work, BN_PARTS, C,
                       sums);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

// y = relu(batchnorm(x)) from azg_bn_sums' sums over n_total rows (this call's x, or every rank's
// when the caller all-reduced them); sv [4C] f32 receives scale, beta, mean, invstd; run_mean /
// run_var updated in place (either may be null)
extern "C" int azg_bn_relu_fwd_from_sums(const float* x, int64_t rows, int32_t C, const double* sums, int64_t n_total,
                                         const float* gamma, const float* beta, float eps, float momentum,
                                         float* run_mean, float* run_var, float* y, float* sv, void* stream) {
    if (!bn_args_ok(x, rows, C) || !sums || n_total < 2 || !gamma || !beta || !y || !sv || ((uintptr_t)y & 15) ||
        ((uintptr_t)sv & 15))
        return AZG_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    const int C4 = C / 4;
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + BN_T - 1) / BN_T), dim3(BN_T), 0, st, sums, C,
                       (long long)n_total, gamma, beta, eps, momentum, run_mean, run_var, sv);
    const long long n4 = rows * C4;
    hipLaunchKernelGGL(bn_apply_relu_kernel, dim3(stream_grid(n4)), dim3(BN_T), 0, st, (const float4*)x,
                       (const float4*)sv, n4, C4, (float4*)y);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

// sums [2C] f64 = per channel (sum g, sum g xhat) over the rows of x / dy (g = dy where the forward's ReLU
// passed); work >= 2 * 512 * C doubles
extern "C" int azg_bn_relu_bwd_sums(const float* x, const float* dy, int64_t rows, int32_t C, const float* sv,
                                    double* sums, double* work, void* stream) {
    if (!bn_args_ok(x, rows, C) || !dy || !sv || !sums || !work || ((uintptr_t)dy & 15) || ((uintptr_t)sv & 15))
        return AZG_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(BN_PARTS), dim3(BN_T), 0, st, (const float4*)x, (const float4*)dy,
                       (const float4*)sv, (long long)rows, C / 4, work);
    hipLaunchKernelGGL(bn_sums_kernel, dim3((C + BN_T / 64 - 1) / (BN_T / 64)), dim3(BN_T), 0, st, work, BN_PARTS, C,
                       sums);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

// dx from azg_bn_relu_bwd_sums' sums over n_total rows (every rank's, data-parallel); dgamma / dbeta
// (may be null) = the sums themselves; co >= 2C f32 scratch
extern "C" int azg_bn_relu_bwd_from_sums(const float* x, const float* dy, int64_t rows, int32_t C, const float* sv,
                                         const double* sums, int64_t n_total, float* dx, float* dgamma, float* dbeta,
                                         float* co, void* stream) {
    if (!bn_args_ok(x, rows, C) || !dy || !sv || !sums || n_total < 2 || !dx || !co || (!dgamma) != (!dbeta) ||
        ((uintptr_t)dy & 15) || ((uintptr_t)dx & 15) || ((uintptr_t)sv & 15) || ((uintptr_t)co & 15))
        return AZG_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    const int C4 = C / 4;
    hipLaunchKernelGGL(bn_bwd_coef_kernel, dim3((C + BN_T - 1) / BN_T), dim3(BN_T), 0, st, sums, C,
                       (long long)n_total, dgamma, dbeta, co);
    const long long n4 = rows * C4;
    hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(stream_grid(n4)), dim3(BN_T), 0, st, (const float4*)x,
                       (const float4*)dy, (const float4*)sv, (const float4*)co, n4, C4, (float4*)dx);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

// *amax = bits of max |dy| and db [C] = dy summed over the rows (db may be null), dy [rows][C] f32;
// work >= 2 * 512 * C doubles + 512 floats
extern "C" int azg_wt_dy_stats(const float* dy, int64_t rows, int32_t C, uint32_t* amax, float* db, double* work,
                               void* stream) {
    if (!bn_args_ok(dy, rows, C) || !amax || !work) return AZG_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    float* pmax = reinterpret_cast<float*>(work + (size_t)2 * BN_PARTS * C);
    hipLaunchKernelGGL(dy_part_kernel, dim3(BN_PARTS), dim3(BN_T), 0, st, (const float4*)dy, (long long)rows, C / 4,
                       work, pmax);
    hipLaunchKernelGGL(dy_finish_kernel, dim3((C + BN_T / 64 - 1) / (BN_T / 64)), dim3(BN_T), 0, st, work, pmax,
                       BN_PARTS, C, db, amax);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

// One process: azg_bn_sums + azg_bn_relu_fwd_from_sums (work >= 2 * 512 * C + 2 C doubles: the partials,
// then the sums)
extern "C" int azg_bn_relu_fwd(const float* x, int64_t rows, int32_t C, const float* gamma, const float* beta,
                               float eps, float momentum, float* run_mean, float* run_var, float* y, float* sv,
                               double* work, void* stream) {
    if (!work) return AZG_ERR_ARG;
    double* sums = work + (size_t)2 * BN_PARTS * C;
    int rc = azg_bn_sums(x, rows, C, sums, work, stream);
    if (rc) return rc;
    return azg_bn_relu_fwd_from_sums(x, rows, C, sums, rows, gamma, beta, eps, momentum, run_mean, run_var, y, sv,
                                     stream);
}

// One process: azg_bn_relu_bwd_sums + azg_bn_relu_bwd_from_sums (dgamma, dbeta written, not accumulated;
// work as azg_bn_relu_fwd's)
extern "C" int azg_bn_relu_bwd(const float* x, const float* dy, int64_t rows, int32_t C, const float* sv, float* dx,
                               float* dgamma, float* dbeta, float* co, double* work, void* stream) {
    if (!work || !dgamma || !dbeta) return AZG_ERR_ARG;
    double* sums = work + (size_t)2 * BN_PARTS * C;
    int rc = azg_bn_relu_bwd_sums(x, dy, rows, C, sv, sums, work, stream);
    if (rc) return rc;
    return azg_bn_relu_bwd_from_sums(x, dy, rows, C, sv, sums, rows, dx, dgamma, dbeta, co, stream);
}
