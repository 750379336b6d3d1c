// azg_train_loss.hip -- the training step's heads and losses (NNet.py:57-61, 96-100; InflexionNNet.py:54):
//   log p = log_softmax(x3), v = tanh(z4),
//   l_pi = -sum_b sum_a t_pi[b][a] log p[b][a] / B,   l_v = sum_b (t_v[b] - v[b])^2 / B,
// and their gradients, in three launches instead of torch's ~16 small kernels per step (log_softmax, tanh,
// the products, sums, negation and divisions, forward and backward).
//
//   loss_rows_kernel : one wave per row: m = max x, ls = log sum exp(x - m) (the row statistics the backward
//                      reuses), the row's -sum t (x - m - ls) and (t_v - tanh z)^2
//   loss_sum_kernel  : one block sums the rows' terms in a fixed order (f64), / B -> l_pi, l_v
//   loss_bwd_kernel  : one wave per row: dx = g_pi (softmax(x) sum_a t - t) / B (log_softmax's adjoint of
//                      -g_pi t / B), dz = g_v (-2 (t_v - v)) (1 - v^2) / B (tanh's adjoint as torch forms it)
//
// f32 arithmetic per element as torch forms it (log p = (x - m) - log s, exp(log p) for the softmax); the
// sums are in a fixed order (deterministic), not torch's reduction order (within f32 rounding of it).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "../../include/azg.h"

namespace {

constexpr int WAVE = 64;

__device__ __forceinline__ float wave_max(float x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o));
    return x;
}
__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    return x;
}

// rows: [B][4] = (row l_pi term, row l_v term, m, ls)
__global__ __launch_bounds__(256) void loss_rows_kernel(const float* __restrict__ x3, int ld3,
                                                        const float* __restrict__ z4, int ld4,
                                                        const float* __restrict__ tpi, int ldt,
                                                        const float* __restrict__ tv, int B, int A,
                                                        float* __restrict__ rows) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= B) return;  // wave-uniform
    const float* x = x3 + (long long)b * ld3;
    const float* t = tpi + (long long)b * ldt;
    float m = -INFINITY;
    for (int a = lane; a < A; a += WAVE) m = fmaxf(m, x[a]);
    m = wave_max(m);
    float s = 0.f;
    for (int a = lane; a < A; a += WAVE) s += expf(x[a] - m);
    s = wave_sum(s);
    const float ls = logf(s);
    float lp = 0.f;
    for (int a = lane; a < A; a += WAVE) lp += t[a] * ((x[a] - m) - ls);
    lp = wave_sum(lp);
    if (lane == 0) {
        const float v = tanhf(z4[(long long)b * ld4]);
        const float d = tv[b] - v;
        float* r = rows + 4LL * b;
        r[0] = -lp;
        r[1] = d * d;
        r[2] = m;
        r[3] = ls;
    }
}

__global__ __launch_bounds__(256) void loss_sum_kernel(const float* __restrict__ rows, int B, float* __restrict__ out) {
    __shared__ double sp[256], sv[256];
    const int tid = threadIdx.x;
    double p = 0.0, v = 0.0;
    for (int b = tid; b < B; b += 256) {  // thread tid's rows in order, then the threads' sums in a fixed tree
        p += (double)rows[4LL * b];
        v += (double)rows[4LL * b + 1];
    }
    sp[tid] = p;
    sv[tid] = v;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (tid < w) {
            sp[tid] += sp[tid + w];
            sv[tid] += sv[tid + w];
        }
        __syncthreads();
    }
    if (tid == 0) {
        out[0] = (float)sp[0] / (float)B;
        out[1] = (float)sv[0] / (float)B;
    }
}

__global__ __launch_bounds__(256) void loss_bwd_kernel(const float* __restrict__ x3, int ld3,
                                                       const float* __restrict__ z4, int ld4,
                                                       const float* __restrict__ tpi, int ldt,
                                                       const float* __restrict__ tv, const float* __restrict__ rows,
                                                       int B, int A, const float* __restrict__ g,
                                                       float* __restrict__ dx3, int lddx, float* __restrict__ dz4,
                                                       int lddz) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= B) return;
    const float* x = x3 + (long long)b * ld3;
    const float* t = tpi + (long long)b * ldt;
    const float m = rows[4LL * b + 2], ls = rows[4LL * b + 3];
    const float invB = 1.0f / (float)B;
    const float gp = g[0] * invB;  // the adjoint of l_pi = -sum t logp / B w.r.t. logp is -gp t
    float st = 0.f;
    for (int a = lane; a < A; a += WAVE) st += -gp * t[a];
    st = wave_sum(st);  // sum_a of log_softmax's output gradient
    float* dx = dx3 + (long long)b * lddx;
    for (int a = lane; a < A; a += WAVE) {
        const float go = -gp * t[a];
        dx[a] = go - expf((x[a] - m) - ls) * st;  // log_softmax backward: go - exp(out) sum(go)
    }
    if (lane == 0) {
        const float v = tanhf(z4[(long long)b * ld4]);
        const float gv = g[1] * invB;
        const float go = gv * (-2.0f * (tv[b] - v));  // d/dv of (t - v)^2, scaled
        dz4[(long long)b * lddz] = go * (1.0f - v * v);
    }
}

}  // namespace

extern "C" int azg_train_loss_fwd(const float* x3, int32_t ld3, const float* z4, int32_t ld4, const float* tpi,
                                  int32_t ldt, const float* tv, int32_t B, int32_t A, float* rows, float* out,
                                  void* stream) {
    if (!x3 || !z4 || !tpi || !tv || !rows || !out || B <= 0 || A <= 0 || ld3 < A || ldt < A || ld4 < 1)
        return AZG_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(loss_rows_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, x3, ld3, z4, ld4, tpi, ldt,
                       tv, B, A, rows);
    hipLaunchKernelGGL(loss_sum_kernel, dim3(1), dim3(256), 0, st, rows, B, out);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_train_loss_bwd(const float* x3, int32_t ld3, const float* z4, int32_t ld4, const float* tpi,
                                  int32_t ldt, const float* tv, const float* rows, int32_t B, int32_t A, const float* g,
                                  float* dx3, int32_t lddx, float* dz4, int32_t lddz, void* stream) {
    if (!x3 || !z4 || !tpi || !tv || !rows || !g || !dx3 || !dz4 || B <= 0 || A <= 0 || ld3 < A || ldt < A ||
        lddx < A || ld4 < 1 || lddz < 1)
        return AZG_ERR_ARG;
    hipLaunchKernelGGL(loss_bwd_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, (hipStream_t)stream, x3, ld3, z4,
                       ld4, tpi, ldt, tv, rows, B, A, g, dx3, lddx, dz4, lddz);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}
