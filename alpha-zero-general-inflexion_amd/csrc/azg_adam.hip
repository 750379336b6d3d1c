// azg_adam.hip -- the trainer's Adam step (NNet.py:37: optim.Adam(self.nnet.parameters()), lr 1e-3,
// betas (0.9, 0.999), eps 1e-8) over every parameter tensor in ONE launch.
//
// torch's capturable foreach Adam (torch/optim/adam.py _multi_tensor_adam, the form the GPU trainer
// replays inside its HIP graph) costs ~20 multi-tensor launches per step plus ~54 per-parameter
// scalar kernels for the bias corrections (`_foreach_pow(beta, steps)` has no multi-tensor form):
// ~470 us of a 3.0 ms 512-example step (profiles/r06_prof_train_probe.md), for 12.6 M parameters
// whose whole update is 7 x 50 MB of HBM traffic (~70 us).  Here one kernel reads p, g, m, v and
// writes p, m, v once, with float4 accesses, and follows the foreach form's f32 arithmetic:
//
//   t = step + 1 (the device counter, bumped by adam_bump_kernel first)
//   step_size = 1 / ((beta1^t - 1) / lr)        (negative; _foreach_pow / sub_ / div_ / reciprocal_)
//   bc2_sqrt  = sqrt(-(beta2^t - 1))
//   m = m + (1 - beta1) (g - m)                  (lerp_, weight < 0.5)
//   v = v beta2;  v = v + (1 - beta2) g g        (mul_, addcmul_)
//   p = p + step_size (m / (sqrt(v) / bc2_sqrt + eps))   (addcdiv_)
//
// Parameters and gradients are separate tensors (segment i: params[i], grads[i], counts[i]); the
// state m, v is two flat buffers with segment i at offset off[i] (counts rounded up to 4, so every
// segment's state is 16-B aligned).  The segment table travels as the kernel's by-value argument,
// so a captured launch replays with the pointers it was captured with (the graph trainer's
// gradients live at fixed addresses in the graph's pool).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/azg.h"

int azg_host_fail(int code, const std::string& msg);  // azg_capi.cpp

namespace {

constexpr int ADAM_T = 256;
constexpr int ADAM_VEC = 4;                        // floats per thread per iteration (float4)
constexpr int ADAM_CHUNK = ADAM_T * ADAM_VEC * 4;  // elements per block

struct AdamArgs {
    float* p[AZG_ADAM_MAX_SEG];
    const float* g[AZG_ADAM_MAX_SEG];
    long long cnt[AZG_ADAM_MAX_SEG];
    long long off[AZG_ADAM_MAX_SEG];       // state offset of each segment (multiple of 4)
    int blk[AZG_ADAM_MAX_SEG + 1];         // first block of each segment (prefix of ceil(cnt / CHUNK))
    int nseg;
    float lr, beta1, beta2, eps, one_minus_beta1, one_minus_beta2;
};

__global__ void adam_bump_kernel(float* step) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *step = *step + 1.0f;
}

__device__ __forceinline__ float adam_elem(float& p, float g, float& m, float& v, float step_size, float bc2,
                                           const AdamArgs& a) {
    m = m + a.one_minus_beta1 * (g - m);
    v = v * a.beta2;
    v = v + a.one_minus_beta2 * g * g;
    const float denom = sqrtf(v) / bc2 + a.eps;
    p = p + step_size * (m / denom);
    return p;
}

__global__ __launch_bounds__(ADAM_T) void adam_kernel(AdamArgs a, float* __restrict__ m, float* __restrict__ v,
                                                      const float* __restrict__ step) {
    const int b = blockIdx.x;
    int s = 0;
    while (s + 1 < a.nseg && a.blk[s + 1] <= b) ++s;
    const float t = *step;
    float bc1 = powf(a.beta1, t);
    bc1 = bc1 - 1.0f;
    bc1 = bc1 / a.lr;
    const float step_size = 1.0f / bc1;
    float bc2 = powf(a.beta2, t);
    bc2 = bc2 - 1.0f;
    bc2 = -bc2;
    bc2 = sqrtf(bc2);
    const long long n = a.cnt[s];
    const long long c0 = (long long)(b - a.blk[s]) * ADAM_CHUNK;
    const long long c1 = c0 + ADAM_CHUNK < n ? c0 + ADAM_CHUNK : n;
    float* __restrict__ P = a.p[s];
    const float* __restrict__ G = a.g[s];
    float* __restrict__ M = m + a.off[s];
    float* __restrict__ V = v + a.off[s];
    const bool vec = ((reinterpret_cast<uintptr_t>(P) | reinterpret_cast<uintptr_t>(G)) & 15) == 0;
    long long i = c0 + (long long)threadIdx.x * ADAM_VEC;
    if (vec) {
        for (; i + ADAM_VEC <= c1; i += (long long)ADAM_T * ADAM_VEC) {
            float4 pp = *reinterpret_cast<const float4*>(P + i);
            const float4 gg = *reinterpret_cast<const float4*>(G + i);
            float4 mm = *reinterpret_cast<const float4*>(M + i);
            float4 vv = *reinterpret_cast<const float4*>(V + i);
            adam_elem(pp.x, gg.x, mm.x, vv.x, step_size, bc2, a);
            adam_elem(pp.y, gg.y, mm.y, vv.y, step_size, bc2, a);
            adam_elem(pp.z, gg.z, mm.z, vv.z, step_size, bc2, a);
            adam_elem(pp.w, gg.w, mm.w, vv.w, step_size, bc2, a);
            *reinterpret_cast<float4*>(P + i) = pp;
            *reinterpret_cast<float4*>(M + i) = mm;
            *reinterpret_cast<float4*>(V + i) = vv;
        }
    }
    // the tail (fewer than 4 left in this thread's stride) or unaligned tensors: element by element
    for (; i < c1; i += (long long)ADAM_T * ADAM_VEC)
        for (long long j = i; j < i + ADAM_VEC && j < c1; ++j) {
            float pp = P[j], mm = M[j], vv = V[j];
            adam_elem(pp, G[j], mm, vv, step_size, bc2, a);
            P[j] = pp;
            M[j] = mm;
            V[j] = vv;
        }
}

}  // namespace

extern "C" int azg_adam_step(int32_t nseg, float* const* params, const float* const* grads, const int64_t* counts,
                             float* m, float* v, float* step, double lr, double beta1, double beta2, double eps,
                             void* stream) {
    if (nseg < 1 || nseg > AZG_ADAM_MAX_SEG)
        return azg_host_fail(AZG_ERR_ARG, "azg_adam_step: 1 <= nseg <= AZG_ADAM_MAX_SEG");
    if (!params || !grads || !counts || !m || !v || !step)
        return azg_host_fail(AZG_ERR_ARG, "azg_adam_step: null pointer");
    if ((reinterpret_cast<uintptr_t>(m) | reinterpret_cast<uintptr_t>(v)) & 15)
        return azg_host_fail(AZG_ERR_ARG, "azg_adam_step: m and v must be 16-B aligned");
    AdamArgs a{};
    long long off = 0;
    long long blocks = 0;
    for (int s = 0; s < nseg; ++s) {
        if (!params[s] || !grads[s] || counts[s] < 0)
            return azg_host_fail(AZG_ERR_ARG, "azg_adam_step: null segment or negative count");
        a.p[s] = params[s];
        a.g[s] = grads[s];
        a.cnt[s] = counts[s];
        a.off[s] = off;
        a.blk[s] = (int)blocks;
        off += (counts[s] + 3) / 4 * 4;
        blocks += (counts[s] + ADAM_CHUNK - 1) / ADAM_CHUNK;
    }
    if (blocks < 1 || blocks >= (1LL << 31)) return azg_host_fail(AZG_ERR_ARG, "azg_adam_step: no elements");
    a.blk[nseg] = (int)blocks;
    a.nseg = nseg;
    // Python floats cast to f32 where torch's ops meet the f32 tensors (1 - beta formed in f64 first)
    a.lr = (float)lr;
    a.beta1 = (float)beta1;
    a.beta2 = (float)beta2;
    a.eps = (float)eps;
    a.one_minus_beta1 = (float)(1.0 - beta1);
    a.one_minus_beta2 = (float)(1.0 - beta2);
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(adam_bump_kernel, dim3(1), dim3(64), 0, st, step);
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(ADAM_T), 0, st, a, m, v, step);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return azg_host_fail(AZG_ERR_HIP, std::string("azg_adam_step: ") + hipGetErrorString(e));
    return AZG_OK;
}
