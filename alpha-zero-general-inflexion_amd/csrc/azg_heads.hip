// azg_heads.hip -- the leaf network's fully connected tail (InflexionNNet.py:47-54,
// BN folded) around split-fp16 GEMMs, as the two epilogue kernels the GEMMs need:
//
//   fc1 -> fc2 -> [fc3 | fc4]: each GEMM is one fp16 hipBLASLt GEMM with f32
//   accumulation over split operands, A rows [hi | lo | hi] times the weights stacked
//   [hi; hi; lo] (= hi Wh + lo Wh + hi Wl, f32-accurate products as the Winograd GEMMs,
//   DESIGN.md 4.1); the weights are pre-scaled by a power of two that `scale` undoes.
//
//  * fc_act_split: y = relu(bias + scale * m) of one FC layer (m summed over the parts
//    of a split-K GEMM first, fc1 on libazg's split GEMM) written straight as the
//    next layer's A operand, one fp16 row [hi | lo | hi] per leaf (AZG_WINO_SPLIT), so
//    the activation never exists in f32; |y| > 65504 or NaN sets *overflow (the
//    InferenceNet range flag).  HBM-bound: 4 values per lane, float4 loads.
//  * policy_value: P = softmax(bias[:A] + scale * m[:, :A]) (= exp(log_softmax),
//    NNet.py:94) and v = tanh(bias[A] + scale * m[:, A]) from the stacked fc3 | fc4
//    GEMM, one wave per leaf (max and sum as __shfl_xor butterflies), written in the
//    [G, A] / [G] layout azg_sim_end reads.
#include <hip/hip_runtime.h>

#include "../../include/azg.h"
#include "azg_ptr.h"

namespace {

__global__ __launch_bounds__(256) void fc_act_split_kernel(const float4* __restrict__ m, int parts,
                                                           long long pstride4, const float4* __restrict__ bias,
                                                           float scale, ushort4* __restrict__ out, long long rows,
                                                           int n4, int relu, int* overflow) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows * n4) return;
    const long long r = i / n4;
    const int c4 = (int)(i - r * n4);
    float4 x = m[i];
    for (int p = 1; p < parts; ++p) {  // split-K parts, summed in order
        const float4 t = m[p * pstride4 + i];
        x = make_float4(x.x + t.x, x.y + t.y, x.z + t.z, x.w + t.w);
    }
    const float4 b = bias[c4];
    float y[4] = {b.x + scale * x.x, b.y + scale * x.y, b.z + scale * x.z, b.w + scale * x.w};
    unsigned short hi[4], lo[4];
    bool bad = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (relu) y[j] = fmaxf(y[j], 0.f);
        const _Float16 h = (_Float16)y[j];  // round to nearest even
        const _Float16 l = (_Float16)(y[j] - (float)h);
        hi[j] = __builtin_bit_cast(unsigned short, h);
        lo[j] = __builtin_bit_cast(unsigned short, l);
        bad |= !(fabsf(y[j]) <= 65504.f);
    }
    ushort4* row = out + r * 3 * n4;
    const ushort4 H = {hi[0], hi[1], hi[2], hi[3]}, L = {lo[0], lo[1], lo[2], lo[3]};
    row[c4] = H;
    row[n4 + c4] = L;
    row[2 * n4 + c4] = H;
    if (bad) atomicOr(overflow, 1);
}

constexpr int PV_MAX_PER_LANE = 16;  // up to 1024 actions per leaf (9x9 Inflexion: 567)

template <int PV_PER_LANE>
__global__ __launch_bounds__(256) void policy_value_kernel(const float* __restrict__ m, int ldm,
                                                           const float* __restrict__ bias, float scale,
                                                           float* __restrict__ P, float* __restrict__ v, int rows,
                                                           int A) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= rows) return;  // wave-uniform
    const float* mr = m + (long long)r * ldm;
    float x[PV_PER_LANE];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < PV_PER_LANE; ++j) {
        const int a = lane + 64 * j;
        x[j] = a < A ? bias[a] + scale * mr[a] : -INFINITY;
        mx = fmaxf(mx, x[j]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < PV_PER_LANE; ++j) {
        x[j] = lane + 64 * j < A ? expf(x[j] - mx) : 0.f;
        s += x[j];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    const float inv = 1.f / s;
    float* pr = P + (long long)r * A;
#pragma unroll
    for (int j = 0; j < PV_PER_LANE; ++j) {
        const int a = lane + 64 * j;
        if (a < A) pr[a] = x[j] * inv;
    }
    if (lane == 0) v[r] = tanhf(bias[A] + scale * mr[A]);
}

}  // namespace

extern "C" int azg_fc_act_split(const float* m, int32_t parts, int64_t part_stride, const float* bias, float scale,
                                void* out, int32_t rows, int32_t n, int32_t relu, int32_t* overflow, void* stream) {
    if (!m || !bias || !out || !azg_device_writable(overflow) || rows <= 0 || n <= 0 || n % 4 || parts < 1 || part_stride % 4 ||
        (parts > 1 && part_stride < (int64_t)rows * n) || ((uintptr_t)m & 15) || ((uintptr_t)bias & 15) ||
        ((uintptr_t)out & 7))
        return AZG_ERR_ARG;
    const long long items = (long long)rows * (n / 4);
    hipLaunchKernelGGL(fc_act_split_kernel, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (const float4*)m, parts, (long long)(part_stride / 4), (const float4*)bias, scale,
                       (ushort4*)out, (long long)rows, n / 4, relu, overflow);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_policy_value(const float* m, int32_t ldm, const float* bias, float scale, float* P, float* v,
                                int32_t rows, int32_t actions, void* stream) {
    if (!m || !bias || !P || !v || rows <= 0 || actions <= 0 || actions > 64 * PV_MAX_PER_LANE || ldm < actions + 1)
        return AZG_ERR_ARG;
    const dim3 grid((unsigned)((rows + 3) / 4));
    if (actions <= 64 * 8)
        hipLaunchKernelGGL(policy_value_kernel<8>, grid, dim3(256), 0, (hipStream_t)stream, m, ldm, bias, scale, P, v,
                           rows, actions);
    else
        hipLaunchKernelGGL(policy_value_kernel<PV_MAX_PER_LANE>, grid, dim3(256), 0, (hipStream_t)stream, m, ldm,
                           bias, scale, P, v, rows, actions);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}
