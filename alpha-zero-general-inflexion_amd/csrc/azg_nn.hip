// azg_nn.hip -- epilogue kernels for the leaf network (NHWC activations).
//
// The implicit-GEMM convolutions run without a bias; this kernel applies the
// BatchNorm-folded bias and the ReLU in ONE read-modify-write pass over the
// NHWC output (instead of a bias pass plus a ReLU pass).  HBM-bound: 8 bytes
// moved per element, float4 per lane, grid-stride over >= 8 waves per CU.
#include <hip/hip_runtime.h>

#include "../../include/azg.h"

namespace {
__global__ __launch_bounds__(256) void bias_relu_nhwc_kernel(float4* __restrict__ x, const float4* __restrict__ b,
                                                             long long n4, int c4) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        float4 v = x[i];
        const float4 bb = b[i % c4];
        v.x = fmaxf(v.x + bb.x, 0.0f);
        v.y = fmaxf(v.y + bb.y, 0.0f);
        v.z = fmaxf(v.z + bb.z, 0.0f);
        v.w = fmaxf(v.w + bb.w, 0.0f);
        x[i] = v;
    }
}
}  // namespace

extern "C" int azg_bias_relu_nhwc(float* x, const float* bias, int64_t rows, int32_t channels, void* stream) {
    if (!x || !bias || rows < 0 || channels <= 0 || channels % 4 || ((uintptr_t)x & 15) || ((uintptr_t)bias & 15))
        return AZG_ERR_ARG;
    const long long n4 = rows * (long long)channels / 4;
    if (n4 == 0) return 0;
    long long blocks = (n4 + 255) / 256;
    if (blocks > 256 * 16) blocks = 256 * 16;
    hipLaunchKernelGGL(bias_relu_nhwc_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       (float4*)x, (const float4*)bias, n4, channels / 4);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}
