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
//  * policy_value: P = exp(log_softmax(bias[:A] + scale * m[:, :A])) (the reference's exp(log_softmax),
//    NNet.py:94) and v = tanh(bias[A] + scale * m[:, A]) from the stacked fc3 | fc4
//    GEMM, one wave per leaf (max and sum as __shfl_xor butterflies), written in the
//    [G, A] / [G] layout azg_sim_end reads.
//
// With fc2 and [fc3 | fc4] on libazg's split GEMM too (azg_fc_act with AZG_WINO_SPLIT2
// output, azg_policy_value_parts), no library GEMM is left in the 4096-leaf forward:
// fc_act writes the next layer's A operand as out_parts K-parts of 32-channel
// [hi(32) | lo(32)] blocks ([part][rows][2 n / out_parts] fp16, the split GEMM's
// operand layout, AZG_WINO_SPLIT2), the next split-K GEMM's parts being its "points";
// policy_value sums that GEMM's parts in order before the softmax / tanh.
#include <hip/hip_runtime.h>

#include "../../include/azg.h"
#include "azg_ptr.h"

namespace {

// PM > 1: up to PM split-K parts, every part's load issued before the in-order sum (one memory
// round trip, not one per part: C2's fc2 sums 16 parts); PM = 0: any number, one part at a time
template <int FMT, int PM>
__global__ __launch_bounds__(256) void fc_act_split_kernel(const float4* __restrict__ m, int parts,
                                                           long long pstride4, const float4* __restrict__ bias,
                                                           float scale, ushort4* __restrict__ out, long long rows,
                                                           int n4, int relu, int out_parts, int* overflow) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows * n4) return;
    const long long r = i / n4;
    const int c4 = (int)(i - r * n4);
    float4 x = m[i];
    if constexpr (PM > 1) {
        float4 t[PM - 1];
#pragma unroll
        for (int p = 1; p < PM; ++p) t[p - 1] = p < parts ? m[p * pstride4 + i] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int p = 1; p < PM; ++p)  // split-K parts, summed in order
            if (p < parts) x = make_float4(x.x + t[p - 1].x, x.y + t[p - 1].y, x.z + t[p - 1].z, x.w + t[p - 1].w);
    } else {
        for (int p = 1; p < parts; ++p) {  // split-K parts, summed in order
            const float4 t = m[p * pstride4 + i];
            x = make_float4(x.x + t.x, x.y + t.y, x.z + t.z, x.w + t.w);
        }
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
    const ushort4 H = {hi[0], hi[1], hi[2], hi[3]}, L = {lo[0], lo[1], lo[2], lo[3]};
    if constexpr (FMT == AZG_WINO_SPLIT) {
        ushort4* row = out + r * 3 * n4;
        row[c4] = H;
        row[n4 + c4] = L;
        row[2 * n4 + c4] = H;
    } else {
        // column c = 4 c4 of part p = c / np: block (c % np) / 32 of its row, hi at
        // 64 block + c % 32 halves, lo 32 halves on (np = n / out_parts columns per part)
        const int np4 = n4 / out_parts, p = c4 / np4, cc4 = c4 - p * np4;
        ushort4* row = out + ((long long)p * rows + r) * 2 * np4;
        const int q = (cc4 >> 3) * 16 + (cc4 & 7);  // in ushort4 units: 16 per 64-half block
        row[q] = H;
        row[q + 8] = L;
    }
    if (bad) atomicOr(overflow, 1);
}

// fc_act with the GEMM's partial products TRANSPOSED, m [parts][n][rows] (the small-batch fc1,
// computed as W x A^T so each weight tile is read once: nnet.InferenceNet._fc_split_azg): a block
// takes 16 features x 64 rows (C2's 1024 x 256: 256 blocks, one per CU), each thread one row of 4
// features with every part's load issued before the in-order sum (up to FT_PMAX parts in flight),
// turns the tile through LDS and writes y = relu(bias + scale m) as the next layer's
// AZG_WINO_SPLIT2 K-parts ([out_parts][rows][2 n / out_parts], 32-channel [hi | lo] blocks), as
// fc_act_split_kernel.  (The first form, 64 x 64 tiles with one load in flight per part: 64 blocks,
// 68.9 us at C2 -- 22.6% of its kernel time, profiles/r05_prof_C2_fc_act_t.md.)
constexpr int FT_PMAX = 32;

__global__ __launch_bounds__(256) void fc_act_t_kernel(const float* __restrict__ m, int parts, long long pstride,
                                                       const float* __restrict__ bias, float scale,
                                                       unsigned short* __restrict__ out, int rows, int n, int relu,
                                                       int out_parts, int* overflow) {
    __shared__ float s[16][65];
    const int t = threadIdx.x, f0 = blockIdx.x * 16, r0 = blockIdx.y * 64;
    {
        const int r = t & 63, fg = t >> 6;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int f = fg + 4 * j;
            const float* p = m + (long long)(f0 + f) * rows + r0 + r;
            float v[FT_PMAX];
#pragma unroll
            for (int q = 0; q < FT_PMAX; ++q) v[q] = q < parts ? __builtin_nontemporal_load(p + q * pstride) : 0.f;
            float x = v[0];
#pragma unroll
            for (int q = 1; q < FT_PMAX; ++q)
                if (q < parts) x += v[q];  // split-K parts, in order
            s[f][r] = x;
        }
    }
    __syncthreads();
    const int r = t >> 2, sub = t & 3;  // row, 4 features
    const int np = n / out_parts, part = f0 / np, cc = f0 - part * np;  // 16 features never straddle a part
    const int c = cc + 4 * sub;  // the thread's first column within its part: 4 columns of one 32-block
    unsigned short* row = out + ((long long)part * rows + r0 + r) * 2 * np + 64 * (c >> 5) + (c & 31);
    bool bad = false;
    using u16x4 = __attribute__((ext_vector_type(4))) unsigned short;
    u16x4 hi, lo;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int f = 4 * sub + j;
        float y = bias[f0 + f] + scale * s[f][r];
        if (relu) y = fmaxf(y, 0.f);
        const _Float16 h = (_Float16)y;
        const _Float16 l = (_Float16)(y - (float)h);
        hi[j] = __builtin_bit_cast(unsigned short, h);
        lo[j] = __builtin_bit_cast(unsigned short, l);
        bad |= !(fabsf(y) <= 65504.f);
    }
    *(u16x4*)row = hi;
    *(u16x4*)(row + 32) = lo;
    if (bad) atomicOr(overflow, 1);
}

constexpr int PV_MAX_PER_LANE = 16;  // up to 1024 actions per leaf (9x9 Inflexion: 567)
constexpr int PV_PMAX = 16;          // split-K parts of the [fc3 | fc4] GEMM

// PM > 1 (the split-K [fc3 | fc4] GEMM's parts, <= PM): every part's loads issued before the
// in-order sums, one memory round trip (C2's 8 parts: 14.8 us with one round trip per part);
// PM = 1: one part
template <int PV_PER_LANE, int PM>
__global__ __launch_bounds__(256) void policy_value_kernel(const float* __restrict__ m, int ldm, int parts,
                                                           long long pstride, const float* __restrict__ bias,
                                                           float scale, float* __restrict__ P,
                                                           float* __restrict__ v, int rows, int A) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= rows) return;  // wave-uniform
    const float* mr = m + (long long)r * ldm;
    float x[PV_PER_LANE];
    float mx = -INFINITY;
    float t[PM][PV_PER_LANE];
#pragma unroll
    for (int p = 0; p < PM; ++p)
#pragma unroll
        for (int j = 0; j < PV_PER_LANE; ++j) {
            const int a = lane + 64 * j;
            t[p][j] = (a < A && p < parts) ? mr[p * pstride + a] : 0.f;
        }
    float tv[PM];  // the value column, lane 0, loaded with the rest
#pragma unroll
    for (int p = 0; p < PM; ++p) tv[p] = (lane == 0 && p < parts) ? mr[p * pstride + A] : 0.f;
#pragma unroll
    for (int j = 0; j < PV_PER_LANE; ++j) {
        const int a = lane + 64 * j;
        float s = t[0][j];
#pragma unroll
        for (int p = 1; p < PM; ++p)
            if (p < parts) s += t[p][j];  // split-K parts, in order
        x[j] = a < A ? bias[a] + scale * s : -INFINITY;
        mx = fmaxf(mx, x[j]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    // P = exp(log_softmax) as the reference forms it (NNet.py:94 on torch's CPU log_softmax:
    // (x - max) - log(sum exp(x - max)), then exp): ONE rounding into the subnormal range.  The direct
    // softmax exp(x - max) / sum rounds twice there, and a peaked network's tiny priors -- the only
    // ones left to explore at a lost position -- then differed from the reference's by subnormal ulps
    // or zero / nonzero, deciding PUCT ties among unvisited edges (tests/golden peaked_* traces)
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < PV_PER_LANE; ++j) {
        x[j] -= mx;
        s += lane + 64 * j < A ? expf(x[j]) : 0.f;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    const float ls = logf(s);
    float* pr = P + (long long)r * A;
#pragma unroll
    for (int j = 0; j < PV_PER_LANE; ++j) {
        const int a = lane + 64 * j;
        if (a < A) pr[a] = expf(x[j] - ls);
    }
    if (lane == 0) {
        float t = tv[0];
#pragma unroll
        for (int p = 1; p < PM; ++p)
            if (p < parts) t += tv[p];
        v[r] = tanhf(bias[A] + scale * t);
    }
}

}  // namespace

extern "C" int azg_fc_act(const float* m, int32_t parts, int64_t part_stride, const float* bias, float scale,
                          void* out, int32_t rows, int32_t n, int32_t relu, int32_t fmt, int32_t out_parts,
                          int32_t* overflow, void* stream) {
    if (!m || !bias || !out || !azg_device_writable(overflow) || rows <= 0 || n <= 0 || n % 4 || parts < 1 ||
        part_stride % 4 || (parts > 1 && part_stride < (int64_t)rows * n) || ((uintptr_t)m & 15) ||
        ((uintptr_t)bias & 15) || ((uintptr_t)out & 7) || (fmt != AZG_WINO_SPLIT && fmt != AZG_WINO_SPLIT2) ||
        (fmt == AZG_WINO_SPLIT && out_parts != 1) ||
        (fmt == AZG_WINO_SPLIT2 && (out_parts < 1 || n % out_parts || (n / out_parts) % 32)))
        return AZG_ERR_ARG;
    const long long items = (long long)rows * (n / 4);
    const dim3 grid((unsigned)((items + 255) / 256));
    auto launch = [&](auto kern, int op) {
        hipLaunchKernelGGL(kern, grid, dim3(256), 0, (hipStream_t)stream, (const float4*)m, parts,
                           (long long)(part_stride / 4), (const float4*)bias, scale, (ushort4*)out, (long long)rows,
                           n / 4, relu, op, overflow);
    };
    if (fmt == AZG_WINO_SPLIT)
        launch(fc_act_split_kernel<AZG_WINO_SPLIT, 0>, 1);
    else if (parts <= 4)
        launch(fc_act_split_kernel<AZG_WINO_SPLIT2, 4>, out_parts);
    else if (parts <= 16)
        launch(fc_act_split_kernel<AZG_WINO_SPLIT2, 16>, out_parts);
    else
        launch(fc_act_split_kernel<AZG_WINO_SPLIT2, 0>, out_parts);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_fc_act_t(const float* m, int32_t parts, int64_t part_stride, const float* bias, float scale,
                            void* out, int32_t rows, int32_t n, int32_t relu, int32_t out_parts, int32_t* overflow,
                            void* stream) {
    if (!m || !bias || !out || !azg_device_writable(overflow) || rows <= 0 || rows % 64 || n <= 0 || n % 64 ||
        parts < 1 || parts > FT_PMAX || (parts > 1 && part_stride < (int64_t)rows * n) || out_parts < 1 ||
        n % out_parts || (n / out_parts) % 64 || ((uintptr_t)out & 15))
        return AZG_ERR_ARG;
    hipLaunchKernelGGL(fc_act_t_kernel, dim3(n / 16, rows / 64), dim3(256), 0, (hipStream_t)stream, m, parts,
                       (long long)part_stride, bias, scale, (unsigned short*)out, rows, n, relu, out_parts, overflow);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_fc_act_split(const float* m, int32_t parts, int64_t part_stride, const float* bias, float scale,
                                void* out, int32_t rows, int32_t n, int32_t relu, int32_t* overflow, void* stream) {
    return azg_fc_act(m, parts, part_stride, bias, scale, out, rows, n, relu, AZG_WINO_SPLIT, 1, overflow, stream);
}

extern "C" int azg_policy_value_parts(const float* m, int32_t parts, int64_t part_stride, int32_t ldm,
                                      const float* bias, float scale, float* P, float* v, int32_t rows,
                                      int32_t actions, void* stream) {
    if (!m || !bias || !P || !v || rows <= 0 || actions <= 0 || actions > 64 * PV_MAX_PER_LANE ||
        ldm < actions + 1 || parts < 1 || parts > PV_PMAX || (parts > 1 && part_stride < (int64_t)rows * ldm))
        return AZG_ERR_ARG;
    const dim3 grid((unsigned)((rows + 3) / 4));
    auto launch = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, dim3(256), 0, (hipStream_t)stream, m, ldm, parts, (long long)part_stride,
                           bias, scale, P, v, rows, actions);
    };
    if (actions <= 64 * 8) {
        if (parts == 1)
            launch(policy_value_kernel<8, 1>);
        else if (parts <= 8)
            launch(policy_value_kernel<8, 8>);
        else
            launch(policy_value_kernel<8, PV_PMAX>);
    } else {
        if (parts == 1)
            launch(policy_value_kernel<PV_MAX_PER_LANE, 1>);
        else
            launch(policy_value_kernel<PV_MAX_PER_LANE, PV_PMAX>);
    }
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_policy_value(const float* m, int32_t ldm, const float* bias, float scale, float* P, float* v,
                                int32_t rows, int32_t actions, void* stream) {
    return azg_policy_value_parts(m, 1, 0, ldm, bias, scale, P, v, rows, actions, stream);
}
