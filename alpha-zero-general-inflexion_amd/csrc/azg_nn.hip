// azg_nn.hip -- leaf-network kernels (NHWC activations, f32).
//
//  * bias_relu_nhwc: the BatchNorm-folded bias + ReLU in ONE read-modify-write
//    pass over an NHWC activation (HBM-bound, float4 per lane, grid-stride).
//  * conv3x3 implicit GEMM on f32 MFMA with the bias + ReLU fused into the
//    epilogue (conv2-4 + bn2-4 + relu of InflexionNNet.forward):
//        y[m, n] = relu(bias[n] + sum_k A[m, k] * W[k, n]),
//        m = output pixel (b, oy, ox), k = tap * C + c, tap = dy * 3 + dx,
//        A[m, k] = x[b, oy + dy - pad, ox + dx - pad, c] (0 outside the image),
//    W pre-transposed to [9*C][N] (k-major).  Per 256-thread workgroup a
//    128 (pixels) x BN (channels) tile, K in steps of BK; the 4 waves form a
//    2x2 grid, each owning 64 x BN/2 as (BN/64) x 2 v_mfma_f32_32x32x2_f32
//    accumulators.  A is gathered with zero padding (unconditional loads from
//    a zero page), transposed into a k-major LDS image (conflict-free fragment
//    reads) through registers; B (a plain row copy) goes global -> LDS by
//    global_load_lds.  Both are double-buffered: stage k+1's loads are issued
//    before stage k's MFMAs.  The channel tiles of one pixel tile get block ids
//    that are equal mod 8 (one XCD under round-robin dispatch) so the gathered
//    pixels are re-read from that XCD's L2 -- a speed choice only.
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

using f32x16 = __attribute__((ext_vector_type(16))) float;
using f32x4 = __attribute__((ext_vector_type(4))) float;

// byte offset of a __shared__ address inside the workgroup's LDS (operand of ds_* asm)
__device__ __forceinline__ unsigned lds_addr(const float* p) {
    return (unsigned)(size_t)(const __attribute__((address_space(3))) float*)p;
}
constexpr int CBM = 128;

// Zero page for the padding taps: every A load is unconditional (a select
// between a load and 0 makes hipcc wait for the load right after issuing it).
__device__ __attribute__((aligned(16))) float g_zero_page[64];

template <int BN, int BK, int MINB>
__global__ __launch_bounds__(256, MINB) void conv3x3_bias_relu_kernel(
    const float* __restrict__ x, const float* __restrict__ wt, const float* __restrict__ bias,
    float* __restrict__ y, int M, int HWo, int Wo, int Hi, int Wi, int pad, int C, int N) {
    constexpr int STAGE = BK * (CBM + BN);
    constexpr int TN = BN / 64;              // 32-col MFMA tiles per wave (wave covers BN/2 columns)
    constexpr int AV = BK / 8;               // float4 of A per thread per stage (2 threads per pixel)
    constexpr int BI = BK * BN / 256 / 4;    // global_load_lds (1 KB each) per wave per stage
    constexpr int BROWS = 256 / BN;          // B rows per global_load_lds
    __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int ntn = N / BN;
    const int grp = blockIdx.x / (8 * ntn), rr = blockIdx.x % (8 * ntn);
    const int mt = grp * 8 + (rr & 7), nt = rr >> 3;
    const int m0 = mt * CBM, n0 = nt * BN;
    if (m0 >= M) return;  // grid rounded up to whole XCD groups

    // A staging: pixel ap (0..127), channel half ah (BK/2 channels each)
    const int ap = tid >> 1, ah = tid & 1;
    const int am = m0 + ap;
    const bool a_ok = am < M;
    const int amc = a_ok ? am : 0;
    const int bimg = amc / HWo, rem = amc - bimg * HWo, oy = rem / Wo, ox = rem - (rem / Wo) * Wo;
    const float* xb = x + (size_t)bimg * Hi * Wi * C + (BK / 2) * ah;
    // B staging: wave-instruction i of wave w fills rows [(w*BI + i) * BROWS, +BROWS) of [BK][BN]
    const int brow = (lane * 4) / BN, bcol = (lane * 4) % BN;
    const float* wb = wt + (size_t)brow * N + n0 + bcol;

    float4 ra[AV];
    auto load_b = [&](int ks, int buf) {
        float* Bs = smem + buf * STAGE + BK * CBM;
        const float* src = wb + (size_t)ks * BK * N;
#pragma unroll
        for (int i = 0; i < BI; ++i) {
            const int r0 = (wid * BI + i) * BROWS;
            __builtin_amdgcn_global_load_lds((const void*)(src + (size_t)r0 * N), (void*)(Bs + r0 * BN), 16, 0, 0);
        }
    };
    auto load_a = [&](int ks) {
        const int k0 = ks * BK, tap = k0 / C, c0 = k0 - tap * C;
        const int dy = tap / 3, dx = tap - (tap / 3) * 3;
        const int iy = oy + dy - pad, ix = ox + dx - pad;
        const bool ok = a_ok && iy >= 0 && iy < Hi && ix >= 0 && ix < Wi;
        const float4* src = ok ? (const float4*)(xb + ((size_t)iy * Wi + ix) * C + c0) : (const float4*)g_zero_page;
#pragma unroll
        for (int i = 0; i < AV; ++i) ra[i] = src[i];
    };
    auto store_a = [&](int buf) {
        float* As = smem + buf * STAGE;
#pragma unroll
        for (int i = 0; i < AV; ++i) {
            const int k = (BK / 2) * ah + 4 * i;
            As[(k + 0) * CBM + ap] = ra[i].x;
            As[(k + 1) * CBM + ap] = ra[i].y;
            As[(k + 2) * CBM + ap] = ra[i].z;
            As[(k + 3) * CBM + ap] = ra[i].w;
        }
    };

    f32x16 acc[2][TN];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};
    const int wm = (wid >> 1) * 64, wn = (wid & 1) * (BN / 2);
    const int li = lane & 31, lk = lane >> 5;
    const int nks = 9 * C / BK;
    load_b(0, 0);
    load_a(0);
    store_a(0);
    __syncthreads();
    for (int ks = 0; ks < nks; ++ks) {
        const int cur = ks & 1;
        // unconditional (the last iteration reloads its own stage into the idle buffer):
        // guarded loads/stores let hipcc merge the guards and hoist the LDS writes
        const int nx = ks + 1 < nks ? ks + 1 : ks;
        load_b(nx, cur ^ 1);  // retired by the barrier's vmcnt(0) below
        load_a(nx);
        __builtin_amdgcn_sched_barrier(0);  // the next stage's loads go out before this stage's MFMAs
        const float* As = smem + cur * STAGE + wm + li + lk * CBM;
        const float* Bs = smem + cur * STAGE + BK * CBM + wn + li + lk * BN;
        // fragments of k-step kk+1 are read while the MFMAs of kk run
        float a[2], b[TN];
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = As[32 * i];
#pragma unroll
        for (int j = 0; j < TN; ++j) b[j] = Bs[32 * j];
#pragma unroll
        for (int kk = 0; kk < BK / 2; ++kk) {
            float na[2] = {0.f, 0.f}, nb[TN];
#pragma unroll
            for (int j = 0; j < TN; ++j) nb[j] = 0.f;
            if (kk + 1 < BK / 2) {
#pragma unroll
                for (int i = 0; i < 2; ++i) na[i] = As[(2 * kk + 2) * CBM + 32 * i];
#pragma unroll
                for (int j = 0; j < TN; ++j) nb[j] = Bs[(2 * kk + 2) * BN + 32 * j];
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 2; ++i) a[i] = na[i];
#pragma unroll
            for (int j = 0; j < TN; ++j) b[j] = nb[j];
        }
        store_a(cur ^ 1);
        __syncthreads();
    }
    // epilogue: C/D map col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn + 32 * j + li;
        const float bn = bias[n];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
                if (m < M) y[(size_t)m * N + n] = fmaxf(acc[i][j][r] + bn, 0.0f);
            }
        }
    }
}

// v2: both operands by LDS-DMA into a 3-stage ring, one raw barrier per stage.
// Tile 128 x 128 x 16.  A image per stage: [128 pixels][16 k] (64 B rows) with
// the 16-B chunk c of pixel m stored at slot c ^ ((m >> 2) & 3), so the
// ds_read_b128 fragment reads are bank-conflict free; lane half h of an MFMA
// reads chunk 2q + h and uses its 4 values for 4 MFMA k-steps, i.e. step
// (q, j) contracts k = 8q + j (h = 0) and k = 8q + 4 + j (h = 1).  B image
// [16 k][128 n] read with the same k permutation.  Per wave and stage: 2 A + 2 B
// global_load_lds (16 B/lane); stage ks+2 is issued right after the barrier
// that publishes stage ks, so two stages are always in flight.
constexpr int R_BK = 16, R_BN = 128, R_ASTAGE = CBM * R_BK, R_STAGE = R_ASTAGE + R_BK * R_BN;  // 3 ring slots

__global__ __launch_bounds__(256, 3) void conv3x3_ring_kernel(const float* __restrict__ x, const float* __restrict__ wt,
                                                              const float* __restrict__ bias, float* __restrict__ y,
                                                              const float* __restrict__ zero_page, int M, int HWo,
                                                              int Wo, int Hi, int Wi, int pad, int C, int N) {
    __shared__ __attribute__((aligned(16))) float ring0[R_STAGE];
    __shared__ __attribute__((aligned(16))) float ring1[R_STAGE];
    __shared__ __attribute__((aligned(16))) float ring2[R_STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int ntn = N / R_BN;
    const int grp = blockIdx.x / (8 * ntn), rr = blockIdx.x % (8 * ntn);
    const int mt = grp * 8 + (rr & 7), nt = rr >> 3;
    const int m0 = mt * CBM, n0 = nt * R_BN;
    if (m0 >= M) return;

    // A DMA: wave w fills pixels 32w + 16t + lane/4 (t = 0, 1), slot lane%4 holding chunk slot^((m>>2)&3)
    // a_px: input address of output pixel (oy, ox) at tap (pad, pad) — each stage adds a
    // wave-uniform tap/channel offset; rows outside M get oy = -Hi so every tap is masked
    const float* a_px[2];
    int a_oy[2], a_ox[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int mloc = 32 * wid + 16 * t + (lane >> 2);
        const int am = m0 + mloc;
        const int amc = am < M ? am : 0;
        const int b = amc / HWo, rem = amc - b * HWo;
        a_oy[t] = am < M ? rem / Wo - pad : -4 * Hi;
        a_ox[t] = rem - (rem / Wo) * Wo - pad;
        a_px[t] = x + (((size_t)b * Hi + (rem / Wo)) * Wi + (rem - (rem / Wo) * Wo)) * C +
                  4 * ((lane & 3) ^ ((mloc >> 2) & 3));
    }
    // B DMA: wave w fills rows 4w + 2t + lane/32, 4 channels from (lane%32)*4
    const float* wb = wt + (size_t)(4 * wid + (lane >> 5)) * N + n0 + (lane & 31) * 4;

    auto issue = [&](int ks, float* As) {
        float* Bs = As + R_ASTAGE;
        const int k0 = ks * R_BK, tap = k0 / C, c0 = k0 - tap * C;
        const int dy = tap / 3, dx = tap - (tap / 3) * 3;
        const long off = ((long)(dy - pad) * Wi + (dx - pad)) * C + c0;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const bool ok = (unsigned)(a_oy[t] + dy) < (unsigned)Hi && (unsigned)(a_ox[t] + dx) < (unsigned)Wi;
            const float* src = ok ? a_px[t] + off : zero_page;
            __builtin_amdgcn_global_load_lds((const void*)src, (void*)(As + (32 * wid + 16 * t) * R_BK), 16, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < 2; ++t)
            __builtin_amdgcn_global_load_lds((const void*)(wb + (size_t)(k0 + 2 * t) * N),
                                             (void*)(Bs + (4 * wid + 2 * t) * R_BN), 16, 0, 0);
    };

    f32x16 acc00 = {}, acc01 = {}, acc10 = {}, acc11 = {};
    const int wm = (wid >> 1) * 64, wn = (wid & 1) * 64;
    const int li = lane & 31, h = lane >> 5;
    const int sw = (li >> 2) & 3;  // swizzle of rows wm + li and wm + 32 + li
    const int nks = 9 * C / R_BK;
    // one stage: wait for this wave's stage-ks DMA, barrier (every wave's landed,
    // stage ks-1 consumed), issue stage ks+2 into the slot stage ks-1 used, compute ks
    auto stage = [&](int ks, const float* As, float* next2) {
        if (ks + 1 < nks)
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (ks + 2 < nks) issue(ks + 2, next2);
        // LDS operand reads in asm: hipcc's waitcnt pass cannot tell the in-flight
        // DMA slots from the one read here and would drain vmcnt before every
        // compiler-visible ds_read. Waits for these reads are explicit below.
        const unsigned a_q0 = lds_addr(As + (wm + li) * R_BK + ((0 + h) ^ sw) * 4);
        const unsigned a_q1 = lds_addr(As + (wm + li) * R_BK + ((2 + h) ^ sw) * 4);
        const unsigned b_ad = lds_addr(As + R_ASTAGE + wn + li + 4 * h * R_BN);
        f32x4 a0[2], a1[2];
        float b0[2][4], b1[2][4];
        asm volatile(
            "ds_read_b128 %0, %16\n\t"
            "ds_read_b128 %1, %16 offset:2048\n\t"
            "ds_read_b32 %4, %18 offset:0\n\t"
            "ds_read_b32 %8, %18 offset:128\n\t"
            "ds_read_b32 %5, %18 offset:512\n\t"
            "ds_read_b32 %9, %18 offset:640\n\t"
            "ds_read_b32 %6, %18 offset:1024\n\t"
            "ds_read_b32 %10, %18 offset:1152\n\t"
            "ds_read_b32 %7, %18 offset:1536\n\t"
            "ds_read_b32 %11, %18 offset:1664\n\t"
            "ds_read_b128 %2, %17\n\t"
            "ds_read_b128 %3, %17 offset:2048\n\t"
            "ds_read_b32 %12, %18 offset:4096\n\t"
            "ds_read_b32 %13, %18 offset:4608\n\t"
            "ds_read_b32 %14, %18 offset:5120\n\t"
            "ds_read_b32 %15, %18 offset:5632\n\t"
            : "=&v"(a0[0]), "=&v"(a1[0]), "=&v"(a0[1]), "=&v"(a1[1]), "=&v"(b0[0][0]), "=&v"(b0[0][1]),
              "=&v"(b0[0][2]), "=&v"(b0[0][3]), "=&v"(b1[0][0]), "=&v"(b1[0][1]), "=&v"(b1[0][2]),
              "=&v"(b1[0][3]), "=&v"(b0[1][0]), "=&v"(b0[1][1]), "=&v"(b0[1][2]), "=&v"(b0[1][3])
            : "v"(a_q0), "v"(a_q1), "v"(b_ad)
            : "memory");
        asm volatile(
            "ds_read_b32 %0, %4 offset:4224\n\t"
            "ds_read_b32 %1, %4 offset:4736\n\t"
            "ds_read_b32 %2, %4 offset:5248\n\t"
            "ds_read_b32 %3, %4 offset:5760\n\t"
            : "=&v"(b1[1][0]), "=&v"(b1[1][1]), "=&v"(b1[1][2]), "=&v"(b1[1][3])
            : "v"(b_ad)
            : "memory");
        // q = 0 operands are the first 10 reads issued: 10 of 20 may still be pending
        asm volatile("s_waitcnt lgkmcnt(10)"
                     : "+v"(a0[0]), "+v"(a1[0]), "+v"(b0[0][0]), "+v"(b0[0][1]), "+v"(b0[0][2]), "+v"(b0[0][3]),
                       "+v"(b1[0][0]), "+v"(b1[0][1]), "+v"(b1[0][2]), "+v"(b1[0][3]));
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            if (q == 1) __builtin_amdgcn_sched_barrier(0);  // keep the q = 0 MFMAs ahead of this wait
            if (q == 1)
                asm volatile("s_waitcnt lgkmcnt(0)"
                             : "+v"(a0[1]), "+v"(a1[1]), "+v"(b0[1][0]), "+v"(b0[1][1]), "+v"(b0[1][2]),
                               "+v"(b0[1][3]), "+v"(b1[1][0]), "+v"(b1[1][1]), "+v"(b1[1][2]), "+v"(b1[1][3]));
#pragma unroll
            for (int j = 0; j < 4; ++j) {  // k = 8q + 4h + j
                acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[q][j], b0[q][j], acc00, 0, 0, 0);
                acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[q][j], b1[q][j], acc01, 0, 0, 0);
                acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[q][j], b0[q][j], acc10, 0, 0, 0);
                acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[q][j], b1[q][j], acc11, 0, 0, 0);
            }
        }
    };
    // three named slots (distinct LDS objects), loop unrolled by 3: hipcc can then
    // prove the in-flight DMA never targets the slot being read and leaves it in flight
    issue(0, ring0);
    if (nks > 1) issue(1, ring1);
    for (int ks = 0; ks < nks; ks += 3) {  // nks = 9 C / 16 is a multiple of 3
        stage(ks, ring0, ring2);
        stage(ks + 1, ring1, ring0);
        stage(ks + 2, ring2, ring1);
    }
    const int nA = n0 + wn + li, nB = nA + 32;
    const float bA = bias[nA], bB = bias[nB];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int mA = m0 + wm + row, mB = mA + 32;
        if (mA < M) {
            y[(size_t)mA * N + nA] = fmaxf(acc00[r] + bA, 0.0f);
            y[(size_t)mA * N + nB] = fmaxf(acc01[r] + bB, 0.0f);
        }
        if (mB < M) {
            y[(size_t)mB * N + nA] = fmaxf(acc10[r] + bA, 0.0f);
            y[(size_t)mB * N + nB] = fmaxf(acc11[r] + bB, 0.0f);
        }
    }
}

int launch_ring(const float* x, const float* wt, const float* bias, float* y, int batch, int h_in, int pad, int c_in,
                int c_out, hipStream_t st) {
    const int h_out = h_in + 2 * pad - 2;
    if (c_in % R_BK || c_out % R_BN) return AZG_ERR_ARG;
    const int M = batch * h_out * h_out;
    const int ntn = c_out / R_BN;
    const int mtiles = (M + CBM - 1) / CBM, groups = (mtiles + 7) / 8;
    static const float* zero_page = nullptr;
    if (!zero_page && hipGetSymbolAddress((void**)&zero_page, HIP_SYMBOL(g_zero_page)) != hipSuccess)
        return AZG_ERR_HIP;
    hipLaunchKernelGGL(conv3x3_ring_kernel, dim3(groups * 8 * ntn), dim3(256), 0, st, x, wt, bias, y, zero_page,
                       M, h_out * h_out, h_out, h_in, h_in, pad, c_in, c_out);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

template <int BN, int BK, int MINB>
int launch_conv(const float* x, const float* wt, const float* bias, float* y, int batch, int h_in, int pad, int c_in,
                int c_out, hipStream_t st) {
    const int h_out = h_in + 2 * pad - 2;
    if (c_in % BK || c_out % BN) return AZG_ERR_ARG;
    const int M = batch * h_out * h_out;
    const int ntn = c_out / BN;
    const int mtiles = (M + CBM - 1) / CBM, groups = (mtiles + 7) / 8;
    hipLaunchKernelGGL((conv3x3_bias_relu_kernel<BN, BK, MINB>), dim3(groups * 8 * ntn), dim3(256), 0, st, x, wt,
                       bias, y, M, h_out * h_out, h_out, h_in, h_in, pad, c_in, c_out);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}
}  // namespace

extern "C" int azg_conv3x3_variant(int variant, const float* x, const float* wt, const float* bias, float* y,
                                   int32_t batch, int32_t h_in, int32_t pad, int32_t c_in, int32_t c_out,
                                   void* stream) {
    const int h_out = h_in + 2 * pad - 2;
    if (!x || !wt || !bias || !y || batch <= 0 || h_out <= 0 || ((uintptr_t)x & 15) || ((uintptr_t)wt & 15))
        return AZG_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    switch (variant) {
        case 0: return launch_conv<128, 32, 2>(x, wt, bias, y, batch, h_in, pad, c_in, c_out, st);
        case 1: return launch_conv<128, 16, 3>(x, wt, bias, y, batch, h_in, pad, c_in, c_out, st);
        case 2: return launch_conv<256, 16, 2>(x, wt, bias, y, batch, h_in, pad, c_in, c_out, st);
        case 3: return launch_conv<256, 32, 1>(x, wt, bias, y, batch, h_in, pad, c_in, c_out, st);
        case 4: return launch_ring(x, wt, bias, y, batch, h_in, pad, c_in, c_out, st);
        default: return AZG_ERR_ARG;
    }
}

extern "C" int azg_conv3x3_bias_relu_nhwc(const float* x, const float* wt, const float* bias, float* y,
                                          int32_t batch, int32_t h_in, int32_t pad, int32_t c_in, int32_t c_out,
                                          void* stream) {
    // variant 1 (BN 128, BK 16, 3+ blocks per CU) measured fastest on conv2-4 at 4096 leaves
    // (profiles/r01_conv_probe.json)
    return azg_conv3x3_variant(1, x, wt, bias, y, batch, h_in, pad, c_in, c_out, stream);
}

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
