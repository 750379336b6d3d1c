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
    // biases first, retired before the first store: vmcnt also counts stores, so a
    // bias load left pending behind the guarded stores serialises every store
    float bn[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) bn[j] = bias[n0 + wn + 32 * j + li];
#pragma unroll
    for (int j = 0; j < TN; ++j) asm volatile("s_waitcnt vmcnt(0)" : "+v"(bn[j]));
    const bool full = m0 + CBM <= M;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn + 32 * j + li;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
                if (full || m < M) y[(size_t)m * N + n] = fmaxf(acc[i][j][r] + bn[j], 0.0f);
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

// One wave's MFMA operands of one stage: A rows wm+li / wm+32+li as two b128
// chunks (q = 0, 1), B columns wn+li / wn+32+li at the 8 k of each q.
struct RingFrag {
    f32x4 a0[2], a1[2];
    float b0[2][4], b1[2][4];
};

// LDS operand reads in asm: hipcc's waitcnt pass cannot tell the in-flight DMA
// slots from the one read here (no alias scopes on LDS-DMA) and would drain
// vmcnt before every compiler-visible ds_read.  The waits are explicit
// (ring_wait_q0 / ring_wait_all); issue order: q = 0 operands first.
__device__ __forceinline__ void ring_read(RingFrag& f, unsigned a_q0, unsigned a_q1, unsigned b_ad) {
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
        : "=&v"(f.a0[0]), "=&v"(f.a1[0]), "=&v"(f.a0[1]), "=&v"(f.a1[1]), "=&v"(f.b0[0][0]), "=&v"(f.b0[0][1]),
          "=&v"(f.b0[0][2]), "=&v"(f.b0[0][3]), "=&v"(f.b1[0][0]), "=&v"(f.b1[0][1]), "=&v"(f.b1[0][2]),
          "=&v"(f.b1[0][3]), "=&v"(f.b0[1][0]), "=&v"(f.b0[1][1]), "=&v"(f.b0[1][2]), "=&v"(f.b0[1][3])
        : "v"(a_q0), "v"(a_q1), "v"(b_ad)
        : "memory");
    asm volatile(
        "ds_read_b32 %0, %4 offset:4224\n\t"
        "ds_read_b32 %1, %4 offset:4736\n\t"
        "ds_read_b32 %2, %4 offset:5248\n\t"
        "ds_read_b32 %3, %4 offset:5760\n\t"
        : "=&v"(f.b1[1][0]), "=&v"(f.b1[1][1]), "=&v"(f.b1[1][2]), "=&v"(f.b1[1][3])
        : "v"(b_ad)
        : "memory");
}

// q = 0 operands are the first 10 of the 20 reads
__device__ __forceinline__ void ring_wait_q0(RingFrag& f) {
    asm volatile("s_waitcnt lgkmcnt(10)"
                 : "+v"(f.a0[0]), "+v"(f.a1[0]), "+v"(f.b0[0][0]), "+v"(f.b0[0][1]), "+v"(f.b0[0][2]),
                   "+v"(f.b0[0][3]), "+v"(f.b1[0][0]), "+v"(f.b1[0][1]), "+v"(f.b1[0][2]), "+v"(f.b1[0][3]));
}

__device__ __forceinline__ void ring_wait_all(RingFrag& f) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(f.a0[0]), "+v"(f.a1[0]), "+v"(f.b0[0][0]), "+v"(f.b0[0][1]), "+v"(f.b0[0][2]),
                   "+v"(f.b0[0][3]), "+v"(f.b1[0][0]), "+v"(f.b1[0][1]), "+v"(f.b1[0][2]), "+v"(f.b1[0][3]));
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(f.a0[1]), "+v"(f.a1[1]), "+v"(f.b0[1][0]), "+v"(f.b0[1][1]), "+v"(f.b0[1][2]),
                   "+v"(f.b0[1][3]), "+v"(f.b1[1][0]), "+v"(f.b1[1][1]), "+v"(f.b1[1][2]), "+v"(f.b1[1][3]));
}

__device__ __forceinline__ void ring_mma(const RingFrag& f, int q, f32x16& acc00, f32x16& acc01, f32x16& acc10,
                                         f32x16& acc11) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // k = 8q + 4h + j
        acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(f.a0[q][j], f.b0[q][j], acc00, 0, 0, 0);
        acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(f.a0[q][j], f.b1[q][j], acc01, 0, 0, 0);
        acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(f.a1[q][j], f.b0[q][j], acc10, 0, 0, 0);
        acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(f.a1[q][j], f.b1[q][j], acc11, 0, 0, 0);
    }
}

// PIPE = false (variant 4): per stage, wait + barrier, issue stage ks+2, read and
// compute stage ks.  PIPE = true (variant 5): three stages in flight; stage ks
// computes from registers read during stage ks-1: q = 0 MFMAs, then the barrier
// that publishes stage ks+1 (and frees slot ks for stage ks+3's DMA), then the
// reads of stage ks+1 overlap the q = 1 MFMAs.
// Tile schedule with a split-K tail.  The T = mtiles x ntn output tiles are
// ordered so that the ntn channel tiles of 8 consecutive pixel tiles share
// block ids equal mod 8 (one XCD under round-robin dispatch, so a pixel
// tile's gathered inputs are re-read from one L2).  With P blocks resident on
// the chip, T tiles run as ceil(T / P) rounds; the last r = T mod P tiles would
// leave most of the chip idle in the final round, so each of them is split
// into S K-ranges (S = P / r) whose partial tiles go to a workspace and are
// summed in a fixed order (deterministic) by ring_tail_reduce_kernel.
struct RingSched {
    int mtiles, ntn, t_full, S, ntrip;  // t_full = T - r unsplit tiles; ntrip = nks / 3
    float* ws;                          // [r][S][64][256] partial accumulators
};

__device__ __forceinline__ void ring_tile(int t, int mtiles, int ntn, int& mt, int& nt) {
    const int mfull = mtiles & ~7, tg = mfull * ntn;
    if (t < tg) {
        const int grp = t / (8 * ntn), rr = t - grp * 8 * ntn;
        mt = grp * 8 + (rr & 7);
        nt = rr >> 3;
    } else {  // the last, partial group of pixel tiles
        const int rem = mtiles - mfull, u = t - tg;
        mt = mfull + u % rem;
        nt = u / rem;
    }
}

template <bool PIPE>
__global__ __launch_bounds__(256, 3) void conv3x3_ring_kernel(const float* __restrict__ x, const float* __restrict__ wt,
                                                              const float* __restrict__ bias, float* __restrict__ y,
                                                              const float* __restrict__ zero_page, int M, int HWo,
                                                              int Wo, int Hi, int Wi, int pad, int C, int N,
                                                              RingSched sc) {
    __shared__ __attribute__((aligned(16))) float ring0[R_STAGE];
    __shared__ __attribute__((aligned(16))) float ring1[R_STAGE];
    __shared__ __attribute__((aligned(16))) float ring2[R_STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    int t = blockIdx.x, part = -1, ks_begin = 0, ks_end = sc.ntrip * 3;
    if (t >= sc.t_full) {  // split tail tile: K-range `part` of S
        const int u = t - sc.t_full;
        part = u % sc.S;
        t = sc.t_full + u / sc.S;
        ks_begin = 3 * (part * sc.ntrip / sc.S);
        ks_end = 3 * ((part + 1) * sc.ntrip / sc.S);
    }
    int mt, nt;
    ring_tile(t, sc.mtiles, sc.ntn, mt, nt);
    const int m0 = mt * CBM, n0 = nt * R_BN;

    // A DMA: wave w fills pixels 32w + 16t + lane/4 (t = 0, 1), slot lane%4 holding chunk slot^((m>>2)&3)
    // a_px: input address of output pixel (oy, ox) at tap (pad, pad) -- each stage adds a
    // wave-uniform tap/channel offset; rows outside M get oy = -4 Hi so every tap is masked
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
    // stages are issued in increasing order: the next stage's (tap dy/dx, channel
    // c0) and weight row advance incrementally (no divisions on the issue path)
    int nc0, ndy, ndx;
    {
        const int k0 = ks_begin * R_BK, tap = k0 / C;
        nc0 = k0 - tap * C;
        ndy = tap / 3;
        ndx = tap - ndy * 3;
        wb += (size_t)k0 * N;
    }
    auto issue = [&](int, float* As) {
        float* Bs = As + R_ASTAGE;
        const long off = ((long)(ndy - pad) * Wi + (ndx - pad)) * C + nc0;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const bool ok = (unsigned)(a_oy[t] + ndy) < (unsigned)Hi && (unsigned)(a_ox[t] + ndx) < (unsigned)Wi;
            const float* src = ok ? a_px[t] + off : zero_page;
            __builtin_amdgcn_global_load_lds((const void*)src, (void*)(As + (32 * wid + 16 * t) * R_BK), 16, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < 2; ++t)
            __builtin_amdgcn_global_load_lds((const void*)(wb + (size_t)(2 * t) * N),
                                             (void*)(Bs + (4 * wid + 2 * t) * R_BN), 16, 0, 0);
        wb += (size_t)R_BK * N;
        nc0 += R_BK;
        if (nc0 == C) {
            nc0 = 0;
            if (++ndx == 3) {
                ndx = 0;
                ++ndy;
            }
        }
    };

    f32x16 acc00 = {}, acc01 = {}, acc10 = {}, acc11 = {};
    const int wm = (wid >> 1) * 64, wn = (wid & 1) * 64;
    const int li = lane & 31, h = lane >> 5;
    const int sw = (li >> 2) & 3;  // swizzle of rows wm + li and wm + 32 + li
    auto read = [&](RingFrag& f, const float* As) {
        ring_read(f, lds_addr(As + (wm + li) * R_BK + ((0 + h) ^ sw) * 4),
                  lds_addr(As + (wm + li) * R_BK + ((2 + h) ^ sw) * 4), lds_addr(As + R_ASTAGE + wn + li + 4 * h * R_BN));
    };
    if constexpr (!PIPE) {
        // one stage: wait for this wave's stage-ks DMA, barrier (every wave's landed,
        // stage ks-1 consumed), issue stage ks+2 into the slot stage ks-1 used, compute ks
        auto stage = [&](int ks, const float* As, float* next2) {
            if (ks + 1 < ks_end)
                asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            if (ks + 2 < ks_end) issue(ks + 2, next2);
            RingFrag f;
            read(f, As);
            ring_wait_q0(f);
            ring_mma(f, 0, acc00, acc01, acc10, acc11);
            __builtin_amdgcn_sched_barrier(0);  // keep the q = 0 MFMAs ahead of the next wait
            ring_wait_all(f);
            ring_mma(f, 1, acc00, acc01, acc10, acc11);
        };
        // three named slots (distinct LDS objects), loop unrolled by 3: every access
        // names a fixed object
        issue(ks_begin, ring0);
        issue(ks_begin + 1, ring1);
        for (int ks = ks_begin; ks < ks_end; ks += 3) {  // K ranges are whole multiples of 3 stages
            stage(ks, ring0, ring2);
            stage(ks + 1, ring1, ring0);
            stage(ks + 2, ring2, ring1);
        }
    } else {
        RingFrag cur;
        auto stage = [&](int ks, const float* As_next, float* dma_slot) {
            ring_mma(cur, 0, acc00, acc01, acc10, acc11);
            RingFrag nx;
            const bool more = ks + 1 < ks_end;
            if (more) {
                if (ks + 2 < ks_end)
                    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // stage ks+1 landed (this wave)
                else
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();  // every wave's stage ks+1 landed, slot ks read
                if (ks + 3 < ks_end) issue(ks + 3, dma_slot);
                read(nx, As_next);
            }
            __builtin_amdgcn_sched_barrier(0);
            ring_mma(cur, 1, acc00, acc01, acc10, acc11);
            if (more) {
                __builtin_amdgcn_sched_barrier(0);
                ring_wait_all(nx);
                cur = nx;
            }
        };
        issue(ks_begin, ring0);
        issue(ks_begin + 1, ring1);
        issue(ks_begin + 2, ring2);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        read(cur, ring0);
        ring_wait_all(cur);
        for (int ks = ks_begin; ks < ks_end; ks += 3) {  // stage ks reads slot (ks+1)%3, refills slot ks%3
            stage(ks, ring1, ring0);
            stage(ks + 1, ring2, ring1);
            stage(ks + 2, ring0, ring2);
        }
    }
    if (part >= 0) {  // partial tile: registers to the workspace, coalesced per register
        float* w = sc.ws + ((size_t)(t - sc.t_full) * sc.S + part) * 64 * 256 + tid;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            w[(r + 0) * 256] = acc00[r];
            w[(r + 16) * 256] = acc01[r];
            w[(r + 32) * 256] = acc10[r];
            w[(r + 48) * 256] = acc11[r];
        }
        return;
    }
    const int nA = n0 + wn + li, nB = nA + 32;
    float bA = bias[nA], bB = bias[nB];
    // retire the bias loads before the first store (vmcnt also counts stores: a
    // pending load behind guarded stores serialises every store)
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(bA), "+v"(bB));
    const bool full = m0 + CBM <= M;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int mA = m0 + wm + row, mB = mA + 32;
        if (full || mA < M) {
            y[(size_t)mA * N + nA] = fmaxf(acc00[r] + bA, 0.0f);
            y[(size_t)mA * N + nB] = fmaxf(acc01[r] + bB, 0.0f);
        }
        if (full || mB < M) {
            y[(size_t)mB * N + nA] = fmaxf(acc10[r] + bA, 0.0f);
            y[(size_t)mB * N + nB] = fmaxf(acc11[r] + bB, 0.0f);
        }
    }
}

// Sum the S partial tiles of each split tail tile in part order, then bias +
// ReLU + store -- the epilogue conv3x3_ring_kernel skipped for them.
__global__ __launch_bounds__(256) void ring_tail_reduce_kernel(const float* __restrict__ bias, float* __restrict__ y,
                                                               int M, int N, RingSched sc) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int t = sc.t_full + blockIdx.x;
    int mt, nt;
    ring_tile(t, sc.mtiles, sc.ntn, mt, nt);
    const int m0 = mt * CBM, n0 = nt * R_BN;
    const int wm = (wid >> 1) * 64, wn = (wid & 1) * 64, li = lane & 31, h = lane >> 5;
    const float* w = sc.ws + (size_t)blockIdx.x * sc.S * 64 * 256 + tid;
    const int nA = n0 + wn + li, nB = nA + 32;
    const float bA = bias[nA], bB = bias[nB];
    for (int r = 0; r < 16; ++r) {
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float a = w[(r + 16 * q) * 256];
            for (int p = 1; p < sc.S; ++p) a += w[((size_t)p * 64 + r + 16 * q) * 256];
            v[q] = a;
        }
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int mA = m0 + wm + row, mB = mA + 32;
        if (mA < M) {
            y[(size_t)mA * N + nA] = fmaxf(v[0] + bA, 0.0f);
            y[(size_t)mA * N + nB] = fmaxf(v[1] + bB, 0.0f);
        }
        if (mB < M) {
            y[(size_t)mB * N + nA] = fmaxf(v[2] + bA, 0.0f);
            y[(size_t)mB * N + nB] = fmaxf(v[3] + bB, 0.0f);
        }
    }
}

// device-wide workspace for split tails (grown on demand: the first call of a
// shape allocates, so capture a HIP graph only after an eager call)
float* g_ring_ws = nullptr;
size_t g_ring_ws_bytes = 0;

template <bool PIPE>
int launch_ring(const float* x, const float* wt, const float* bias, float* y, int batch, int h_in, int pad, int c_in,
                int c_out, hipStream_t st) {
    const int h_out = h_in + 2 * pad - 2;
    if (c_in % R_BK || c_out % R_BN) return AZG_ERR_ARG;  // nks = 9 c_in / 16: a multiple of 9
    const int M = batch * h_out * h_out;
    const int ntn = c_out / R_BN;
    const int mtiles = (M + CBM - 1) / CBM;
    static const float* zero_page = nullptr;
    if (!zero_page && hipGetSymbolAddress((void**)&zero_page, HIP_SYMBOL(g_zero_page)) != hipSuccess)
        return AZG_ERR_HIP;
    static int resident = 0, cus = 0;  // blocks the whole chip holds at once; CUs
    if (!resident) {
        int dev = 0, per_cu = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, conv3x3_ring_kernel<PIPE>, 256, 0) != hipSuccess)
            return AZG_ERR_HIP;
        resident = cus * (per_cu > 0 ? per_cu : 1);
    }
    RingSched sc;
    sc.mtiles = mtiles;
    sc.ntn = ntn;
    sc.ntrip = 9 * c_in / R_BK / 3;
    // A tail of at most one block per CU runs alone on its CU, i.e. at up to 3x the
    // shared speed, and costs ~1/3 of a round: splitting it measured slower
    // (conv2/3 at 4096 leaves).  Split only a tail of more than one block per CU.
    const int T = mtiles * ntn, r = T % resident;
    sc.S = r > cus ? resident / r : 1;
    if (sc.S > sc.ntrip / 2) sc.S = sc.ntrip / 2;
    if (sc.S < 2) {
        sc.S = 1;
        sc.t_full = T;
        sc.ws = nullptr;
    } else {
        sc.t_full = T - r;
        const size_t need = (size_t)r * sc.S * 64 * 256 * sizeof(float);
        if (need > g_ring_ws_bytes) {
            if (g_ring_ws) (void)hipFree(g_ring_ws);
            g_ring_ws = nullptr;
            g_ring_ws_bytes = 0;
            if (hipMalloc((void**)&g_ring_ws, need) != hipSuccess) return AZG_ERR_HIP;
            g_ring_ws_bytes = need;
        }
        sc.ws = g_ring_ws;
    }
    const int blocks = sc.t_full + (T - sc.t_full) * sc.S;
    hipLaunchKernelGGL(conv3x3_ring_kernel<PIPE>, dim3(blocks), dim3(256), 0, st, x, wt, bias, y, zero_page, M,
                       h_out * h_out, h_out, h_in, h_in, pad, c_in, c_out, sc);
    if (hipGetLastError() != hipSuccess) return AZG_ERR_HIP;
    if (sc.S > 1) {
        hipLaunchKernelGGL(ring_tail_reduce_kernel, dim3(T - sc.t_full), dim3(256), 0, st, bias, y, M, c_out, sc);
        if (hipGetLastError() != hipSuccess) return AZG_ERR_HIP;
    }
    return 0;
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
        case 4: return launch_ring<false>(x, wt, bias, y, batch, h_in, pad, c_in, c_out, st);
        case 5: return launch_ring<true>(x, wt, bias, y, batch, h_in, pad, c_in, c_out, st);
        default: return AZG_ERR_ARG;
    }
}

extern "C" int azg_conv3x3_bias_relu_nhwc(const float* x, const float* wt, const float* bias, float* y,
                                          int32_t batch, int32_t h_in, int32_t pad, int32_t c_in, int32_t c_out,
                                          void* stream) {
    // variant 4 (LDS-DMA ring, split-K tail) measured fastest of libazg's on conv2-4 at 4096 leaves
    // (profiles/r01_conv_probe.json)
    return azg_conv3x3_variant(4, x, wt, bias, y, batch, h_in, pad, c_in, c_out, stream);
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
