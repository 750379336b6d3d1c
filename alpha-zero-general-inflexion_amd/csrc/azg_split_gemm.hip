// azg_split_gemm.hip -- the Winograd GEMMs of the leaf network (azg_winograd.hip)
// as an error-compensated fp16 MFMA GEMM, hand-written for gfx950.
//
// Per transformed point e:  M_e [T x K] (f32) = V_e [T x C] x U_e [C x K], with both
// f32 operands split exactly into fp16 halves, v = vh + vl (+ 2^-22 |v|), and
//     M = Vh Uh + Vl Uh + Vh Ul      (the 2^-22 Vl Ul term dropped)
// computed by v_mfma_f32_16x16x32_f16 with f32 accumulation: f32-accurate products
//  at the fp16 MFMA rate.  Operands are stored once per half:
//   A = V_e : [T][2C] fp16 rows [hi(C) | lo(C)]     (the transforms write them)
//   B = U_e : [K][2C] fp16 rows [hi(C) | lo(C)]     (U^T, formed once per weight set)
// i.e. 4 bytes per operand element, as f32, where a library GEMM needs the A
// row [hi | lo | hi] (6 bytes).  U is pre-scaled by a power of two that the
// output transform undoes.
//
// Tiling: 256 x 256 output tile per 512-thread workgroup (8 waves as 2 (rows) x 4
// (cols), 128 x 64 per wave = 8 x 4 accumulators of 16 x 16), 32 channels per
// K stage.  Both operands go global -> LDS by LDS-DMA (global_load_lds_dwordx4,
// 1 KB per wave-instruction) into two stage buffers of 64 KB; an LDS row is one
// tile row's 32 channels: hi (4 x 16 B) then lo (4 x 16 B), 16-B chunk c stored at
// c ^ ((row >> 1) & 7), so each 16-lane group of a ds_read_b128 (16 rows, one
// chunk) covers all 16 slots of the 256-B bank row (conflict-free).  Per stage a
// wave reads its operands (16 A + 8 B ds_read_b128), issues the next stage's DMA
// (8 per wave), then runs 96 MFMAs; a vmcnt(0) + barrier closes the stage, so the
// DMA lands under the MFMAs and the reads never wait on a DMA in flight.
//
// The tiles of all GEMMs of a layer (runs of points with equal T) are one grid;
// block ids are dealt to the 8 XCDs round-robin, so the mapping gives each XCD a
// contiguous range of tiles: a row tile's two column tiles run side by side on
// one XCD and share its A tile through that L2.
#include <hip/hip_runtime.h>

#include "../../include/azg.h"

namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;
using f16x8 = __attribute__((ext_vector_type(8))) _Float16;

constexpr int SG_BM = 256, SG_BN = 256, SG_BK = 32;
constexpr int SG_ROWB = 128;                 // LDS bytes per tile row per stage (hi + lo)
constexpr int SG_TILEB = SG_BM * SG_ROWB;    // 32 KB per operand per stage
constexpr int SG_STAGEB = 2 * SG_TILEB;      // A then B
constexpr int SG_MAXRUNS = 4;

struct SGArgs {
    const _Float16* A;
    const _Float16* Bt;
    float* M;
    int nruns, C, K, ntn;  // ntn = K / 256 column tiles
    int total;             // tiles of all runs
    int points[SG_MAXRUNS], rows[SG_MAXRUNS], mtiles[SG_MAXRUNS], tile0[SG_MAXRUNS + 1], b_pt0[SG_MAXRUNS];
    long long a_off[SG_MAXRUNS], m_off[SG_MAXRUNS];
};

__global__ __launch_bounds__(512, 1) void split_gemm_kernel(SGArgs g) {
    __shared__ __attribute__((aligned(16))) char smem[2 * SG_STAGEB];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

    // block -> tile: each XCD (bid % 8) takes one contiguous range (bijective)
    int L;
    {
        const int bid = blockIdx.x, xcd = bid % 8, q = g.total / 8, rr = g.total % 8;
        L = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
    }
    int r = 0;
    while (r + 1 < g.nruns && L >= g.tile0[r + 1]) ++r;
    const int u = L - g.tile0[r];
    const int nt = u % g.ntn;
    const int mt = (u / g.ntn) % g.mtiles[r];
    const int e = u / (g.ntn * g.mtiles[r]);
    const int T = g.rows[r], C = g.C, K = g.K, C2 = 2 * C;
    const int m0 = mt * SG_BM, n0 = nt * SG_BN;
    const _Float16* Ae = g.A + g.a_off[r] + (long long)e * T * C2;
    const _Float16* Be = g.Bt + (long long)(g.b_pt0[r] + e) * K * C2;
    float* Me = g.M + g.m_off[r] + (long long)e * T * K;

    // DMA sources: wave w fills tile rows 32w + 8i + lane/8 (i < 4) of A and of B;
    // lane%8 is the physical 16-B chunk, holding logical chunk lc = phys ^ ((row>>1)&7):
    // hi channels 8lc.. (lc < 4) or lo channels 8(lc-4).. of the stage
    const _Float16* asrc[4];
    const _Float16* bsrc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int R = 32 * wid + 8 * i + (lane >> 3);
        const int lc = (lane & 7) ^ ((R >> 1) & 7);
        const int col = lc < 4 ? 8 * lc : C + 8 * (lc - 4);
        const int arow = m0 + R < T ? m0 + R : T - 1;  // rows past T: loaded, never stored
        asrc[i] = Ae + (long long)arow * C2 + col;
        bsrc[i] = Be + (long long)(n0 + R) * C2 + col;
    }
    auto issue = [&](int ks, int buf) {
        char* base = smem + buf * SG_STAGEB + (32 * wid) * SG_ROWB;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + ks * SG_BK),
                                             (__attribute__((address_space(3))) void*)(base + 8 * i * SG_ROWB), 16, 0,
                                             0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + ks * SG_BK),
                                             (__attribute__((address_space(3))) void*)(base + SG_TILEB +
                                                                                      8 * i * SG_ROWB),
                                             16, 0, 0);
    };

    // operand reads: wave (wm, wn) = rows 128 wm.., cols 64 wn..; lane holds row lane%16
    // of a 16-row block, channels 8 (lane/16).. of the 32 (hi) and the same of lo
    const int wm = wid >> 2, wn = wid & 3;
    const int lr = lane & 15, sw = lr >> 1;  // (row >> 1) & 7 of every 16-row block
    const int ch = lane >> 4;
    const int a_hi = (wm * 128 + lr) * SG_ROWB + 16 * (ch ^ sw);
    const int a_lo = (wm * 128 + lr) * SG_ROWB + 16 * ((4 + ch) ^ sw);
    const int b_hi = SG_TILEB + (wn * 64 + lr) * SG_ROWB + 16 * (ch ^ sw);
    const int b_lo = SG_TILEB + (wn * 64 + lr) * SG_ROWB + 16 * ((4 + ch) ^ sw);

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nks = C / SG_BK;
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int ks = 0; ks < nks; ++ks) {
        const char* st = smem + (ks & 1) * SG_STAGEB;
        f16x8 ah[8], al[8], bh[4], bl[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            bh[j] = *(const f16x8*)(st + b_hi + 16 * j * SG_ROWB);
            bl[j] = *(const f16x8*)(st + b_lo + 16 * j * SG_ROWB);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            ah[i] = *(const f16x8*)(st + a_hi + 16 * i * SG_ROWB);
            al[i] = *(const f16x8*)(st + a_lo + 16 * i * SG_ROWB);
        }
        if (ks + 1 < nks) issue(ks + 1, (ks + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);  // the DMA issue stays ahead of the MFMAs
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
            }
        __builtin_amdgcn_sched_barrier(0);  // ... and the stage's closing wait behind them
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    // epilogue: C/D map of 16x16x32: col = lane % 16, row = 4 (lane / 16) + reg
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = m0 + wm * 128 + 16 * i + 4 * ch + q;
            if (row >= T) continue;
            float* out = Me + (long long)row * K + n0 + wn * 64 + lr;
#pragma unroll
            for (int j = 0; j < 4; ++j) out[16 * j] = acc[i][j][q];
        }
    }
}

}  // namespace

extern "C" int azg_split_gemm(const void* A, const void* Bt, float* M, int32_t nruns, const int32_t* points,
                              const int32_t* rows, int32_t c, int32_t k, void* stream) {
    if (!A || !Bt || !M || !points || !rows || nruns < 1 || nruns > SG_MAXRUNS || c <= 0 || c % SG_BK ||
        k <= 0 || k % SG_BN || ((uintptr_t)A & 15) || ((uintptr_t)Bt & 15) || ((uintptr_t)M & 15))
        return AZG_ERR_ARG;
    SGArgs g{};
    g.A = (const _Float16*)A;
    g.Bt = (const _Float16*)Bt;
    g.M = M;
    g.nruns = nruns;
    g.C = c;
    g.K = k;
    g.ntn = k / SG_BN;
    long long a = 0, m = 0;
    int tiles = 0, pt = 0;
    for (int r = 0; r < nruns; ++r) {
        if (points[r] <= 0 || rows[r] <= 0) return AZG_ERR_ARG;
        g.points[r] = points[r];
        g.rows[r] = rows[r];
        g.mtiles[r] = (rows[r] + SG_BM - 1) / SG_BM;
        g.tile0[r] = tiles;
        g.a_off[r] = a;
        g.m_off[r] = m;
        g.b_pt0[r] = pt;
        const long long t = (long long)points[r] * g.mtiles[r] * g.ntn;
        if (tiles + t > (1ll << 30)) return AZG_ERR_ARG;
        tiles += (int)t;
        a += (long long)points[r] * rows[r] * 2 * c;
        m += (long long)points[r] * rows[r] * k;
        pt += points[r];
    }
    g.tile0[nruns] = tiles;
    g.total = tiles;
    hipLaunchKernelGGL(split_gemm_kernel, dim3(tiles), dim3(512), 0, (hipStream_t)stream, g);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}
