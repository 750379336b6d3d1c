// azg_split_gemm.hip -- the Winograd GEMMs of the leaf network (azg_winograd.hip)
// as an error-compensated fp16 MFMA GEMM, hand-written for gfx950.
//
// Per transformed point e:  M_e [T x K] (f32) = V_e [T x C] x U_e [C x K], with both
// f32 operands split exactly into fp16 halves, v = vh + vl (+ 2^-22 |v|), and
//     M = Vh Uh + Vl Uh + Vh Ul      (the 2^-22 Vl Ul term dropped)
// computed by v_mfma_f32_16x16x32_f16 with f32 accumulation: f32-accurate products
//  at the fp16 MFMA rate.  Operands are stored once per half:
//   A = V_e : [T][2C] fp16 rows of 32-channel blocks [hi(32) | lo(32)] (the transforms
//             write them, AZG_WINO_SPLIT2)
//   B = U_e : [K][2C] fp16 rows, the same blocks (U^T, formed once per weight set)
// i.e. 4 bytes per operand element, as f32, where a library GEMM needs the A
// row [hi | lo | hi] (6 bytes).  U is pre-scaled by a power of two that the
// output transform undoes.
//
// Tiling: 256 x 256 output tile per 512-thread workgroup (8 waves as 2 (rows) x 4
// (cols), 128 x 64 per wave = 8 x 4 accumulators of 16 x 16), 32 channels per
// K stage.  Both operands go global -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds,
// 1 KB per wave-instruction) into two stage buffers of 64 KB; an LDS row is one
// tile row's 32 channels: hi (4 x 16 B) then lo (4 x 16 B), 16-B chunk c stored at
// c ^ ((row >> 1) & 7), so each 16-lane group of a ds_read_b128 (16 rows, one
// chunk) covers all 16 slots of the 256-B bank row (conflict-free).  A stage is
// 16 A + 8 B ds_read_b128 and 96 MFMAs per wave plus 8 DMA issues; variant 0 runs
// them in that order with a vmcnt(0) + barrier per stage, one tile per workgroup;
// variant 4 (default) is variant 0 as a persistent kernel (one workgroup per CU,
// the next tile's first stage loaded under the current tile's last); variant 1
// overlaps each phase's reads with the previous phase's MFMAs, variant 2 runs one
// wave per SIMD on 128 x 128 per wave, variant 3 spreads the DMA issue between the
// MFMAs.  Measured on conv2's shape (tools/split_gemm_bench.py, round-robin medians,
// profiles/r01_split_gemm_bench.json), TF/s of fp16 MFMA work: variant 4 1116,
// 7 1091, 12 1073, 0 1072; hipBLASLt on the [hi|lo|hi] form 903.  PMC
// (tools/split_gemm_pmc.py): no LDS bank conflicts, MFMA busy 61% (variant 4).  The
// bound is the global -> LDS operand feed (~5.8 TB/s chip-wide; zeroing either
// operand's DMA runs 33% faster, both 50%: variants 6, 15, 16), which is why the
// operand rows are 32-channel [hi | lo] blocks (one 128-B line per row per stage).
//
// The tiles of all GEMMs of a layer (runs of points with equal T) are one grid;
// block ids are dealt to the 8 XCDs round-robin, so the mapping gives each XCD a
// contiguous range of tiles: a row tile's two column tiles run side by side on
// one XCD and share its A tile through that L2.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "../../include/azg.h"

namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;
using f16x8 = __attribute__((ext_vector_type(8))) _Float16;

constexpr int SG_BM = 256, SG_BN = 256, SG_BK = 32;
constexpr int SG_ROWB = 128;                 // LDS bytes per tile row per stage (hi + lo)
constexpr int SG_TILEB = SG_BM * SG_ROWB;    // 32 KB per operand per stage
constexpr int SG_STAGEB = 2 * SG_TILEB;      // A then B
constexpr int SG_MAXRUNS = 4;
// Operand rows are 32-channel blocks [hi(32) | lo(32)] (AZG_WINO_SPLIT2): stage ks of a
// row is the one 128-B line at byte 128 ks, logical chunk lc (hi 8 lc.. for lc < 4, lo
// 8 (lc - 4).. after) at 16 lc within it.
constexpr int SG_STAGE_SOFF = 2 * SG_BK * 2;

struct SGArgs {
    const _Float16* A;
    const _Float16* Bt;
    float* M;
    int nruns, C, K, ntn;  // ntn = K / 256 column tiles
    int total;             // tiles of all runs
    int points[SG_MAXRUNS], rows[SG_MAXRUNS], mtiles[SG_MAXRUNS], tile0[SG_MAXRUNS + 1], b_pt0[SG_MAXRUNS];
    long long a_off[SG_MAXRUNS], m_off[SG_MAXRUNS];
    unsigned long long* stamps;  // diagnostic build only: per-wave segment cycle sums
};

// B tile row R of the LDS image (column block j = (R % 64) / 16, lane lr = R % 16 of
// a wave's 64 columns) holds output column 64 (R / 64) + 4 lr + j: lane lr's four
// column blocks are then four adjacent columns, stored as one 16-B write per row in
// the epilogue.  LDS rows R and R + 16 (j, j + 1) are adjacent columns, so the B
// DMA's second descriptor starts one row on.
__device__ __forceinline__ int b_col(int R) { return (R & ~63) | ((R & 15) << 2) | ((R >> 4) & 3); }

// byte address of a __shared__ location in the workgroup's LDS (operand of ds_* asm)
[[maybe_unused]] __device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p;
}

// Variant 0: per stage, all operand reads, then the next stage's DMA, then 96 MFMAs,
// then vmcnt(0) + barrier (reads and MFMAs of a wave do not overlap).
// Variant 3 (ILV = true): the same, with the next stage's 8 DMA pieces issued one per
// row block between the MFMAs instead of in one burst before them.
// Variant 17 (BM = 128): variant 0 on 128 x 256 tiles (64 x 64 per wave, 48 MFMAs per
// stage, 48 KB stage buffers): twice the tiles of the 256-row form for launches that
// fill less than a round of the chip (a few hundred leaves: conv3 / conv4 at 256
// leaves are 98 / 50 tiles of 256 rows on 256 CUs), at twice the A-operand bytes per
// flop; azg_split_gemm picks it by round count (split_gemm_pick).  Variant 18 (BM = 64)
// is the same on 64 x 256 tiles (32 x 64 per wave).
template <bool ILV, int BM = SG_BM>
__global__ __launch_bounds__(512, 1) void split_gemm_kernel(SGArgs g) {
    static_assert(BM == 256 || ((BM == 128 || BM == 64) && !ILV), "row tile");
    constexpr int ATILEB = BM * SG_ROWB;       // A bytes per stage
    constexpr int STAGEB = ATILEB + SG_TILEB;  // A then B (256 rows)
    constexpr int NI = BM / 32;                // 16-row blocks per wave
    constexpr int AP = BM / 64;                // A DMA pieces (8 rows each) per wave
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGEB];
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
    const int m0 = mt * BM, n0 = nt * SG_BN;
    const _Float16* Ae = g.A + g.a_off[r] + (long long)e * T * C2;
    const _Float16* Be = g.Bt + (long long)(g.b_pt0[r] + e) * K * C2;
    float* Me = g.M + g.m_off[r] + (long long)e * T * K;

    // (Non-temporal A-operand loads (aux 2) were A/B'd in round 4: C4 neutral, C2 +0.9% -- within the ~1.5%
// box-to-box spread of C2's A/B pairs -- but +8% PMC bytes per launch at C4 (1.004 vs 0.925 GB): the two
// column tiles of a row tile no longer share its A tile through the XCD's L2.  Not kept; nor non-temporal
// M stores (C4 -0.7%, C2 +1.9% / -1% on two boxes).  profiles/r04_ab_gemm_nt_a, r04_ab_gemm_nt_m.)
// DMA sources: wave w fills A tile rows (BM/8) w + 8i + lane/8 (i < AP) and B tile
    // rows 32w + 8i + lane/8 (i < 4); lane%8 is the physical 16-B chunk, holding logical
    // chunk lc = phys ^ ((row>>1)&7): hi channels 8lc.. (lc < 4) or lo channels 8(lc-4)..
    // of the stage
    // DMA by buffer_load ... lds: two descriptors per operand (SGPRs), the second
    // based 16 rows further on with 16 rows fewer in range, serve row groups i < 2
    // and i >= 2 with the same two lane offsets (the chunk swizzle differs between
    // even and odd i); the wave-uniform soffset is the stage's column (inside the
    // row), so the range check decides on the row alone: A rows past T load as
    // zeros (never stored), nothing past the operand is read
    const auto ar0 = __builtin_amdgcn_make_buffer_rsrc((void*)Ae, 0, T * C2 * 2, 0x00020000);
    const auto ar1 = __builtin_amdgcn_make_buffer_rsrc((void*)(Ae + 16 * C2), 0, (T > 16 ? T - 16 : 0) * C2 * 2,
                                                       0x00020000);
    const auto br0 = __builtin_amdgcn_make_buffer_rsrc((void*)Be, 0, K * C2 * 2, 0x00020000);
    const auto br1 = __builtin_amdgcn_make_buffer_rsrc((void*)(Be + C2), 0, (K - 1) * C2 * 2, 0x00020000);
    int aoff[2], boff[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int RA = (BM / 8) * wid + 8 * i + (lane >> 3);
        const int R = 32 * wid + 8 * i + (lane >> 3);
        aoff[i] = ((m0 + RA) * C2 + 8 * ((lane & 7) ^ ((RA >> 1) & 7))) * 2;
        boff[i] = ((n0 + b_col(R)) * C2 + 8 * ((lane & 7) ^ ((R >> 1) & 7))) * 2;
    }
    auto issue = [&](int ks, int buf) {
        char* abase = smem + buf * STAGEB + ((BM / 8) * wid) * SG_ROWB;
        char* bbase = smem + buf * STAGEB + ATILEB + (32 * wid) * SG_ROWB;
#pragma unroll
        for (int i = 0; i < AP; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(i < 2 ? ar0 : ar1,
                                                     (__attribute__((address_space(3))) void*)(abase + 8 * i * SG_ROWB),
                                                     16, aoff[i & 1], ks * SG_STAGE_SOFF, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(i < 2 ? br0 : br1,
                                                     (__attribute__((address_space(3))) void*)(bbase + 8 * i * SG_ROWB),
                                                     16, boff[i & 1], ks * SG_STAGE_SOFF, 0, 0);
    };
    // DMA piece p of a stage (p < 4: A row group p, else B row group p - 4)
    auto issue_piece = [&](int ks, int buf, int p) {
        char* base = smem + buf * STAGEB + (32 * wid) * SG_ROWB;
        const int q = p & 3;
        if (p < 4)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(q < 2 ? ar0 : ar1,
                                                     (__attribute__((address_space(3))) void*)(base + 8 * q * SG_ROWB),
                                                     16, aoff[q & 1], ks * SG_STAGE_SOFF, 0, 0);
        else
            __builtin_amdgcn_raw_ptr_buffer_load_lds(q < 2 ? br0 : br1,
                                                     (__attribute__((address_space(3))) void*)(base + ATILEB +
                                                                                              8 * q * SG_ROWB),
                                                     16, boff[q & 1], ks * SG_STAGE_SOFF, 0, 0);
    };

    // operand reads: wave (wm, wn) = rows (BM/2) wm.., cols 64 wn..; lane holds row
    // lane%16 of a 16-row block, channels 8 (lane/16).. of the 32 (hi) and the same of lo
    const int wm = wid >> 2, wn = wid & 3;
    const int lr = lane & 15, sw = lr >> 1;  // (row >> 1) & 7 of every 16-row block
    const int ch = lane >> 4;
    const int a_hi = (wm * (BM / 2) + lr) * SG_ROWB + 16 * (ch ^ sw);
    const int a_lo = (wm * (BM / 2) + lr) * SG_ROWB + 16 * ((4 + ch) ^ sw);
    const int b_hi = ATILEB + (wn * 64 + lr) * SG_ROWB + 16 * (ch ^ sw);
    const int b_lo = ATILEB + (wn * 64 + lr) * SG_ROWB + 16 * ((4 + ch) ^ sw);

    f32x4 acc[NI][4];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nks = C / SG_BK;
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int ks = 0; ks < nks; ++ks) {
        const char* st = smem + (ks & 1) * STAGEB;
        f16x8 ah[NI], al[NI], bh[4], bl[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            bh[j] = *(const f16x8*)(st + b_hi + 16 * j * SG_ROWB);
            bl[j] = *(const f16x8*)(st + b_lo + 16 * j * SG_ROWB);
        }
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            ah[i] = *(const f16x8*)(st + a_hi + 16 * i * SG_ROWB);
            al[i] = *(const f16x8*)(st + a_lo + 16 * i * SG_ROWB);
        }
        if (!ILV && ks + 1 < nks) issue(ks + 1, (ks + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);  // the DMA issue stays ahead of the MFMAs
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            if (ILV && ks + 1 < nks) {
                issue_piece(ks + 1, (ks + 1) & 1, i);
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
            }
            if (ILV) __builtin_amdgcn_sched_barrier(0);
        }
        __builtin_amdgcn_sched_barrier(0);  // ... and the stage's closing wait behind them
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    // epilogue: C/D map of 16x16x32: col = lane % 16, row = 4 (lane / 16) + reg; the
    // lane's four column blocks are adjacent columns (b_col): one 16-B store per row
#pragma unroll
    for (int i = 0; i < NI; ++i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = m0 + wm * (BM / 2) + 16 * i + 4 * ch + q;
            if (row >= T) continue;
            *(f32x4*)(Me + (long long)row * K + n0 + wn * 64 + 4 * lr) =
                f32x4{acc[i][0][q], acc[i][1][q], acc[i][2][q], acc[i][3][q]};
        }
    }
}

// Variant 4: variant 0 as a persistent kernel.  One workgroup per CU walks a
// strided sequence of tiles inside its XCD's contiguous range; the last stage of a
// tile issues the next tile's stage-0 DMA (its first-stage load latency hides
// under the last stage's MFMAs), and a tile's epilogue stores drain under the next
// tile's first stage (the stage's closing vmcnt(0) is the first wait on them).
struct SGTile {
    const _Float16* Ae;
    const _Float16* Be;
    float* Me;
    int T, m0, n0;
};

__device__ __forceinline__ SGTile sg_tile(const SGArgs& g, int L) {
    int r = 0;
    while (r + 1 < g.nruns && L >= g.tile0[r + 1]) ++r;
    const int u = L - g.tile0[r];
    const int nt = u % g.ntn;
    const int mt = (u / g.ntn) % g.mtiles[r];
    const int e = u / (g.ntn * g.mtiles[r]);
    const int T = g.rows[r], C2 = 2 * g.C, K = g.K;
    SGTile t;
    t.Ae = g.A + g.a_off[r] + (long long)e * T * C2;
    t.Be = g.Bt + (long long)(g.b_pt0[r] + e) * K * C2;
    t.Me = g.M + g.m_off[r] + (long long)e * T * K;
    t.T = T;
    t.m0 = mt * SG_BM;
    t.n0 = nt * SG_BN;
    return t;
}

// DW = waves that issue the DMA: 8 (variant 4: 4 pieces per operand each) or 4
// (variant 5: waves 0-3, one per SIMD, 8 pieces per operand each, so on every SIMD
// one wave's DMA issue runs beside the other wave's MFMAs)
// PROBE = true (variant 6, timing probe only, wrong results): every descriptor has
// zero records, so the DMA moves no global data (LDS gets zeros) while the
// instruction stream, waits and barriers stay: prices the operand traffic
// (MI355X_MICROARCH.md / cdna_hip_programming.md, zero-record descriptor).
//
// PP = true (variant 7, with DW = 4): ping-pong.  Waves 0-3 (X: one per SIMD, rows
// 0-127 of the tile) and waves 4-7 (Y, rows 128-255) run half a stage apart, a
// barrier per half-stage: while one wave of a SIMD reads its operands from LDS the
// other runs its 96 MFMAs, so the MFMA pipe does not stand idle behind every
// stage's operand reads.  X issues the DMA (its own and Y's rows) right after its
// reads of stage j, into the buffer Y finished reading a half-stage earlier, and
// waits for it at the end of its MFMA half-step.
// SPR = true (variant 8): the non-ping-pong loop issues a row block's hi.hi,
// lo.hi, hi.lo MFMAs 4 apart instead of back to back on one accumulator.
// STAMP = true (azg_split_gemm_stamps, a diagnostic build, never the product path):
// s_memtime stamps split each stage into [operand reads + DMA issue, reads landed],
// [MFMA issue], [vmcnt(0)], [barrier] and the epilogue; per-wave sums go to g.stamps
// (MI355X guide, in-kernel stamps: read the shares, not the length).
[[maybe_unused]] __device__ __forceinline__ unsigned long long sg_stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

// DEF = true (variant 11): deferred epilogue.  A tile's accumulators are stored
// during the next tile's first stage, each row block's four rows just before that
// row block's first MFMAs overwrite them, so the chip-wide burst of M stores at the
// end of every tile (all CUs finish their tiles together) runs under MFMAs instead
// of stalling every wave (the stamp build put the epilogue at 11% of wave time).
// PZ = 1 / 2 (variants 15 / 16, timing probes only, wrong results): as PROBE, but only
// the B (15) or only the A (16) descriptors have zero records, pricing each operand's
// share of the global -> LDS feed.
template <int DW, bool PROBE = false, bool PP = false, bool SPR = false, bool STAMP = false, bool DEF = false,
          int PZ = 0>
__global__ __launch_bounds__(512, 1) void split_gemm_persist_kernel(SGArgs g) {
    __shared__ __attribute__((aligned(16))) char smem[2 * SG_STAGEB];
    // wid through readfirstlane: the compiler then knows it is wave-uniform (DW < 8 branches on it)
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int C = g.C, K = g.K, C2 = 2 * C;

    // this block's tiles: its XCD's contiguous range (as the one-tile variants deal
    // it), strided by the number of blocks on the XCD
    const int xcd = blockIdx.x % 8, kb = blockIdx.x / 8;
    const int nblk = ((int)gridDim.x - xcd + 7) / 8;
    const int q8 = g.total / 8, rr = g.total % 8;
    const int start = xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8;
    const int cnt = q8 + (xcd < rr ? 1 : 0);
    if (kb >= cnt) return;

    // per-lane DMA geometry (tile independent part): wave w fills LDS rows
    // 32 w + 8 i + lane / 8 (i < 4) of A and of B; with DW = 4, waves 0-3 also fill
    // the rows of waves 4-7 (128 rows on: b_col(R + 128) = b_col(R) + 128)
    int arow[2], brow[2], dcol[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int R = 32 * wid + 8 * i + (lane >> 3);
        const int lc = (lane & 7) ^ ((R >> 1) & 7);
        dcol[i] = 8 * lc;
        arow[i] = R;
        brow[i] = b_col(R);
    }
    const int wm = wid >> 2, wn = wid & 3;
    const int lr = lane & 15, sw = lr >> 1;
    const int ch = lane >> 4;
    const int a_hi = (wm * 128 + lr) * SG_ROWB + 16 * (ch ^ sw);
    const int a_lo = (wm * 128 + lr) * SG_ROWB + 16 * ((4 + ch) ^ sw);
    const int b_hi = SG_TILEB + (wn * 64 + lr) * SG_ROWB + 16 * (ch ^ sw);
    const int b_lo = SG_TILEB + (wn * 64 + lr) * SG_ROWB + 16 * ((4 + ch) ^ sw);

    // DMA of stage ks of tile t into buffer buf (descriptors as variant 0; the
    // second half's 128 rows on)
    auto issue = [&](const SGTile& t, int ks, int buf) {
        if (DW < 8 && wid >= DW) return;
#pragma unroll
        for (int h = 0; h < 8 / DW; ++h) {
            const int T = t.T - 128 * h;
            const _Float16* Ae = t.Ae + 128 * h * C2;
            const _Float16* Be = t.Be + 128 * h * C2;
            constexpr bool ZA = PROBE || PZ == 2, ZB = PROBE || PZ == 1;
            const auto ar0 = __builtin_amdgcn_make_buffer_rsrc((void*)Ae, 0, ZA ? 0 : (T > 0 ? T : 0) * C2 * 2,
                                                               0x00020000);
            const auto ar1 = __builtin_amdgcn_make_buffer_rsrc((void*)(Ae + 16 * C2), 0,
                                                               ZA ? 0 : (T > 16 ? T - 16 : 0) * C2 * 2, 0x00020000);
            const auto br0 = __builtin_amdgcn_make_buffer_rsrc((void*)Be, 0, ZB ? 0 : (K - 128 * h) * C2 * 2,
                                                               0x00020000);
            const auto br1 = __builtin_amdgcn_make_buffer_rsrc((void*)(Be + C2), 0,
                                                               ZB ? 0 : (K - 128 * h - 1) * C2 * 2, 0x00020000);
            char* base = smem + buf * SG_STAGEB + (32 * wid + 128 * h) * SG_ROWB;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(i < 2 ? ar0 : ar1,
                                                         (__attribute__((address_space(3))) void*)(base + 8 * i * SG_ROWB),
                                                         16, ((t.m0 + arow[i & 1]) * C2 + dcol[i & 1]) * 2,
                                                         ks * SG_STAGE_SOFF, 0, 0);
#pragma unroll
            for (int i = 0; i < 4; ++i)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(i < 2 ? br0 : br1,
                                                         (__attribute__((address_space(3))) void*)(base + SG_TILEB +
                                                                                                  8 * i * SG_ROWB),
                                                         16, ((t.n0 + brow[i & 1]) * C2 + dcol[i & 1]) * 2,
                                                         ks * SG_STAGE_SOFF, 0, 0);
        }
    };

    const int nks = C / SG_BK;  // even: every tile starts in buffer 0
    SGTile cur = sg_tile(g, start + kb);
    issue(cur, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned long long stq[5] = {0, 0, 0, 0, 0};
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    SGTile prev = cur;  // DEF: the tile whose accumulators are still to be stored
    bool have_prev = false;
    // rows 4 ch + q of row block i of tile t, 4 adjacent columns per lane (b_col)
    auto store_rows = [&](const SGTile& t, int i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = t.m0 + wm * 128 + 16 * i + 4 * ch + q;
            if (row < t.T)
                *(f32x4*)(t.Me + (long long)row * K + t.n0 + wn * 64 + 4 * lr) =
                    f32x4{acc[i][0][q], acc[i][1][q], acc[i][2][q], acc[i][3][q]};
        }
    };
    for (int it = kb;;) {
        const int nx = it + nblk;
        const bool more = nx < cnt;
        const SGTile nxt = sg_tile(g, start + (more ? nx : it));

        if constexpr (!DEF) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        if constexpr (PP) {
            const bool X = wid < 4;
            f16x8 ah[8], al[8], bh[4], bl[4];
            auto read = [&](int ks) {
                const char* st = smem + (ks & 1) * SG_STAGEB;
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
            };
            auto mma = [&]() {  // per row block: hi.hi, lo.hi, hi.lo of its 4 accumulators, 4 MFMAs apart
#pragma unroll
                for (int i = 0; i < 8; ++i) {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                }
            };
            // half-step hs: X reads stage hs/2 (even hs; + the next stage's DMA) and
            // computes stage (hs-1)/2 (odd hs); Y reads at odd hs and computes at even
            // hs > 0, one stage behind.  One instance of each body (register phis).
            for (int hs = 0; hs <= 2 * nks; ++hs) {
                const bool odd = hs & 1;
                const bool do_read = X ? (!odd && hs < 2 * nks) : odd;
                const bool do_mma = X ? odd : (!odd && hs > 0);
                const int ks = X ? (hs >> 1) : ((hs - 1) >> 1);
                if (do_read) {
                    read(ks);
                    if (X) {
                        if (ks + 1 < nks) issue(cur, ks + 1, (ks + 1) & 1);
                        else if (more) issue(nxt, 0, 0);
                    }
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                }
                __builtin_amdgcn_sched_barrier(0);
                if (do_mma) {
                    mma();
                    __builtin_amdgcn_sched_barrier(0);
                    if (X) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_barrier();
            }
        } else
        for (int ks = 0; ks < nks; ++ks) {
            unsigned long long t0 = 0;
            if constexpr (STAMP) t0 = sg_stamp();
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
            if (ks + 1 < nks) issue(cur, ks + 1, (ks + 1) & 1);
            else if (more) issue(nxt, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            unsigned long long t1 = 0;
            if constexpr (STAMP) t1 = sg_stamp();
            if constexpr (SPR) {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                }
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    if (DEF && ks == 0) {
                        if (have_prev) store_rows(prev, i);
#pragma unroll
                        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                    }
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            unsigned long long t2 = 0, t3 = 0, t4 = 0;
            if constexpr (STAMP) t2 = sg_stamp();
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if constexpr (STAMP) t3 = sg_stamp();
            __syncthreads();
            if constexpr (STAMP) {
                t4 = sg_stamp();
                stq[0] += t1 - t0;
                stq[1] += t2 - t1;
                stq[2] += t3 - t2;
                stq[3] += t4 - t3;
            }
        }
        unsigned long long te = 0;
        if constexpr (STAMP) te = sg_stamp();
        if constexpr (DEF) {
            prev = cur;
            have_prev = true;
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) store_rows(cur, i);
        }
        if constexpr (STAMP) stq[4] += sg_stamp() - te;
        if (!more) break;
        it = nx;
        cur = nxt;
    }
    if constexpr (DEF) {
#pragma unroll
        for (int i = 0; i < 8; ++i) store_rows(prev, i);
    }
    if constexpr (STAMP) {
        if (lane == 0)
            for (int i = 0; i < 5; ++i) g.stamps[((size_t)blockIdx.x * 8 + wid) * 5 + i] = stq[i];
    }
}

#ifdef AZG_SG_PROBES
// ---------------------------------------------------------------------------
// Probe-only schedules (variants 1, 2, 3, 5-8, 10-12, 15, 16, 19): measured, recorded in
// HISTORY.md 4.1 / 6b, none faster than variant 4.  Built only into tools/libazg_probes.so
// (tools/Makefile, -DAZG_SG_PROBES), never into the product libazg.so.
// Variant 12: ping-pong with the DMA split evenly and one stage stream across tiles.
// Waves 0-3 (X, rows 0-127 of the tile, one per SIMD) and 4-7 (Y, rows 128-255) run
// half a stage apart, one barrier per half-step: while one wave of a SIMD reads its
// operands the other runs its 96 MFMAs.  Every wave issues the DMA of its own 32 LDS
// rows (as variant 4), X for stage s + 1 right after its reads of stage s, Y for
// stage s + 2 right after its reads of stage s (into the buffer it has just read;
// X read it a half-step earlier), so both groups' reading half-steps carry 8 DMA
// issues per wave (variant 7 put all 16 on X).  The stages of a block's tiles form
// one stream (s = tile * nks + k-stage): a group stores its accumulators right after
// its last MFMA half-step of a tile, and the other group keeps computing meanwhile,
// so no half-step stands empty between tiles.  Landing: X waits vmcnt(0) at the end
// of its MFMA half-step (its stage s + 1 part); Y at the end of its reading
// half-step waits for all but the 8 DMA pieces it has just issued (its stage s + 1
// part, issued a stage earlier), before the barrier that precedes X's read of s + 1.
__global__ __launch_bounds__(512, 1) void split_gemm_pp2_kernel(SGArgs g) {
    __shared__ __attribute__((aligned(16))) char smem[2 * SG_STAGEB];
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int C = g.C, K = g.K, C2 = 2 * C;
    const int xcd = blockIdx.x % 8, kb = blockIdx.x / 8;
    const int nblk = ((int)gridDim.x - xcd + 7) / 8;
    const int q8 = g.total / 8, rr = g.total % 8;
    const int start = xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8;
    const int cnt = q8 + (xcd < rr ? 1 : 0);
    if (kb >= cnt) return;  // uniform over the workgroup
    const int nks = C / SG_BK;
    const int S = ((cnt - kb + nblk - 1) / nblk) * nks;  // this block's stages
    const bool X = wid < 4;

    int arow[2], brow[2], dcol[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int R = 32 * wid + 8 * i + (lane >> 3);
        const int lc = (lane & 7) ^ ((R >> 1) & 7);
        dcol[i] = 8 * lc;
        arow[i] = R;
        brow[i] = b_col(R);
    }
    const int wm = wid >> 2, wn = wid & 3;
    const int lr = lane & 15, sw = lr >> 1;
    const int ch = lane >> 4;
    const int a_hi = (wm * 128 + lr) * SG_ROWB + 16 * (ch ^ sw);
    const int a_lo = (wm * 128 + lr) * SG_ROWB + 16 * ((4 + ch) ^ sw);
    const int b_hi = SG_TILEB + (wn * 64 + lr) * SG_ROWB + 16 * (ch ^ sw);
    const int b_lo = SG_TILEB + (wn * 64 + lr) * SG_ROWB + 16 * ((4 + ch) ^ sw);

    auto tile_of = [&](int s) { return sg_tile(g, start + kb + (s / nks) * nblk); };
    // this wave's 8 DMA pieces of stream stage s (its 32 rows of A and of B)
    auto issue = [&](int s) {
        const SGTile t = tile_of(s);
        const int ks = s % nks;
        const int T = t.T;
        const auto ar0 = __builtin_amdgcn_make_buffer_rsrc((void*)t.Ae, 0, T * C2 * 2, 0x00020000);
        const auto ar1 = __builtin_amdgcn_make_buffer_rsrc((void*)(t.Ae + 16 * C2), 0, (T > 16 ? T - 16 : 0) * C2 * 2,
                                                           0x00020000);
        const auto br0 = __builtin_amdgcn_make_buffer_rsrc((void*)t.Be, 0, K * C2 * 2, 0x00020000);
        const auto br1 = __builtin_amdgcn_make_buffer_rsrc((void*)(t.Be + C2), 0, (K - 1) * C2 * 2, 0x00020000);
        char* base = smem + (s & 1) * SG_STAGEB + (32 * wid) * SG_ROWB;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(i < 2 ? ar0 : ar1,
                                                     (__attribute__((address_space(3))) void*)(base + 8 * i * SG_ROWB),
                                                     16, ((t.m0 + arow[i & 1]) * C2 + dcol[i & 1]) * 2,
                                                     ks * SG_STAGE_SOFF, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(i < 2 ? br0 : br1,
                                                     (__attribute__((address_space(3))) void*)(base + SG_TILEB +
                                                                                              8 * i * SG_ROWB),
                                                     16, ((t.n0 + brow[i & 1]) * C2 + dcol[i & 1]) * 2,
                                                     ks * SG_STAGE_SOFF, 0, 0);
    };

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    f16x8 ah[8], al[8], bh[4], bl[4];

    issue(0);
    if (!X && S > 1) issue(1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    // half-step hs: X reads stage hs/2 (even hs) and computes stage (hs-1)/2 (odd hs);
    // Y reads stage (hs-1)/2 (odd hs) and computes stage hs/2 - 1 (even hs > 0)
    for (int hs = 0; hs <= 2 * S; ++hs) {
        const bool odd = hs & 1;
        const bool do_read = X ? (!odd && hs < 2 * S) : odd;
        const bool do_mma = X ? odd : (!odd && hs > 0);
        const int s = odd ? (hs - 1) >> 1 : (X ? hs >> 1 : (hs >> 1) - 1);
        bool issued = false;
        if (do_read) {
            const char* st = smem + (s & 1) * SG_STAGEB;
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
            if (X) {
                if (s + 1 < S) issue(s + 1);  // the other buffer: both groups finished stage s - 1
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            } else {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this buffer's reads landed ...
                if (s + 2 < S) {                                      // ... before it is refilled
                    issue(s + 2);
                    issued = true;
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        if (do_mma) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                }
            if ((s + 1) % nks == 0) {  // the tile's last stage: store and clear
                const SGTile t = tile_of(s);
#pragma unroll
                for (int i = 0; i < 8; ++i)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int row = t.m0 + wm * 128 + 16 * i + 4 * ch + q;
                        if (row < t.T)
                            *(f32x4*)(t.Me + (long long)row * K + t.n0 + wn * 64 + 4 * lr) =
                                f32x4{acc[i][0][q], acc[i][1][q], acc[i][2][q], acc[i][3][q]};
                    }
#pragma unroll
                for (int i = 0; i < 8; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        if (odd) {
            if (X || !issued) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        }
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
    }
}

// ---------------------------------------------------------------------------
// Variant 1: the stage's 96 MFMAs in 4 phases of 2 row blocks (24 MFMAs);
// each phase's ds_reads (the next phase's A fragments; in phase 3 the next stage's
// B fragments and phase-0 A) are issued before its MFMAs and land under them, so a
// wave's MFMAs never wait for a whole stage of reads.  The reads are inline asm:
// hipcc counts no LDS-DMA alias scopes and would otherwise drain vmcnt (the next
// stage's DMA, in flight) before every ds_read.  Each read is waited for by an
// explicit lgkmcnt(0) naming its destinations ("+v") at the start of the phase
// that consumes it.  One barrier per stage, after phase 2: this wave's reads of
// the stage buffer are complete (lgkmcnt) and the next stage's DMA has landed
// (vmcnt(0): nothing else is outstanding), so in phase 3 every wave may read the
// next buffer and refill this one (stage s+2).  B fragments alternate between two
// register sets by stage parity (loop unrolled by 2), A fragments between two sets
// by phase parity: no register copies.
template <unsigned V>
struct UC {
    static constexpr unsigned value = V;
};
struct Frag2 {
    f16x8 h[2], l[2];
};
struct Frag4 {
    f16x8 h[4], l[4];
};

// A fragments of phase P (row blocks 2P, 2P+1): hi and lo, 4 ds_read_b128; OFF is
// the stage buffer's byte offset, folded into the instruction's 16-bit offset
template <int P, unsigned OFF>
__device__ __forceinline__ void read_a(Frag2& a, unsigned hi, unsigned lo) {
    asm volatile(
        "ds_read_b128 %0, %4 offset:%c6\n\t"
        "ds_read_b128 %1, %4 offset:%c7\n\t"
        "ds_read_b128 %2, %5 offset:%c6\n\t"
        "ds_read_b128 %3, %5 offset:%c7"
        : "=v"(a.h[0]), "=v"(a.h[1]), "=v"(a.l[0]), "=v"(a.l[1])
        : "v"(hi), "v"(lo), "i"(OFF + P * 2 * 16 * SG_ROWB), "i"(OFF + (P * 2 + 1) * 16 * SG_ROWB));
}
// B fragments of column block J: hi and lo, 2 ds_read_b128
template <int J, unsigned OFF>
__device__ __forceinline__ void read_b(Frag4& b, unsigned hi, unsigned lo) {
    asm volatile(
        "ds_read_b128 %0, %2 offset:%c4\n\t"
        "ds_read_b128 %1, %3 offset:%c4"
        : "=v"(b.h[J]), "=v"(b.l[J])
        : "v"(hi), "v"(lo), "i"(OFF + J * 16 * SG_ROWB));
}
__device__ __forceinline__ void wait_a(Frag2& a) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a.h[0]), "+v"(a.h[1]), "+v"(a.l[0]), "+v"(a.l[1]));
}
__device__ __forceinline__ void wait_ab(Frag2& a, Frag4& b) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(a.h[0]), "+v"(a.h[1]), "+v"(a.l[0]), "+v"(a.l[1]), "+v"(b.h[0]), "+v"(b.h[1]),
                   "+v"(b.h[2]), "+v"(b.h[3]), "+v"(b.l[0]), "+v"(b.l[1]), "+v"(b.l[2]), "+v"(b.l[3]));
}
// 24 MFMAs of row blocks I0, I0+1: hi.hi, lo.hi, hi.lo per accumulator, the three
// products of one accumulator 8 MFMAs apart
template <int I0>
__device__ __forceinline__ void mma_phase(f32x4 (&acc)[8][4], const Frag2& a, const Frag4& b) {
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[I0 + ii][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a.h[ii], b.h[j], acc[I0 + ii][j], 0, 0, 0);
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[I0 + ii][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a.l[ii], b.h[j], acc[I0 + ii][j], 0, 0, 0);
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[I0 + ii][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a.h[ii], b.l[j], acc[I0 + ii][j], 0, 0, 0);
}
// The 6 MFMAs of row blocks I0, I0+1 with column block J (phase 3 retires the B
// fragments one column block at a time so the next stage's reuse their registers)
template <int I0, int J>
__device__ __forceinline__ void mma_col(f32x4 (&acc)[8][4], const Frag2& a, const Frag4& b) {
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) acc[I0 + ii][J] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a.h[ii], b.h[J], acc[I0 + ii][J], 0, 0, 0);
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) acc[I0 + ii][J] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a.l[ii], b.h[J], acc[I0 + ii][J], 0, 0, 0);
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) acc[I0 + ii][J] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a.h[ii], b.l[J], acc[I0 + ii][J], 0, 0, 0);
}

__global__ __launch_bounds__(512, 1) void split_gemm_pipe_kernel(SGArgs g) {
    __shared__ __attribute__((aligned(16))) char smem[2 * SG_STAGEB];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
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

    // DMA by buffer_load ... lds: two descriptors per operand (SGPRs), the second
    // based 16 rows further on with 16 rows fewer in range, serve row groups i < 2
    // and i >= 2 with the same two lane offsets (the chunk swizzle differs between
    // even and odd i); the wave-uniform soffset is the stage's column (inside the
    // row), so the range check decides on the row alone: A rows past T load as
    // zeros (never stored), nothing past the operand is read
    const auto ar0 = __builtin_amdgcn_make_buffer_rsrc((void*)Ae, 0, T * C2 * 2, 0x00020000);
    const auto ar1 = __builtin_amdgcn_make_buffer_rsrc((void*)(Ae + 16 * C2), 0, (T > 16 ? T - 16 : 0) * C2 * 2,
                                                       0x00020000);
    const auto br0 = __builtin_amdgcn_make_buffer_rsrc((void*)Be, 0, K * C2 * 2, 0x00020000);
    const auto br1 = __builtin_amdgcn_make_buffer_rsrc((void*)(Be + C2), 0, (K - 1) * C2 * 2, 0x00020000);
    int aoff[2], boff[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int R = 32 * wid + 8 * i + (lane >> 3);
        const int lc = (lane & 7) ^ ((R >> 1) & 7);
        const int col = 8 * lc;
        aoff[i] = ((m0 + R) * C2 + col) * 2;
        boff[i] = ((n0 + b_col(R)) * C2 + col) * 2;
    }
    // LDS: [A stage 0 | A stage 1 | B stage 0 | B stage 1], 32 KB each, so every
    // operand read is one of four base registers plus an immediate offset
    auto issue = [&](int ks, int buf) {
        char* base = smem + buf * SG_TILEB + (32 * wid) * SG_ROWB;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(i < 2 ? ar0 : ar1,
                                                     (__attribute__((address_space(3))) void*)(base + 8 * i * SG_ROWB),
                                                     16, aoff[i & 1], ks * SG_STAGE_SOFF, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(i < 2 ? br0 : br1,
                                                     (__attribute__((address_space(3))) void*)(base + 2 * SG_TILEB +
                                                                                              8 * i * SG_ROWB),
                                                     16, boff[i & 1], ks * SG_STAGE_SOFF, 0, 0);
    };

    const int wm = wid >> 2, wn = wid & 3;
    const int lr = lane & 15, sw = lr >> 1, ch = lane >> 4;
    const unsigned s0 = lds_addr(smem);
    const unsigned a_hi = s0 + (wm * 128 + lr) * SG_ROWB + 16 * (ch ^ sw);
    const unsigned a_lo = s0 + (wm * 128 + lr) * SG_ROWB + 16 * ((4 + ch) ^ sw);
    const unsigned b_hi = s0 + 2 * SG_TILEB + (wn * 64 + lr) * SG_ROWB + 16 * (ch ^ sw);
    const unsigned b_lo = s0 + 2 * SG_TILEB + (wn * 64 + lr) * SG_ROWB + 16 * ((4 + ch) ^ sw);

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nks = C / SG_BK;  // even (C % 64 == 0)
    Frag2 ax, ay;
    Frag4 b;
    issue(0, 0);
    issue(1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // stage 0 landed (this wave)
    __builtin_amdgcn_s_barrier();
    read_b<0, 0>(b, b_hi, b_lo);
    read_b<1, 0>(b, b_hi, b_lo);
    read_b<2, 0>(b, b_hi, b_lo);
    read_b<3, 0>(b, b_hi, b_lo);
    read_a<0, 0>(ax, a_hi, a_lo);

    // one stage, its buffer at byte offset CO (of the A and of the B region), the
    // next stage's at NO
    auto stage = [&](int ks, auto co_t) {
        constexpr unsigned CO = decltype(co_t)::value, NO = SG_TILEB - CO;
        wait_ab(ax, b);
        read_a<1, CO>(ay, a_hi, a_lo);
        mma_phase<0>(acc, ax, b);
        __builtin_amdgcn_sched_barrier(0);
        wait_a(ay);
        read_a<2, CO>(ax, a_hi, a_lo);
        mma_phase<2>(acc, ay, b);
        __builtin_amdgcn_sched_barrier(0);
        wait_a(ax);
        read_a<3, CO>(ay, a_hi, a_lo);
        mma_phase<4>(acc, ax, b);
        __builtin_amdgcn_sched_barrier(0);
        wait_a(ay);  // this wave's reads of the stage buffer are done
        if (ks + 1 < nks) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stage ks+1 landed (this wave)
            __builtin_amdgcn_s_barrier();                     // ... for every wave; buffer CO free
            if (ks + 2 < nks) issue(ks + 2, ks & 1);
            read_a<0, NO>(ax, a_hi, a_lo);
            mma_col<6, 0>(acc, ay, b);
            __builtin_amdgcn_sched_barrier(0);
            read_b<0, NO>(b, b_hi, b_lo);
            mma_col<6, 1>(acc, ay, b);
            __builtin_amdgcn_sched_barrier(0);
            read_b<1, NO>(b, b_hi, b_lo);
            mma_col<6, 2>(acc, ay, b);
            __builtin_amdgcn_sched_barrier(0);
            read_b<2, NO>(b, b_hi, b_lo);
            mma_col<6, 3>(acc, ay, b);
            __builtin_amdgcn_sched_barrier(0);
            read_b<3, NO>(b, b_hi, b_lo);
        } else {
            mma_phase<6>(acc, ay, b);
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    for (int ks = 0; ks < nks; ks += 2) {
        stage(ks, UC<0>{});
        stage(ks + 1, UC<SG_TILEB>{});
    }

#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = m0 + wm * 128 + 16 * i + 4 * ch + q;
            if (row >= T) continue;
            *(f32x4*)(Me + (long long)row * K + n0 + wn * 64 + 4 * lr) =
                f32x4{acc[i][0][q], acc[i][1][q], acc[i][2][q], acc[i][3][q]};
        }
    }
}

// ---------------------------------------------------------------------------
// Variant 2: one wave per SIMD (4 waves, 2 x 2, 128 x 128 per wave = 8 x 8
// accumulators of 16 x 16, 256 accumulator registers held in AGPRs).  Against the
// 8-wave variants each A element is read from LDS by 2 waves instead of 4: 128 KB
// of ds_read per stage instead of 192 KB for the same 256 x 256 x 32 work.  A wave
// keeps the stage's 8 B fragments (hi, lo) in registers and streams its 8 A
// fragments through a 4-slot ring, two row blocks ahead.  One barrier per stage,
// at row block 6: the wave's reads of the stage buffer have all landed (A[7] was
// issued at row block 5) and the next stage's DMA has landed (vmcnt(0)); after it
// the stage buffer is refilled (stage + 2) and row blocks 6 and 7 run column block
// by column block, each column block's B fragments replaced by the next stage's
// as soon as its 6 MFMAs are issued.  Operand reads are inline-asm ds_read_b128 with explicit lgkmcnt waits
// (as variant 1); LDS is [A stage 0 | A stage 1 | B stage 0 | B stage 1].
constexpr int W4_ROWB = SG_ROWB;
constexpr int W4_TILEB = SG_TILEB;

// wave column tile of 128: LDS row R (block j = (R % 128) / 16, lane lr = R % 16)
// holds output column 128 (R / 128) + 8 lr + j, so a lane's 8 column blocks are 8
// adjacent columns (two 16-B stores per row in the epilogue)
__device__ __forceinline__ int b_col128(int R) { return (R & ~127) | ((R & 15) << 3) | ((R >> 4) & 7); }

struct FragA {
    f16x8 h, l;
};
struct FragB8 {
    f16x8 h[8], l[8];
};

template <unsigned OFF>
__device__ __forceinline__ void w4_read_a(FragA& a, unsigned hi, unsigned lo) {
    asm volatile(
        "ds_read_b128 %0, %2 offset:%c4\n\t"
        "ds_read_b128 %1, %3 offset:%c4"
        : "=v"(a.h), "=v"(a.l)
        : "v"(hi), "v"(lo), "i"(OFF));
}
// B fragments of column block J (hi, lo)
template <int J, unsigned OFF>
__device__ __forceinline__ void w4_read_b(FragB8& b, unsigned hi, unsigned lo) {
    asm volatile(
        "ds_read_b128 %0, %2 offset:%c4\n\t"
        "ds_read_b128 %1, %3 offset:%c4"
        : "=v"(b.h[J]), "=v"(b.l[J])
        : "v"(hi), "v"(lo), "i"(OFF + J * 16 * W4_ROWB));
}
// s_waitcnt lgkmcnt(N) that the compiler sees as defining the awaited registers
template <int N>
__device__ __forceinline__ void w4_wait(FragA& a) {
    asm volatile("s_waitcnt lgkmcnt(%c2)" : "+v"(a.h), "+v"(a.l) : "i"(N));
}
template <int N>
__device__ __forceinline__ void w4_wait(FragA& a, FragB8& b) {
    asm volatile("s_waitcnt lgkmcnt(%c18)"
                 : "+v"(a.h), "+v"(a.l), "+v"(b.h[0]), "+v"(b.l[0]), "+v"(b.h[1]), "+v"(b.l[1]), "+v"(b.h[2]),
                   "+v"(b.l[2]), "+v"(b.h[3]), "+v"(b.l[3]), "+v"(b.h[4]), "+v"(b.l[4]), "+v"(b.h[5]), "+v"(b.l[5]),
                   "+v"(b.h[6]), "+v"(b.l[6]), "+v"(b.h[7]), "+v"(b.l[7])
                 : "i"(N));
}
// One MFMA accumulating in place in AGPRs ("+a"): left to itself, hipcc keeps
// part of the 256 accumulators in VGPRs and shuffles them between the register
// files every stage.  MFMA-to-MFMA accumulator chains are interlocked in hardware;
// the epilogue waits out the last results (s_nop) before reading them.
__device__ __forceinline__ void w4_mfma(f32x4& c, const f16x8& a, const f16x8& b) {
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
// the 24 MFMAs of row block I: hi.hi, lo.hi, hi.lo for the 8 column blocks
template <int I>
__device__ __forceinline__ void w4_mma(f32x4 (&acc)[8][8], const FragA& a, const FragB8& b) {
#pragma unroll
    for (int j = 0; j < 8; ++j) w4_mfma(acc[I][j], a.h, b.h[j]);
#pragma unroll
    for (int j = 0; j < 8; ++j) w4_mfma(acc[I][j], a.l, b.h[j]);
#pragma unroll
    for (int j = 0; j < 8; ++j) w4_mfma(acc[I][j], a.h, b.l[j]);
}
// the 6 MFMAs of row blocks 6, 7 with column block J (the stage's last two row
// blocks retire the B fragments one column block at a time, so the next stage's
// are read into the same registers)
template <int J>
__device__ __forceinline__ void w4_mma_col(f32x4 (&acc)[8][8], const FragA& a6, const FragA& a7, const FragB8& b) {
    w4_mfma(acc[6][J], a6.h, b.h[J]);
    w4_mfma(acc[7][J], a7.h, b.h[J]);
    w4_mfma(acc[6][J], a6.l, b.h[J]);
    w4_mfma(acc[7][J], a7.l, b.h[J]);
    w4_mfma(acc[6][J], a6.h, b.l[J]);
    w4_mfma(acc[7][J], a7.h, b.l[J]);
}

__global__ __launch_bounds__(256, 1) void split_gemm_w4_kernel(SGArgs g) {
    __shared__ __attribute__((aligned(16))) char smem[4 * W4_TILEB];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
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

    // DMA: wave w fills LDS rows 64 w + 8 i + lane / 8 (i < 8) of A and of B.  Row
    // groups 2d and 2d + 1 share descriptor d (based 16 rows on for A, one column
    // row on for B: b_col128), with one lane offset for even and one for odd i;
    // the soffset is the stage's column, so the range check decides on the row
    const auto mk = [&](const _Float16* base, int nrows) {
        return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (nrows > 0 ? nrows : 0) * C2 * 2, 0x00020000);
    };
    const auto ar0 = mk(Ae, T), ar1 = mk(Ae + 16 * C2, T - 16), ar2 = mk(Ae + 32 * C2, T - 32),
               ar3 = mk(Ae + 48 * C2, T - 48);
    const auto br0 = mk(Be, K), br1 = mk(Be + C2, K - 1), br2 = mk(Be + 2 * C2, K - 2), br3 = mk(Be + 3 * C2, K - 3);
    int aoff[2], boff[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int R = 64 * wid + 8 * i + (lane >> 3);
        const int lc = (lane & 7) ^ ((R >> 1) & 7);
        const int col = 8 * lc;
        aoff[i] = ((m0 + R) * C2 + col) * 2;
        boff[i] = ((n0 + b_col128(R)) * C2 + col) * 2;
    }
    auto issue = [&](int ks, int buf) {
        char* abase = smem + buf * W4_TILEB + (64 * wid) * W4_ROWB;
        char* bbase = abase + 2 * W4_TILEB;
        const int so = ks * SG_STAGE_SOFF;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const auto rs = i < 2 ? ar0 : i < 4 ? ar1 : i < 6 ? ar2 : ar3;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(abase + 8 * i * W4_ROWB),
                                                     16, aoff[i & 1], so, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const auto rs = i < 2 ? br0 : i < 4 ? br1 : i < 6 ? br2 : br3;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(bbase + 8 * i * W4_ROWB),
                                                     16, boff[i & 1], so, 0, 0);
        }
    };

    // operand reads: wave (wm, wn) = rows 128 wm.., cols 128 wn..; lane holds row (col)
    // lane % 16 of a 16-block, channels 8 (lane / 16).. of hi and of lo
    const int wm = wid >> 1, wn = wid & 1;
    const int lr = lane & 15, sw = lr >> 1, ch = lane >> 4;
    const unsigned s0 = lds_addr(smem);
    const unsigned a_hi = s0 + (wm * 128 + lr) * W4_ROWB + 16 * (ch ^ sw);
    const unsigned a_lo = s0 + (wm * 128 + lr) * W4_ROWB + 16 * ((4 + ch) ^ sw);
    const unsigned b_hi = s0 + 2 * W4_TILEB + (wn * 128 + lr) * W4_ROWB + 16 * (ch ^ sw);
    const unsigned b_lo = s0 + 2 * W4_TILEB + (wn * 128 + lr) * W4_ROWB + 16 * ((4 + ch) ^ sw);

    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nks = C / SG_BK;  // even (C % 64 == 0)
    FragA a[4];
    FragB8 b;
    constexpr unsigned RB = 16 * W4_ROWB;  // bytes per 16-row block
    issue(0, 0);
    issue(1, 1);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // stage 0 landed (this wave)
    __builtin_amdgcn_s_barrier();
    // read order of a stage's first fragments: A[0], B[0..7], A[1]
    w4_read_a<0>(a[0], a_hi, a_lo);
    w4_read_b<0, 0>(b, b_hi, b_lo);
    w4_read_b<1, 0>(b, b_hi, b_lo);
    w4_read_b<2, 0>(b, b_hi, b_lo);
    w4_read_b<3, 0>(b, b_hi, b_lo);
    w4_read_b<4, 0>(b, b_hi, b_lo);
    w4_read_b<5, 0>(b, b_hi, b_lo);
    w4_read_b<6, 0>(b, b_hi, b_lo);
    w4_read_b<7, 0>(b, b_hi, b_lo);
    w4_read_a<RB>(a[1], a_hi, a_lo);

    // one stage, its buffer at byte offset CO of the A and of the B region; the last
    // stage (LAST) reads nothing further.  Straight-line per stage (no register
    // phis), the loop unrolled by 2 for the buffer parity, the last 2 stages peeled
    auto stage = [&](int ks, auto co_t, auto last_t) {
        constexpr unsigned CO = decltype(co_t)::value, NO = W4_TILEB - CO;
        constexpr bool LAST = decltype(last_t)::value;
        w4_wait<2>(a[0], b);  // B and A[0] landed (A[1] may be in flight)
        w4_read_a<CO + 2 * RB>(a[2], a_hi, a_lo);
        w4_mma<0>(acc, a[0], b);
        w4_wait<2>(a[1]);
        w4_read_a<CO + 3 * RB>(a[3], a_hi, a_lo);
        w4_mma<1>(acc, a[1], b);
        w4_wait<2>(a[2]);
        w4_read_a<CO + 4 * RB>(a[0], a_hi, a_lo);
        w4_mma<2>(acc, a[2], b);
        w4_wait<2>(a[3]);
        w4_read_a<CO + 5 * RB>(a[1], a_hi, a_lo);
        w4_mma<3>(acc, a[3], b);
        w4_wait<2>(a[0]);
        w4_read_a<CO + 6 * RB>(a[2], a_hi, a_lo);
        w4_mma<4>(acc, a[0], b);
        w4_wait<2>(a[1]);
        w4_read_a<CO + 7 * RB>(a[3], a_hi, a_lo);
        w4_mma<5>(acc, a[1], b);
        w4_wait<0>(a[2]);  // A[6], A[7]: this wave's reads of the stage buffer are done
        w4_wait<0>(a[3]);
        if constexpr (!LAST) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stage ks+1 landed (this wave)
            __builtin_amdgcn_s_barrier();                     // ... for every wave; buffer CO free
            if (ks + 2 < nks) issue(ks + 2, ks & 1);
            w4_read_a<NO>(a[0], a_hi, a_lo);
            w4_mma_col<0>(acc, a[2], a[3], b);
            w4_read_b<0, NO>(b, b_hi, b_lo);
            w4_mma_col<1>(acc, a[2], a[3], b);
            w4_read_b<1, NO>(b, b_hi, b_lo);
            w4_mma_col<2>(acc, a[2], a[3], b);
            w4_read_b<2, NO>(b, b_hi, b_lo);
            w4_mma_col<3>(acc, a[2], a[3], b);
            w4_read_b<3, NO>(b, b_hi, b_lo);
            w4_mma_col<4>(acc, a[2], a[3], b);
            w4_read_b<4, NO>(b, b_hi, b_lo);
            w4_mma_col<5>(acc, a[2], a[3], b);
            w4_read_b<5, NO>(b, b_hi, b_lo);
            w4_mma_col<6>(acc, a[2], a[3], b);
            w4_read_b<6, NO>(b, b_hi, b_lo);
            w4_mma_col<7>(acc, a[2], a[3], b);
            w4_read_b<7, NO>(b, b_hi, b_lo);
            w4_read_a<NO + RB>(a[1], a_hi, a_lo);
        } else {
            w4_mma<6>(acc, a[2], b);
            w4_mma<7>(acc, a[3], b);
        }
    };
    for (int ks = 0; ks < nks - 2; ks += 2) {
        stage(ks, UC<0>{}, std::false_type{});
        stage(ks + 1, UC<W4_TILEB>{}, std::false_type{});
    }
    stage(nks - 2, UC<0>{}, std::false_type{});
    stage(nks - 1, UC<W4_TILEB>{}, std::true_type{});

    // epilogue: lane (lr, ch) holds rows 4 ch + q of each row block, columns
    // 8 lr .. 8 lr + 7 of the wave's 128 (b_col128): two 16-B stores per row.
    // The last MFMAs' results are waited out first (asm MFMAs carry no hazard
    // tracking): 4 x s_nop 15 > the 16x16x32 result latency
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = m0 + wm * 128 + 16 * i + 4 * ch + q;
            if (row >= T) continue;
            float* out = Me + (long long)row * K + n0 + wn * 128 + 8 * lr;
            *(f32x4*)out = f32x4{acc[i][0][q], acc[i][1][q], acc[i][2][q], acc[i][3][q]};
            *(f32x4*)(out + 4) = f32x4{acc[i][4][q], acc[i][5][q], acc[i][6][q], acc[i][7][q]};
        }
    }
}

// ---------------------------------------------------------------------------
// Variant 19: variant 4 on 384 x 256 tiles.  The operand feed (global -> LDS by
// LDS-DMA) sets variant 4's stage time, so the lever is operand bytes per flop:
// a tile of M x N moves (M + N) 128 B per 32-channel stage for 3 * 2 M N 32 flop,
// 1.5 M N / (M + N) flop per byte -- 192 at 256 x 256, 230 at 384 x 256 (+20%).
// The accumulators bound the tile (f32 acc of 384 x 256 = 384 KB of the CU's
// 512 KB register file): 8 waves (2 x 4) of 192 x 64, 12 x 4 accumulators of 16 x 16
// = 192 registers per lane, which two waves per SIMD (256 registers each) only
// hold if the A fragments are not all resident: a wave keeps the stage's 4 B
// fragments (hi, lo: 32 registers) and streams its 12 A row blocks one ahead (2 x 8
// registers), each read issued under the previous row block's 12 MFMAs.  Stage
// buffers are 48 KB of A + 32 KB of B, two of them fill the 160 KB of LDS.  Each wave
// issues 10 DMA pieces per stage (6 A, 4 B), one ahead of each of its first 10 row
// blocks' MFMAs instead of in one burst.  Accumulators, MFMA order per accumulator
// (stage by stage, hi.hi, lo.hi, hi.lo) and so every result are variant 4's.
constexpr int S3_BM = 384;
constexpr int S3_ATILEB = S3_BM * SG_ROWB;      // 48 KB
constexpr int S3_STAGEB = S3_ATILEB + SG_TILEB;  // 80 KB

__global__ __launch_bounds__(512, 1) void split_gemm_384_kernel(SGArgs g) {
    __shared__ __attribute__((aligned(16))) char smem[2 * S3_STAGEB];
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int C = g.C, K = g.K, C2 = 2 * C;

    // this block's tiles: its XCD's contiguous range, strided by the XCD's block count (variant 4)
    const int xcd = blockIdx.x % 8, kb = blockIdx.x / 8;
    const int nblk = ((int)gridDim.x - xcd + 7) / 8;
    const int q8 = g.total / 8, rr = g.total % 8;
    const int start = xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8;
    const int cnt = q8 + (xcd < rr ? 1 : 0);
    if (kb >= cnt) return;

    auto tile_of = [&](int L) {
        SGTile t = sg_tile(g, L);
        int r = 0;
        while (r + 1 < g.nruns && L >= g.tile0[r + 1]) ++r;
        t.m0 = ((L - g.tile0[r]) / g.ntn % g.mtiles[r]) * S3_BM;
        return t;
    };

    // DMA geometry.  A: wave w fills tile rows 48 w + 8 i + lane / 8 (i < 6); the
    // chunk swizzle (row >> 1) & 7 depends on i's parity only, so two lane offsets
    // serve the six pieces, with descriptors based 0 / 16 / 32 rows on (range check
    // on the row: rows past T load zeros).  B as variant 4: rows 32 w + 8 i + lane / 8.
    // The lane offsets are formed once per tile (4 registers: the accumulators leave
    // few); the swizzled chunk is that of both operands' rows: (4 i + lane / 16) & 7.
    const int wm = wid >> 2, wn = wid & 3;
    const int lr = lane & 15, ch = lane >> 4;
    // fragment rows: the lo chunk of a row is its hi chunk ^ 4 (ch < 4), i.e. byte ^ 64
    const int a_hi = (wm * 192 + lr) * SG_ROWB + 16 * (ch ^ (lr >> 1));
    const int b_hi = S3_ATILEB + (wn * 64 + lr) * SG_ROWB + 16 * (ch ^ (lr >> 1));
    int aoff[2], boff[2];
    auto tile_offsets = [&](const SGTile& t) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int R = 8 * i + (lane >> 3);
            const int col = 8 * ((lane & 7) ^ ((R >> 1) & 7));
            aoff[i] = ((t.m0 + 48 * wid + R) * C2 + col) * 2;
            boff[i] = ((t.n0 + b_col(32 * wid + R)) * C2 + col) * 2;
        }
    };

    // DMA piece p (< 6: A row group p, else B row group p - 6) of stage ks of tile t
    // (offsets of that tile in aoff / boff)
    auto piece = [&](const SGTile& t, int ks, int buf, int p) {
        char* base = smem + buf * S3_STAGEB;
        if (p < 6) {
            const int d = p >> 1;  // descriptor: rows 16 d on
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(t.Ae + 16 * d * C2), 0, (t.T - 16 * d > 0 ? t.T - 16 * d : 0) * C2 * 2, 0x00020000);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rs, (__attribute__((address_space(3))) void*)(base + (48 * wid + 8 * p) * SG_ROWB), 16,
                aoff[p & 1], ks * SG_STAGE_SOFF, 0, 0);
        } else {
            const int q = p - 6, d = q >> 1;  // descriptor: one column row on for q >= 2
            const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(t.Be + d * C2), 0, (K - d) * C2 * 2,
                                                              0x00020000);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rs, (__attribute__((address_space(3))) void*)(base + S3_ATILEB + (32 * wid + 8 * q) * SG_ROWB), 16,
                boff[q & 1], ks * SG_STAGE_SOFF, 0, 0);
        }
    };

    const int nks = C / SG_BK;  // even: every tile starts in buffer 0
    SGTile cur = tile_of(start + kb);
    tile_offsets(cur);
#pragma unroll
    for (int p = 0; p < 10; ++p) piece(cur, 0, 0, p);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    f32x4 acc[12][4];
    for (int it = kb;;) {
        const int nx = it + nblk;
        const bool more = nx < cnt;
        const SGTile nxt = tile_of(start + (more ? nx : it));
#pragma unroll
        for (int i = 0; i < 12; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int ks = 0; ks < nks; ++ks) {
            const char* st = smem + (ks & 1) * S3_STAGEB;
            const bool has_next = ks + 1 < nks || more;
            const SGTile& dt = ks + 1 < nks ? cur : nxt;
            const int dks = ks + 1 < nks ? ks + 1 : 0, dbuf = (ks + 1) & 1;
            if (ks + 1 == nks && more) tile_offsets(nxt);  // the next tile's stage 0 goes out now
            f16x8 bh[4], bl[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                bh[j] = *(const f16x8*)(st + b_hi + 16 * j * SG_ROWB);
                bl[j] = *(const f16x8*)(st + (b_hi ^ 64) + 16 * j * SG_ROWB);
            }
#pragma unroll
            for (int i = 0; i < 12; ++i) {
                // one A fragment pair in flight: the partner wave of the SIMD covers its latency
                const f16x8 ah = *(const f16x8*)(st + a_hi + 16 * i * SG_ROWB);
                const f16x8 al = *(const f16x8*)(st + (a_hi ^ 64) + 16 * i * SG_ROWB);
                if (i < 10 && has_next) piece(dt, dks, dbuf, i);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[j], acc[i][j], 0, 0, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        // epilogue: rows 4 ch + q of each row block, 4 adjacent columns per lane (b_col)
#pragma unroll
        for (int i = 0; i < 12; ++i) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = cur.m0 + wm * 192 + 16 * i + 4 * ch + q;
                if (row < cur.T)
                    *(f32x4*)(cur.Me + (long long)row * K + cur.n0 + wn * 64 + 4 * lr) =
                        f32x4{acc[i][0][q], acc[i][1][q], acc[i][2][q], acc[i][3][q]};
            }
        }
        if (!more) break;
        it = nx;
        cur = nxt;
    }
}

#endif  // AZG_SG_PROBES
}  // namespace

// cap on the persistent grid (azg_set_gemm_blocks; 0: one block per CU)
static int g_block_cap = 0;

// one workgroup per CU (a block fills a CU: 128 KB of LDS), at most one per tile
static unsigned persistent_blocks(int tiles) {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    const int n = g_block_cap > 0 && g_block_cap < cus ? g_block_cap : cus;
    return (unsigned)(tiles < n ? tiles : n);
}

// Persistent split-GEMM launches use at most `blocks` workgroups (CUs) from now on, leaving
// the other CUs to kernels of another stream (two half-batches on two streams: one's GEMM
// beside the other's HBM-bound transforms); 0 restores one block per CU.  Process-wide.
// Rounded down to a multiple of 8 (at least 8): the persistent kernels deal each XCD
// (blockIdx % 8) a contiguous tile range, so every XCD needs a block.
extern "C" int azg_set_gemm_blocks(int32_t blocks) {
    if (blocks < 0) return AZG_ERR_ARG;
    g_block_cap = blocks == 0 ? 0 : (blocks < 8 ? 8 : blocks & ~7);
    return 0;
}

static int split_gemm_launch(int variant, const void* A, const void* Bt, float* M, int32_t nruns,
                             const int32_t* points, const int32_t* rows, int32_t c, int32_t k, void* stream,
                             unsigned long long* stamps = nullptr) {
    if (!A || !Bt || !M || !points || !rows || nruns < 1 || nruns > SG_MAXRUNS || c <= 0 || c % (2 * SG_BK) ||
        k <= 0 || k % SG_BN || ((uintptr_t)A & 15) || ((uintptr_t)Bt & 15) || ((uintptr_t)M & 15) || variant < 0 ||
        variant > 19 || variant == 9 || variant == 13 || variant == 14 || (variant == 10) != (stamps != nullptr))
        return AZG_ERR_ARG;
#ifndef AZG_SG_PROBES
    // the product schedules: 0 (one tile per workgroup), 4 (persistent, default), 17 / 18
    // (128 / 64-row tiles for short launches); the others exist in the probe build only
    if (variant != 0 && variant != 4 && variant != 17 && variant != 18) return AZG_ERR_ARG;
    const int bm = variant == 17 ? 128 : variant == 18 ? 64 : SG_BM;
#else
    const int bm = variant == 17 ? 128 : variant == 18 ? 64 : variant == 19 ? S3_BM : SG_BM;
#endif
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
        g.mtiles[r] = (rows[r] + bm - 1) / bm;
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
    g.stamps = stamps;
    if (variant == 0)
        hipLaunchKernelGGL(split_gemm_kernel<false>, dim3(tiles), dim3(512), 0, (hipStream_t)stream, g);
    else if (variant == 17)
        hipLaunchKernelGGL((split_gemm_kernel<false, 128>), dim3(tiles), dim3(512), 0, (hipStream_t)stream, g);
    else if (variant == 18)
        hipLaunchKernelGGL((split_gemm_kernel<false, 64>), dim3(tiles), dim3(512), 0, (hipStream_t)stream, g);
    else if (variant == 4)
        hipLaunchKernelGGL(split_gemm_persist_kernel<8>, dim3(persistent_blocks(tiles)), dim3(512), 0,
                           (hipStream_t)stream, g);
#ifdef AZG_SG_PROBES
    else if (variant == 3)
        hipLaunchKernelGGL(split_gemm_kernel<true>, dim3(tiles), dim3(512), 0, (hipStream_t)stream, g);
    else if (variant == 1)
        hipLaunchKernelGGL(split_gemm_pipe_kernel, dim3(tiles), dim3(512), 0, (hipStream_t)stream, g);
    else if (variant == 5)
        hipLaunchKernelGGL(split_gemm_persist_kernel<4>, dim3(persistent_blocks(tiles)), dim3(512), 0,
                           (hipStream_t)stream, g);
    else if (variant == 6)
        hipLaunchKernelGGL((split_gemm_persist_kernel<8, true>), dim3(persistent_blocks(tiles)), dim3(512), 0,
                           (hipStream_t)stream, g);
    else if (variant == 7)
        hipLaunchKernelGGL((split_gemm_persist_kernel<4, false, true>), dim3(persistent_blocks(tiles)), dim3(512), 0,
                           (hipStream_t)stream, g);
    else if (variant == 8)
        hipLaunchKernelGGL((split_gemm_persist_kernel<8, false, false, true>), dim3(persistent_blocks(tiles)),
                           dim3(512), 0, (hipStream_t)stream, g);
    else if (variant == 11)
        hipLaunchKernelGGL((split_gemm_persist_kernel<8, false, false, false, false, true>),
                           dim3(persistent_blocks(tiles)), dim3(512), 0, (hipStream_t)stream, g);
    else if (variant == 12)
        hipLaunchKernelGGL(split_gemm_pp2_kernel, dim3(persistent_blocks(tiles)), dim3(512), 0, (hipStream_t)stream, g);
    else if (variant == 15)
        hipLaunchKernelGGL((split_gemm_persist_kernel<8, false, false, false, false, false, 1>),
                           dim3(persistent_blocks(tiles)), dim3(512), 0, (hipStream_t)stream, g);
    else if (variant == 16)
        hipLaunchKernelGGL((split_gemm_persist_kernel<8, false, false, false, false, false, 2>),
                           dim3(persistent_blocks(tiles)), dim3(512), 0, (hipStream_t)stream, g);
    else if (variant == 10)
        hipLaunchKernelGGL((split_gemm_persist_kernel<8, false, false, false, true>), dim3(persistent_blocks(tiles)),
                           dim3(512), 0, (hipStream_t)stream, g);
    else if (variant == 19)
        hipLaunchKernelGGL(split_gemm_384_kernel, dim3(persistent_blocks(tiles)), dim3(512), 0, (hipStream_t)stream, g);
    else
        hipLaunchKernelGGL(split_gemm_w4_kernel, dim3(tiles), dim3(256), 0, (hipStream_t)stream, g);
#endif
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

// The default schedule for a launch: variant 4 (256-row tiles, persistent) unless a
// short launch needs fewer weighted rounds of the chip on 128-row (variant 17) or
// 64-row tiles (variant 18), a round of those costing about 5/8 and 4/8 of a 256-row
// round (tools/split_gemm_bench.py with AZG_SG_LEAVES = 128-4096,
// profiles/r02_split_gemm_bench_smallbatch.json); ties keep the larger tile.
static int split_gemm_pick(int32_t nruns, const int32_t* points, const int32_t* rows, int32_t k) {
    if (!points || !rows || nruns < 1 || nruns > SG_MAXRUNS || k <= 0) return 4;
    long long t[3] = {0, 0, 0};  // tiles at 256, 128, 64 rows
    for (int r = 0; r < nruns; ++r) {
        if (points[r] <= 0 || rows[r] <= 0) return 4;
        for (int i = 0; i < 3; ++i) t[i] += (long long)points[r] * ((rows[r] + (255 >> i)) / (256 >> i)) * (k / SG_BN);
    }
    const long long cus = persistent_blocks(1 << 30);
    const int weight[3] = {8, 5, 4}, variant[3] = {4, 17, 18};
    int best = 0;
    long long best_cost = 0;
    for (int i = 0; i < 3; ++i) {
        const long long cost = (t[i] + cus - 1) / cus * weight[i];
        if (i == 0 || cost < best_cost) best = i, best_cost = cost;
    }
    return variant[best];
}

extern "C" int azg_split_gemm(const void* A, const void* Bt, float* M, int32_t nruns, const int32_t* points,
                              const int32_t* rows, int32_t c, int32_t k, void* stream) {
    return split_gemm_launch(split_gemm_pick(nruns, points, rows, k), A, Bt, M, nruns, points, rows, c, k, stream);
}

extern "C" int azg_split_gemm_pick(int32_t nruns, const int32_t* points, const int32_t* rows, int32_t k) {
    return split_gemm_pick(nruns, points, rows, k);
}

extern "C" int azg_split_gemm_variant(int32_t variant, const void* A, const void* Bt, float* M, int32_t nruns,
                                      const int32_t* points, const int32_t* rows, int32_t c, int32_t k, void* stream) {
    return split_gemm_launch(variant, A, Bt, M, nruns, points, rows, c, k, stream);
}

#ifdef AZG_SG_PROBES
// probe build only (tools/split_gemm_stamps.py): per-wave phase stamps of variant 4
extern "C" int azg_split_gemm_stamps(const void* A, const void* Bt, float* M, int32_t nruns, const int32_t* points,
                                     const int32_t* rows, int32_t c, int32_t k, uint64_t* stamps, int64_t cap,
                                     void* stream) {
    if (!stamps || cap < (int64_t)persistent_blocks(1 << 30) * 8 * 5) return AZG_ERR_ARG;
    return split_gemm_launch(10, A, Bt, M, nruns, points, rows, c, k, stream, (unsigned long long*)stamps);
}
#endif  // AZG_SG_PROBES
