// azg_small_mfma.hip -- the small-batch 3x3 convolutions (1-4 leaves: the drop-in MCTS's one leaf per
// simulation, C1) on the f32 MFMA, bit-identical to azg_small.hip's VALU kernels.
//
// At one leaf a 512-channel layer is 49 / 25 / 9 output pixels x 512 channels x 4608 products: the
// VALU kernels (small_conv_sk_kernel, small_conv_kernel) spread it over 512 blocks but each lane still
// runs a chain of up to 1,152 dependent multiply-adds fed from LDS: conv12 19.0, conv3 18.1, conv4
// 9.5 us (profiles/r05_small_layer_bench.json), 0.065 of HBM on a 9.4 MB weight stream.
//
// The arithmetic those kernels perform, per output (leaf pixel p, channel co):
//   the K products of a layer part q (KG parts of Cin / KG input channels; KG = 4 for conv12, 8 for the
//   split-K conv3, 1 for conv4) are cut into KSL contiguous slices of `per` float4 steps (k = tap *
//   Cq + ci, tap-major); each slice is an fmaf chain from 0 in k order (zero-padded taps skipped);
//   part_q = the slices summed in slice order from 0; y = relu((sum of the parts in order from 0) + b).
// v_mfma_f32_16x16x4_f32 is bit for bit a k-ordered f32 fmaf chain per output (D = fma(a3, b3, ...
// fma(a0, b0, C)), cdna_hip_programming.md 'FP32-input MFMA'), so a chain of MFMAs over a slice's k
// in order, from a zero accumulator, IS that slice's chain for 16 pixels x 16 channels at once (a
// skipped padded tap contributes fma(w, 0, acc) = acc exactly: the accumulator is never -0).  Hence:
//
//  * one block per (16-channel tile, 16-row tile, part q, slice group): each wave runs SPW slices'
//    MFMA chains (independent accumulators), the B operand (weights) streamed from a packed copy
//    Wm[q][co][slice][j][t] (lane (co, j) reads its `per` values contiguously: slot j of step t is
//    k = 4t + j), the A operand (the im2col inputs) read per lane from the previous layer's NHWC
//    rows in L2 -- or, for conv12, from conv1's output computed into LDS by conv1_sparse exactly as
//    small_conv_sk_kernel does;
//  * a block covering a whole part sums its slices in order through LDS and publishes the part sum;
//    with KG = 1 (conv4) a block covers a few slices and publishes the raw chains (a part of one
//    slice: 0 + chain = chain exactly), so the layer spreads over 256 blocks instead of 32;
//  * the published tiles meet as in azg_small.hip: write-through stores drained, one relaxed ticket
//    per (channel tile, row tile), the last block sums them in order, adds the bias, applies ReLU.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../include/azg.h"
#include "../alpha-zero-general-inflexion_amd/csrc/azg_conv1.h"
#include "azg_small_probes.h"

#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "azg_small_mfma.hip's hand-off assumes the gfx950 memory model (see azg_small.hip)"
#endif

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int SM_MAXW = 8;      // waves per block
// conv12: conv1's output for the tile's leaves, <= 2 x 49 cells x (128 + 4) floats at the 7x7 board
// (52 KB: two blocks per CU with the chains' LDS; 8x8 boards take the VALU kernels)
constexpr int SM_LDS = 52 * 1024;

struct SmArgs {
    const float* x;       // NHWC rows of the previous layer (sB per leaf, sY, sX; channels contiguous) or,
                          // with w1, the NCHW leaf planes [B][D][n][n]
    long long sB;
    int sY, sX;
    int B, H, pad, Ho;    // batch, input side, padding, output side
    const float* wm;      // packed weights [KG][Cout][KSL][4][TP]
    int Cin, Cout, KG, KSL, per, SPB;  // parts, slices per part, float4 steps per slice, slices per block
    const float* bias;
    int relu;
    float* y;
    int ldy;
    float* work;          // [tiles][KG or KSL][256]
    unsigned* tickets;    // [tiles]
    const float* w1;      // conv1 (conv12): [C][3][3][D], b1 [C]
    const float* b1;
    int D;
};

__device__ __forceinline__ void st_wt(float* p, float v) {  // write-through (agent-scope relaxed atomic store)
    __hip_atomic_store((unsigned*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_coh(const float* p) {
    return __uint_as_float(__hip_atomic_load((const unsigned*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// F1 > 0: conv12 (conv1 of the leaf planes fused, board side F1); SPW: slices per wave; PER: float4
// steps per slice (a.per)
template <int F1, int SPW, int PER>
__global__ __launch_bounds__(64 * SM_MAXW) __attribute__((amdgpu_waves_per_eu(1, 2))) void small_mfma_conv_kernel(SmArgs a) {
    __shared__ __attribute__((aligned(16))) float lds[F1 > 0 ? SM_LDS / 4 : 1];
    __shared__ float red[F1 > 0 ? 1 : 1][16 * SM_MAXW * SPW][17];  // [slice][row][co] chains of the block
    __shared__ unsigned s_last;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int nw = blockDim.x >> 6;
    const int cot = blockIdx.x, rt = blockIdx.y;
    const int groups = a.KSL / a.SPB;       // slice groups per part
    const int q = blockIdx.z / groups, g = blockIdx.z - q * groups;
    const int Cq = a.Cin / a.KG, hw = a.Ho * a.Ho, rows = a.B * hw;
    const int co = cot * 16 + (lane & 15), j = lane >> 4;
    // the lane's A row (pixel) for the MFMA A operand: row l & 15 of the tile
    const int row = rt * 16 + (lane & 15);
    const bool rok = row < rows;
    const int leaf = rok ? row / hw : 0, pix = rok ? row - leaf * hw : 0;
    const int oy = pix / a.Ho, ox = pix - oy * a.Ho;
    const int leaf0 = (rt * 16) / hw;       // first leaf of the tile (conv12 staging)
    const int P = Cq + 4;                   // LDS pitch of a staged pixel (conv12)
    if constexpr (F1 > 0) {
        // conv1 for this part's Cq channels at every cell of the tile's leaves (<= 2 for hw >= 16):
        // relu(b1 + conv1_sparse(planes)), as small_conv_sk_body stages it
        constexpr int NN = F1 * F1;
        const int leaf1 = min(a.B - 1, (rt * 16 + 15) / hw);
        const int ci_base = q * Cq;
        for (int item = wv; item < (leaf1 - leaf0 + 1) * ((Cq + 63) / 64); item += nw) {
            const int lf = leaf0 + item / ((Cq + 63) / 64), cb = item % ((Cq + 63) / 64);
            const int c = min(cb * 64 + lane, Cq - 1);
            float acc1[NN];
            conv1_sparse<F1>(a.x + lf * a.sB, a.w1 + (long long)(ci_base + c) * 9 * a.D, a.D, lane, acc1, 1, a.D);
            const float bc = a.b1[ci_base + c];
            if (cb * 64 + lane < Cq) {
#pragma unroll
                for (int r = 0; r < NN; ++r) lds[((lf - leaf0) * NN + r) * P + c] = fmaxf(acc1[r] + bc, 0.f);
            }
        }
        __syncthreads();
    }
    // this wave's slices: s = g * SPB + wv * SPW + u.  Every operand of the wave's chains is loaded
    // first (PER weights and PER inputs per slice and lane: one memory round trip), then the MFMAs.
    f32x4 acc[SPW];
    const int s0 = g * a.SPB + wv * SPW;
    const bool active = wv * SPW < a.SPB;
    if (active) {
        constexpr int TP = (PER + 3) / 4 * 4;
        float bv[SPW][TP], av[SPW][PER];
#pragma unroll
        for (int u = 0; u < SPW; ++u) {
            const int s = s0 + u;
            const float4* __restrict__ wb =
                (const float4*)(a.wm + ((((long long)q * a.Cout + co) * a.KSL + s) * 4 + j) * TP);
#pragma unroll
            for (int t4 = 0; t4 < TP / 4; ++t4) {
                const float4 w4 = wb[t4];
                bv[u][4 * t4] = w4.x, bv[u][4 * t4 + 1] = w4.y, bv[u][4 * t4 + 2] = w4.z, bv[u][4 * t4 + 3] = w4.w;
            }
            // slot j of step t: k = 4 (s PER + t) + j within the part (tap-major); Cq % 4 == 0, so the
            // tap advances only where ci wraps
            int k = 4 * s * PER + j;
            int tap = k / Cq, ci = k - tap * Cq;
            // branch-free: every lane loads from an in-bounds address (a padded tap reads cell (0, 0)) and
            // selects 0 for it, so all PER loads issue before the first wait (a load under a divergent
            // branch was waited for inside the branch: one memory round trip per step)
#pragma unroll
            for (int t = 0; t < PER; ++t) {
                const int iy = oy + tap / 3 - a.pad, ix = ox + tap % 3 - a.pad;
                const bool ok = rok && iy >= 0 && iy < a.H && ix >= 0 && ix < a.H;
                const int iyc = ok ? iy : 0, ixc = ok ? ix : 0;
                float v;
                if constexpr (F1 > 0)
                    v = lds[((leaf - leaf0) * F1 * F1 + iyc * F1 + ixc) * P + ci];
                else
                    v = a.x[leaf * a.sB + (long long)iyc * a.sY + (long long)ixc * a.sX + q * Cq + ci];
                av[u][t] = ok ? v : 0.f;
                ci += 4;
                if (ci >= Cq) ci -= Cq, ++tap;
            }
        }
#pragma unroll
        for (int u = 0; u < SPW; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < PER; ++t)
#pragma unroll
            for (int u = 0; u < SPW; ++u)  // (the slices' chains interleaved: independent accumulators)
                acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u][t], bv[u][t], acc[u], 0, 0, 0);
    }
    // the chains to LDS: D[row 4 (l >> 4) + r][col l & 15]
    if (active) {
#pragma unroll
        for (int u = 0; u < SPW; ++u)
#pragma unroll
            for (int r = 0; r < 4; ++r) red[0][(wv * SPW + u) * 16 + 4 * (lane >> 4) + r][lane & 15] = acc[u][r];
    }
    __syncthreads();
    const int tiles_x = gridDim.x;
    const long long tile = (long long)rt * tiles_x + cot;
    const bool whole = a.SPB == a.KSL;  // the block covers part q: publish its ordered slice sum
    const int nslots = whole ? a.KG : a.KSL;
    float* wt = a.work + tile * nslots * 256;
    if (tid < 256) {
        const int r = tid >> 4, c = tid & 15;
        if (whole) {
            float sum = 0.f;
            for (int s = 0; s < a.SPB; ++s) sum += red[0][s * 16 + r][c];  // slice order
            st_wt(wt + q * 256 + tid, sum);
        } else {
            for (int s = 0; s < a.SPB; ++s) st_wt(wt + (g * a.SPB + s) * 256 + tid, red[0][s * 16 + r][c]);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const unsigned expect = whole ? (unsigned)a.KG : (unsigned)groups;  // (KG == 1 when !whole)
    if (tid == 0) s_last = __hip_atomic_fetch_add(a.tickets + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                           expect - 1;
    __syncthreads();
    if (!s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (compiler order only: the loads are sc1)
    if (tid < 256) {
        const int r = tid >> 4, c = tid & 15;
        const int orow = rt * 16 + r, oco = cot * 16 + c;
        if (orow < rows) {
            float sum = 0.f;
            for (int p = 0; p < nslots; ++p) sum += ld_coh(wt + p * 256 + tid);  // part / slice order
            float o = sum + (a.bias ? a.bias[oco] : 0.f);
            if (a.relu) o = fmaxf(o, 0.f);
            a.y[(long long)orow * a.ldy + oco] = o;
        }
    }
    if (tid == 0) __hip_atomic_store(a.tickets + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the slicing azg_small.hip's kernels use for this layer (see the header): KG, KSL, per
bool small_layout(int H, int pad, int Cin, int Cout, bool conv12, int* kg, int* ksl, int* per) {
    const int Ho = H + 2 * pad - 2, n = Ho * Ho;
    if (Ho <= 0 || n > 256) return false;
    const int pxl = n <= 16 ? 16 : n <= 32 ? 32 : n <= 64 ? 64 : n <= 128 ? 128 : 256;
    int KG;
    if (conv12) KG = 4;                                          // SK_KG1
    else if (n > 16 && Cin % 32 == 0 && Cout % 8 == 0) KG = 8;  // the split-K form (SK_KG)
    else KG = 1;                                                 // small_conv_kernel (VEC)
    if (Cin % (4 * KG)) return false;
    const int KSL = 512 / pxl, KS = 9 * (Cin / KG) / 4;
    const int pr = (KS + KSL - 1) / KSL;
    if (pr * KSL != KS) return false;  // (ragged slices: not implemented here)
    *kg = KG, *ksl = KSL, *per = pr;
    return true;
}

}  // namespace

extern "C" int azg_small_mfma_layout(int32_t H, int32_t pad, int32_t Cin, int32_t Cout, int32_t conv12, int32_t* out) {
    int kg, ksl, per;
    if (!out || Cin <= 0 || Cout <= 0 || !small_layout(H, pad, Cin, Cout, conv12 != 0, &kg, &ksl, &per))
        return AZG_ERR_ARG;
    out[0] = kg;
    out[1] = ksl;
    out[2] = per;
    out[3] = (per + 3) / 4 * 4;
    return AZG_OK;
}

extern "C" int azg_small_conv_mfma(const float* x, int64_t sB, int32_t sY, int32_t sX, int32_t batch, int32_t H,
                                   int32_t pad, const float* wm, int32_t Cin, int32_t Cout, const float* bias,
                                   int32_t relu, float* y, int32_t ldy, float* work, int64_t work_floats,
                                   uint32_t* tickets, int32_t n_tickets, const float* w1, const float* b1, int32_t D,
                                   void* stream) {
    const bool c12 = w1 != nullptr;
    int kg, ksl, per;
    if (!x || !wm || !y || !work || !tickets || batch <= 0 || batch > 4 || pad < 0 || pad > 1 || Cout % 16 ||
        ldy < Cout || !small_layout(H, pad, Cin, Cout, c12, &kg, &ksl, &per) || ((uintptr_t)wm & 15))
        return AZG_ERR_ARG;
    const int Ho = H + 2 * pad - 2, rows = batch * Ho * Ho;
    const int rtiles = (rows + 15) / 16, ctiles = Cout / 16;
    if (c12) {
        // conv1 of the tile's leaves in LDS: <= 2 leaves of the board (hw >= 16) x Cq channels
        if (!b1 || D < 1 || D > 4 || H < 6 || H > 8 || pad != 1 || Ho * Ho < 16 ||
            (size_t)2 * H * H * (Cin / kg + 4) * 4 > (size_t)SM_LDS)
            return AZG_ERR_ARG;
    } else if (sY < 0 || sX < 0 || sB < 0) {
        return AZG_ERR_ARG;
    }
    // slices per wave / per block: a whole part per block when it has several parts (in-block slice
    // sums), else (KG 1: conv4) 4 slices per block, one per wave
    int spw, spb;
    if (kg > 1) {
        spb = ksl;
        spw = ksl <= 8 ? (ksl + 3) / 4 : (ksl + 7) / 8;
        spw = spw <= 1 ? 1 : spw <= 2 ? 2 : 4;
        if (spb > spw * SM_MAXW) return AZG_ERR_ARG;
    } else {
        spw = 1;
        spb = ksl % 4 == 0 ? 4 : 1;
    }
    const int nslots = spb == ksl ? kg : ksl;
    if (n_tickets < rtiles * ctiles || work_floats < (long long)rtiles * ctiles * nslots * 256) return AZG_ERR_ARG;
    SmArgs a{};
    a.x = x, a.sB = sB, a.sY = sY, a.sX = sX, a.B = batch, a.H = H, a.pad = pad, a.Ho = Ho;
    a.wm = wm, a.Cin = Cin, a.Cout = Cout, a.KG = kg, a.KSL = ksl, a.per = per, a.SPB = spb;
    a.bias = bias, a.relu = relu, a.y = y, a.ldy = ldy, a.work = work, a.tickets = tickets;
    a.w1 = w1, a.b1 = b1, a.D = D;
    const int waves = (spb + spw - 1) / spw;
    const dim3 grid((unsigned)ctiles, (unsigned)rtiles, (unsigned)(kg * (ksl / spb)));
    const dim3 block((unsigned)(64 * (waves < 4 ? 4 : waves)));  // >= 256 threads: the combine's 16 x 16 outputs
    hipStream_t st = (hipStream_t)stream;
    bool known = true;
    auto go = [&](auto F_, auto S_) {
        constexpr int F = decltype(F_)::value, SW = decltype(S_)::value;
        if (per == 36) hipLaunchKernelGGL((small_mfma_conv_kernel<F, SW, 36>), grid, block, 0, st, a);
        else if (per == 9) hipLaunchKernelGGL((small_mfma_conv_kernel<F, SW, 9>), grid, block, 0, st, a);
        else known = false;
    };
    auto by_spw = [&](auto F_) {
        if (spw == 1) go(F_, std::integral_constant<int, 1>{});
        else if (spw == 2) go(F_, std::integral_constant<int, 2>{});
        else go(F_, std::integral_constant<int, 4>{});
    };
    if (!c12) by_spw(std::integral_constant<int, 0>{});
    else if (H == 6) by_spw(std::integral_constant<int, 6>{});
    else if (H == 7) by_spw(std::integral_constant<int, 7>{});
    else by_spw(std::integral_constant<int, 8>{});
    if (!known) return AZG_ERR_ARG;  // (slice lengths other than the boards' layers': the VALU kernels)
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}
