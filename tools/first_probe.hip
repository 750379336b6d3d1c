// first_probe.hip -- probe build (not the product): winograd_first_kernel's write path
// in other shapes, to find what holds it at ~5.1 TB/s (HISTORY.md 6b).
// Every variant computes exactly the product kernel's values and layout (conv1_sparse,
// in_tile, the AZG_WINO_SPLIT2 rows); only the store shape and the block / grid shape
// differ:
//   S = 0: the product's two 2-byte stores per lane (one 128-B line each, permlane32_swap)
//   S = 1: one 4-byte store per lane (the wave's whole 256-B row segment in one store;
//          each lane's pair of halves gathered with two ds_bpermute)
//   WPB  : waves per block (1: the product; 4, 8: channel blocks of one image together)
//   P    : persistent grid (each wave loops over (image, channel block) items)
// Built by tools/Makefile into tools/libfirst_probe.so; driven by tools/first_probe.py.
#include "../alpha-zero-general-inflexion_amd/csrc/azg_winograd_kern.h"

namespace {

template <int S, bool NT>
__device__ __forceinline__ bool store_seg(unsigned short* rowp, unsigned lane, float v) {
    const _Float16 hi = (_Float16)v;
    const _Float16 lo = (_Float16)(v - (float)hi);
    if constexpr (S == 0) {
        return store_v2_wave<NT>(rowp, lane, v);
    } else {
        // segment halves 2L, 2L+1: block L/32; within it q = 2 (L % 32): hi (q < 32) or lo
        // (q >= 32) of channels 32 (L/32) + q % 32 and + 1
        const unsigned hl = (unsigned)__builtin_bit_cast(unsigned short, hi) |
                            ((unsigned)__builtin_bit_cast(unsigned short, lo) << 16);
        const unsigned l31 = lane & 31u;
        const unsigned src = (lane & 32u) + ((2u * l31) & 31u);
        const unsigned a = (unsigned)__builtin_amdgcn_ds_bpermute((int)(src * 4), (int)hl);
        const unsigned b = (unsigned)__builtin_amdgcn_ds_bpermute((int)((src + 1) * 4), (int)hl);
        const unsigned out = l31 < 16 ? ((a & 0xffffu) | (b << 16)) : ((a >> 16) | (b & 0xffff0000u));
        unsigned* p = (unsigned*)rowp + lane;
        if constexpr (NT) __builtin_nontemporal_store(out, p);
        else *p = out;
        return !(fabsf(v) <= 65504.f);
    }
}

template <int S, bool NT, int NPARTS = 2>
__device__ __forceinline__ void plane_to_V_probe(const float (&ys)[49], long long b, int c0, unsigned lane, int C,
                                                 long long B, void* __restrict__ Vout, int* overflow, int only_row = -1) {
    constexpr int HO = 7;
    const WSeq Sq(HO);
    bool bad = false;
    for_tiles<HO>(Sq, [&](auto A_, auto B_, int i, int j) {
        constexpr int MA = decltype(A_)::value, MB = decltype(B_)::value;
        if (only_row >= 0 && (NPARTS == 2 ? i : i * 2 + j) != only_row) return;  // (wave-uniform)
        const long long row = Sq.row0(i, j, b, B), ps = Sq.pstride(i, j, B);
        const int y0 = Sq.off(i) - 1, x0 = Sq.off(j) - 1;
        float d[MA + 2][MB + 2];
#pragma unroll
        for (int u = 0; u < MA + 2; ++u)
#pragma unroll
            for (int v = 0; v < MB + 2; ++v) {
                const int iy = y0 + u, ix = x0 + v;
                d[u][v] = (iy >= 0 && iy < 7 && ix >= 0 && ix < 7) ? ys[iy * 7 + ix] : 0.f;
            }
        float Vt[MA + 2][MB + 2];
        in_tile<MA, MB>(d, Vt);
#pragma unroll
        for (int e = 0; e < (MA + 2) * (MB + 2); ++e)
            bad |= store_seg<S, NT>((unsigned short*)Vout + (row + e * ps) * 2 * C + 2 * c0, lane,
                                    Vt[e / (MB + 2)][e % (MB + 2)]);
    });
    if (bad) atomicOr(overflow, 1);
}

template <int S, int WPB, bool P, bool NT, int HALVES = 1>
__global__ __launch_bounds__(64 * WPB) void first_probe_kernel(const float* __restrict__ planes,
                                                               const float* __restrict__ w1,
                                                               const float* __restrict__ b1, void* __restrict__ Vout,
                                                               int depth, int C, long long B, int* overflow) {
    const unsigned lane = threadIdx.x & 63u;
    const unsigned w = WPB > 1 ? (unsigned)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0u;  // wave-uniform
    const int cblocks = C / 64;
    const long long items = B * cblocks * HALVES;
    auto body = [&](long long it2) {
        const int half = HALVES > 1 ? (int)(it2 % HALVES) : -1;
        const long long it = it2 / HALVES;
        const long long b = it / cblocks;
        const int k0 = (int)(it % cblocks) * 64, k = k0 + (int)lane;
        const float bk = b1[k];
        float acc[49];
        conv1_sparse<7>(planes + b * depth * 49, w1 + (size_t)k * depth * 9, depth, lane, acc);
        if constexpr (S == 0 && HALVES == 1) {
            Plane<7> ys;
#pragma unroll
            for (int q = 0; q < 49; ++q) ys.put(q, fmaxf(acc[q] + bk, 0.f));
            plane_to_V<7, AZG_WINO_SPLIT2, 1, NT>(ys, 7, b, k0, lane, C, B, Vout, overflow);
        } else {
            float ys[49];
#pragma unroll
            for (int q = 0; q < 49; ++q) ys[q] = fmaxf(acc[q] + bk, 0.f);
            plane_to_V_probe<S, NT, HALVES>(ys, b, k0, lane, C, B, Vout, overflow, half);
        }
    };
    const long long it0 = (long long)blockIdx.x * WPB + w;
    if constexpr (P) {
        for (long long it = it0; it < items; it += (long long)gridDim.x * WPB) body(it);
    } else {
        body(it0);  // the grid is exact (items % WPB == 0, checked by the launcher)
    }
}

}  // namespace

// variant: 0 the product kernel; 1.. the probe shapes below.  grid_waves: persistent
// variants' total waves (0: 16 per CU)
extern "C" int first_probe(int variant, const float* planes, const float* w1, const float* b1, void* V, int batch,
                           int depth, int c, int* overflow, int grid_waves, void* stream) {
    if (!planes || !w1 || !b1 || !V || batch <= 0 || depth < 1 || depth > 4 || c % 64) return AZG_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    const long long B = batch, items = B * (c / 64);
    const int gw = grid_waves > 0 ? grid_waves : 256 * 16;
    if (items % 8) return AZG_ERR_ARG;
    auto go = [&](auto kern, int wpb, bool persist, int halves = 1) {
        long long blocks = persist ? gw / wpb : (items * halves + wpb - 1) / wpb;
        hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(64 * wpb), 0, st, planes, w1, b1, V, depth, c, B,
                           overflow);
    };
    switch (variant) {
        case 0:
            hipLaunchKernelGGL((winograd_first_kernel<7, AZG_WINO_SPLIT2>), dim3((unsigned)items), dim3(64), 0, st,
                               planes, w1, b1, V, depth, 7, c, B, overflow);
            break;
        case 1: go(first_probe_kernel<0, 1, false, true>, 1, false); break;
        case 2: go(first_probe_kernel<1, 1, false, true>, 1, false); break;
        case 3: go(first_probe_kernel<0, 4, false, true>, 4, false); break;
        case 4: go(first_probe_kernel<1, 4, false, true>, 4, false); break;
        case 5: go(first_probe_kernel<0, 8, false, true>, 8, false); break;
        case 6: go(first_probe_kernel<1, 8, false, true>, 8, false); break;
        case 7: go(first_probe_kernel<0, 1, true, true>, 1, true); break;
        case 8: go(first_probe_kernel<1, 1, true, true>, 1, true); break;
        case 9: go(first_probe_kernel<1, 4, true, true>, 4, true); break;
        case 10: go(first_probe_kernel<1, 1, false, false>, 1, false); break;
        case 11: go(first_probe_kernel<0, 1, false, false>, 1, false); break;
        case 12: go(first_probe_kernel<0, 1, false, true, 2>, 1, false, 2); break;  // tile rows over 2 waves
        case 13: go(first_probe_kernel<1, 1, false, true, 2>, 1, false, 2); break;
        case 14: go(first_probe_kernel<0, 4, false, true, 2>, 4, false, 2); break;
        case 15: go(first_probe_kernel<0, 1, false, true, 4>, 1, false, 4); break;  // one tile per wave
        case 16: go(first_probe_kernel<0, 4, false, true, 4>, 4, false, 4); break;
        case 17: go(first_probe_kernel<0, 2, false, true, 2>, 2, false, 2); break;
        default: return AZG_ERR_ARG;
    }
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}
