// azg_small.hip -- the leaf network at one to four leaves (C1: one game, one leaf per
// simulation; the drop-in MCTS; small arenas): conv1-4 (3x3, BN folded, bias + ReLU,
// InflexionNNet.py:39-45) and fc1 / fc2 / [fc3 | fc4] (:47-54), one launch per layer, meant
// to be replayed from a HIP graph (the drop-in captures each call's simulations).
//
// At one leaf a layer is a weight stream with little reuse: conv2 is 49 pixels x 512
// channels x 4608 products against 9.4 MB of weights, fc1 1024 x 4608 against 18.9 MB.
// The cost that matters is latency -- dependent memory round trips and the serial chain of
// multiply-adds in one lane -- so both kernels spread every layer over the whole chip and
// keep each lane's chain short:
//
//  * small_conv_kernel<PXL, CO_PB, VEC, WLDS>: block = CO_PB output channels x the output
//    pixels of one leaf at a time, 512 threads = PXL pixels x (512 / PXL) K-slices.  The leaf's
//    input plane (one burst of loads, rows padded so a ds_read_b128 phase is conflict-free) and
//    the block's weight rows (WLDS, when both fit the CU's 160 KB) are staged in LDS, so the
//    multiply-adds wait on one memory round trip, not on one per step.  Thread (p, s) sums,
//    for its pixel p, the products of its contiguous slice of k = tap * Cin + ci (float4 steps
//    along ci for NHWC inputs: VEC), then the slices' partial sums are added through LDS in
//    slice order, + bias, ReLU, written as NHWC rows.  PXL is the smallest of 16 / 32 / 64 /
//    128 / 256 that holds one leaf's output pixels, so conv3 / conv4's 25 / 9 pixels cut K
//    into 16 / 32 slices and the lanes stay busy; each leaf is summed in the same order
//    whatever the batch (batch-invariant).  A lane's chain is CO_PB x 9 Cin / slices
//    multiply-adds (conv2: 1152).
//  * small_fc_kernel<NPB, BMAX>: block = NPB output rows, 256 threads split K in float4
//    steps (lane-contiguous: 1 KB of weights per wave-instruction), each thread holding
//    NPB x B sums; a wave butterfly then an LDS step across the 4 waves, in a fixed order.
//
// Everything is f32 with a fixed summation order (deterministic; per leaf the same whatever the batch);
// P and v stay within the north_star's 1e-5 of the reference module
// (tests/test_gpu_nn.py::test_small_forward_matches_reference).  The softmax / tanh heads are
// azg_policy_value (azg_heads.hip).  Replaces round 3's split-K partial / reduce GEMMs and
// one-launch layer (3.4-3.7 ms per 25-simulation drop-in call against the library form's
// 3.0; HISTORY.md 6b).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "../../include/azg.h"
#include "azg_conv1.h"
#ifdef AZG_SMALL_PROBES
#include "../../tools/azg_small_probes.h"
#endif

// The split-K hand-off below (partials stored with relaxed agent-scope atomic stores, every
// wave draining them with `s_waitcnt vmcnt(0)`, one relaxed ticket per block, the last block
// reading with relaxed agent-scope loads) relies on the gfx9 memory model as gfx950 implements
// it: vmcnt counts stores as well as loads, and agent-scope atomic stores and loads bypass the
// non-coherent caches (sc1), so a drained store is visible to every CU.  The HIP / C++ model
// alone does not promise that (a target that counts stores separately, vscnt, would need the
// release on the ticket); this file is built for gfx950 only.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "azg_small.hip's split-K hand-off assumes the gfx950 memory model (see the comment above)"
#endif

#ifdef AZG_SMALL_TIMING  // probe build only (tools/Makefile libazg_small_timing.so, tools/sk_stamps.py)
// per-block wall-clock stamps of the split-K conv's phases: [block][8] (vector stores from lane 0)
__device__ unsigned long long azg_sk_stamps[1024 * 8];
#define SK_STAMP(i)                                                                                     \
    do {                                                                                                \
        if (threadIdx.x == 0 && bid < 1024)                                                             \
            __builtin_nontemporal_store(wall_clock64(), azg_sk_stamps + bid * 8 + (i) + threadIdx.x); \
    } while (0)
#else
#define SK_STAMP(i) \
    do {            \
    } while (0)
#endif

namespace {

constexpr int SC_T = 512;  // small_conv threads
constexpr size_t SC_LDS_MAX = 160 * 1024;  // the CU's whole LDS: one block per CU
constexpr int SC_UNR = 16;   // input staging loads in flight per thread
constexpr int SC_UNRW = 6;   // weight staging loads per thread (2 x 4608 floats: 4.5)
constexpr int SF_T = 256;  // small_fc threads

// LDS row pitch (floats) of a staged input pixel: channels rounded up to float4, + 4 so that
// the 16 lanes of a ds_read_b128 phase (16 neighbouring pixels) start on 16 different
// 4-bank groups (pitch % 64 == 4 for Cin % 64 == 0)
__host__ __device__ constexpr int sc_pitch(int cin) { return ((cin + 3) & ~3) + 4; }

// COH (the fused forward, small_net_kernel): activations another block of the same launch wrote
// are read with device-scope (sc1) loads and written with agent-scope (write-through) stores -- the
// split-K hand-off's rule (see above) applied to every layer boundary inside the launch.  The loads
// are 128-bit buffer loads with the sc1 cache policy from a wave-uniform base (one instruction per
// float4; relaxed agent-scope atomic loads are 32-bit, four instructions per float4).  (Ordinary loads
// after an agent-scope acquire fence instead -- buffer_inv sc1 per wave at each layer, dropping the
// XCD's L2 weights with the stale lines -- measured 192 us per forward against these loads' 130 us,
// profiles/r05_small_net_probe_*.json.)
constexpr int BUF_SC1 = 16;  // cache-policy bit of sc1 in the buffer intrinsics' aux operand (gfx940+)

[[maybe_unused]] __device__ __forceinline__ __amdgpu_buffer_rsrc_t coh_rsrc(const float* base) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7fffffff, 0x00020000);
}

template <bool COH>
__device__ __forceinline__ float4 ld4(const float* base, long long off) {  // base: wave-uniform
    if constexpr (COH)
        return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(coh_rsrc(base), (int)(off * 4), 0,
                                                                                BUF_SC1));
    else
        return *(const float4*)(base + off);
}
template <bool COH>
__device__ __forceinline__ float ld1(const float* base, long long off) {  // base: wave-uniform
    if constexpr (COH)
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(coh_rsrc(base), (int)(off * 4), 0,
                                                                              BUF_SC1));
    else
        return base[off];
}
template <bool COH>
__device__ __forceinline__ void st1(float* p, float v) {
    if constexpr (COH)
        __hip_atomic_store((unsigned*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        *p = v;
}

template <int PXL, int CO_PB, bool VEC, bool WLDS, bool COH = false>
__device__ __forceinline__ void small_conv_body(int bid, float* __restrict__ lds, const float* __restrict__ x,
                                                long long sB, int sY, int sX, int sC, int B, int H, int pad,
                                                const float* __restrict__ w, int Cin, int Cout,
                                                const float* __restrict__ bias, int relu, float* __restrict__ y,
                                                int ldy) {
    constexpr int KSL = SC_T / PXL;  // K slices
    const int tid = threadIdx.x;
    const int p = tid % PXL, s = tid / PXL;
    const int co0 = bid * CO_PB;
    const int Ho = H + 2 * pad - 2, hw = Ho * Ho;
    const int K = 9 * Cin, P = sc_pitch(Cin);
    float* xs = lds;                          // [H * H][P] one leaf's input
    float* ws = xs + H * H * P;               // [CO_PB][K] the block's weights (WLDS)
    float* red = ws + (WLDS ? CO_PB * K : 0);  // [KSL][PXL][CO_PB]
    constexpr int STEP = VEC ? 4 : 1;
    const int KS = K / STEP;
    const int per = (KS + KSL - 1) / KSL;
    const int k0 = s * per, k1 = min(KS, k0 + per);
    // staging: every thread's loads are issued together (UNR float4 in flight per thread, one memory
    // round trip per UNR x 8 KB), then stored to LDS.  UNR: SC_UNR, or 8 for <= 16 output pixels
    // (conv4: a 5 x 5 x 512 plane is 6.25 vectors per thread; 16 in flight held 256 VGPRs + 48 B of
    // scratch, 8 fit)
    constexpr int UNR = PXL <= 16 ? 8 : SC_UNR;
    const int nw4 = WLDS ? CO_PB * K / 4 : 0;  // the block's weights: CO_PB contiguous rows
    const float4* __restrict__ w4 = (const float4*)(w + (long long)co0 * K);
    int oy = 0, ox = 0;
    if (p < hw) oy = p / Ho, ox = p - (p / Ho) * Ho;
    for (int b = 0; b < B; ++b) {
        // stage leaf b's input plane into LDS (NHWC float4 rows, or any strides element-wise);
        // with the weights on the first leaf
        const float* __restrict__ xb = x + b * sB;
        if constexpr (VEC) {
            const int c4 = Cin / 4, nx4 = H * H * c4;
            // one batch of input vectors from `base` (and with WW the block's weights: their loads
            // issued first, their stores after the batch's loads are in flight)
            auto batch = [&](int base, auto WW) {
                constexpr bool WITHW = decltype(WW)::value;
                float4 rw[WITHW ? SC_UNRW : 1];
                if constexpr (WITHW) {
#pragma unroll
                    for (int u = 0; u < SC_UNRW; ++u) rw[u] = w4[min(tid + u * SC_T, nw4 - 1)];
                }
                float4 r[UNR];
#pragma unroll
                for (int u = 0; u < UNR; ++u) {  // past the end: a duplicate load, not stored
                    const int i = min(base + u * SC_T, nx4 - 1);
                    const int pix = i / c4, c = (i - pix * c4) * 4, iy = pix / H, ix = pix - iy * H;
                    r[u] = ld4<COH>(xb, (long long)iy * sY + (long long)ix * sX + c);
                }
                if constexpr (WITHW) {
#pragma unroll
                    for (int u = 0; u < SC_UNRW; ++u)  // past the end: rewrites the last vector with its own value
                        ((float4*)ws)[min(tid + u * SC_T, nw4 - 1)] = rw[u];
                    for (int i = tid + SC_UNRW * SC_T; i < nw4; i += SC_T) ((float4*)ws)[i] = w4[i];
                }
#pragma unroll
                for (int u = 0; u < UNR; ++u) {
                    const int i = base + u * SC_T;
                    if (i < nx4) {
                        const int pix = i / c4, c = (i - pix * c4) * 4;
                        *(float4*)(xs + pix * P + c) = r[u];
                    }
                }
            };
            if (WLDS && b == 0) batch(tid, std::true_type{});
            else batch(tid, std::false_type{});
            for (int base = tid + SC_T * UNR; base < nx4; base += SC_T * UNR) batch(base, std::false_type{});
        } else {
            if (b == 0)
                for (int i = tid; i < nw4; i += SC_T) ((float4*)ws)[i] = w4[i];
            const int n = H * H * Cin;
            for (int i = tid; i < n; i += SC_T) {
                const int pix = i / Cin, c = i - pix * Cin, iy = pix / H, ix = pix - iy * H;
                xs[pix * P + c] = ld1<COH>(xb, (long long)iy * sY + (long long)ix * sX + (long long)c * sC);
            }
        }
        __syncthreads();
        float acc[CO_PB];
#pragma unroll
        for (int c = 0; c < CO_PB; ++c) acc[c] = 0.f;
        if (p < hw) {
            int kk = k0;
            while (kk < k1) {  // k runs tap-major: a slice is a few runs of one tap each
                const int k = kk * STEP;
                const int tap = k / Cin, ci0 = k - tap * Cin;
                const int run = min(k1 - kk, (Cin - ci0) / STEP);
                const int iy = oy + tap / 3 - pad, ix = ox + tap % 3 - pad;
                if (iy >= 0 && iy < H && ix >= 0 && ix < H) {
                    const float* xp = xs + (iy * H + ix) * P + ci0;
                    if constexpr (VEC) {
#pragma unroll 4
                        for (int j = 0; j < run; ++j) {
                            const float4 xv = *(const float4*)(xp + 4 * j);
#pragma unroll
                            for (int c = 0; c < CO_PB; ++c) {
                                const float4 wv = WLDS ? *(const float4*)(ws + c * K + k + 4 * j)
                                                       : *(const float4*)(w + (long long)(co0 + c) * K + k + 4 * j);
                                float a = acc[c];
                                a = fmaf(wv.x, xv.x, a);
                                a = fmaf(wv.y, xv.y, a);
                                a = fmaf(wv.z, xv.z, a);
                                a = fmaf(wv.w, xv.w, a);
                                acc[c] = a;
                            }
                        }
                    } else {
                        for (int j = 0; j < run; ++j) {
                            const float xv = xp[j];
#pragma unroll
                            for (int c = 0; c < CO_PB; ++c)
                                acc[c] = fmaf(WLDS ? ws[c * K + k + j] : w[(long long)(co0 + c) * K + k + j], xv, acc[c]);
                        }
                    }
                }
                kk += run;
            }
        }
#pragma unroll
        for (int c = 0; c < CO_PB; ++c) red[(s * PXL + p) * CO_PB + c] = acc[c];
        __syncthreads();
        for (int t = tid; t < hw * CO_PB; t += SC_T) {
            const int pp = t / CO_PB, c = t - pp * CO_PB;
            float sum = 0.f;
            for (int q = 0; q < KSL; ++q) sum += red[(q * PXL + pp) * CO_PB + c];  // slice order
            float o = sum + (bias ? bias[co0 + c] : 0.f);
            if (relu) o = fmaxf(o, 0.f);
            st1<COH>(y + (long long)(b * hw + pp) * ldy + co0 + c, o);
        }
        __syncthreads();  // xs and red are rewritten for the next leaf
    }
}

template <int PXL, int CO_PB, bool VEC, bool WLDS>
__global__ __launch_bounds__(SC_T) void small_conv_kernel(const float* __restrict__ x, long long sB, int sY, int sX,
                                                          int sC, int B, int H, int pad,
                                                          const float* __restrict__ w, int Cin, int Cout,
                                                          const float* __restrict__ bias, int relu,
                                                          float* __restrict__ y, int ldy) {
    __shared__ __attribute__((aligned(16))) float lds[SC_LDS_MAX / 4];
    small_conv_body<PXL, CO_PB, VEC, WLDS>(blockIdx.x, lds, x, sB, sY, sX, sC, B, H, pad, w, Cin, Cout, bias, relu, y,
                                           ldy);
}

// Split-K form for the 512-channel layers (conv2-4): block (co group of SK_CO = 8 channels, ci
// part kg of KG: 8 for conv3 / conv4, 4 for conv12), 512 threads = PXL pixels x (512 / PXL) slices of the part's
// 9 x Cin / 4 products.  Eight output channels per lane reuse each staged input vector 8
// times (LDS traffic per multiply-add a quarter of the 2-channel form's), and the quarter's
// input (H * H x Cin / 4) and weights (8 x 9 x Cin / 4) are a quarter of the plane.  The four
// quarters' partial sums meet in a workspace: each block publishes its [leaf][pixel][8] partials
// (write-through stores, drained, then one relaxed atomic ticket per co group) and the LAST of the
// four blocks to arrive sums them in quarter order 0..3 (deterministic whatever the arrival order),
// adds the bias, applies ReLU, writes the output and resets the ticket for the next launch.  No
// block waits on another.
// KG = SK_KG = 8 K-parts for conv3 / conv4 (staged input eighth + weights + slice partials, n <= 8,
// Cin = 512: <= 52 KB, two blocks per CU) and SK_KG1 = 4 for conv12, whose conv1 registers
// allow one 512-thread block per CU (<= 87 KB; 8 parts at two blocks per CU spill 258 VGPRs)
// (4 / 8 / 16 K-parts for conv3 at one leaf: 16.2 / 14.3 / 19.0 us; 16 fit two blocks per CU for 1024
// blocks, two rounds; tools/small_layer_bench.py)
constexpr int SK_CO = 8, SK_KG = 8, SK_KG1 = 4;
__host__ __device__ constexpr size_t sk_lds(int kg) { return kg == SK_KG1 ? 96 * 1024 : 56 * 1024; }
__host__ __device__ constexpr int sk_wpf(int kg) { return kg == SK_KG1 ? 5 : 3; }  // 8 x 9 x 512 / kg / 4 / 512

// F1 > 0 (conv1 fused, conv2 only; F1 = the board side, 6..8): x is then the NCHW leaf planes
// [B][D][F1][F1] (sB per leaf) and the staged quarter is conv1's output for that quarter's
// channels, relu(b1 + conv1(planes)) with w1 [Cin][3][3][D] (channels_last, BN folded) --
// computed by the block's first Cq / 64 waves, one channel per lane and the leaf's planes read as
// wave-uniform scalars (conv1_sparse, azg_conv1.h: constant planes one multiply-add per output,
// 0/1 planes only their nonzero cells), instead of a launch of its own, while the other waves
// stage the block's weight quarter (azg_small_conv12's LDS bound keeps Cq <= 188: at least five
// staging waves).
// The block's weight quarter is loaded into registers first (SC_WPF float4 per thread) and
// written to LDS once the leaf's input loads are in flight: one memory round trip for both.
template <int PXL, int F1, int KG, bool COH = false>
__device__ __forceinline__ void small_conv_sk_body(int bid, int nblk, float* __restrict__ lds, unsigned& s_last,
                                                   const float* __restrict__ x, long long sB, int sY, int sX, int B,
                                                   int H, int pad, const float* __restrict__ w, int Cin,
                                                   const float* __restrict__ bias, int relu, float* __restrict__ y,
                                                   int ldy, float* __restrict__ part, unsigned* __restrict__ ticket,
                                                   const float* __restrict__ w1, const float* __restrict__ b1, int D) {
    constexpr int KSL = SC_T / PXL;
    constexpr int SC_WPF = sk_wpf(KG);
    SK_STAMP(0);
    const int tid = threadIdx.x;
    const int p = tid % PXL, s = tid / PXL;
    const int cg = bid / KG, kg = bid % KG;
    const int co0 = cg * SK_CO;
    const int Cq = Cin / KG, ci_base = kg * Cq;
    const int Ho = H + 2 * pad - 2, hw = Ho * Ho;
    const int P = Cq + 4;                       // LDS pitch of a staged pixel
    const int Kq = 9 * Cq;                      // this quarter's products per output
    float* xs = lds;                            // [H * H][P]
    // the quarter's weights w[co0 + c][tap][ci_base + ci], k = tap * Cq + ci:
    //  * CM (conv3 / conv4): channel-major, ws[c * Kq + k] -- float4 i of the slice at ws[4 i], one
    //    conflict-free ds_write_b128 each (the k-major layout's four strided ds_write_b32 per float4
    //    conflict 32 ways: staging 8.6 -> 2.6 us per block at one leaf, tools/sk_stamps.py);
    //  * conv12 (F1 > 0): k-major, ws[k * 8 + c], the 8 channels of a k adjacent (its weights are staged
    //    under conv1's arithmetic; channel-major measured slower there, 7.0 -> 9.0 us of products)
    constexpr bool CM = F1 == 0;
    float* ws = xs + H * H * P;                 // [SK_CO][Kq] (CM) or [Kq][SK_CO]
    float* red = ws + Kq * SK_CO;               // [KSL][PXL][SK_CO]
    const int q4 = Cq / 4, nw4 = SK_CO * 9 * q4;
    // float4 i of the slice: channel c = i / (9 q4), then (tap, ci), so that (CM) ws[4 i] is its place
    // (conv12's staging is bound by conv1's arithmetic, not by its strided stores: c fastest, 4-way
    // instead of 32-way conflicts, left its 8.0 us unchanged, tools/sk_stamps.py)
    auto wcoord = [&](int i, int& c, int& tap, int& ci) {
        c = i / (9 * q4);
        const int r = i - c * 9 * q4;
        tap = r / q4, ci = (r - tap * q4) * 4;
    };
    auto wload = [&](int i) {
        int c, tap, ci;
        wcoord(i, c, tap, ci);
        return *(const float4*)(w + ((long long)(co0 + c) * 9 + tap) * Cin + ci_base + ci);
    };
    auto wstore = [&](int i, float4 v) {
        if constexpr (CM) {
            *(float4*)(ws + 4 * i) = v;
        } else {
            int c, tap, ci;
            wcoord(i, c, tap, ci);
            float* d = ws + (tap * Cq + ci) * SK_CO + c;
            d[0] = v.x;
            d[SK_CO] = v.y;
            d[2 * SK_CO] = v.z;
            d[3 * SK_CO] = v.w;
        }
    };
    float4 wpf[F1 > 0 ? 1 : SC_WPF];  // (conv12: the waves that compute no conv1 stage the weights)
    if constexpr (F1 == 0) {
#pragma unroll
        for (int u = 0; u < SC_WPF; ++u) {
            const int i = tid + u * SC_T;
            if (i < nw4) wpf[u] = wload(i);
        }
    }
    bool w_staged = F1 > 0;
    auto stage_w = [&]() {  // (block-uniform)
        if (w_staged) return;
#pragma unroll
        for (int u = 0; u < SC_WPF; ++u) {
            const int i = tid + u * SC_T;
            if (i < nw4) wstore(i, wpf[u]);
        }
        for (int i = tid + SC_WPF * SC_T; i < nw4; i += SC_T) wstore(i, wload(i));
        w_staged = true;
    };
    int oy = 0, ox = 0;
    if (p < hw) oy = p / Ho, ox = p - (p / Ho) * Ho;
    const int KS = Kq / 4;  // float4 steps
    const int per = (KS + KSL - 1) / KSL;
    const int k0 = s * per, k1 = min(KS, k0 + per);
    for (int b = 0; b < B; ++b) {
        if constexpr (F1 > 0) {
            constexpr int NN = F1 * F1;
            const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
            const unsigned lane = tid & 63;
            const int nconv = (Cq + 63) / 64;  // conv1 waves; the others stage the weights (first leaf)
            if (wv < nconv) {
                const int c = min(wv * 64 + (int)lane, Cq - 1);  // (lanes past the quarter: a duplicate, not stored)
                float acc1[NN];
                conv1_sparse<F1>(x + b * sB, w1 + (long long)(ci_base + c) * 9 * D, D, lane, acc1, 1, D);
                const float bc = b1[ci_base + c];
                if (wv * 64 + (int)lane < Cq) {
#pragma unroll
                    for (int q = 0; q < NN; ++q) xs[q * P + c] = fmaxf(acc1[q] + bc, 0.f);
                }
            } else if (b == 0) {
                constexpr int U = 6;
                const int t0 = tid - nconv * 64, nst = SC_T - nconv * 64;
                for (int i0 = t0; i0 < nw4; i0 += nst * U) {
                    float4 r[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) r[u] = wload(min(i0 + u * nst, nw4 - 1));
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        if (i0 + u * nst < nw4) wstore(i0 + u * nst, r[u]);
                }
            }
        }
        const float* __restrict__ xb = x + b * sB + ci_base;
        const int c4 = Cq / 4, n4 = F1 > 0 ? 0 : H * H * c4;
        // input loads in flight per thread: 4 (a one-leaf eighth of conv3's input is 784 float4, two per
        // thread; 16 in flight cost 64 VGPRs and spilled under the two-blocks-per-CU bound)
        constexpr int UNR = 4;
        for (int base = tid; base < n4; base += SC_T * UNR) {
            const int rem = n4 - (base - tid);  // (block-uniform: no load past the block's last float4)
            float4 r[UNR];
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                if (u * SC_T >= rem) break;
                const int i = min(base + u * SC_T, n4 - 1);
                const int pix = i / c4, c = (i - pix * c4) * 4, iy = pix / H, ix = pix - iy * H;
                r[u] = ld4<COH>(xb, (long long)iy * sY + (long long)ix * sX + c);
            }
            stage_w();  // the weights' stores once the first input loads are in flight
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                const int i = base + u * SC_T;
                if (i < n4) {
                    const int pix = i / c4, c = (i - pix * c4) * 4;
                    *(float4*)(xs + pix * P + c) = r[u];
                }
            }
        }
        stage_w();
        __syncthreads();
        SK_STAMP(1);
        float acc[SK_CO];
#pragma unroll
        for (int c = 0; c < SK_CO; ++c) acc[c] = 0.f;
        if (p < hw) {
            int kk = k0;
            while (kk < k1) {  // k = tap * Cq + ci: a slice is a few runs of one tap each
                const int k = kk * 4;
                const int tap = k / Cq, ci0 = k - tap * Cq;
                const int run = min(k1 - kk, (Cq - ci0) / 4);
                const int iy = oy + tap / 3 - pad, ix = ox + tap % 3 - pad;
                if (iy >= 0 && iy < H && ix >= 0 && ix < H) {
                    const float* xp = xs + (iy * H + ix) * P + ci0;
                    if constexpr (CM) {
                        const float* wp = ws + k;
#pragma unroll 2
                        for (int j = 0; j < run; ++j) {
                            const float4 xv = *(const float4*)(xp + 4 * j);
#pragma unroll
                            for (int c = 0; c < SK_CO; ++c) {  // per channel its four k in order
                                const float4 wv = *(const float4*)(wp + c * Kq + 4 * j);
                                acc[c] = fmaf(wv.x, xv.x, acc[c]);
                                acc[c] = fmaf(wv.y, xv.y, acc[c]);
                                acc[c] = fmaf(wv.z, xv.z, acc[c]);
                                acc[c] = fmaf(wv.w, xv.w, acc[c]);
                            }
                        }
                    } else {
                        const float* wp = ws + k * SK_CO;
#pragma unroll 2
                        for (int j = 0; j < run; ++j) {
                            const float4 xv = *(const float4*)(xp + 4 * j);
                            const float xs4[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
                            for (int e = 0; e < 4; ++e) {
                                const float4 wa = *(const float4*)(wp + (4 * j + e) * SK_CO);
                                const float4 wb = *(const float4*)(wp + (4 * j + e) * SK_CO + 4);
                                acc[0] = fmaf(wa.x, xs4[e], acc[0]);
                                acc[1] = fmaf(wa.y, xs4[e], acc[1]);
                                acc[2] = fmaf(wa.z, xs4[e], acc[2]);
                                acc[3] = fmaf(wa.w, xs4[e], acc[3]);
                                acc[4] = fmaf(wb.x, xs4[e], acc[4]);
                                acc[5] = fmaf(wb.y, xs4[e], acc[5]);
                                acc[6] = fmaf(wb.z, xs4[e], acc[6]);
                                acc[7] = fmaf(wb.w, xs4[e], acc[7]);
                            }
                        }
                    }
                }
                kk += run;
            }
        }
        float4* r4 = (float4*)(red + (s * PXL + p) * SK_CO);
        r4[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
        r4[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
        __syncthreads();
        SK_STAMP(2);
        // the block's partial for leaf b, slices summed in order -> part[kg][b][pixel][8]
        for (int t = tid; t < hw * SK_CO; t += SC_T) {
            const int pp = t / SK_CO, c = t - pp * SK_CO;
            float sum = 0.f;
            for (int q = 0; q < KSL; ++q) sum += red[(q * PXL + pp) * SK_CO + c];
            // write-through (sc1) stores: published by the drain below, no release fence
            __hip_atomic_store((unsigned*)(part + (((long long)kg * (nblk / KG) + cg) * B + b) * hw * SK_CO + t),
                               __float_as_uint(sum), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();  // xs and red are rewritten for the next leaf
    }
    // publish (MI355X hand-off, cdna_hip_programming.md Guideline 16 R1): every wave drains its
    // write-through partial stores, then one relaxed ticket per block; the last of the co group's
    // KG blocks combines the quarters in order, reading them with sc1 loads only (no fences:
    // a __threadfence by every wave of every block -- an L2 write-back and invalidate each --
    // held these kernels at 64-91 us per leaf, the drop-in call at 6.7 ms instead of 2.7)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    SK_STAMP(3);
    if (tid == 0)
        s_last = __hip_atomic_fetch_add(ticket + cg, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == KG - 1;
    __syncthreads();
    SK_STAMP(4);
    if (!s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (compiler order only: every load below is sc1)
    const int G = nblk / KG;
    for (int t = tid; t < B * hw * SK_CO; t += SC_T) {
        const int c = t % SK_CO, bp = t / SK_CO;  // bp = b * hw + pixel
        float sum = 0.f;
#pragma unroll
        for (int q = 0; q < KG; ++q) {  // coherent (agent-scope) loads: other CUs wrote them
            const unsigned u = __hip_atomic_load((const unsigned*)(part + (((long long)q * G + cg) * B) * hw * SK_CO + t),
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sum += __uint_as_float(u);
        }
        float o = sum + (bias ? bias[co0 + c] : 0.f);
        if (relu) o = fmaxf(o, 0.f);
        st1<COH>(y + (long long)bp * ldy + co0 + c, o);
    }
    // every block of the group has arrived: ready for the next launch (or the fused forward's next layer)
    if (tid == 0) __hip_atomic_store(ticket + cg, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    SK_STAMP(5);
}

// conv3 / conv4 (F1 == 0): two 512-thread blocks per CU (4 waves per SIMD, <= 128 VGPRs) so that all
// 512 blocks of a layer are resident at once -- at 167 VGPRs the second half started only as the first
// finished (11 us of start spread, tools/sk_stamps.py); conv12 (F1 > 0, 96 KB of LDS) is one block per CU
template <int PXL, int F1, int KG>
__global__ __launch_bounds__(SC_T) __attribute__((amdgpu_waves_per_eu(F1 > 0 ? 1 : 4)))
void small_conv_sk_kernel(const float* __restrict__ x, long long sB, int sY,
                                                             int sX, int B, int H, int pad,
                                                             const float* __restrict__ w, int Cin,
                                                             const float* __restrict__ bias, int relu,
                                                             float* __restrict__ y, int ldy,
                                                             float* __restrict__ part, unsigned* __restrict__ ticket,
                                                             const float* __restrict__ w1, const float* __restrict__ b1,
                                                             int D) {
    __shared__ __attribute__((aligned(16))) float lds[sk_lds(KG) / 4];
    __shared__ unsigned s_last;
    small_conv_sk_body<PXL, F1, KG>(blockIdx.x, gridDim.x, lds, s_last, x, sB, sY, sX, B, H, pad, w, Cin, bias, relu,
                                    y, ldy, part, ticket, w1, b1, D);
}

// HEADS ([fc3 | fc4] + the heads, InflexionNNet.py:51-54 and NNet.py:94): y receives the
// logits (no bias); each block then takes a ticket, and the last of the grid's blocks reads all
// rows back (agent-scope loads) and writes P = softmax(hb[:A] + y[:A]) and v = tanh(hb[A] + y[A])
// per leaf -- the arithmetic of azg_policy_value, one wave per leaf -- and resets the ticket.
// tid: the thread's index in the (virtual) block of SF_T threads; valid = false: a block half with no
// row group in this round (the fused kernel runs two groups per 512-thread block) -- it computes and
// stores nothing, takes no ticket, but meets every barrier of the block
template <int NPB, int BMAX, bool HEADS, bool COH = false>
__device__ __forceinline__ void small_fc_body(int bid, int nblk, int tid, bool valid, float (*red)[NPB * BMAX],
                                              unsigned& s_last, const float* __restrict__ x, int ldx, int B,
                                              const float* __restrict__ w, int K, int N,
                                              const float* __restrict__ bias, int relu, float* __restrict__ y,
                                              int ldy, const float* __restrict__ hb, float* __restrict__ P,
                                              float* __restrict__ V, unsigned* __restrict__ ticket) {
    constexpr int T = SF_T;
    const int lane = tid & 63, wv = tid >> 6;
    const int n0 = bid * NPB;
    const int K4 = K / 4;
    float acc[NPB][BMAX];
#pragma unroll
    for (int r = 0; r < NPB; ++r)
#pragma unroll
        for (int b = 0; b < BMAX; ++b) acc[r][b] = 0.f;
#pragma unroll 8
    for (int k4 = tid; k4 < (valid ? K4 : 0); k4 += T) {
        float4 xv[BMAX];
#pragma unroll
        for (int b = 0; b < BMAX; ++b)
            xv[b] = b < B ? ld4<COH>(x + (long long)b * ldx, 4 * k4) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int r = 0; r < NPB; ++r) {
            if (n0 + r >= N) break;
            const float4 wr = *(const float4*)(w + (long long)(n0 + r) * K + 4 * k4);
#pragma unroll
            for (int b = 0; b < BMAX; ++b) {
                float a = acc[r][b];
                a = fmaf(wr.x, xv[b].x, a);
                a = fmaf(wr.y, xv[b].y, a);
                a = fmaf(wr.z, xv[b].z, a);
                a = fmaf(wr.w, xv[b].w, a);
                acc[r][b] = a;
            }
        }
    }
    // wave butterfly, then the 4 waves' sums in wave order (fixed: deterministic)
#pragma unroll
    for (int r = 0; r < NPB; ++r)
#pragma unroll
        for (int b = 0; b < BMAX; ++b) {
            float v = acc[r][b];
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
            if (lane == 0) red[wv][r * BMAX + b] = v;
        }
    __syncthreads();
    if (tid < NPB * BMAX && valid) {
        const int r = tid / BMAX, b = tid - r * BMAX;
        if (n0 + r < N && b < B) {
            float sum = 0.f;
#pragma unroll
            for (int q = 0; q < T / 64; ++q) sum += red[q][tid];
            float o = sum + (bias ? bias[n0 + r] : 0.f);
            if (relu) o = fmaxf(o, 0.f);
            if constexpr (HEADS)  // write-through (sc1): read back by the grid's last block
                __hip_atomic_store((unsigned*)(y + (long long)b * ldy + n0 + r), __float_as_uint(o), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            else
                st1<COH>(y + (long long)b * ldy + n0 + r, o);
        }
    }
    if constexpr (COH && !HEADS) __syncthreads();  // red is rewritten by the block's next row group
    if constexpr (HEADS) {
        // publish as small_conv_sk_kernel does: drain, one relaxed ticket, sc1 loads in the last block
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0)
            s_last = valid && __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                                  (unsigned)nblk - 1;
        __syncthreads();
        if (!s_last) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (compiler order only: the loads are sc1)
        const int A = N - 1;
        if (wv < B) {  // one wave per leaf
            const float* yr = y + (long long)wv * ldy;
            auto ld = [&](int a) {
                return __uint_as_float(__hip_atomic_load((const unsigned*)(yr + a), __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT));
            };
            constexpr int PL = 16;  // up to 1024 actions
            float xa[PL];
            float mx = -INFINITY;
#pragma unroll
            for (int j = 0; j < PL; ++j) {
                const int a = lane + 64 * j;
                xa[j] = a < A ? hb[a] + ld(a) : -INFINITY;
                mx = fmaxf(mx, xa[j]);
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
            // exp(log_softmax) in the reference's order (azg_heads.hip policy_value_kernel)
            float sm = 0.f;
#pragma unroll
            for (int j = 0; j < PL; ++j) {
                xa[j] -= mx;
                sm += lane + 64 * j < A ? expf(xa[j]) : 0.f;
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) sm += __shfl_xor(sm, o);
            const float ls = logf(sm);
#pragma unroll
            for (int j = 0; j < PL; ++j) {
                const int a = lane + 64 * j;
                if (a < A) P[(long long)wv * A + a] = expf(xa[j] - ls);
            }
            if (lane == 0) V[wv] = tanhf(hb[A] + ld(A));
        }
        if (tid == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <int NPB, int BMAX, bool HEADS>
__global__ __launch_bounds__(SF_T) void small_fc_kernel(const float* __restrict__ x, int ldx, int B,
                                                        const float* __restrict__ w, int K, int N,
                                                        const float* __restrict__ bias, int relu,
                                                        float* __restrict__ y, int ldy, const float* __restrict__ hb,
                                                        float* __restrict__ P, float* __restrict__ V,
                                                        unsigned* __restrict__ ticket) {
    __shared__ float red[SF_T / 64][NPB * BMAX];
    __shared__ unsigned s_last;
    small_fc_body<NPB, BMAX, HEADS>(blockIdx.x, gridDim.x, threadIdx.x, true, red, s_last, x, ldx, B, w, K, N, bias,
                                    relu, y, ldy, hb, P, V, ticket);
}

#ifdef AZG_SMALL_PROBES  // the one-launch form: probe build only (tools/Makefile libazg_small_probes.so)
// ---- the whole forward in one launch (small_net_kernel) ---------------------------------------
// conv1 + conv2 (split-K, 4 K-parts), conv3 (split-K, 8 K-parts), conv4 (2-channel blocks), fc1, fc2,
// [fc3 | fc4] + heads: the same block bodies as the per-layer kernels above (same arithmetic, same
// summation orders: bit-identical results), in one grid of at most one 512-thread block per CU.
//
// The layers' block bodies are ITEMS of one in-order work queue (layer 0's items first, then layer
// 1's, ...): a block takes the next item with one atomic, and before an item of layer L it waits
// until every item of layer L-1 is done (a per-layer done counter).  An item is handed out only
// after every item of the layers before it, to a block that is already running, and the items a
// block waits for were all handed out earlier -- so the launch completes whatever number of its
// blocks is resident at once (a GPU shared with another process, or other kernels in flight): no
// grid barrier, which a persistent grid can only pass when all of its blocks are co-resident (two
// processes' launches each holding part of the CUs timed out before, tests/test_gpu_dist.py).
// Activations cross the layers as write-through stores drained before the done count and agent-scope
// loads after the wait (the split-K hand-off's rule).  Each block prefetches its next item while it
// works on the current one; the last block to leave resets the counters for the next launch.  A wait
// gives up after ~2^24 polls (setting *err) rather than hang.
struct SmallNetArgs {
    const float* planes;
    const float *w1, *b1, *w2, *b2, *w3, *b3, *w4, *b4, *fw1, *fb1, *fw2, *fb2, *fw34, *fb34;
    float *y2, *y3, *y4, *h1, *h2, *logits, *P, *v;
    float* part;
    unsigned* tickets;
    unsigned* heads_ticket;
    unsigned* sched;  // [0] next item, [1] blocks finished, [2 + L] items of layer L done (L < 5)
    int* err;
    int B, D, C, A, N1, N2;
};

constexpr int SN_POOL = 96 * 1024;  // LDS of the fused kernel: the largest layer's (conv1 + conv2's split-K block)
constexpr int SN_SCHED_WORDS = 8;

template <int NB, int BMAX, bool WLDS3, bool WLDS4>
__global__ __launch_bounds__(SC_T) void small_net_kernel(SmallNetArgs a) {
    __shared__ __attribute__((aligned(16))) float pool[SN_POOL / 4];
    __shared__ unsigned s_last;
    __shared__ unsigned s_half[2];
    __shared__ int s_next;
    constexpr int H3 = NB - 2, H4 = NB - 4;  // conv3's and conv4's output sides (pads 1, 1, 0, 0)
    constexpr int P12 = NB * NB <= 64 ? 64 : 128, P3 = H3 * H3 <= 16 ? 16 : H3 * H3 <= 32 ? 32 : 64,
                  P4 = H4 * H4 <= 16 ? 16 : 32;
    const int C = a.C, B = a.B, tid = threadIdx.x;
    const int K1 = H4 * H4 * C, half = tid / SF_T, ht = tid % SF_T;
    // items per layer: conv12 split-K blocks; conv3 split-K blocks (or 2-channel blocks for <= 16
    // output pixels, 6x6 boards); conv4 2-channel blocks; fc1 / fc2 / heads row-group pairs (one group
    // per 256-thread half, each exactly the per-layer small_fc_kernel's block)
    const int nsk = C / SK_CO * SK_KG1;
    const int n3 = H3 * H3 > 16 ? C / SK_CO * SK_KG : C / 2;
    const int npb1 = a.N1 >= 2048 ? 4 : a.N1 >= 1024 ? 2 : 1, npb2 = a.N2 >= 2048 ? 4 : a.N2 >= 1024 ? 2 : 1;
    const int ng1 = (a.N1 + npb1 - 1) / npb1, ng2 = (a.N2 + npb2 - 1) / npb2, ng3 = (a.A + 1 + 3) / 4;
    // (scalars, not arrays: a dynamically indexed local array lives in scratch memory)
    const int e0 = nsk, e1 = e0 + n3, e2 = e1 + C / 2, e3 = e2 + (ng1 + 1) / 2, e4 = e3 + (ng2 + 1) / 2,
              e5 = e4 + (ng3 + 1) / 2;
    unsigned* q = a.sched;

    auto fc = [&](auto NPB_, auto HEADS_, int g0, int nrow, const float* x, int ldx, const float* w, int K,
                  const float* bias, int relu, float* y, int ldy, const float* hb, float* P, float* V,
                  unsigned* ticket) {
        constexpr int NPB = decltype(NPB_)::value;
        constexpr bool HD = decltype(HEADS_)::value;
        const int ng = (nrow + NPB - 1) / NPB;
        float(*red)[NPB * BMAX] = (float(*)[NPB * BMAX])(pool + half * (SF_T / 64) * NPB * BMAX);
        small_fc_body<NPB, BMAX, HD, true>(g0 + half, ng, ht, g0 + half < ng, red, s_half[half], x, ldx, B, w, K,
                                           nrow, bias, relu, y, ldy, hb, P, V, ticket);
    };

    // One loop per layer, in layer order (the queue's order): a block runs the items it takes while
    // they belong to layer L, and carries the first item past it to the next layer's loop.  The layers'
    // code sits in separate loops, so their hoisted invariants are live in their own loop only (one
    // loop with a switch over the six bodies spilled 464 B per thread).
    if (tid == 0) s_next = (int)__hip_atomic_fetch_add(q, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    int item = s_next;
    // wait until layer L-1's `target` items are done (and so every layer before it: its items waited in turn)
    auto wait_layer = [&](int L, int target) {
        if (tid == 0) {
            // polls back off (64 .. 512 clocks apart): up to 256 blocks poll one counter, and the blocks
            // still working on layer L-1 increment it through the same memory channel
            for (unsigned spins = 0;
                 __hip_atomic_load(q + 2 + (L - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)target;) {
                if (spins < 4) __builtin_amdgcn_s_sleep(1);
                else if (spins < 16) __builtin_amdgcn_s_sleep(4);
                else __builtin_amdgcn_s_sleep(8);
                if (++spins > (1u << 22)) {  // an item never finished: report instead of hanging the GPU
                    atomicOr(a.err, 1);
                    break;
                }
            }
        }
        __syncthreads();
    };
    // run the items of layer L in [lo, hi): body(i) per item, each counted done after its stores landed
    auto layer = [&](int L, int lo, int hi, auto&& body) {
        if (item >= hi) return;
        if (L > 0) wait_layer(L, lo - (L == 1 ? 0 : L == 2 ? e0 : L == 3 ? e1 : L == 4 ? e2 : e3));
        while (item < hi) {
            unsigned nxt = 0;  // the next item, fetched while this one runs (thread 0)
            if (tid == 0) nxt = __hip_atomic_fetch_add(q, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            body(item - lo);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this item's write-through stores have landed
            __syncthreads();
            if (tid == 0) {
                if (L < 5) __hip_atomic_fetch_add(q + 2 + L, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                s_next = (int)nxt;
            }
            __syncthreads();
            item = s_next;
            __syncthreads();  // every thread has read s_next before thread 0 writes it again
        }
    };
    layer(0, 0, e0, [&](int i) {
        small_conv_sk_body<P12, NB, SK_KG1, true>(i, nsk, pool, s_last, a.planes, (long long)a.D * NB * NB, 0, 0, B,
                                                  NB, 1, a.w2, C, a.b2, 1, a.y2, C, a.part, a.tickets, a.w1, a.b1,
                                                  a.D);
    });
    layer(1, e0, e1, [&](int i) {
        if constexpr (H3 * H3 > 16)  // conv3 as the per-layer path runs it: split-K in 8 K-parts ...
            small_conv_sk_body<P3, 0, SK_KG, true>(i, n3, pool, s_last, a.y2, (long long)NB * NB * C, NB * C, C, B,
                                                   NB, 0, a.w3, C, a.b3, 1, a.y3, C, a.part, a.tickets, nullptr,
                                                   nullptr, 0);
        else  // ... or, for <= 16 output pixels (6x6 boards), in 2-channel blocks
            small_conv_body<P3, 2, true, WLDS3, true>(i, pool, a.y2, (long long)NB * NB * C, NB * C, C, 1, B, NB, 0,
                                                      a.w3, C, C, a.b3, 1, a.y3, C);
    });
    layer(2, e1, e2, [&](int i) {
        small_conv_body<P4, 2, true, WLDS4, true>(i, pool, a.y3, (long long)H3 * H3 * C, H3 * C, C, 1, B, H3, 0, a.w4,
                                                  C, C, a.b4, 1, a.y4, C);
    });
    layer(3, e2, e3, [&](int i) {
        if (npb1 == 4) fc(std::integral_constant<int, 4>{}, std::false_type{}, 2 * i, a.N1, a.y4, K1, a.fw1, K1, a.fb1,
                          1, a.h1, a.N1, nullptr, nullptr, nullptr, nullptr);
        else if (npb1 == 2) fc(std::integral_constant<int, 2>{}, std::false_type{}, 2 * i, a.N1, a.y4, K1, a.fw1, K1,
                               a.fb1, 1, a.h1, a.N1, nullptr, nullptr, nullptr, nullptr);
        else fc(std::integral_constant<int, 1>{}, std::false_type{}, 2 * i, a.N1, a.y4, K1, a.fw1, K1, a.fb1, 1, a.h1,
                a.N1, nullptr, nullptr, nullptr, nullptr);
    });
    layer(4, e3, e4, [&](int i) {
        if (npb2 == 4) fc(std::integral_constant<int, 4>{}, std::false_type{}, 2 * i, a.N2, a.h1, a.N1, a.fw2, a.N1,
                          a.fb2, 1, a.h2, a.N2, nullptr, nullptr, nullptr, nullptr);
        else if (npb2 == 2) fc(std::integral_constant<int, 2>{}, std::false_type{}, 2 * i, a.N2, a.h1, a.N1, a.fw2,
                               a.N1, a.fb2, 1, a.h2, a.N2, nullptr, nullptr, nullptr, nullptr);
        else fc(std::integral_constant<int, 1>{}, std::false_type{}, 2 * i, a.N2, a.h1, a.N1, a.fw2, a.N1, a.fb2, 1,
                a.h2, a.N2, nullptr, nullptr, nullptr, nullptr);
    });
    layer(5, e4, e5, [&](int i) {
        fc(std::integral_constant<int, 4>{}, std::true_type{}, 2 * i, a.A + 1, a.h2, a.N2, a.fw34, a.N2, nullptr, 0,
           a.logits, a.A + 1, a.fb34, a.P, a.v, a.heads_ticket);
    });
    // the last block to leave resets the queue for the next launch (every block has taken its last item)
    if (tid == 0 &&
        __hip_atomic_fetch_add(q + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1u)
        for (int w = 0; w < SN_SCHED_WORDS; ++w) __hip_atomic_store(q + w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

#endif  // AZG_SMALL_PROBES

template <int PXL, bool VEC>
int launch_conv(dim3 grid, hipStream_t st, const float* x, long long sB, int sY, int sX, int sC, int B, int H,
                int pad, const float* w, int Cin, int Cout, const float* bias, int relu, float* y, int ldy) {
    constexpr int CO_PB = 2;
    const size_t xs = (size_t)H * H * sc_pitch(Cin) * 4, red = (size_t)SC_T * CO_PB * 4, wb = (size_t)CO_PB * 9 * Cin * 4;
    if (xs + red > SC_LDS_MAX) return AZG_ERR_ARG;
    if (xs + red + wb <= SC_LDS_MAX && ((uintptr_t)w & 15) == 0 && Cin % 4 == 0)
        hipLaunchKernelGGL((small_conv_kernel<PXL, CO_PB, VEC, true>), grid, dim3(SC_T), 0, st, x, sB, sY, sX, sC, B,
                           H, pad, w, Cin, Cout, bias, relu, y, ldy);
    else
        hipLaunchKernelGGL((small_conv_kernel<PXL, CO_PB, VEC, false>), grid, dim3(SC_T), 0, st, x, sB, sY, sX, sC, B,
                           H, pad, w, Cin, Cout, bias, relu, y, ldy);
    return 0;
}

template <int PXL, int F1 = 0, int KG = SK_KG>
void launch_conv_sk(hipStream_t st, const float* x, long long sB, int sY, int sX, int B, int H, int pad,
                    const float* w, int Cin, int Cout, const float* bias, int relu, float* y, int ldy, float* work,
                    unsigned* tickets, const float* w1 = nullptr, const float* b1 = nullptr, int D = 0) {
    hipLaunchKernelGGL((small_conv_sk_kernel<PXL, F1, KG>), dim3((unsigned)(Cout / SK_CO * KG)), dim3(SC_T), 0, st, x,
                       sB, sY, sX, B, H, pad, w, Cin, bias, relu, y, ldy, work, tickets, w1, b1, D);
}

}  // namespace

extern "C" int azg_small_conv3x3(const float* x, int64_t sB, int32_t sY, int32_t sX, int32_t sC, int32_t batch,
                                 int32_t H, int32_t pad, const float* w, int32_t Cin, int32_t Cout,
                                 const float* bias, int32_t relu, float* y, int32_t ldy, float* work,
                                 int64_t work_floats, uint32_t* tickets, int32_t n_tickets, void* stream) {
    const int Ho = H + 2 * pad - 2;
    if (!x || !w || !y || batch <= 0 || batch > 4 || H <= 0 || H > 16 || Ho <= 0 || pad < 0 || pad > 1 || Cin <= 0 ||
        Cout <= 0 || Cout % 2 || ldy < Cout || Ho * Ho > 256 || sB < 0 || sY < 0 || sX < 0 || sC < 0)
        return AZG_ERR_ARG;
    // NHWC input with float4 along the channels (aligned rows), else element-wise staging
    const bool vec = sC == 1 && Cin % 4 == 0 && sX % 4 == 0 && sY % 4 == 0 && sB % 4 == 0 &&
                     ((uintptr_t)x & 15) == 0 && ((uintptr_t)w & 15) == 0;
    hipStream_t st = (hipStream_t)stream;
    const int n = Ho * Ho;  // output pixels of one leaf: the leaves run one after another
    // the split-K form (8 channels x a quarter of the input channels per block, quarters combined
    // by the last block of each group) when the workspace holds the partials and the tickets
    const long long need = (long long)SK_KG * Cout * batch * n;
    // (not for <= 16 output pixels, conv4: there the combine's round trips cost more than the
    // 2-channel form's longer K loop, 13.0-13.3 vs 11.4-11.9 us at one leaf, tools/small_layer_bench.py)
    const bool sk = n > 16 && vec && Cin % (4 * SK_KG) == 0 && Cout % SK_CO == 0 && work && tickets &&
                    work_floats >= need && n_tickets >= Cout / SK_CO && ((uintptr_t)work & 15) == 0 &&
                    (size_t)H * H * (Cin / SK_KG + 4) * 4 + (size_t)9 * Cin / SK_KG * SK_CO * 4 +
                            (size_t)SC_T * SK_CO * 4 <= sk_lds(SK_KG);
    if (sk) {
        if (n <= 16) launch_conv_sk<16>(st, x, sB, sY, sX, batch, H, pad, w, Cin, Cout, bias, relu, y, ldy, work, tickets);
        else if (n <= 32) launch_conv_sk<32>(st, x, sB, sY, sX, batch, H, pad, w, Cin, Cout, bias, relu, y, ldy, work, tickets);
        else if (n <= 64) launch_conv_sk<64>(st, x, sB, sY, sX, batch, H, pad, w, Cin, Cout, bias, relu, y, ldy, work, tickets);
        else if (n <= 128) launch_conv_sk<128>(st, x, sB, sY, sX, batch, H, pad, w, Cin, Cout, bias, relu, y, ldy, work, tickets);
        else launch_conv_sk<256>(st, x, sB, sY, sX, batch, H, pad, w, Cin, Cout, bias, relu, y, ldy, work, tickets);
        return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
    }
    const dim3 grid((unsigned)(Cout / 2));
    int rc = 0;
    auto go = [&](auto V_) {
        constexpr bool V = decltype(V_)::value;
        if (n <= 16) rc = launch_conv<16, V>(grid, st, x, sB, sY, sX, sC, batch, H, pad, w, Cin, Cout, bias, relu, y, ldy);
        else if (n <= 32) rc = launch_conv<32, V>(grid, st, x, sB, sY, sX, sC, batch, H, pad, w, Cin, Cout, bias, relu, y, ldy);
        else if (n <= 64) rc = launch_conv<64, V>(grid, st, x, sB, sY, sX, sC, batch, H, pad, w, Cin, Cout, bias, relu, y, ldy);
        else if (n <= 128) rc = launch_conv<128, V>(grid, st, x, sB, sY, sX, sC, batch, H, pad, w, Cin, Cout, bias, relu, y, ldy);
        else rc = launch_conv<256, V>(grid, st, x, sB, sY, sX, sC, batch, H, pad, w, Cin, Cout, bias, relu, y, ldy);
    };
    if (vec) go(std::true_type{});
    else go(std::false_type{});
    if (rc) return rc;
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_small_conv12(const float* planes, int32_t batch, int32_t depth, int32_t n, const float* w1,
                                const float* b1, const float* w2, const float* b2, int32_t C, float* y, int32_t ldy,
                                float* work, int64_t work_floats, uint32_t* tickets, int32_t n_tickets, void* stream) {
    const int hw = n * n;
    if (!planes || !w1 || !b1 || !w2 || !y || !work || !tickets || batch <= 0 || batch > 4 || depth < 1 || depth > 4 ||
        n < 6 || n > 8 || C <= 0 || C % (4 * SK_KG1) || C % SK_CO || ldy < C ||
        work_floats < (long long)SK_KG1 * C * batch * hw || n_tickets < C / SK_CO || ((uintptr_t)w2 & 15) ||
        ((uintptr_t)work & 15) ||
        (size_t)hw * (C / SK_KG1 + 4) * 4 + (size_t)9 * C / SK_KG1 * SK_CO * 4 + (size_t)SC_T * SK_CO * 4 >
            sk_lds(SK_KG1))
        return AZG_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    const long long sB = (long long)depth * hw;
    auto go = [&](auto N_) {
        launch_conv_sk<64, decltype(N_)::value, SK_KG1>(st, planes, sB, 0, 0, batch, n, 1, w2, C, C, b2, 1, y, ldy,
                                                        work, tickets, w1, b1, depth);
    };
    switch (n) {  // the boards' sides: conv1's output plane in registers (conv1_sparse)
        case 6: go(std::integral_constant<int, 6>{}); break;
        case 7: go(std::integral_constant<int, 7>{}); break;
        case 8: go(std::integral_constant<int, 8>{}); break;
        default: return AZG_ERR_ARG;
    }
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_small_fc(const float* x, int32_t ldx, int32_t batch, const float* w, int32_t K, int32_t N,
                            const float* bias, int32_t relu, float* y, int32_t ldy, void* stream) {
    if (!x || !w || !y || batch <= 0 || batch > 4 || K <= 0 || K % 4 || N <= 0 || ldx % 4 || ldx < K ||
        ldy < N || ((uintptr_t)x & 15) || ((uintptr_t)w & 15))
        return AZG_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    // rows per block: at least ~512 blocks (two per CU), so a layer's weight stream is spread
    // over the whole chip (fc2's 512 rows were 128 blocks at 4 per block)
    auto go = [&](auto NPB_) {
        constexpr int NPB = decltype(NPB_)::value;
        const dim3 grid((unsigned)((N + NPB - 1) / NPB));
        if (batch == 1)
            hipLaunchKernelGGL((small_fc_kernel<NPB, 1, false>), grid, dim3(SF_T), 0, st, x, ldx, batch, w, K, N, bias,
                               relu, y, ldy, nullptr, nullptr, nullptr, nullptr);
        else
            hipLaunchKernelGGL((small_fc_kernel<NPB, 4, false>), grid, dim3(SF_T), 0, st, x, ldx, batch, w, K, N, bias,
                               relu, y, ldy, nullptr, nullptr, nullptr, nullptr);
    };
    if (N >= 2048) go(std::integral_constant<int, 4>{});
    else if (N >= 1024) go(std::integral_constant<int, 2>{});
    else go(std::integral_constant<int, 1>{});
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_small_heads(const float* x, int32_t ldx, int32_t batch, const float* w34, int32_t K, int32_t A,
                               const float* b34, float* logits, float* P, float* v, uint32_t* ticket, void* stream) {
    if (!x || !w34 || !b34 || !logits || !P || !v || !ticket || batch <= 0 || batch > 4 || K <= 0 || K % 4 ||
        A < 1 || A > 1023 || ldx % 4 || ldx < K || ((uintptr_t)x & 15) || ((uintptr_t)w34 & 15))
        return AZG_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    const int N = A + 1;
    // 4 rows per block: the last-arriver ticket is a fan-in over the grid, and one row per block
    // (344 arrivals instead of 86) measured 7.5 -> 9.7 us
    const dim3 grid((unsigned)((N + 3) / 4));
    if (batch == 1)
        hipLaunchKernelGGL((small_fc_kernel<4, 1, true>), grid, dim3(SF_T), 0, st, x, ldx, batch, w34, K, N, nullptr, 0,
                           logits, N, b34, P, v, ticket);
    else
        hipLaunchKernelGGL((small_fc_kernel<4, 4, true>), grid, dim3(SF_T), 0, st, x, ldx, batch, w34, K, N, nullptr, 0,
                           logits, N, b34, P, v, ticket);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

#ifdef AZG_SMALL_PROBES
// grid of azg_small_net (azg_small_net_blocks; 0: one block per CU)
static int g_small_net_blocks = 0;

extern "C" int azg_small_net_blocks(int32_t blocks) {
    if (blocks < 0) return AZG_ERR_ARG;
    g_small_net_blocks = blocks;
    return 0;
}

// The whole small-batch forward in one launch (small_net_kernel above).  w: 14 device pointers
// w1 b1 w2 b2 w3 b3 w4 b4 fw1 fb1 fw2 fb2 fw34 fb34 (BN folded, conv weights [co][3][3][ci] as the
// per-layer kernels take them, w1 [co][3][3][depth]); acts: the activations (y2 | y3 | y4 | h1 | h2 |
// logits, sized by the caller); sched: the work queue's SN_SCHED_WORDS u32 counters (zero before the
// first launch; every launch leaves them zero); err: set when a wait gave up (the caller zeroes sched then).
extern "C" int azg_small_net(const float* planes, int32_t batch, int32_t depth, int32_t n, int32_t C, int32_t A,
                             int32_t n1, int32_t n2, const float* const* w, float* acts, int64_t acts_floats, float* P,
                             float* v, float* work, int64_t work_floats, uint32_t* tickets, int32_t n_tickets,
                             uint32_t* sched, int32_t* err, void* stream) {
    if (!planes || !w || !acts || !P || !v || !work || !tickets || !sched || !err || batch <= 0 || batch > 4 ||
        depth < 1 || depth > 4 || n < 6 || n > 8 || C <= 0 || C % (4 * SK_KG1) || C % SK_CO || A < 1 || A > 1023 ||
        n1 <= 0 || n1 % 4 || n2 <= 0 || n2 % 4 || n_tickets < C / SK_CO + 1 || ((uintptr_t)work & 15) ||
        ((uintptr_t)acts & 15))
        return AZG_ERR_ARG;
    for (int i = 0; i < 14; ++i)
        if (!w[i] || ((uintptr_t)w[i] & 15)) return AZG_ERR_ARG;
    const int hw = n * n, h3 = n - 2, h4 = n - 4;
    const long long need_acts = (long long)batch * (hw * C + h3 * h3 * C + h4 * h4 * C + n1 + n2 + (A + 1));
    if (acts_floats < need_acts || work_floats < (long long)SK_KG1 * C * batch * hw) return AZG_ERR_ARG;
    // LDS: conv1 + conv2 and conv3 as split-K blocks, conv4 as 2-channel blocks (weights in LDS if they fit)
    const size_t sk12 = (size_t)hw * (C / SK_KG1 + 4) * 4 + (size_t)9 * C / SK_KG1 * SK_CO * 4 + (size_t)SC_T * SK_CO * 4;
    const size_t c3 = (size_t)hw * sc_pitch(C) * 4 + (size_t)SC_T * 2 * 4;  // conv3 in 2-channel blocks (6x6)
    const size_t c4 = (size_t)h3 * h3 * sc_pitch(C) * 4 + (size_t)SC_T * 2 * 4, w4b = (size_t)2 * 9 * C * 4;
    if (sk12 > SN_POOL || c4 > SN_POOL || (h3 * h3 <= 16 && c3 > SN_POOL)) return AZG_ERR_ARG;
    // conv3's split-K form (> 16 output pixels) as azg_small_conv3x3 takes it: C % (4 SK_KG), its LDS
    if (h3 * h3 > 16 && (C % (4 * SK_KG) || (size_t)hw * (C / SK_KG + 4) * 4 + (size_t)9 * C / SK_KG * SK_CO * 4 +
                                                     (size_t)SC_T * SK_CO * 4 > (size_t)SN_POOL))
        return AZG_ERR_ARG;
    const bool wlds3 = c3 + w4b <= SN_POOL, wlds4 = c4 + w4b <= SN_POOL;
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            return AZG_ERR_HIP;
    }
    SmallNetArgs a{};
    a.planes = planes;
    a.w1 = w[0], a.b1 = w[1], a.w2 = w[2], a.b2 = w[3], a.w3 = w[4], a.b3 = w[5], a.w4 = w[6], a.b4 = w[7];
    a.fw1 = w[8], a.fb1 = w[9], a.fw2 = w[10], a.fb2 = w[11], a.fw34 = w[12], a.fb34 = w[13];
    a.y2 = acts;
    a.y3 = a.y2 + (long long)batch * hw * C;
    a.y4 = a.y3 + (long long)batch * h3 * h3 * C;
    a.h1 = a.y4 + (long long)batch * h4 * h4 * C;
    a.h2 = a.h1 + (long long)batch * n1;
    a.logits = a.h2 + (long long)batch * n2;
    a.P = P, a.v = v, a.part = work, a.tickets = tickets, a.heads_ticket = tickets + C / SK_CO;
    a.sched = sched, a.err = err;
    a.B = batch, a.D = depth, a.C = C, a.A = A, a.N1 = n1, a.N2 = n2;
    const int blocks = g_small_net_blocks > 0 && g_small_net_blocks < cus ? g_small_net_blocks : cus;
    const dim3 grid((unsigned)blocks);
    hipStream_t st = (hipStream_t)stream;
    auto go = [&](auto N_, auto B_, auto W3_, auto W4_) {
        hipLaunchKernelGGL((small_net_kernel<decltype(N_)::value, decltype(B_)::value, decltype(W3_)::value,
                                             decltype(W4_)::value>),
                           grid, dim3(SC_T), 0, st, a);
    };
    auto by_w = [&](auto N_, auto B_) {  // (WLDS3 matters for 6x6 boards only)
        if (wlds3 && wlds4) go(N_, B_, std::true_type{}, std::true_type{});
        else if (wlds4) go(N_, B_, std::false_type{}, std::true_type{});
        else go(N_, B_, std::false_type{}, std::false_type{});
    };
    auto by_b = [&](auto N_) {
        if (batch == 1) by_w(N_, std::integral_constant<int, 1>{});
        else by_w(N_, std::integral_constant<int, 4>{});
    };
    switch (n) {
        case 6: by_b(std::integral_constant<int, 6>{}); break;
        case 7: by_b(std::integral_constant<int, 7>{}); break;
        default: by_b(std::integral_constant<int, 8>{}); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}
#endif  // AZG_SMALL_PROBES

#ifdef AZG_SMALL_TIMING
// the stamps of the last launch(es) and the wall clock's rate (kHz)
extern "C" int azg_sk_stamps_read(unsigned long long* out, int32_t n, int32_t* khz) {
    if (!out || n <= 0 || n > 1024 * 8 || !khz) return AZG_ERR_ARG;
    int dev = 0, rate = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, dev) != hipSuccess)
        return AZG_ERR_HIP;
    *khz = rate;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(azg_sk_stamps), (size_t)n * 8) == hipSuccess ? 0 : AZG_ERR_HIP;
}
#endif
