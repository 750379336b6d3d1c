// azg_small.hip -- the leaf network at a few leaves (C1: one game, one leaf per
// simulation; anything below the Winograd path's 64 leaves): conv1-4 (3x3, BN folded,
// bias + ReLU, InflexionNNet.py:39-45) and fc1 / fc2 / [fc3 | fc4] (:47-54) as one
// small f32 GEMM each,
//     out[px][co] = sum_k W[co][k] * X[k][px],   k = tap * Cin + ci,
// px = (leaf, y, x) output pixels (taps = 9; the FC layers are taps = 1, one pixel per
// leaf), W the folded weights as [co][ky][kx][ci] (a channels_last conv weight; an FC
// weight [co][ci]).  At one leaf a layer
// is 49 pixels x 512 channels x 4608 products (231 MFLOP) against 9.4 MB of weights: a
// weight stream, so the K dimension is what spreads it over the chip.
//
//  * small_gemm_partial: block (co tile of 128, px tile of 64, K-split z) accumulates its
//    K range slab by slab (kc <= 64 consecutive k of one tap, a power of two): the slab's
//    weights and the matching im2col values (zero padding, any input strides: NCHW leaf
//    planes or the NHWC activations this file writes) go through LDS, each thread keeps
//    4 x 4 outputs, f32 fmaf in k order.  Partial sums to part[z][px][co].
//  * small_gemm_reduce: out[px][co] = sum_z part[z][px][co] in z order, + bias, ReLU,
//    written NHWC (the next layer's input, or the FC rows).  Deterministic.
// Two launches per layer, no library: this path replaces MIOpen and hipBLASLt below
// the batched forward's sizes.
#include <hip/hip_runtime.h>

#include "../../include/azg.h"

namespace {

constexpr int SM_CO = 128;    // co tile (512 threads: 32 rows of 4 co)
constexpr int SM_T = 64;      // px tile (16 columns of 4 px)
constexpr int SM_KMAX = 64;   // slab of K in LDS (a power of two, within one tap)
constexpr int SM_PW = SM_CO + 4, SM_PX = SM_T + 4;  // LDS row pitches: 16-B aligned float4 reads
constexpr int SM_PERW = SM_CO * SM_KMAX / 512, SM_PERX = SM_T * SM_KMAX / 512;  // loads in flight per thread

// Block (co tile of 128, px tile of 64, K-split z), 512 threads of 4 x 4 outputs, over its
// slabs: each slab (KC = 2^kc_shift consecutive k of one tap, KC | Cin) is staged in two
// phases -- every thread issues all its weight and im2col loads into registers, then
// stores them to LDS -- and the next slab's loads are issued before this slab's
// multiply-adds (software pipeline); the pixel decomposition is computed once.
__global__ __launch_bounds__(512) void small_gemm_partial_kernel(const float* __restrict__ x, long long sB, int sY,
                                                                 int sX, int sC, int H, int W, int pad, int taps,
                                                                 int Ho, int Wo, int npx,
                                                                 const float* __restrict__ w, int Cin, int Cout,
                                                                 int kc_shift, int slabs_per_split,
                                                                 float* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) float sw[SM_KMAX * SM_PW];  // [kk][co]
    __shared__ __attribute__((aligned(16))) float sx[SM_KMAX * SM_PX];  // [kk][px]
    __shared__ long long s_base[SM_T];      // input offset of the pixel's leaf
    __shared__ int s_oy[SM_T], s_ox[SM_T];   // its output position (-1 past npx)
    const int tid = threadIdx.x, KC = 1 << kc_shift;
    const int co0 = blockIdx.x * SM_CO, px0 = blockIdx.y * SM_T, z = blockIdx.z;
    const int ty = tid >> 4, tx = tid & 15;  // outputs co0 + 4 ty .., px0 + 4 tx ..
    const int K = Cin * taps;
    if (tid < SM_T) {
        const int px = px0 + tid, hw = Ho * Wo;
        const int b = px / hw, r = px - b * hw;
        s_base[tid] = (long long)b * sB;
        s_oy[tid] = px < npx ? r / Wo : -1;
        s_ox[tid] = r % Wo;
    }
    float acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
    __syncthreads();

    const int nw = SM_CO << kc_shift, nx = SM_T << kc_shift;
    // slab sl's weights and im2col values into registers (all loads issued together)
    float tw[SM_PERW], tv[SM_PERX];
    auto load = [&](int sl) {
        const int k0 = (z * slabs_per_split + sl) << kc_shift;
        const int tap = k0 / Cin, ci0 = k0 - tap * Cin;
        const int dy = taps == 9 ? tap / 3 - pad : 0, dx = taps == 9 ? tap % 3 - pad : 0;
#pragma unroll
        for (int r = 0; r < SM_PERW; ++r) {
            const int i = tid + 512 * r;
            tw[r] = 0.f;
            if (i < nw) {
                const int row = i >> kc_shift, kk = i & (KC - 1);
                if (co0 + row < Cout) tw[r] = w[(long long)(co0 + row) * K + k0 + kk];
            }
        }
#pragma unroll
        for (int r = 0; r < SM_PERX; ++r) {
            const int i = tid + 512 * r;
            tv[r] = 0.f;
            if (i < nx) {
                const int row = i >> kc_shift, kk = i & (KC - 1);
                const int oy = s_oy[row];
                const int iy = oy + dy, ix = s_ox[row] + dx;
                if (oy >= 0 && iy >= 0 && iy < H && ix >= 0 && ix < W)
                    tv[r] = x[s_base[row] + (long long)iy * sY + (long long)ix * sX + (long long)(ci0 + kk) * sC];
            }
        }
    };
    load(0);
    for (int sl = 0; sl < slabs_per_split; ++sl) {
#pragma unroll
        for (int r = 0; r < SM_PERW; ++r) {
            const int i = tid + 512 * r;
            if (i < nw) sw[(i & (KC - 1)) * SM_PW + (i >> kc_shift)] = tw[r];
        }
#pragma unroll
        for (int r = 0; r < SM_PERX; ++r) {
            const int i = tid + 512 * r;
            if (i < nx) sx[(i & (KC - 1)) * SM_PX + (i >> kc_shift)] = tv[r];
        }
        __syncthreads();
        if (sl + 1 < slabs_per_split) load(sl + 1);
        for (int kk = 0; kk < KC; ++kk) {
            const float4 a = *(const float4*)(sw + kk * SM_PW + 4 * ty);
            const float4 c = *(const float4*)(sx + kk * SM_PX + 4 * tx);
            const float av[4] = {a.x, a.y, a.z, a.w}, cv[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], cv[j], acc[i][j]);
        }
        __syncthreads();
    }
    float* pz = part + (long long)z * npx * Cout;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int px = px0 + 4 * tx + j;
        if (px >= npx) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int co = co0 + 4 * ty + i;
            if (co < Cout) pz[(long long)px * Cout + co] = acc[i][j];
        }
    }
}

__global__ __launch_bounds__(256) void small_gemm_reduce_kernel(const float* __restrict__ part, int ksplit, int npx,
                                                                int Cout, const float* __restrict__ bias, int relu,
                                                                float* __restrict__ y, int ldy) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)npx * Cout) return;
    const int px = (int)(i / Cout), co = (int)(i - (long long)px * Cout);
    // in split order; the loads 8 at a time (independent), the adds in sequence
    const long long stride = (long long)npx * Cout;
    float s = part[i];
    int z = 1;
    for (; z + 8 <= ksplit; z += 8) {
        float t[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) t[j] = part[(z + j) * stride + i];
#pragma unroll
        for (int j = 0; j < 8; ++j) s += t[j];
    }
    for (; z < ksplit; ++z) s += part[z * stride + i];
    if (bias) s += bias[co];
    if (relu) s = fmaxf(s, 0.f);
    y[(long long)px * ldy + co] = s;
}

// ---------------------------------------------------------------------------
// small_layer: one whole layer per launch, no partial sums in HBM (one leaf to a few).
// The partial + reduce pair above spreads a layer over the chip by splitting K, which at
// one leaf writes and re-reads K-split x 49 x 512 partials and costs two launches.  Here
// block (co group of COB, pixel group) owns its outputs outright: its 512 threads split
// K (thread t: k pairs 2t, 2t + 1024, ...; 128 consecutive k of a wave lie in one tap),
// each keeps NPG x COB accumulators in registers, and the block sums the 512 partials of
// each output through LDS.  Per leaf the whole input activation (H x W x Cin f32, 100 KB
// for 7 x 7 x 512) is copied into LDS by LDS-DMA (no registers, every piece in flight at
// once) and read as float2 -- an input value feeds COB = 8 co -- while all of a thread's
// weight pairs (at most MAXM per co) are loaded into registers up front, under that copy.
// At one leaf conv2-4 are 64 co groups x ceil(49 / 13) pixel groups = 256 / 128 / 64
// blocks; an FC layer (H = W = 1, taps 1) is ceil(Cout / COB) blocks of one pixel.  f32
// fmaf in a fixed order (per thread k in order; the upper half's partials added to the
// lower's, then four quarter sums combined pairwise): deterministic.
constexpr int SL_THREADS = 512;
constexpr int SL_LDS = 32768 + 1024;  // floats: an 8 x 8 x 512 input, or the 256 x (13 x 8 + 1) partials

template <int NPG, int COB, int MAXM>
__global__ __launch_bounds__(SL_THREADS) void small_layer_kernel(const float* __restrict__ x, long long sB, int sY,
                                                                 int sX, int sC, int H, int W, int pad, int taps,
                                                                 int Ho, int Wo, const float* __restrict__ w, int Cin,
                                                                 int Cout, const float* __restrict__ bias, int relu,
                                                                 float* __restrict__ y, int ldy, int B, int npg) {
    __shared__ __attribute__((aligned(16))) float smem[SL_LDS];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int co0 = blockIdx.x * COB, g = blockIdx.y;
    const int NP = Ho * Wo, K = taps * Cin, KP = K >> 1;
    // pixel group g: [p0, p0 + npb), groups as equal as possible
    const int base = NP / npg, extra = NP % npg;
    const int p0 = g * base + (g < extra ? g : extra), npb = base + (g < extra ? 1 : 0);
    int oy[NPG], ox[NPG];
#pragma unroll
    for (int i = 0; i < NPG; ++i) {
        const int p = p0 + (i < npb ? i : 0);
        oy[i] = p / Wo;
        ox[i] = p - (p / Wo) * Wo;
    }
    const int nin = H * W * Cin;
    constexpr int R = NPG * COB + 1;  // partials row pitch (odd: conflict-free)
    // a leaf's input is one contiguous [iy][ix][ci] block for NHWC activations and FC rows
    const bool dense = sC == 1 && sX == Cin && sY == W * Cin && ((uintptr_t)x & 15) == 0 && (sB & 3) == 0;
    for (int b = 0; b < B; ++b) {
        const float* xb = x + (long long)b * sB;
        if (dense) {  // LDS-DMA: 1 KB per wave-instruction, bytes past the input read as 0
            const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)xb, 0, nin * 4, 0x00020000);
            const int nq = (nin * 4 + 1023) >> 10;
            for (int q = wid; q < nq; q += SL_THREADS / 64)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rs, (__attribute__((address_space(3))) void*)((char*)smem + (q << 10)), 16, (q << 10) + 16 * lane,
                    0, 0, 0);
        } else {
            for (int e = tid; e < nin; e += SL_THREADS) {
                const int pix = e / Cin, ci = e - pix * Cin;
                const int iy = pix / W, ix = pix - (pix / W) * W;
                smem[e] = xb[(long long)iy * sY + (long long)ix * sX + (long long)ci * sC];
            }
        }
        float acc[NPG][COB];
#pragma unroll
        for (int i = 0; i < NPG; ++i)
#pragma unroll
            for (int c = 0; c < COB; ++c) acc[i][c] = 0.f;
        for (int m0 = 0; m0 * SL_THREADS < KP; m0 += MAXM) {
            // the thread's weight pairs of MAXM k pairs, all loads in flight together
            float2 wv[MAXM][COB];
#pragma unroll
            for (int m = 0; m < MAXM; ++m) {
                const int j = tid + SL_THREADS * (m0 + m);
#pragma unroll
                for (int c = 0; c < COB; ++c)
                    wv[m][c] = j < KP && co0 + c < Cout ? *(const float2*)(w + (long long)(co0 + c) * K + 2 * j)
                                                        : make_float2(0.f, 0.f);
            }
            if (m0 == 0) {  // the input copy has landed (this thread's pieces, then everyone's)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
            }
#pragma unroll
            for (int m = 0; m < MAXM; ++m) {
                const int j = tid + SL_THREADS * (m0 + m);
                if (j >= KP) break;
                const int k = 2 * j, tap = k / Cin, ci = k - tap * Cin;
                const int dy = taps == 9 ? tap / 3 - pad : 0, dx = taps == 9 ? tap % 3 - pad : 0;
                // the pair's inputs at the block's pixels, all LDS reads issued before the
                // multiply-adds; a pixel outside the image or the group reads word 0, zeroed
                float2 v[NPG];
#pragma unroll
                for (int i = 0; i < NPG; ++i) {
                    const int iy = oy[i] + dy, ix = ox[i] + dx;
                    const bool ok = i < npb && iy >= 0 && iy < H && ix >= 0 && ix < W;
                    v[i] = *(const float2*)(smem + (ok ? (iy * W + ix) * Cin + ci : 0));
                    if (!ok) v[i] = make_float2(0.f, 0.f);
                }
#pragma unroll
                for (int i = 0; i < NPG; ++i)
#pragma unroll
                    for (int c = 0; c < COB; ++c) {
                        acc[i][c] = fmaf(wv[m][c].x, v[i].x, acc[i][c]);
                        acc[i][c] = fmaf(wv[m][c].y, v[i].y, acc[i][c]);
                    }
            }
        }
        __syncthreads();  // every thread is done with the input: the partials reuse its LDS
        const int row = tid & 255;
        if (tid >= 256) {
#pragma unroll
            for (int i = 0; i < NPG; ++i)
#pragma unroll
                for (int c = 0; c < COB; ++c)
                    if (i < npb) smem[row * R + i * COB + c] = acc[i][c];
        }
        __syncthreads();
        if (tid < 256) {
#pragma unroll
            for (int i = 0; i < NPG; ++i)
#pragma unroll
                for (int c = 0; c < COB; ++c)
                    if (i < npb) smem[row * R + i * COB + c] = acc[i][c] + smem[row * R + i * COB + c];
        }
        __syncthreads();
        // output o = (i, c): four threads sum 64 rows each in row order, combined pairwise
        const int o = tid >> 2, qt = tid & 3;
        float s = 0.f;
        if (o < npb * COB)
            for (int t0 = 64 * qt; t0 < 64 * qt + 64; t0 += 16) {
                float q[16];  // 16 independent LDS reads in flight, then the adds in order
#pragma unroll
                for (int u = 0; u < 16; ++u) q[u] = smem[(t0 + u) * R + o];
#pragma unroll
                for (int u = 0; u < 16; ++u) s += q[u];
            }
        s += __shfl_xor(s, 1);
        s += __shfl_xor(s, 2);
        if (qt == 0 && o < npb * COB) {
            const int i = o / COB, c = o - (o / COB) * COB, co = co0 + c;
            if (co < Cout) {
                float r = s;
                if (bias) r += bias[co];
                if (relu) r = fmaxf(r, 0.f);
                y[((long long)b * NP + p0 + i) * ldy + co] = r;
            }
        }
        __syncthreads();  // the partials are read before the next leaf's input lands
    }
}

// small_row: a 3x3 conv layer at one leaf to a few with one output row per block.  The
// block (8 co, output row oy) stages only the three input rows its window reads (<= 3 x 8
// x 512 f32 = 48 KB, by LDS-DMA) and its LDS (<= 66.5 KB with the partials) lets two
// blocks share a CU, so one block's weight and input round trips run under the other's
// multiply-adds; 256 threads split K as small_layer's, accumulators for the row's Wo <= 8
// pixels x 8 co in registers, the 256 partials summed through LDS in a fixed order.
constexpr int SR_THREADS = 256;
constexpr int SR_LDS = 256 * (8 * 8 + 1);  // floats: the partials, or three input rows at a 1-KB multiple pitch

template <int NPG, int COB, int MAXM>
__global__ __launch_bounds__(SR_THREADS, 2) void small_row_kernel(const float* __restrict__ x, long long sB, int sY,
                                                                  int sX, int sC, int H, int W, int pad, int Ho,
                                                                  int Wo, const float* __restrict__ w, int Cin,
                                                                  int Cout, const float* __restrict__ bias, int relu,
                                                                  float* __restrict__ y, int ldy, int B) {
    __shared__ __attribute__((aligned(16))) float smem[SR_LDS];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int co0 = blockIdx.x * COB, oy = blockIdx.y;
    const int K = 9 * Cin, KP = K >> 1, iy0 = oy - pad, rowf = W * Cin;
    const int nq = (rowf * 4 + 1023) >> 10, rpf = nq << 8;  // 1-KB DMA pieces per row; LDS row pitch (floats)
    constexpr int R = NPG * COB + 1;
    const bool dense = sC == 1 && sX == Cin && sY == W * Cin && ((uintptr_t)x & 15) == 0 && (sB & 3) == 0 &&
                       (rowf & 3) == 0;
    for (int b = 0; b < B; ++b) {
        const float* xb = x + (long long)b * sB;
        // window rows r = 0..2 (input row iy0 + r; rows outside the image are never read)
        if (dense) {  // a piece writes a whole KB (zeros past the row): rows rpf apart
            for (int t = wid; t < 3 * nq; t += SR_THREADS / 64) {
                const int r = t / nq, q = t - r * nq, iy = iy0 + r;
                if (iy < 0 || iy >= H) continue;
                const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(xb + (long long)iy * sY), 0, rowf * 4,
                                                                  0x00020000);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rs, (__attribute__((address_space(3))) void*)((char*)smem + r * rpf * 4 + (q << 10)), 16,
                    (q << 10) + 16 * lane, 0, 0, 0);
            }
        } else {
            for (int e = tid; e < 3 * rowf; e += SR_THREADS) {
                const int r = e / rowf, rem = e - r * rowf, ix = rem / Cin, ci = rem - ix * Cin, iy = iy0 + r;
                if (iy >= 0 && iy < H)
                    smem[r * rpf + rem] = xb[(long long)iy * sY + (long long)ix * sX + (long long)ci * sC];
            }
        }
        float acc[NPG][COB];
#pragma unroll
        for (int i = 0; i < NPG; ++i)
#pragma unroll
            for (int c = 0; c < COB; ++c) acc[i][c] = 0.f;
        // weight chunks of MAXM k pairs, double-buffered: chunk n + 1's loads are issued
        // before chunk n's multiply-adds, so each round trip runs under the previous chunk
        auto wload = [&](int m0, float2 (&wv)[MAXM][COB]) {
#pragma unroll
            for (int m = 0; m < MAXM; ++m) {
                const int j = tid + SR_THREADS * (m0 + m);
#pragma unroll
                for (int c = 0; c < COB; ++c)
                    wv[m][c] = j < KP && co0 + c < Cout ? *(const float2*)(w + (long long)(co0 + c) * K + 2 * j)
                                                        : make_float2(0.f, 0.f);
            }
        };
        auto compute = [&](int m0, const float2 (&wv)[MAXM][COB]) {
#pragma unroll
            for (int m = 0; m < MAXM; ++m) {
                const int j = tid + SR_THREADS * (m0 + m);
                if (j >= KP) break;
                const int k = 2 * j, tap = k / Cin, ci = k - tap * Cin, ky = tap / 3, kx = tap - ky * 3;
                const bool rok = iy0 + ky >= 0 && iy0 + ky < H;
                float2 v[NPG];
#pragma unroll
                for (int i = 0; i < NPG; ++i) {
                    const int ix = i + kx - pad;
                    const bool ok = rok && i < Wo && ix >= 0 && ix < W;
                    v[i] = *(const float2*)(smem + (ok ? ky * rpf + ix * Cin + ci : 0));
                    if (!ok) v[i] = make_float2(0.f, 0.f);
                }
#pragma unroll
                for (int i = 0; i < NPG; ++i)
#pragma unroll
                    for (int c = 0; c < COB; ++c) {
                        acc[i][c] = fmaf(wv[m][c].x, v[i].x, acc[i][c]);
                        acc[i][c] = fmaf(wv[m][c].y, v[i].y, acc[i][c]);
                    }
            }
        };
        const int nchunk = (KP + SR_THREADS * MAXM - 1) / (SR_THREADS * MAXM);
        float2 wa[MAXM][COB], wb[MAXM][COB];
        wload(0, wa);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the rows and chunk 0 have landed
        __syncthreads();
        for (int n = 0; n < nchunk; n += 2) {
            if (n + 1 < nchunk) wload((n + 1) * MAXM, wb);
            compute(n * MAXM, wa);
            if (n + 1 >= nchunk) break;
            if (n + 2 < nchunk) wload((n + 2) * MAXM, wa);
            compute((n + 1) * MAXM, wb);
        }
        __syncthreads();  // the input rows are read: the partials reuse the LDS
#pragma unroll
        for (int i = 0; i < NPG; ++i)
#pragma unroll
            for (int c = 0; c < COB; ++c)
                if (i < Wo) smem[tid * R + i * COB + c] = acc[i][c];
        __syncthreads();
        // output o = (i, c): four threads sum 64 partials each in thread order, combined pairwise
        const int o = tid >> 2, qt = tid & 3, nout = Wo * COB;
        float s = 0.f;
        if (o < nout)
            for (int t0 = 64 * qt; t0 < 64 * qt + 64; t0 += 16) {
                float q[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) q[u] = smem[(t0 + u) * R + o];
#pragma unroll
                for (int u = 0; u < 16; ++u) s += q[u];
            }
        s += __shfl_xor(s, 1);
        s += __shfl_xor(s, 2);
        if (qt == 0 && o < nout) {
            const int i = o / COB, c = o - (o / COB) * COB, co = co0 + c;
            if (co < Cout) {
                float r = s;
                if (bias) r += bias[co];
                if (relu) r = fmaxf(r, 0.f);
                y[((long long)b * Ho * Wo + oy * Wo + i) * ldy + co] = r;
            }
        }
        __syncthreads();
    }
}

}  // namespace

// One layer (3x3 conv, taps 9, or FC, taps 1; + bias, ReLU) on small_layer_kernel:
// batch leaves, input x with element strides (sB, sY, sX, sC), weights [Cout][taps * Cin]
// (k = tap * Cin + ci), output rows y[(leaf * Ho * Wo + pixel) * ldy + co].  Needs Cin even,
// the input of one leaf (H * W * Cin floats) in 128 KB of LDS and w 8-B aligned.
extern "C" int azg_small_layer(const float* x, int64_t sB, int32_t sY, int32_t sX, int32_t sC, int32_t batch,
                               int32_t H, int32_t W, int32_t pad, int32_t taps, const float* w, int32_t Cin,
                               int32_t Cout, const float* bias, int32_t relu, float* y, int32_t ldy, void* stream) {
    if (!x || !w || !y || batch <= 0 || H <= 0 || W <= 0 || (taps != 1 && taps != 9) || Cin <= 0 || (Cin & 1) ||
        Cout <= 0 || ldy < Cout || pad < 0 || (taps == 1 && (pad || H != 1 || W != 1)) || ((uintptr_t)w & 7))
        return AZG_ERR_ARG;
    const int Ho = taps == 9 ? H + 2 * pad - 2 : 1, Wo = taps == 9 ? W + 2 * pad - 2 : 1;
    if (Ho <= 0 || Wo <= 0 || (long long)H * W * Cin > 32768 || (long long)taps * Cin > (1 << 24)) return AZG_ERR_ARG;
    const hipStream_t st = (hipStream_t)stream;
    if (taps == 9 && Wo <= 8 && W <= 8 && 3LL * ((W * Cin * 4LL + 1023) / 1024) * 256 <= SR_LDS) {  // one row per block
        const dim3 grid((unsigned)((Cout + 7) / 8), (unsigned)Ho);
        hipLaunchKernelGGL((small_row_kernel<8, 8, 2>), grid, dim3(SR_THREADS), 0, st, x, (long long)sB, sY, sX, sC, H,
                           W, pad, Ho, Wo, w, Cin, Cout, bias, relu, y, ldy, batch);
    } else if (taps == 9) {
        constexpr int NPG = 13, COB = 8;
        const int np = Ho * Wo, npg = (np + NPG - 1) / NPG;
        const dim3 grid((unsigned)((Cout + COB - 1) / COB), (unsigned)npg);
        hipLaunchKernelGGL((small_layer_kernel<NPG, COB, 3>), grid, dim3(SL_THREADS), 0, st, x, (long long)sB, sY, sX, sC,
                           H, W, pad, taps, Ho, Wo, w, Cin, Cout, bias, relu, y, ldy, batch, npg);
    } else {
        constexpr int COB = 4;
        const dim3 grid((unsigned)((Cout + COB - 1) / COB), 1u);
        hipLaunchKernelGGL((small_layer_kernel<1, COB, 8>), grid, dim3(SL_THREADS), 0, st, x, (long long)sB, sY, sX, sC, H,
                           W, pad, taps, Ho, Wo, w, Cin, Cout, bias, relu, y, ldy, batch, 1);
    }
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_small_gemm_partial(const float* x, int64_t sB, int32_t sY, int32_t sX, int32_t sC, int32_t batch,
                                      int32_t H, int32_t W, int32_t pad, int32_t taps, const float* w, int32_t Cin,
                                      int32_t Cout, int32_t kc, int32_t ksplit, float* part, void* stream) {
    if (!x || !w || !part || batch <= 0 || H <= 0 || W <= 0 || (taps != 1 && taps != 9) || Cin <= 0 || Cout <= 0 ||
        kc <= 0 || kc > SM_KMAX || (kc & (kc - 1)) || Cin % kc || ksplit <= 0 || pad < 0 || (taps == 1 && pad))
        return AZG_ERR_ARG;
    int kc_shift = 0;
    while ((1 << kc_shift) < kc) ++kc_shift;
    const int Ho = taps == 9 ? H + 2 * pad - 2 : H, Wo = taps == 9 ? W + 2 * pad - 2 : W;
    if (Ho <= 0 || Wo <= 0) return AZG_ERR_ARG;
    const long long npx = (long long)batch * Ho * Wo;
    const int slabs = taps * Cin / kc;
    if (npx > (1 << 24) || ksplit > slabs || slabs % ksplit) return AZG_ERR_ARG;
    const dim3 grid((unsigned)((Cout + SM_CO - 1) / SM_CO), (unsigned)((npx + SM_T - 1) / SM_T), (unsigned)ksplit);
    hipLaunchKernelGGL(small_gemm_partial_kernel, grid, dim3(512), 0, (hipStream_t)stream, x, (long long)sB, sY, sX,
                       sC, H, W, pad, taps, Ho, Wo, (int)npx, w, Cin, Cout, kc_shift, slabs / ksplit, part);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_small_gemm_reduce(const float* part, int32_t ksplit, int32_t npx, int32_t Cout, const float* bias,
                                     int32_t relu, float* y, int32_t ldy, void* stream) {
    if (!part || !y || ksplit <= 0 || npx <= 0 || Cout <= 0 || ldy < Cout) return AZG_ERR_ARG;
    const long long n = (long long)npx * Cout;
    hipLaunchKernelGGL(small_gemm_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, part, ksplit, npx, Cout, bias, relu, y, ldy);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}
