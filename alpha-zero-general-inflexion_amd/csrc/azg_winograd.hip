// azg_winograd.hip -- the leaf network's 3x3 convolutions as Winograd F(m x m, 3x3).
//
// conv2-4 of InflexionNNet.forward (InflexionNNet.py:43-45, BN folded) are
// y = relu(bias + conv3x3(x, w)).  With m x m output tiles (n = m + 2 input
// points per side), each tile is
//     Y = A^T [ U (.) V ] A,   U = G g G^T (per (c, k)),   V = B^T d B (per (tile, c)),
// and the sum over input channels c of U (.) V is, for each of the n*n tile
// positions e, one GEMM  M_e[T x K] = V_e[T x C] x U_e[C x K]  (T = tiles).
// Multiply-adds per output: n^2 / m^2 instead of 9 -- F(2,3): 4, F(3,3): 2.78 --
// less the tile padding of outputs that are not a multiple of m.  The GEMMs
// are f32 (hipBLASLt through torch.bmm); these kernels are the two transforms,
// HBM-bound and coalesced (4 channels per lane as float4, consecutive lanes on
// consecutive channels):
//   * winograd_in : NHWC input (zero padding; optionally the previous layer's
//                   bias + ReLU applied on load) -> V [n*n][T][C]
//   * winograd_out: M [n*n][T][K] -> NHWC output, bias + ReLU fused, tile
//                   padding cropped.
// B and A have small integer entries (F(2,3): 0, +-1; F(3,3): up to 4), so the
// transforms are adds and exact scalings except F(3,3)'s x3; U is formed in f64
// by the caller (G has entries 1/2, 1/3, 1/6).  F(3,3)'s larger constants make
// its f32 error ~3x F(2,3)'s.
#include <hip/hip_runtime.h>

#include "../../include/azg.h"

namespace {

__device__ __forceinline__ float4 f4add(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float4 f4scale(float c, float4 a) { return make_float4(c * a.x, c * a.y, c * a.z, c * a.w); }

// transform tables: B^T [n][n] (input), A^T [m][n] (output)
template <int M>
struct WinoT;
template <>
struct WinoT<2> {
    static constexpr int N = 4;
    static constexpr float BT[4][4] = {{1, 0, -1, 0}, {0, 1, 1, 0}, {0, -1, 1, 0}, {0, 1, 0, -1}};
    static constexpr float AT[2][4] = {{1, 1, 1, 0}, {0, 1, -1, -1}};
};
template <>
struct WinoT<3> {
    static constexpr int N = 5;  // interpolation points 0, 1, -1, 2, inf
    static constexpr float BT[5][5] = {
        {2, -1, -2, 1, 0}, {0, -2, -1, 1, 0}, {0, 2, -3, 1, 0}, {0, -1, 0, 1, 0}, {0, 2, -1, -2, 1}};
    static constexpr float AT[3][5] = {{1, 1, 1, 1, 0}, {0, 1, -1, 2, 0}, {0, 1, 1, 4, 1}};
};

// sum_j coef[j] * x[j], skipping zero coefficients at compile time (x1 folds)
template <int L>
__device__ __forceinline__ float4 combine(const float (&coef)[L], const float4* x) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    bool first = true;
#pragma unroll
    for (int j = 0; j < L; ++j) {
        if (coef[j] == 0.f) continue;
        const float4 term = coef[j] == 1.f ? x[j] : f4scale(coef[j], x[j]);
        acc = first ? term : f4add(acc, term);
        first = false;
    }
    return acc;
}

// One V element: f32, or its fp16 (hi, lo, hi) triple at columns c, C + c, 2C + c
// of a 3C-wide row.
template <bool SPLIT>
__device__ __forceinline__ void store_v(void* V, long long row, int C, int c, float v, int* overflow) {
    if constexpr (!SPLIT) {
        ((float*)V)[row * C + c] = v;
    } else {
        const _Float16 hi = (_Float16)v;  // round to nearest even
        const _Float16 lo = (_Float16)(v - (float)hi);
        _Float16* r = (_Float16*)V + row * 3 * C;
        r[c] = hi;
        r[C + c] = lo;
        r[2 * C + c] = hi;
        if (!(fabsf(v) <= 65504.f)) atomicOr(overflow, 1);
    }
}

// Four consecutive channels (c4 = c / 4) of one V row.
template <bool SPLIT>
__device__ __forceinline__ void store_v4(void* V, long long row, int C4, int c4, float4 v, int* overflow) {
    if constexpr (!SPLIT) {
        ((float4*)V)[row * C4 + c4] = v;
    } else {
        const float x[4] = {v.x, v.y, v.z, v.w};
        union {
            _Float16 h[4];
            uint2 u;
        } hi, lo;
        bool bad = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            hi.h[j] = (_Float16)x[j];
            lo.h[j] = (_Float16)(x[j] - (float)hi.h[j]);
            bad |= !(fabsf(x[j]) <= 65504.f);
        }
        uint2* r = (uint2*)V + row * 3 * C4;
        r[c4] = hi.u;
        r[C4 + c4] = lo.u;
        r[2 * C4 + c4] = hi.u;
        if (bad) atomicOr(overflow, 1);
    }
}

// Work item of a thread: block ids are dealt round-robin to the 8 XCDs, so the
// block -> work mapping gives each XCD one contiguous eighth of the work:
// neighbouring tiles, which share input halo pixels, then hit the same L2.
__device__ __forceinline__ long long xcd_item() {
    const unsigned per = gridDim.x / 8;  // the grid is a multiple of 8 blocks
    const unsigned vb = (blockIdx.x % 8) * per + blockIdx.x / 8;
    return (long long)vb * blockDim.x + threadIdx.x;
}

// tile index t = (b * tiles + ty) * tiles + tx
// in_bias != null: x is the previous layer's raw output and relu(x + in_bias)
// is applied on load (that layer's bias + ReLU fused here; padding stays 0)
template <int M, bool SPLIT>
__global__ __launch_bounds__(256) void winograd_in_kernel(const float4* __restrict__ x,
                                                          const float4* __restrict__ in_bias, void* __restrict__ V,
                                                          int H, int pad, int C4, int tiles, long long T,
                                                          int* overflow) {
    using W = WinoT<M>;
    constexpr int N = W::N;
    const long long i = xcd_item();
    if (i >= T * C4) return;
    const int c4 = (int)(i % C4);
    const long long t = i / C4;
    const int tx = (int)(t % tiles);
    const long long r = t / tiles;
    const int ty = (int)(r % tiles);
    const long long b = r / tiles;
    const float4 ib = in_bias ? in_bias[c4] : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 d[N][N];
#pragma unroll
    for (int u = 0; u < N; ++u) {
        const int iy = M * ty - pad + u;
#pragma unroll
        for (int v = 0; v < N; ++v) {
            const int ix = M * tx - pad + v;
            float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
            if (iy >= 0 && iy < H && ix >= 0 && ix < H) {
                z = x[((b * H + iy) * H + ix) * C4 + c4];
                if (in_bias) {
                    z = f4add(z, ib);
                    z.x = fmaxf(z.x, 0.f);
                    z.y = fmaxf(z.y, 0.f);
                    z.z = fmaxf(z.z, 0.f);
                    z.w = fmaxf(z.w, 0.f);
                }
            }
            d[u][v] = z;
        }
    }
    // s = B^T d (rows), then V = s B (columns)
    float4 s[N][N];
#pragma unroll
    for (int v = 0; v < N; ++v) {
        float4 col[N];
#pragma unroll
        for (int u = 0; u < N; ++u) col[u] = d[u][v];
#pragma unroll
        for (int a = 0; a < N; ++a) s[a][v] = combine<N>(W::BT[a], col);
    }
#pragma unroll
    for (int a = 0; a < N; ++a) {
#pragma unroll
        for (int bb = 0; bb < N; ++bb)
            store_v4<SPLIT>(V, (long long)(a * N + bb) * T + t, C4, c4, combine<N>(W::BT[bb], s[a]), overflow);
    }
}

template <int M>
__global__ __launch_bounds__(256) void winograd_out_kernel(const float4* __restrict__ Min,
                                                           const float4* __restrict__ bias, float4* __restrict__ y,
                                                           int Ho, int K4, int tiles, long long T, int relu,
                                                           float mscale) {
    using W = WinoT<M>;
    constexpr int N = W::N;
    const long long i = xcd_item();
    if (i >= T * K4) return;
    const int k4 = (int)(i % K4);
    const long long t = i / K4;
    const int tx = (int)(t % tiles);
    const long long r = t / tiles;
    const int ty = (int)(r % tiles);
    const long long b = r / tiles;
    float4 m[N][N];
#pragma unroll
    for (int e = 0; e < N * N; ++e) m[e / N][e % N] = f4scale(mscale, Min[((long long)e * T + t) * K4 + k4]);
    // s = A^T m (rows), then Y = s A (columns)
    float4 s[M][N];
#pragma unroll
    for (int v = 0; v < N; ++v) {
        float4 col[N];
#pragma unroll
        for (int u = 0; u < N; ++u) col[u] = m[u][v];
#pragma unroll
        for (int a = 0; a < M; ++a) s[a][v] = combine<N>(W::AT[a], col);
    }
    const float4 bb = bias[k4];
#pragma unroll
    for (int a = 0; a < M; ++a) {
        const int oy = M * ty + a;
#pragma unroll
        for (int c = 0; c < M; ++c) {
            const int ox = M * tx + c;
            if (oy < Ho && ox < Ho) {
                float4 z = f4add(combine<N>(W::AT[c], s[a]), bb);
                if (relu) {
                    z.x = fmaxf(z.x, 0.f);
                    z.y = fmaxf(z.y, 0.f);
                    z.z = fmaxf(z.z, 0.f);
                    z.w = fmaxf(z.w, 0.f);
                }
                y[((b * Ho + oy) * Ho + ox) * K4 + k4] = z;
            }
        }
    }
}

// scalar (one channel) tile transforms: y = A^T m A (m x m) and V = B^T d B (n x n)
template <int MI>
__device__ __forceinline__ void out_tile(const float (&mm)[WinoT<MI>::N][WinoT<MI>::N], float (&y)[MI][MI]) {
    using W = WinoT<MI>;
    constexpr int N = W::N;
    float sr[MI][N];
#pragma unroll
    for (int v = 0; v < N; ++v)
#pragma unroll
        for (int a = 0; a < MI; ++a) {
            float acc = 0.f;
            bool first = true;
#pragma unroll
            for (int u = 0; u < N; ++u) {
                if (W::AT[a][u] == 0.f) continue;
                const float term = W::AT[a][u] == 1.f ? mm[u][v] : W::AT[a][u] * mm[u][v];
                acc = first ? term : acc + term;
                first = false;
            }
            sr[a][v] = acc;
        }
#pragma unroll
    for (int a = 0; a < MI; ++a)
#pragma unroll
        for (int q = 0; q < MI; ++q) {
            float acc = 0.f;
            bool first = true;
#pragma unroll
            for (int v = 0; v < N; ++v) {
                if (W::AT[q][v] == 0.f) continue;
                const float term = W::AT[q][v] == 1.f ? sr[a][v] : W::AT[q][v] * sr[a][v];
                acc = first ? term : acc + term;
                first = false;
            }
            y[a][q] = acc;
        }
}

template <int MO>
__device__ __forceinline__ void in_tile(const float (&d)[WinoT<MO>::N][WinoT<MO>::N],
                                        float (&V)[WinoT<MO>::N][WinoT<MO>::N]) {
    using W = WinoT<MO>;
    constexpr int N = W::N;
    float sr[N][N];
#pragma unroll
    for (int v = 0; v < N; ++v)
#pragma unroll
        for (int a = 0; a < N; ++a) {
            float acc = 0.f;
            bool first = true;
#pragma unroll
            for (int u = 0; u < N; ++u) {
                if (W::BT[a][u] == 0.f) continue;
                const float term = W::BT[a][u] == 1.f ? d[u][v] : W::BT[a][u] * d[u][v];
                acc = first ? term : acc + term;
                first = false;
            }
            sr[a][v] = acc;
        }
#pragma unroll
    for (int a = 0; a < N; ++a)
#pragma unroll
        for (int bb = 0; bb < N; ++bb) {
            float acc = 0.f;
            bool first = true;
#pragma unroll
            for (int v = 0; v < N; ++v) {
                if (W::BT[bb][v] == 0.f) continue;
                const float term = W::BT[bb][v] == 1.f ? sr[a][v] : W::BT[bb][v] * sr[a][v];
                acc = first ? term : acc + term;
                first = false;
            }
            V[a][bb] = acc;
        }
}

// A lane's private h x h plane: in registers when the side is a compile-time
// HC (loops fully unrolled, every index constant), else in its own LDS column.
template <int HC>
struct Plane {
    float r[HC > 0 ? HC * HC : 1];
    float* lds;
    int lane;
    __device__ __forceinline__ void put(int i, float v) {
        if constexpr (HC > 0) r[i] = v;
        else lds[i * 64 + lane] = v;
    }
    __device__ __forceinline__ float get(int i) const {
        if constexpr (HC > 0) return r[i];
        else return lds[i * 64 + lane];
    }
};

// Next layer's input transform (pad `pad`) of the lane's h x h plane: V tiles out.
template <int MO, int HC, bool SPLIT, class P>
__device__ __forceinline__ void plane_to_V(const P& ys, int h, int pad, long long b, int c, int C, long long To,
                                           void* __restrict__ Vout, int* overflow) {
    constexpr int NO = WinoT<MO>::N;
    const int to = (h + 2 * pad - 2 + MO - 1) / MO;
#pragma unroll
    for (int ty = 0; ty < to; ++ty)
#pragma unroll
        for (int tx = 0; tx < to; ++tx) {
            const long long t = (b * to + ty) * to + tx;
            float d[NO][NO];
#pragma unroll
            for (int u = 0; u < NO; ++u)
#pragma unroll
                for (int v = 0; v < NO; ++v) {
                    const int iy = MO * ty - pad + u, ix = MO * tx - pad + v;
                    d[u][v] = (iy >= 0 && iy < h && ix >= 0 && ix < h) ? ys.get(iy * h + ix) : 0.f;
                }
            float V[NO][NO];
            in_tile<MO>(d, V);
#pragma unroll
            for (int a = 0; a < NO; ++a)
#pragma unroll
                for (int bb = 0; bb < NO; ++bb)
                    store_v<SPLIT>(Vout, (long long)(a * NO + bb) * To + t, C, c, V[a][bb], overflow);
        }
}

// Layer i's output transform fused with layer i+1's input transform (pad 0
// between them, as conv2->conv3->conv4): one wave per (image, 64 channels),
// each lane owning one channel.  The lane's h x h output plane of layer i
// (bias + ReLU applied) is kept in registers (compile-time side HC) or its own
// LDS column -- only that lane reads it back, so no barrier -- and the next
// layer's tiles are transformed from it: layer i's activation never goes to HBM.
template <int MI, int MO, int HC, bool SPLIT>
__global__ __launch_bounds__(64) void winograd_mid_kernel(const float* __restrict__ Min, const float* __restrict__ bias,
                                                          void* __restrict__ Vout, int h_rt, int C, long long Ti,
                                                          long long To, float mscale, int* overflow) {
    constexpr int NI = WinoT<MI>::N;
    extern __shared__ float ys_raw[];  // [h * h][64] when HC == 0
    const int h = HC > 0 ? HC : h_rt;
    const int lane = threadIdx.x;
    const int cblocks = C / 64;
    const long long b = blockIdx.x / cblocks;
    const int c = (blockIdx.x % cblocks) * 64 + lane;
    const int ti = (h + MI - 1) / MI;
    const float bc = bias[c];
    Plane<HC> ys;
    ys.lds = ys_raw;
    ys.lane = lane;
#pragma unroll
    for (int ty = 0; ty < ti; ++ty)
#pragma unroll
        for (int tx = 0; tx < ti; ++tx) {
            const long long t = (b * ti + ty) * ti + tx;
            float mm[NI][NI];
#pragma unroll
            for (int e = 0; e < NI * NI; ++e) mm[e / NI][e % NI] = mscale * Min[((long long)e * Ti + t) * C + c];
            float y[MI][MI];
            out_tile<MI>(mm, y);
#pragma unroll
            for (int a = 0; a < MI; ++a)
#pragma unroll
                for (int q = 0; q < MI; ++q) {
                    const int oy = MI * ty + a, ox = MI * tx + q;
                    if (oy < h && ox < h) ys.put(oy * h + ox, fmaxf(y[a][q] + bc, 0.f));
                }
        }
    plane_to_V<MO, HC, SPLIT>(ys, h, 0, b, c, C, To, Vout, overflow);
}

// The network's first two layers' front end in one pass: conv1 (depth -> C
// channels, 3x3, pad 1) + bias + ReLU computed directly from the NCHW leaf
// planes, then conv2's Winograd input transform (pad 1) -- conv1's activation
// never leaves the chip.  One wave per (image, 64 output channels of conv1),
// one channel per lane: the image's planes are shared through LDS, the lane's
// depth*9 weights and its n x n output plane sit in registers (compile-time
// side NC) or its own LDS column.
template <int MO, int NC, bool SPLIT>
__global__ __launch_bounds__(64) void winograd_first_kernel(const float* __restrict__ planes,
                                                            const float* __restrict__ w1,
                                                            const float* __restrict__ b1, void* __restrict__ Vout,
                                                            int depth, int n_rt, int C, long long To, int* overflow) {
    constexpr int DMAX = 4;
    extern __shared__ float lds[];
    float* xs = lds;  // [depth][n][n], then (NC == 0) the lanes' planes [n * n][64]
    const int n = NC > 0 ? NC : n_rt;
    const int lane = threadIdx.x;
    const int cblocks = C / 64;
    const long long b = blockIdx.x / cblocks;
    const int k = (blockIdx.x % cblocks) * 64 + lane;
    for (int i = lane; i < depth * n * n; i += 64) xs[i] = planes[b * depth * n * n + i];
    float w[DMAX * 9];
#pragma unroll
    for (int j = 0; j < DMAX * 9; ++j) w[j] = j < depth * 9 ? w1[(size_t)k * depth * 9 + j] : 0.f;
    const float bk = b1[k];
    __syncthreads();
    Plane<NC> ys;
    ys.lds = lds + DMAX * 81;
    ys.lane = lane;
#pragma unroll
    for (int y = 0; y < n; ++y)
#pragma unroll
        for (int x = 0; x < n; ++x) {
            float acc = 0.f;
#pragma unroll
            for (int c = 0; c < DMAX; ++c) {
                if (c >= depth) break;
#pragma unroll
                for (int dy = 0; dy < 3; ++dy) {
                    const int iy = y + dy - 1;
                    if (iy < 0 || iy >= n) continue;
#pragma unroll
                    for (int dx = 0; dx < 3; ++dx) {
                        const int ix = x + dx - 1;
                        if (ix < 0 || ix >= n) continue;
                        acc = fmaf(w[c * 9 + dy * 3 + dx], xs[(c * n + iy) * n + ix], acc);
                    }
                }
            }
            ys.put(y * n + x, fmaxf(acc + bk, 0.f));
        }
    plane_to_V<MO, NC, SPLIT>(ys, n, 1, b, k, C, To, Vout, overflow);
}

// one thread per work item, rounded up to whole groups of 8 blocks (xcd_item)
unsigned grid_for(long long n) {
    const long long blocks = (n + 255) / 256;
    return (unsigned)(((blocks + 7) / 8) * 8);
}

bool bad_fmt(int vfmt, const int* overflow) {
    return !(vfmt == AZG_WINO_F32 || (vfmt == AZG_WINO_SPLIT && overflow));
}
}  // namespace

extern "C" int azg_winograd_in_nhwc(const float* x, const float* in_bias, void* V, int32_t batch, int32_t h_in,
                                    int32_t pad, int32_t c, int32_t m, int32_t vfmt, int32_t* overflow,
                                    void* stream) {
    const int h_out = h_in + 2 * pad - 2;
    if (!x || !V || batch <= 0 || h_out <= 0 || c <= 0 || c % 4 || (m != 2 && m != 3) || ((uintptr_t)x & 15) ||
        ((uintptr_t)V & 15) || ((uintptr_t)in_bias & 15) || bad_fmt(vfmt, overflow) ||
        (long long)batch * ((h_out + m - 1) / m) * ((h_out + m - 1) / m) * (c / 4) > (1ll << 38))
        return AZG_ERR_ARG;
    const int tiles = (h_out + m - 1) / m;
    const long long T = (long long)batch * tiles * tiles;
    const dim3 grid(grid_for(T * (c / 4)));
    hipStream_t st = (hipStream_t)stream;
#define AZG_IN(MM, SP)                                                                                             \
    if (m == MM && (vfmt == AZG_WINO_SPLIT) == SP)                                                                 \
        hipLaunchKernelGGL((winograd_in_kernel<MM, SP>), grid, dim3(256), 0, st, (const float4*)x,                 \
                           (const float4*)in_bias, V, h_in, pad, c / 4, tiles, T, overflow);
    AZG_IN(2, false)
    AZG_IN(3, false)
    AZG_IN(2, true)
    AZG_IN(3, true)
#undef AZG_IN
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_winograd_out_nhwc(const float* M, const float* bias, float* y, int32_t batch, int32_t h_out,
                                     int32_t k, int32_t m, int32_t relu, float mscale, void* stream) {
    if (!M || !bias || !y || batch <= 0 || h_out <= 0 || k <= 0 || k % 4 || (m != 2 && m != 3) ||
        ((uintptr_t)M & 15) || ((uintptr_t)bias & 15) || ((uintptr_t)y & 15) ||
        (long long)batch * ((h_out + m - 1) / m) * ((h_out + m - 1) / m) * (k / 4) > (1ll << 38))
        return AZG_ERR_ARG;
    const int tiles = (h_out + m - 1) / m;
    const long long T = (long long)batch * tiles * tiles;
    if (m == 2)
        hipLaunchKernelGGL(winograd_out_kernel<2>, dim3(grid_for(T * (k / 4))), dim3(256), 0, (hipStream_t)stream,
                           (const float4*)M, (const float4*)bias, (float4*)y, h_out, k / 4, tiles, T, relu, mscale);
    else
        hipLaunchKernelGGL(winograd_out_kernel<3>, dim3(grid_for(T * (k / 4))), dim3(256), 0, (hipStream_t)stream,
                           (const float4*)M, (const float4*)bias, (float4*)y, h_out, k / 4, tiles, T, relu, mscale);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_winograd_mid_nhwc(const float* M, const float* bias, void* V, int32_t batch, int32_t h, int32_t c,
                                     int32_t m_in, int32_t m_out, float mscale, int32_t vfmt, int32_t* overflow,
                                     void* stream) {
    if (!M || !bias || !V || batch <= 0 || h < 3 || h > 9 || c <= 0 || c % 64 || (m_in != 2 && m_in != 3) ||
        (m_out != 2 && m_out != 3) || bad_fmt(vfmt, overflow))
        return AZG_ERR_ARG;
    const int ti = (h + m_in - 1) / m_in, to = (h - 2 + m_out - 1) / m_out;
    const long long Ti = (long long)batch * ti * ti, To = (long long)batch * to * to;
    const dim3 grid((unsigned)(batch * (c / 64)));
    const size_t lds = (size_t)h * h * 64 * sizeof(float);
    hipStream_t st = (hipStream_t)stream;
    const bool split = vfmt == AZG_WINO_SPLIT;
    // the board sides of the supported games get register-resident planes
#define AZG_MID(MI, MO, H, SP, L)                                                                          \
    {                                                                                                      \
        hipLaunchKernelGGL((winograd_mid_kernel<MI, MO, H, SP>), grid, dim3(64), L, st, M, bias, V, h, c, Ti, \
                           To, mscale, overflow);                                                          \
        return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;                                          \
    }
#define AZG_MID_REG(MI, MO, H)                                   \
    if (m_in == MI && m_out == MO && h == H) {                   \
        if (split) AZG_MID(MI, MO, H, true, 0) else AZG_MID(MI, MO, H, false, 0) \
    }
    AZG_MID_REG(3, 3, 7)
    AZG_MID_REG(3, 3, 5)
    AZG_MID_REG(3, 3, 8)
    AZG_MID_REG(3, 2, 6)
    AZG_MID_REG(2, 2, 4)
#define AZG_MID_LDS(MI, MO)                                       \
    if (m_in == MI && m_out == MO) {                              \
        if (split) AZG_MID(MI, MO, 0, true, lds) else AZG_MID(MI, MO, 0, false, lds) \
    }
    AZG_MID_LDS(2, 2)
    AZG_MID_LDS(2, 3)
    AZG_MID_LDS(3, 2)
    AZG_MID_LDS(3, 3)
#undef AZG_MID_LDS
#undef AZG_MID_REG
#undef AZG_MID
    return AZG_ERR_ARG;
}

extern "C" int azg_winograd_first_nchw(const float* planes, const float* w1, const float* b1, void* V, int32_t batch,
                                       int32_t depth, int32_t n, int32_t c, int32_t m, int32_t vfmt,
                                       int32_t* overflow, void* stream) {
    if (!planes || !w1 || !b1 || !V || batch <= 0 || depth < 1 || depth > 4 || n < 3 || n > 9 || c <= 0 ||
        c % 64 || (m != 2 && m != 3) || bad_fmt(vfmt, overflow))
        return AZG_ERR_ARG;
    const int to = (n + m - 1) / m;
    const long long To = (long long)batch * to * to;
    const dim3 grid((unsigned)(batch * (c / 64)));
    const size_t lds_reg = 4 * 81 * sizeof(float), lds = (4 * 81 + (size_t)n * n * 64) * sizeof(float);
    hipStream_t st = (hipStream_t)stream;
    const bool split = vfmt == AZG_WINO_SPLIT;
#define AZG_FIRST(MO, N, SP, L)                                                                                  \
    {                                                                                                            \
        hipLaunchKernelGGL((winograd_first_kernel<MO, N, SP>), grid, dim3(64), L, st, planes, w1, b1, V, depth, n, \
                           c, To, overflow);                                                                     \
        return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;                                                \
    }
#define AZG_FIRST_REG(MO, N)                                                  \
    if (m == MO && n == N) {                                                  \
        if (split) AZG_FIRST(MO, N, true, lds_reg) else AZG_FIRST(MO, N, false, lds_reg) \
    }
    AZG_FIRST_REG(3, 7)
    AZG_FIRST_REG(3, 8)
    AZG_FIRST_REG(3, 6)
#undef AZG_FIRST_REG
    if (m == 2) {
        if (split) AZG_FIRST(2, 0, true, lds) else AZG_FIRST(2, 0, false, lds)
    }
    if (split) AZG_FIRST(3, 0, true, lds) else AZG_FIRST(3, 0, false, lds)
#undef AZG_FIRST
}
