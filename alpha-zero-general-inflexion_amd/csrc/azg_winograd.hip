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
template <int M>
__global__ __launch_bounds__(256) void winograd_in_kernel(const float4* __restrict__ x,
                                                          const float4* __restrict__ in_bias, float4* __restrict__ V,
                                                          int H, int pad, int C4, int tiles, long long T) {
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
            V[((long long)(a * N + bb) * T + t) * C4 + c4] = combine<N>(W::BT[bb], s[a]);
    }
}

template <int M>
__global__ __launch_bounds__(256) void winograd_out_kernel(const float4* __restrict__ Min,
                                                           const float4* __restrict__ bias, float4* __restrict__ y,
                                                           int Ho, int K4, int tiles, long long T, int relu) {
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
    for (int e = 0; e < N * N; ++e) m[e / N][e % N] = Min[((long long)e * T + t) * K4 + k4];
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

// Layer i's output transform fused with layer i+1's input transform (pad 0
// between them, as conv2->conv3->conv4): one wave per (image, 64 channels),
// each lane owning one channel.  The lane's h x h output plane of layer i
// (bias + ReLU applied) is staged in LDS -- only that lane reads it back, so
// no barrier -- and the next layer's tiles are transformed from it: layer i's
// NHWC activation never goes to HBM.
template <int MI, int MO>
__global__ __launch_bounds__(64) void winograd_mid_kernel(const float* __restrict__ Min, const float* __restrict__ bias,
                                                          float* __restrict__ Vout, int h, int C, long long Ti,
                                                          long long To) {
    using WI = WinoT<MI>;
    using WO = WinoT<MO>;
    constexpr int NI = WI::N, NO = WO::N;
    extern __shared__ float ys_raw[];  // [h * h][64]
    float(*ys)[64] = reinterpret_cast<float(*)[64]>(ys_raw);
    const int lane = threadIdx.x;
    const int cblocks = C / 64;
    const long long b = blockIdx.x / cblocks;
    const int c = (blockIdx.x % cblocks) * 64 + lane;
    const int ti = (h + MI - 1) / MI, to = (h - 2 + MO - 1) / MO;  // tiles per side: layer i, layer i+1
    const float bc = bias[c];
    for (int ty = 0; ty < ti; ++ty)
        for (int tx = 0; tx < ti; ++tx) {
            const long long t = (b * ti + ty) * ti + tx;
            float mm[NI][NI];
#pragma unroll
            for (int e = 0; e < NI * NI; ++e) mm[e / NI][e % NI] = Min[((long long)e * Ti + t) * C + c];
            float sr[MI][NI];
#pragma unroll
            for (int v = 0; v < NI; ++v)
#pragma unroll
                for (int a = 0; a < MI; ++a) {
                    float acc = 0.f;
                    bool first = true;
#pragma unroll
                    for (int u = 0; u < NI; ++u) {
                        if (WI::AT[a][u] == 0.f) continue;
                        const float term = WI::AT[a][u] == 1.f ? mm[u][v] : WI::AT[a][u] * mm[u][v];
                        acc = first ? term : acc + term;
                        first = false;
                    }
                    sr[a][v] = acc;
                }
#pragma unroll
            for (int a = 0; a < MI; ++a)
#pragma unroll
                for (int q = 0; q < MI; ++q) {
                    const int oy = MI * ty + a, ox = MI * tx + q;
                    if (oy < h && ox < h) {
                        float acc = 0.f;
                        bool first = true;
#pragma unroll
                        for (int v = 0; v < NI; ++v) {
                            if (WI::AT[q][v] == 0.f) continue;
                            const float term = WI::AT[q][v] == 1.f ? sr[a][v] : WI::AT[q][v] * sr[a][v];
                            acc = first ? term : acc + term;
                            first = false;
                        }
                        ys[oy * h + ox][lane] = fmaxf(acc + bc, 0.f);
                    }
                }
        }
    for (int ty = 0; ty < to; ++ty)
        for (int tx = 0; tx < to; ++tx) {
            const long long t = (b * to + ty) * to + tx;
            float d[NO][NO];
#pragma unroll
            for (int u = 0; u < NO; ++u)
#pragma unroll
                for (int v = 0; v < NO; ++v) {
                    const int iy = MO * ty + u, ix = MO * tx + v;
                    d[u][v] = (iy < h && ix < h) ? ys[iy * h + ix][lane] : 0.f;
                }
            float sr[NO][NO];
#pragma unroll
            for (int v = 0; v < NO; ++v)
#pragma unroll
                for (int a = 0; a < NO; ++a) {
                    float acc = 0.f;
                    bool first = true;
#pragma unroll
                    for (int u = 0; u < NO; ++u) {
                        if (WO::BT[a][u] == 0.f) continue;
                        const float term = WO::BT[a][u] == 1.f ? d[u][v] : WO::BT[a][u] * d[u][v];
                        acc = first ? term : acc + term;
                        first = false;
                    }
                    sr[a][v] = acc;
                }
#pragma unroll
            for (int a = 0; a < NO; ++a)
#pragma unroll
                for (int bb = 0; bb < NO; ++bb) {
                    float acc = 0.f;
                    bool first = true;
#pragma unroll
                    for (int v = 0; v < NO; ++v) {
                        if (WO::BT[bb][v] == 0.f) continue;
                        const float term = WO::BT[bb][v] == 1.f ? sr[a][v] : WO::BT[bb][v] * sr[a][v];
                        acc = first ? term : acc + term;
                        first = false;
                    }
                    Vout[((long long)(a * NO + bb) * To + t) * C + c] = acc;
                }
        }
}

// The network's first two layers' front end in one pass: conv1 (depth -> C
// channels, 3x3, pad 1) + bias + ReLU computed directly from the NCHW leaf
// planes, then conv2's Winograd input transform (pad 1) -- conv1's activation
// never leaves the chip.  One wave per (image, 64 output channels of conv1),
// one channel per lane: the image's planes are shared through LDS, the lane's
// depth*9 weights sit in registers, its n x n output plane in its own LDS
// column (no barrier needed for it).
template <int MO>
__global__ __launch_bounds__(64) void winograd_first_kernel(const float* __restrict__ planes,
                                                            const float* __restrict__ w1,
                                                            const float* __restrict__ b1, float* __restrict__ Vout,
                                                            int depth, int n, int C, long long To) {
    using WO = WinoT<MO>;
    constexpr int NO = WO::N;
    constexpr int DMAX = 4;
    extern __shared__ float lds[];
    float* xs = lds;                                               // [depth][n][n]
    float(*ys)[64] = reinterpret_cast<float(*)[64]>(lds + DMAX * 81);  // [n * n][64]
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
    for (int y = 0; y < n; ++y)
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
            ys[y * n + x][lane] = fmaxf(acc + bk, 0.f);
        }
    const int to = (n + MO - 1) / MO;  // conv2: pad 1, n x n outputs
    for (int ty = 0; ty < to; ++ty)
        for (int tx = 0; tx < to; ++tx) {
            const long long t = (b * to + ty) * to + tx;
            float d[NO][NO];
#pragma unroll
            for (int u = 0; u < NO; ++u)
#pragma unroll
                for (int v = 0; v < NO; ++v) {
                    const int iy = MO * ty - 1 + u, ix = MO * tx - 1 + v;
                    d[u][v] = (iy >= 0 && iy < n && ix >= 0 && ix < n) ? ys[iy * n + ix][lane] : 0.f;
                }
            float sr[NO][NO];
#pragma unroll
            for (int v = 0; v < NO; ++v)
#pragma unroll
                for (int a = 0; a < NO; ++a) {
                    float acc = 0.f;
                    bool first = true;
#pragma unroll
                    for (int u = 0; u < NO; ++u) {
                        if (WO::BT[a][u] == 0.f) continue;
                        const float term = WO::BT[a][u] == 1.f ? d[u][v] : WO::BT[a][u] * d[u][v];
                        acc = first ? term : acc + term;
                        first = false;
                    }
                    sr[a][v] = acc;
                }
#pragma unroll
            for (int a = 0; a < NO; ++a)
#pragma unroll
                for (int bb = 0; bb < NO; ++bb) {
                    float acc = 0.f;
                    bool first = true;
#pragma unroll
                    for (int v = 0; v < NO; ++v) {
                        if (WO::BT[bb][v] == 0.f) continue;
                        const float term = WO::BT[bb][v] == 1.f ? sr[a][v] : WO::BT[bb][v] * sr[a][v];
                        acc = first ? term : acc + term;
                        first = false;
                    }
                    Vout[((long long)(a * NO + bb) * To + t) * C + k] = acc;
                }
        }
}

// one thread per work item, rounded up to whole groups of 8 blocks (xcd_item)
unsigned grid_for(long long n) {
    const long long blocks = (n + 255) / 256;
    return (unsigned)(((blocks + 7) / 8) * 8);
}
}  // namespace

extern "C" int azg_winograd_in_nhwc(const float* x, const float* in_bias, float* V, int32_t batch, int32_t h_in,
                                    int32_t pad, int32_t c, int32_t m, void* stream) {
    const int h_out = h_in + 2 * pad - 2;
    if (!x || !V || batch <= 0 || h_out <= 0 || c <= 0 || c % 4 || (m != 2 && m != 3) || ((uintptr_t)x & 15) ||
        ((uintptr_t)V & 15) || ((uintptr_t)in_bias & 15) ||
        (long long)batch * ((h_out + m - 1) / m) * ((h_out + m - 1) / m) * (c / 4) > (1ll << 38))
        return AZG_ERR_ARG;
    const int tiles = (h_out + m - 1) / m;
    const long long T = (long long)batch * tiles * tiles;
    if (m == 2)
        hipLaunchKernelGGL(winograd_in_kernel<2>, dim3(grid_for(T * (c / 4))), dim3(256), 0, (hipStream_t)stream,
                           (const float4*)x, (const float4*)in_bias, (float4*)V, h_in, pad, c / 4, tiles, T);
    else
        hipLaunchKernelGGL(winograd_in_kernel<3>, dim3(grid_for(T * (c / 4))), dim3(256), 0, (hipStream_t)stream,
                           (const float4*)x, (const float4*)in_bias, (float4*)V, h_in, pad, c / 4, tiles, T);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_winograd_out_nhwc(const float* M, const float* bias, float* y, int32_t batch, int32_t h_out,
                                     int32_t k, int32_t m, int32_t relu, void* stream) {
    if (!M || !bias || !y || batch <= 0 || h_out <= 0 || k <= 0 || k % 4 || (m != 2 && m != 3) ||
        ((uintptr_t)M & 15) || ((uintptr_t)bias & 15) || ((uintptr_t)y & 15) ||
        (long long)batch * ((h_out + m - 1) / m) * ((h_out + m - 1) / m) * (k / 4) > (1ll << 38))
        return AZG_ERR_ARG;
    const int tiles = (h_out + m - 1) / m;
    const long long T = (long long)batch * tiles * tiles;
    if (m == 2)
        hipLaunchKernelGGL(winograd_out_kernel<2>, dim3(grid_for(T * (k / 4))), dim3(256), 0, (hipStream_t)stream,
                           (const float4*)M, (const float4*)bias, (float4*)y, h_out, k / 4, tiles, T, relu);
    else
        hipLaunchKernelGGL(winograd_out_kernel<3>, dim3(grid_for(T * (k / 4))), dim3(256), 0, (hipStream_t)stream,
                           (const float4*)M, (const float4*)bias, (float4*)y, h_out, k / 4, tiles, T, relu);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_winograd_mid_nhwc(const float* M, const float* bias, float* V, int32_t batch, int32_t h, int32_t c,
                                     int32_t m_in, int32_t m_out, void* stream) {
    if (!M || !bias || !V || batch <= 0 || h < 3 || h > 9 || c <= 0 || c % 64 || (m_in != 2 && m_in != 3) ||
        (m_out != 2 && m_out != 3))
        return AZG_ERR_ARG;
    const int ti = (h + m_in - 1) / m_in, to = (h - 2 + m_out - 1) / m_out;
    const long long Ti = (long long)batch * ti * ti, To = (long long)batch * to * to;
    const dim3 grid((unsigned)(batch * (c / 64)));
    const size_t lds = (size_t)h * h * 64 * sizeof(float);
    hipStream_t st = (hipStream_t)stream;
    if (m_in == 2 && m_out == 2)
        hipLaunchKernelGGL((winograd_mid_kernel<2, 2>), grid, dim3(64), lds, st, M, bias, V, h, c, Ti, To);
    else if (m_in == 2)
        hipLaunchKernelGGL((winograd_mid_kernel<2, 3>), grid, dim3(64), lds, st, M, bias, V, h, c, Ti, To);
    else if (m_out == 2)
        hipLaunchKernelGGL((winograd_mid_kernel<3, 2>), grid, dim3(64), lds, st, M, bias, V, h, c, Ti, To);
    else
        hipLaunchKernelGGL((winograd_mid_kernel<3, 3>), grid, dim3(64), lds, st, M, bias, V, h, c, Ti, To);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_winograd_first_nchw(const float* planes, const float* w1, const float* b1, float* V, int32_t batch,
                                       int32_t depth, int32_t n, int32_t c, int32_t m, void* stream) {
    if (!planes || !w1 || !b1 || !V || batch <= 0 || depth < 1 || depth > 4 || n < 3 || n > 9 || c <= 0 ||
        c % 64 || (m != 2 && m != 3))
        return AZG_ERR_ARG;
    const int to = (n + m - 1) / m;
    const long long To = (long long)batch * to * to;
    const dim3 grid((unsigned)(batch * (c / 64)));
    const size_t lds = (4 * 81 + (size_t)n * n * 64) * sizeof(float);
    hipStream_t st = (hipStream_t)stream;
    if (m == 2)
        hipLaunchKernelGGL(winograd_first_kernel<2>, grid, dim3(64), lds, st, planes, w1, b1, V, depth, n, c, To);
    else
        hipLaunchKernelGGL(winograd_first_kernel<3>, grid, dim3(64), lds, st, planes, w1, b1, V, depth, n, c, To);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}
