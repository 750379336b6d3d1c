// azg_winograd.hip -- the leaf network's 3x3 convolutions as Winograd F(2x2, 3x3).
//
// conv2-4 of InflexionNNet.forward (InflexionNNet.py:43-45, BN folded) are
// y = relu(bias + conv3x3(x, w)).  With 2x2 output tiles, each tile is
//     Y = A^T [ U (.) V ] A,   U = G g G^T (per (c, k)),   V = B^T d B (per (tile, c)),
// and the sum over input channels c of U (.) V is, for each of the 16 tile
// positions e, one GEMM  M_e[T x K] = V_e[T x C] x U_e[C x K]  (T = tiles).
// That is 16 x 2 T C K multiply-adds instead of 36 per 2x2 outputs: 2.25x
// fewer, less the tile padding (7x7 outputs -> 4x4 tiles: 1.72x; 5x5: 1.56x;
// 3x3: 1.27x).  The GEMMs are f32 (hipBLASLt through torch.bmm); these
// kernels are the two transforms, HBM-bound and coalesced (4 channels per
// lane as float4, consecutive lanes on consecutive channels):
//   * winograd_in : NHWC input (zero padding) -> V [16][T][C]
//   * winograd_out: M [16][T][K] -> NHWC output, bias + ReLU fused, tile
//                   padding cropped.
// The transforms only add and subtract (B, A have entries 0, +-1), so the f32
// results differ from a direct convolution by summation order alone; U is
// formed in f64 by the caller (G has entries 1/2).
#include <hip/hip_runtime.h>

#include "../../include/azg.h"

namespace {

__device__ __forceinline__ float4 f4add(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float4 f4sub(float4 a, float4 b) { return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }

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
__global__ __launch_bounds__(256) void winograd_in_kernel(const float4* __restrict__ x,
                                                          const float4* __restrict__ in_bias, float4* __restrict__ V,
                                                          int H, int pad, int C4, int tiles, long long T) {
    const long long n = T * C4;
    {
        const long long i = xcd_item();
        if (i >= n) return;
        const int c4 = (int)(i % C4);
        const long long t = i / C4;
        const int tx = (int)(t % tiles);
        const long long r = t / tiles;
        const int ty = (int)(r % tiles);
        const long long b = r / tiles;
        const float4 ib = in_bias ? in_bias[c4] : make_float4(0.f, 0.f, 0.f, 0.f);
        float4 d[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int iy = 2 * ty - pad + u;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int ix = 2 * tx - pad + v;
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
        // B^T d: rows (d0 - d2, d1 + d2, d2 - d1, d1 - d3)
        float4 s[4][4];
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            s[0][v] = f4sub(d[0][v], d[2][v]);
            s[1][v] = f4add(d[1][v], d[2][v]);
            s[2][v] = f4sub(d[2][v], d[1][v]);
            s[3][v] = f4sub(d[1][v], d[3][v]);
        }
        // (B^T d) B: the same on columns
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const float4 v0 = f4sub(s[u][0], s[u][2]), v1 = f4add(s[u][1], s[u][2]);
            const float4 v2 = f4sub(s[u][2], s[u][1]), v3 = f4sub(s[u][1], s[u][3]);
            V[((long long)(u * 4 + 0) * T + t) * C4 + c4] = v0;
            V[((long long)(u * 4 + 1) * T + t) * C4 + c4] = v1;
            V[((long long)(u * 4 + 2) * T + t) * C4 + c4] = v2;
            V[((long long)(u * 4 + 3) * T + t) * C4 + c4] = v3;
        }
    }
}

__global__ __launch_bounds__(256) void winograd_out_kernel(const float4* __restrict__ M, const float4* __restrict__ bias,
                                                           float4* __restrict__ y, int Ho, int K4, int tiles,
                                                           long long T, int relu) {
    const long long n = T * K4;
    {
        const long long i = xcd_item();
        if (i >= n) return;
        const int k4 = (int)(i % K4);
        const long long t = i / K4;
        const int tx = (int)(t % tiles);
        const long long r = t / tiles;
        const int ty = (int)(r % tiles);
        const long long b = r / tiles;
        float4 m[4][4];
#pragma unroll
        for (int e = 0; e < 16; ++e) m[e / 4][e % 4] = M[((long long)e * T + t) * K4 + k4];
        // A^T m: rows (m0 + m1 + m2, m1 - m2 - m3)
        float4 s[2][4];
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            s[0][v] = f4add(f4add(m[0][v], m[1][v]), m[2][v]);
            s[1][v] = f4sub(f4sub(m[1][v], m[2][v]), m[3][v]);
        }
        const float4 bb = bias[k4];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            float4 o[2];
            o[0] = f4add(f4add(s[u][0], s[u][1]), s[u][2]);
            o[1] = f4sub(f4sub(s[u][1], s[u][2]), s[u][3]);
            const int oy = 2 * ty + u;
#pragma unroll
            for (int v = 0; v < 2; ++v) {
                const int ox = 2 * tx + v;
                if (oy < Ho && ox < Ho) {
                    float4 z = f4add(o[v], bb);
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
}

// one thread per work item, rounded up to whole groups of 8 blocks (xcd_item)
unsigned grid_for(long long n) {
    const long long blocks = (n + 255) / 256;
    return (unsigned)(((blocks + 7) / 8) * 8);
}
}  // namespace

extern "C" int azg_winograd_in_nhwc(const float* x, const float* in_bias, float* V, int32_t batch, int32_t h_in,
                                    int32_t pad, int32_t c, void* stream) {
    const int h_out = h_in + 2 * pad - 2;
    if (!x || !V || batch <= 0 || h_out <= 0 || c <= 0 || c % 4 || ((uintptr_t)x & 15) || ((uintptr_t)V & 15) ||
        ((uintptr_t)in_bias & 15) ||
        (long long)batch * ((h_out + 1) / 2) * ((h_out + 1) / 2) * (c / 4) > (1ll << 38))
        return AZG_ERR_ARG;
    const int tiles = (h_out + 1) / 2;
    const long long T = (long long)batch * tiles * tiles;
    hipLaunchKernelGGL(winograd_in_kernel, dim3(grid_for(T * (c / 4))), dim3(256), 0, (hipStream_t)stream,
                       (const float4*)x, (const float4*)in_bias, (float4*)V, h_in, pad, c / 4, tiles, T);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}

extern "C" int azg_winograd_out_nhwc(const float* M, const float* bias, float* y, int32_t batch, int32_t h_out,
                                     int32_t k, int32_t relu, void* stream) {
    if (!M || !bias || !y || batch <= 0 || h_out <= 0 || k <= 0 || k % 4 || ((uintptr_t)M & 15) ||
        ((uintptr_t)bias & 15) || ((uintptr_t)y & 15) ||
        (long long)batch * ((h_out + 1) / 2) * ((h_out + 1) / 2) * (k / 4) > (1ll << 38))
        return AZG_ERR_ARG;
    const int tiles = (h_out + 1) / 2;
    const long long T = (long long)batch * tiles * tiles;
    hipLaunchKernelGGL(winograd_out_kernel, dim3(grid_for(T * (k / 4))), dim3(256), 0, (hipStream_t)stream,
                       (const float4*)M, (const float4*)bias, (float4*)y, h_out, k / 4, tiles, T, relu);
    return hipGetLastError() == hipSuccess ? 0 : AZG_ERR_HIP;
}
