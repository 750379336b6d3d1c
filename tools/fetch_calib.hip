// FETCH_SIZE calibration probe: reads of a KNOWN number of bytes at the
// access widths the tree kernels use (4-B and 8-B lanes) and at the 16-B streaming width the
// gfx950 correction of MI355X_MICROARCH.md was calibrated on, so rocprofv3's FETCH_SIZE can be
// compared with the bytes that crossed HBM for each width.  Every line of the buffer is read
// exactly once, whole (a wave reads 64 consecutive elements), from a buffer far larger than the
// caches; the sum goes to one store per wave so nothing is optimised away.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

template <class T>
__global__ __launch_bounds__(256) void read_kernel(const T* __restrict__ x, long long n, float* __restrict__ out) {
    float acc = 0.f;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const T v = x[i];
        if constexpr (sizeof(T) == 4) acc += __uint_as_float((unsigned)v);
        else if constexpr (sizeof(T) == 8) acc += __uint_as_float((unsigned)v) + __uint_as_float((unsigned)(v >> 32));
        else acc += v.x + v.y + v.z + v.w;
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) out[(blockIdx.x * 256 + threadIdx.x) / 64] = acc;
}

}  // namespace

// width 4, 8 or 16 bytes per lane; bytes read = n_bytes (a multiple of 16); out: grid * 4 floats
extern "C" int fetch_calib_read(const void* x, long long n_bytes, int width, float* out, int grid, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (width == 4)
        hipLaunchKernelGGL(read_kernel<unsigned>, dim3(grid), dim3(256), 0, st, (const unsigned*)x, n_bytes / 4, out);
    else if (width == 8)
        hipLaunchKernelGGL(read_kernel<unsigned long long>, dim3(grid), dim3(256), 0, st,
                           (const unsigned long long*)x, n_bytes / 8, out);
    else if (width == 16)
        hipLaunchKernelGGL(read_kernel<float4>, dim3(grid), dim3(256), 0, st, (const float4*)x, n_bytes / 16, out);
    else
        return -1;
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
