// PMC calibration kernels: known byte counts in the access patterns the ADMM passes use,
// so rocprofv3 FETCH_SIZE / WRITE_SIZE can be converted to bytes (MI355X_MICROARCH.md §HBM:
// only 16-B/lane streaming is calibrated there).  Tools only, not part of the product.
#include <hip/hip_runtime.h>
#include <cstdint>

// pass-A-like: one 8-byte element per lane, consecutive lanes consecutive (512 B per wave-instruction)
__global__ void calib_copy8(const float2* __restrict__ a, float2* __restrict__ b, long long n) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        b[i] = a[i];
}
// the same with non-temporal loads and stores (pass A's cache policy, ADMM_NT)
typedef float v2f __attribute__((ext_vector_type(2)));
__global__ void calib_copy8nt(const float2* __restrict__ a, float2* __restrict__ b, long long n) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        __builtin_nontemporal_store(__builtin_nontemporal_load(reinterpret_cast<const v2f*>(a) + i),
                                    reinterpret_cast<v2f*>(b) + i);
}
// 16-byte per lane streaming (the guide's calibrated case)
__global__ void calib_copy16(const float4* __restrict__ a, float4* __restrict__ b, long long n) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        b[i] = a[i];
}
// pass-B-like: blocks of 8 columns x 64 threads; element (row, col) of an H x N complex plane,
// rows t + 64 j (64-byte segments per row)
__global__ void calib_cols(const float2* __restrict__ a, float2* __restrict__ b, int H, int N, int colblocks) {
    const int c = threadIdx.x % 8, t = threadIdx.x / 8;
    const int p = blockIdx.x / colblocks, cb = blockIdx.x % colblocks;
    const size_t base = (size_t)p * H * N + cb * 8 + c;
    for (int j = 0; j < H / 64; ++j) {
        const size_t i = base + (size_t)(t + 64 * j) * N;
        b[i] = a[i];
    }
}

extern "C" int calib_run(int kind, const void* a, void* b, long long bytes, int H, int N, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    if (kind == 0) {
        hipLaunchKernelGGL(calib_copy8, dim3(8192), dim3(256), 0, s, (const float2*)a, (float2*)b, bytes / 8);
    } else if (kind == 1) {
        hipLaunchKernelGGL(calib_copy16, dim3(8192), dim3(256), 0, s, (const float4*)a, (float4*)b, bytes / 16);
    } else if (kind == 3) {
        hipLaunchKernelGGL(calib_copy8nt, dim3(8192), dim3(256), 0, s, (const float2*)a, (float2*)b, bytes / 8);
    } else {
        const long long planes = bytes / ((long long)H * N * 8);
        const int cbs = N / 8;
        hipLaunchKernelGGL(calib_cols, dim3((unsigned)(planes * cbs)), dim3(512), 0, s, (const float2*)a, (float2*)b, H, N, cbs);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
