// Blocks per CU that the runtime admits for a 512-thread kernel at a given dynamic LDS size
// (does the padded column image, 77,824 B, still fit two blocks in gfx950's 160 KB?).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void __launch_bounds__(512) k_dummy(float* o) {
    extern __shared__ float sm[];
    sm[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (o) o[threadIdx.x] = sm[511 - threadIdx.x];
}
int main() {
    hipFuncSetAttribute((const void*)k_dummy, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    const int sizes[] = {65536, 73728, 74752, 75776, 76800, 77824, 78848, 79872, 81920, 81921};
    for (int b : sizes) {
        int n = -1;
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_dummy, 512, b);
        printf("lds %6d B: %d blocks/CU (%s)\n", b, n, hipGetErrorString(e));
    }
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    printf("sharedMemPerMultiprocessor %zu, sharedMemPerBlock %zu, maxSharedMemoryPerMultiProcessor %zu\n",
           p.sharedMemPerMultiprocessor, p.sharedMemPerBlock, p.maxSharedMemoryPerMultiProcessor);
    return 0;
}
