#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void __launch_bounds__(256) k(float* o) {
    extern __shared__ float s[];
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    o[threadIdx.x] = s[255 - threadIdx.x];
}
int main() {
    for (int b : {40000, 48000, 52000, 53000, 54000, 54528, 54613, 55000, 56000, 65536, 80008, 81920}) {
        int nb = 0;
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, 256, b);
        printf("lds %d -> %d blocks/CU\n", b, nb);
    }
    hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
    printf("sharedMemPerMultiprocessor %zu maxSharedMemoryPerMultiProcessor %zu\n", p.sharedMemPerBlock, p.maxSharedMemoryPerMultiProcessor);
    return 0;
}
