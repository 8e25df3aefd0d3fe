// occupancy probe: what the HIP occupancy API reports for a 256-thread kernel vs dynamic LDS size
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(256) void dummy(double* p) {
  extern __shared__ double s[];
  s[threadIdx.x] = p[threadIdx.x];
  __syncthreads();
  p[threadIdx.x] = s[255 - threadIdx.x];
}
int main() {
  hipDeviceProp_t pr;
  (void)hipGetDeviceProperties(&pr, 0);
  printf("CUs %d sharedMemPerBlock %zu sharedMemPerMultiprocessor %zu maxSharedMemoryPerMultiProcessor %zu\n",
         pr.multiProcessorCount, pr.sharedMemPerBlock, pr.sharedMemPerMultiprocessor, pr.maxSharedMemoryPerMultiProcessor);
  for (int kb : {8, 16, 24, 32, 36, 40, 48, 64, 72, 96, 128, 160}) {
    int n = -1;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(dummy), 256, (size_t)kb * 1024);
    printf("lds %3d KiB -> %d blocks/CU (%s)\n", kb, n, hipGetErrorString(e));
  }
  return 0;
}
