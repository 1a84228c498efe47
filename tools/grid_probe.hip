// Launch-size probe: a grid of more than 2^32 - 1 work-items is not refused by
// the runtime -- it runs (grid mod 2^32) work-items and reports success.
// Why kernels.hip cuts one-shot grids at kMaxGridBlocks.
//   hipcc -O2 --offload-arch=gfx950 tools/grid_probe.hip -o tools/bin/grid_probe
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned *c) { if (threadIdx.x == 0) atomicAdd(c, 1u); }
int main() {
    unsigned *c = nullptr;
    if (hipMalloc(&c, 4) != hipSuccess) return 1;
    for (unsigned blocks : {67108863u, 67109863u, 2147483647u}) {
        if (hipMemset(c, 0, 4) != hipSuccess) return 1;
        hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, c);
        hipError_t e = hipGetLastError();
        hipError_t e2 = hipDeviceSynchronize();
        unsigned h = 0;
        if (hipMemcpy(&h, c, 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        printf("blocks %u x 64: launch %s, sync %s, blocks run %u\n", blocks, hipGetErrorString(e), hipGetErrorString(e2), h);
    }
}
