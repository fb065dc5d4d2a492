// PCIe rates: DMA-engine copies (hipMemcpyAsync) against CU-driven copies (a kernel storing 16 B per
// lane into page-locked host memory / loading from it), each direction alone and both at once.
// hipcc --offload-arch=gfx950 -O3 pcie_kernel.hip -o pcie_kernel && ./pcie_kernel [MB]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

__global__ void __launch_bounds__(256) copy16(const uint4 *__restrict__ s, uint4 *__restrict__ d, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) d[i] = s[i];
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main(int argc, char **argv) {
    const size_t mb = argc > 1 ? atoi(argv[1]) : 90, n = mb << 20;
    uint8_t *hd, *hu, *dd, *du;
    CK(hipHostMalloc((void **)&hd, n, hipHostMallocDefault));
    CK(hipHostMalloc((void **)&hu, n, hipHostMallocDefault));
    CK(hipMalloc((void **)&dd, n));
    CK(hipMalloc((void **)&du, n));
    CK(hipMemset(dd, 1, n));
    for (size_t i = 0; i < n; i++) hu[i] = (uint8_t)i;
    void *hdd, *hud;
    CK(hipHostGetDevicePointer(&hdd, hd, 0));
    CK(hipHostGetDevicePointer(&hud, hu, 0));
    hipStream_t s1, s2;
    CK(hipStreamCreate(&s1));
    CK(hipStreamCreate(&s2));
    const int reps = 10;
    auto run = [&](const char *name, int mode) {
        for (int w = 0; w < 2; w++) {
            CK(hipDeviceSynchronize());
            auto t0 = std::chrono::steady_clock::now();
            for (int r = 0; r < reps; r++) {
                if (mode & 1) CK(hipMemcpyAsync(hd, dd, n, hipMemcpyDeviceToHost, s1));                   // D2H dma
                if (mode & 2) CK(hipMemcpyAsync(du, hu, n, hipMemcpyHostToDevice, s2));                   // H2D dma
                if (mode & 4) hipLaunchKernelGGL(copy16, dim3(1024), dim3(256), 0, s1, (const uint4 *)dd, (uint4 *)hdd, n / 16);  // D2H kernel
                if (mode & 8) hipLaunchKernelGGL(copy16, dim3(1024), dim3(256), 0, s2, (const uint4 *)hud, (uint4 *)du, n / 16);  // H2D kernel
            }
            CK(hipDeviceSynchronize());
            const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            int dirs = ((mode & 5) ? 1 : 0) + ((mode & 10) ? 1 : 0);
            if (w) printf("{\"case\": \"%s\", \"GBs_total\": %.2f}\n", name, (double)n * reps * dirs / s / 1e9);
        }
    };
    run("d2h dma", 1);
    run("d2h kernel", 4);
    run("h2d dma", 2);
    run("h2d kernel", 8);
    run("both dma", 3);
    run("d2h kernel + h2d dma", 6);
    run("both kernel", 12);
    if (hd[n - 1] != 1) printf("bad d2h\n");
    return 0;
}
