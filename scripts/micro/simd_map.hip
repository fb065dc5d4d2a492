// Which SIMD each wave of a workgroup lands on (HW_ID: SIMD_ID bits 5:4, CU_ID 11:8,
// SE_ID 15:13), for the lane kernels' workgroup shapes: 4, 6 and 8 waves with enough
// LDS that one workgroup takes a CU.  The lane kernels place their parser and
// reconstruction waves by wave index, assuming wave w runs on SIMD w % 4.
// hipcc --offload-arch=gfx950 -O3 simd_map.hip -o simd_map && ./simd_map
#include <hip/hip_runtime.h>
#include <cstdio>

template <int NT>
__global__ void __launch_bounds__(NT) k_map(unsigned *out) {
    __shared__ unsigned pad[100 * 1024 / 4];  // one workgroup per CU
    if (threadIdx.x == 0) pad[0] = 0;
    __syncthreads();
    const unsigned id = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 4);  // HW_ID bits 15:0 (size 16)
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + (threadIdx.x >> 6)] = id + pad[0];
}

template <int NT>
void run(unsigned *d, unsigned *h) {
    const int nb = 64, nw = NT / 64;
    hipMemset(d, 0xFF, 64 * 8 * sizeof(unsigned));
    hipLaunchKernelGGL(k_map<NT>, dim3(nb), dim3(NT), 0, 0, d);
    hipMemcpy(h, d, 64 * 8 * sizeof(unsigned), hipMemcpyDeviceToHost);
    int counts[8][4] = {};
    for (int b = 0; b < nb; b++)
        for (int w = 0; w < nw; w++) counts[w][(h[b * 8 + w] >> 4) & 3]++;
    printf("%d waves per workgroup: wave -> SIMD histogram over %d workgroups\n", nw, nb);
    for (int w = 0; w < nw; w++)
        printf("  wave %d: simd0 %2d simd1 %2d simd2 %2d simd3 %2d\n", w, counts[w][0], counts[w][1], counts[w][2],
               counts[w][3]);
    printf("  workgroup 0:");
    for (int w = 0; w < nw; w++) printf(" w%d=simd%u/cu%u/se%u", w, (h[w] >> 4) & 3, (h[w] >> 8) & 15, (h[w] >> 13) & 7);
    printf("\n");
}

int main() {
    unsigned *d, h[64 * 8];
    hipMalloc(&d, sizeof(h));
    run<256>(d, h);
    run<384>(d, h);
    run<512>(d, h);
    return 0;
}
