// Launch-cost microbenchmark: empty-ish kernels at the render kernel's shape (256 threads,
// 128 VGPRs, 3 KB LDS) over grid sizes, timed with HIP events.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void k_empty(int* out) {
    if (threadIdx.x == 1000) out[0] = 1;
}

__global__ __launch_bounds__(256, 4) void k_vgpr(int* out, float s) {
    asm volatile("" ::: "v127");  // allocate 128 VGPRs like the render kernel
    if (threadIdx.x == 1000) out[0] = (int)s;
}

__global__ __launch_bounds__(256) void k_lds(int* out) {
    __shared__ float col[768];
    col[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (col[(threadIdx.x + 1) % 256] == 1000.f) out[0] = 1;
}

int main() {
    int* d;
    (void)hipMalloc(&d, 64);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int grid : {2048, 8192, 32768, 131072}) {
        for (int which = 0; which < 3; ++which) {
            float best = 1e9f;
            for (int rep = 0; rep < 10; ++rep) {
                (void)hipEventRecord(a, 0);
                if (which == 0) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, 0, d);
                if (which == 1) hipLaunchKernelGGL(k_vgpr, dim3(grid), dim3(256), 0, 0, d, 1.0f);
                if (which == 2) hipLaunchKernelGGL(k_lds, dim3(grid), dim3(256), 0, 0, d);
                (void)hipEventRecord(b, 0);
                (void)hipEventSynchronize(b);
                float ms;
                (void)hipEventElapsedTime(&ms, a, b);
                if (ms < best) best = ms;
            }
            printf("grid %7d kernel %s: %.1f us\n", grid, which == 0 ? "empty" : which == 1 ? "vgpr " : "lds  ",
                   best * 1e3f);
        }
    }
    return 0;
}
