// Work-queue grab cost: persistent waves (one per 64-thread workgroup) pull item indices from
// Q counters with one returning atomicAdd per item (lane 0, readfirstlane), do `spin` cycles of
// dummy work per item, until N items are taken.  Prints wall time (HIP events) per (Q, grid,
// spin), against the same items without a queue (static striding).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(64) void queue_kernel(unsigned* ctr, int q, int n_per_q, int spin, unsigned* sink) {
    const int home = blockIdx.x % q;
    unsigned acc = 0;
    for (int k = 0; k < q; ++k) {
        const int list = (home + k) % q;
        while (true) {
            unsigned j = 0;
            if (threadIdx.x == 0) j = atomicAdd(&ctr[list * 64], 1u);
            j = __builtin_amdgcn_readfirstlane(j);
            if ((int)j >= n_per_q) break;
            const long long t0 = wall_clock64();
            while (wall_clock64() - t0 < spin) acc += j;
        }
    }
    if (acc == 0xFFFFFFFFu) sink[0] = acc;
}

__global__ __launch_bounds__(64) void static_kernel(int n, int spin, unsigned* sink) {
    unsigned acc = 0;
    for (int j = blockIdx.x; j < n; j += gridDim.x) {
        const long long t0 = wall_clock64();
        while (wall_clock64() - t0 < spin) acc += j;
    }
    if (acc == 0xFFFFFFFFu) sink[0] = acc;
}

int main() {
    unsigned *ctr, *sink;
    (void)hipMalloc(&ctr, 64 * 64 * sizeof(unsigned));
    (void)hipMalloc(&sink, 64);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int N = 100000;
    // wall_clock64 runs at 100 MHz: spin 100 = 1 us of work per item
    for (int spin : {0, 100, 500}) {
        for (int grid : {2048, 6144}) {
            for (int q : {1, 8, 32}) {
                float best = 1e9f;
                for (int rep = 0; rep < 5; ++rep) {
                    (void)hipMemset(ctr, 0, 64 * 64 * sizeof(unsigned));
                    (void)hipEventRecord(a, 0);
                    hipLaunchKernelGGL(queue_kernel, dim3(grid), dim3(64), 0, 0, ctr, q, N / q, spin, sink);
                    (void)hipEventRecord(b, 0);
                    (void)hipEventSynchronize(b);
                    float ms;
                    (void)hipEventElapsedTime(&ms, a, b);
                    if (ms < best) best = ms;
                }
                printf("queue  spin %4d grid %5d q %2d: %8.1f us  (%.1f ns per item)\n", spin, grid, q, best * 1e3f,
                       best * 1e6f / N);
            }
            float best = 1e9f;
            for (int rep = 0; rep < 5; ++rep) {
                (void)hipEventRecord(a, 0);
                hipLaunchKernelGGL(static_kernel, dim3(grid), dim3(64), 0, 0, N, spin, sink);
                (void)hipEventRecord(b, 0);
                (void)hipEventSynchronize(b);
                float ms;
                (void)hipEventElapsedTime(&ms, a, b);
                if (ms < best) best = ms;
            }
            printf("static spin %4d grid %5d     : %8.1f us\n", spin, grid, best * 1e3f);
        }
    }
    return 0;
}
