// Kernel-to-kernel gap on one stream (the c3 frame loop's ~16 us between render kernels,
// profiles/r05/exp/trace_bench_c3.log): K1 spins ~100 us on every CU and optionally writes
// `mb` MB (plain or nontemporal stores), K2 is an empty-ish kernel.  The gap is measured on the
// device: K1's waves atomicMax their end time, K2's atomicMin their start time (wall_clock64,
// 100 MHz).  Variants: plain launches; K1 launched with hipExtLaunchKernel start/stop events
// (as the render kernel is); K2 behind a hipStreamWaitEvent on an event another stream already
// completed (the render kernel's pdone wait).
// Build: hipcc --offload-arch=gfx950 -O3 scripts/micro/kernel_gap.hip -o build/kernel_gap
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>

__global__ __launch_bounds__(256) void k1(unsigned long long* t, int spin_ticks, unsigned char* buf, size_t bytes,
                                         int nt) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < (unsigned long long)spin_ticks) {
    }
    // write `bytes` spread over the grid, 4 bytes per lane per step
    const size_t n4 = bytes / 4, stride = (size_t)gridDim.x * blockDim.x;
    unsigned* b4 = reinterpret_cast<unsigned*>(buf);
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        if (nt) __builtin_nontemporal_store((unsigned)i, b4 + i);
        else b4[i] = (unsigned)i;
    }
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(&t[0], wall_clock64());
}

__global__ __launch_bounds__(256) void k2(unsigned long long* t) {
    if (threadIdx.x == 0) {
        const unsigned long long now = wall_clock64();
        atomicMin(&t[1], now);
        atomicMax(&t[2], now);
    }
}

// K1 with staggered ends (a persistent grid's tail): block b spins base + (b % 64) * step ticks,
// then writes its share of `bytes` (plain or nontemporal stores)
__global__ __launch_bounds__(256) void k1s(unsigned long long* t, int base, int step, unsigned char* buf = nullptr,
                                          size_t bytes = 0, int nt = 0) {
    const unsigned long long t0 = wall_clock64();
    const unsigned long long d = (unsigned long long)(base + (int)(blockIdx.x % 64) * step);
    while (wall_clock64() - t0 < d) {
    }
    const size_t n4 = bytes / 4, stride = (size_t)gridDim.x * blockDim.x;
    unsigned* b4 = reinterpret_cast<unsigned*>(buf);
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        if (nt) __builtin_nontemporal_store((unsigned)i, b4 + i);
        else b4[i] = (unsigned)i;
    }
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(&t[0], wall_clock64());
}

// The render kernel's shape: 256 threads, 7 blocks per CU, 18 KB of LDS per block, a ~500-byte
// argument block; staggered ends; optionally byte stores (the P6 samples' shape: 3 bytes per pixel)
struct BigArgs {
    unsigned long long* t;
    unsigned char* buf;
    size_t bytes;
    int base, step, bytestores;
    float pad[112];
};
__global__ __launch_bounds__(256, 7) void kr(BigArgs A) {
    __shared__ float lds[18432 / 4];
    lds[threadIdx.x] = (float)threadIdx.x;
    const unsigned long long t0 = wall_clock64();
    if (threadIdx.x == 0) atomicMin(&A.t[1], t0);
    const unsigned long long d = (unsigned long long)(A.base + (int)(blockIdx.x % 64) * A.step);
    while (wall_clock64() - t0 < d) {
    }
    __syncthreads();
    if (A.bytestores) {
        const size_t stride = (size_t)gridDim.x * blockDim.x;
        for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; 3 * i + 2 < A.bytes; i += stride) {
            A.buf[3 * i] = (unsigned char)i;
            A.buf[3 * i + 1] = (unsigned char)(i >> 8);
            A.buf[3 * i + 2] = (unsigned char)lds[(threadIdx.x + 1) & 255];
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(&A.t[0], wall_clock64());
}

int main() {
    unsigned long long* t;
    unsigned char* buf;
    const size_t maxb = size_t(64) << 20;
    (void)hipMalloc(&t, 16);
    (void)hipMalloc(&buf, maxb);
    hipStream_t s, o;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&o, hipStreamNonBlocking);
    hipEvent_t e0, e1, done;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventCreate(&done);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int grid = cus * 8;
    const char* names[] = {"plain", "ext_events", "wait_event", "ext+wait"};
    {  // sixth table: render-shaped kernels back to back (K1 then K2, same kernel); gap = K2's first
       // wave start - K1's last wave end, with t[1] reset between them by a tiny kernel
        unsigned long long* t2;
        (void)hipMalloc(&t2, 64);
        for (int bs = 0; bs < 2; ++bs)
            for (int ev = 0; ev < 2; ++ev) {
                double gap = 0;
                const int reps = 20;
                for (int r = 0; r < reps + 3; ++r) {
                    unsigned long long init[8] = {0ull, ~0ull, 0ull, ~0ull, 0, 0, 0, 0};
                    (void)hipMemcpy(t2, init, 64, hipMemcpyHostToDevice);
                    (void)hipDeviceSynchronize();
                    BigArgs A1{};
                    A1.t = t2;  // K1: end -> t2[0]
                    A1.buf = buf;
                    A1.bytes = size_t(6) << 20;
                    A1.base = 5000;
                    A1.step = 50;
                    A1.bytestores = bs;
                    BigArgs A2 = A1;
                    A2.t = t2 + 2;  // K2: start -> t2[3]
                    if (ev) {
                        hipExtLaunchKernelGGL(kr, dim3(cus * 7), dim3(256), 0, s, e0, e1, 0, A1);
                        hipExtLaunchKernelGGL(kr, dim3(cus * 7), dim3(256), 0, s, e0, e1, 0, A2);
                    } else {
                        hipLaunchKernelGGL(kr, dim3(cus * 7), dim3(256), 0, s, A1);
                        hipLaunchKernelGGL(kr, dim3(cus * 7), dim3(256), 0, s, A2);
                    }
                    (void)hipStreamSynchronize(s);
                    unsigned long long h[8];
                    (void)hipMemcpy(h, t2, 64, hipMemcpyDeviceToHost);
                    if (r >= 3) gap += (double)((long long)h[3] - (long long)h[0]) / 100.0;
                }
                printf("{\"render_shaped\": 1, \"byte_stores_6MB\": %d, \"ext_events\": %d, \"gap_us\": %.2f}\n", bs, ev,
                       gap / reps);
                fflush(stdout);
            }
    }
    // fifth table: staggered K1, then K2 behind a stream wait on `done`, recorded by (a) an event
    // record on stream o, (b) a kernel's stop event on stream o (hipExtLaunchKernel, as the frame's
    // pre-pass records pdone), both complete long before K1 ends; (c) no wait
    (void)hipFree(t);
    (void)hipMalloc(&t, 32);
    for (int how = 0; how < 3; ++how) {
        double gap = 0;
        const int reps = 20;
        for (int r = 0; r < reps + 3; ++r) {
            unsigned long long init[4] = {0ull, ~0ull, 0ull, 0ull};
            (void)hipMemcpy(t, init, 32, hipMemcpyHostToDevice);
            (void)hipDeviceSynchronize();
            hipLaunchKernelGGL(k1s, dim3(cus * 7), dim3(256), 0, s, t, 5000, 50, buf, size_t(0), 0);
            if (how == 0) (void)hipEventRecord(done, o);
            if (how == 1) hipExtLaunchKernelGGL(k2, dim3(8), dim3(256), 0, o, nullptr, done, 0, t + 2);
            if (how < 2) (void)hipStreamWaitEvent(s, done, 0);
            hipLaunchKernelGGL(k2, dim3(cus * 7), dim3(256), 0, s, t);
            (void)hipStreamSynchronize(s);
            unsigned long long h[4];
            (void)hipMemcpy(h, t, 32, hipMemcpyDeviceToHost);
            if (r >= 3) gap += (double)((long long)h[1] - (long long)h[0]) / 100.0;
        }
        const char* hn[] = {"event_record", "kernel_stop_event", "no_wait"};
        printf("{\"staggered\": 1, \"wait_on\": \"%s\", \"gap_us\": %.2f}\n", hn[how], gap / reps);
        fflush(stdout);
    }
    // fourth table: staggered ends with 6 MB written, plain vs ext events, plain vs nontemporal
    (void)hipFree(t);
    (void)hipMalloc(&t, 32);
    for (int mb : {0, 6})
        for (int nt = 0; nt < 2; ++nt)
            for (int ev = 0; ev < 2; ++ev) {
                double gap = 0;
                const int reps = 20;
                for (int r = 0; r < reps + 3; ++r) {
                    unsigned long long init[4] = {0ull, ~0ull, 0ull, 0ull};
                    (void)hipMemcpy(t, init, 32, hipMemcpyHostToDevice);
                    (void)hipDeviceSynchronize();
                    if (ev)
                        hipExtLaunchKernelGGL(k1s, dim3(cus * 7), dim3(256), 0, s, e0, e1, 0, t, 5000, 50, buf,
                                              size_t(mb) << 20, nt);
                    else
                        hipLaunchKernelGGL(k1s, dim3(cus * 7), dim3(256), 0, s, t, 5000, 50, buf, size_t(mb) << 20, nt);
                    hipLaunchKernelGGL(k2, dim3(cus * 7), dim3(256), 0, s, t);
                    (void)hipStreamSynchronize(s);
                    unsigned long long h[4];
                    (void)hipMemcpy(h, t, 32, hipMemcpyDeviceToHost);
                    if (r >= 3) gap += (double)((long long)h[1] - (long long)h[0]) / 100.0;
                }
                printf("{\"staggered\": 1, \"write_MB\": %d, \"nontemporal\": %d, \"ext_events\": %d, \"gap_us\": %.2f}\n", mb,
                       nt, ev, gap / reps);
                fflush(stdout);
            }
    return 0;
    // third table: staggered K1 ends (step 0: all at once) and a K2 of g2 blocks: the gap to K2's
    // first wave and K2's own dispatch spread (last block start - first)
    (void)hipFree(t);
    (void)hipMalloc(&t, 32);
    for (int step : {0, 50, 300})
        for (int g2 : {cus, cus * 7}) {
            double gap = 0, spread = 0;
            const int reps = 20;
            for (int r = 0; r < reps + 3; ++r) {
                unsigned long long init[4] = {0ull, ~0ull, 0ull, 0ull};
                (void)hipMemcpy(t, init, 32, hipMemcpyHostToDevice);
                (void)hipDeviceSynchronize();
                hipLaunchKernelGGL(k1s, dim3(cus * 7), dim3(256), 0, s, t, 5000, step);
                hipLaunchKernelGGL(k2, dim3(g2), dim3(256), 0, s, t);
                (void)hipStreamSynchronize(s);
                unsigned long long h[4];
                (void)hipMemcpy(h, t, 32, hipMemcpyDeviceToHost);
                if (r >= 3) {
                    gap += (double)((long long)h[1] - (long long)h[0]) / 100.0;
                    spread += (double)((long long)h[2] - (long long)h[1]) / 100.0;
                }
            }
            printf("{\"k1_end_step_us\": %.1f, \"k1_end_spread_us\": %.1f, \"k2_grid\": %d, \"gap_us\": %.2f, \"k2_dispatch_spread_us\": %.2f}\n",
                   step / 100.0, step * 63 / 100.0, g2, gap / reps, spread / reps);
            fflush(stdout);
        }
    // second table: K1's spin length and grid, plain launches, no writes unless asked
    for (int spin : {1000, 10000, 30000})
        for (int g : {cus, cus * 8})
            for (int mb : {0, 24}) {
                double sum = 0;
                const int reps = 20;
                for (int r = 0; r < reps + 3; ++r) {
                    unsigned long long init[2] = {0ull, ~0ull};
                    (void)hipMemcpy(t, init, 16, hipMemcpyHostToDevice);
                    (void)hipDeviceSynchronize();
                    hipLaunchKernelGGL(k1, dim3(g), dim3(256), 0, s, t, spin, buf, size_t(mb) << 20, 0);
                    hipLaunchKernelGGL(k2, dim3(cus), dim3(256), 0, s, t);
                    (void)hipStreamSynchronize(s);
                    unsigned long long h[2];
                    (void)hipMemcpy(h, t, 16, hipMemcpyDeviceToHost);
                    if (r >= 3) sum += (double)((long long)h[1] - (long long)h[0]) / 100.0;
                }
                printf("{\"spin_us\": %d, \"grid\": %d, \"write_MB\": %d, \"gap_us_mean\": %.2f}\n", spin / 100, g, mb,
                       sum / reps);
                fflush(stdout);
            }
    for (int mb : {0, 6, 24}) {
        for (int nt = 0; nt < (mb ? 2 : 1); ++nt) {
            for (int v = 0; v < 4; ++v) {
                double sum = 0, best = 1e9;
                const int reps = 30;
                for (int r = 0; r < reps + 3; ++r) {
                    unsigned long long init[2] = {0ull, ~0ull};
                    (void)hipMemcpy(t, init, 16, hipMemcpyHostToDevice);
                    (void)hipEventRecord(done, o);  // complete long before K2
                    (void)hipDeviceSynchronize();
                    if (v == 1 || v == 3)
                        hipExtLaunchKernelGGL(k1, dim3(grid), dim3(256), 0, s, e0, e1, 0, t, 10000, buf,
                                              size_t(mb) << 20, nt);
                    else
                        hipLaunchKernelGGL(k1, dim3(grid), dim3(256), 0, s, t, 10000, buf, size_t(mb) << 20, nt);
                    if (v >= 2) (void)hipStreamWaitEvent(s, done, 0);
                    hipLaunchKernelGGL(k2, dim3(cus), dim3(256), 0, s, t);
                    (void)hipStreamSynchronize(s);
                    unsigned long long h[2];
                    (void)hipMemcpy(h, t, 16, hipMemcpyDeviceToHost);
                    const double gap_us = (double)((long long)h[1] - (long long)h[0]) / 100.0;
                    if (r >= 3) {
                        sum += gap_us;
                        if (gap_us < best) best = gap_us;
                    }
                }
                printf("{\"variant\": \"%s\", \"write_MB\": %d, \"nontemporal\": %d, \"gap_us_mean\": %.2f, \"gap_us_min\": %.2f}\n",
                       names[v], mb, nt, sum / reps, best);
                fflush(stdout);
            }
        }
    }
    return 0;
}
