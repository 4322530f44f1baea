// VALU throughput microbenchmark: streams of one instruction kind, 8 independent chains per
// lane, 8 waves per SIMD, timed with HIP events.  Cycles at the nominal 2.4 GHz.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float v2f __attribute__((ext_vector_type(2)));

template <int KIND>
__global__ __launch_bounds__(256) void k(float* out, float s, int iters) {
    const bool sel = (threadIdx.x & 1) != 0;
    float a[8];
    v2f b[8];
    unsigned u[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[i] = threadIdx.x * 0.001f + i;
        b[i] = (v2f){a[i], a[i] + 1.f};
        u[i] = threadIdx.x + i;
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (KIND == 0) a[i] = __builtin_fmaf(a[i], s, 0.5f);
            if (KIND == 1) b[i] = __builtin_elementwise_fma(b[i], (v2f)(s), (v2f)(0.5f));
            if (KIND == 2) a[i] = __builtin_amdgcn_fmed3f(a[i], s, 0.5f);
            if (KIND == 3) a[i] = a[i] * s;
            if (KIND == 4) a[i] = a[i] + s;
            if (KIND == 5) a[i] = __builtin_fmaxf(a[i], s);
            if (KIND == 6) a[i] = __builtin_fmaxf(__builtin_fmaxf(a[i], s), a[(i + 1) & 7]);
            if (KIND == 7) u[i] = u[i] ^ (u[i] >> 3);
            if (KIND == 8) a[i] = a[i] > s ? a[i] : -a[i];
            if (KIND == 9) a[i] = sel ? a[i] : a[(i + 3) & 7];
            if (KIND == 10) u[i] += (a[i] > s) ? 1u : 0u;
            if (KIND == 11) a[i] = __builtin_fmaxf(__builtin_fmaxf(a[i], a[(i + 1) & 7]), __builtin_fmaxf(a[(i + 2) & 7], s));
        }
    }
    float r = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r += a[i] + b[i].x + b[i].y + (float)u[i];
    if (r == 12345.f) out[0] = r;
}

template <int KIND>
float run(float* d, int grid, int iters) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e9f;
    for (int rep = 0; rep < 5; ++rep) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k<KIND>, dim3(grid), dim3(256), 0, 0, d, 0.999f, iters);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    return best;
}

int main() {
    float* d;
    (void)hipMalloc(&d, 64);
    const int grid = 256 * 8, iters = 4096;
    const char* names[] = {"v_fma_f32", "v_pk_fma_f32", "v_med3_f32", "v_mul_f32", "v_add_f32",
                           "fmaxf (canon + v_max)", "v_max3_f32 (2 maxes)", "v_xor+v_lshr", "v_cmp+v_cndmask(+neg)",
                           "v_cndmask (fixed mask)", "v_cmp+v_addc", "4-way max"};
    float ms[12] = {run<0>(d, grid, iters), run<1>(d, grid, iters), run<2>(d, grid, iters), run<3>(d, grid, iters),
                    run<4>(d, grid, iters), run<5>(d, grid, iters), run<6>(d, grid, iters), run<7>(d, grid, iters),
                    run<8>(d, grid, iters), run<9>(d, grid, iters), run<10>(d, grid, iters), run<11>(d, grid, iters)};
    for (int kind = 0; kind < 12; ++kind) {
        const double instr = 8.0 * iters * 8;  // per SIMD: 8 waves x iters x 8 statements
        printf("%-24s %.3f ms  %.2f cycles per statement per SIMD (2.4 GHz)\n", names[kind], ms[kind],
               ms[kind] * 1e-3 * 2.4e9 / instr);
    }
    return 0;
}
