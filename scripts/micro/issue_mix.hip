// Issue-rate microbenchmark for the render kernel's instruction mix: scalar-ALU streams, vector
// FMA streams, both interleaved in one wave's stream, and v_readlane / v_writelane streams, at 8
// and 2 waves per SIMD (256-thread blocks, grid sized per wave count), timed with HIP events.
// Prints cycles per instruction per SIMD and per CU at the nominal 2.4 GHz: SALU_per_CU tells
// whether the scalar unit is one per CU (4 cycles per SALU per SIMD when every SIMD issues) or
// one per SIMD; MIX tells whether a SALU and a VALU instruction of one wave co-issue.
// (The scalar asm declares its SCC clobber: without it the compiler kept the loop's compare
// result in SCC across the asm and the loop never ended.)
// Build: hipcc --offload-arch=gfx950 -O3 scripts/micro/issue_mix.hip -o build/issue_mix
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int CH = 8;  // independent chains per wave

template <int KIND>
__global__ __launch_bounds__(256) void k(float* out, float s, unsigned su, int iters) {
    float a[CH];
    unsigned x[CH];
    unsigned lanes = threadIdx.x;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
        a[i] = threadIdx.x * 0.001f + i;
        x[i] = __builtin_amdgcn_readfirstlane(su + i);  // wave-uniform: SGPR
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            if (KIND == 0 || KIND == 2)  // SALU: s_add_u32 + s_xor_b32 on one chain (2 SALU)
                asm volatile("s_add_u32 %0, %0, %1\n\ts_xor_b32 %0, %0, %1" : "+s"(x[i]) : "s"(su) : "scc");
            if (KIND == 1 || KIND == 2)  // VALU: two v_fma_f32 on one chain
                asm volatile("v_fma_f32 %0, %0, %1, 0.5\n\tv_fma_f32 %0, %0, %1, 0.5" : "+v"(a[i]) : "v"(s));
            if (KIND == 3)  // v_readlane_b32 into SGPRs (the traversal's pop), two per chain
                asm volatile("v_readlane_b32 %0, %1, 5\n\tv_readlane_b32 %0, %1, 9" : "=s"(x[i]) : "v"(lanes));
            if (KIND == 4)  // v_writelane_b32 from SGPRs (the traversal's push), two per chain
                asm volatile("v_writelane_b32 %0, %1, 5\n\tv_writelane_b32 %0, %1, 9" : "+v"(lanes) : "s"(x[i]));
        }
    }
    float r = 0;
#pragma unroll
    for (int i = 0; i < CH; ++i) r += a[i] + (float)x[i];
    r += (float)lanes;
    if (r == 12345.f) out[threadIdx.x] = r;
}

template <int KIND>
float run(float* d, int grid, int iters) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e9f;
    for (int rep = 0; rep < 5; ++rep) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k<KIND>, dim3(grid), dim3(256), 0, 0, d, 0.999f, 3u, iters);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return best;
}

int main() {
    float* d;
    if (hipMalloc(&d, 256 * sizeof(float)) != hipSuccess) return 1;
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int iters = 4096;
    const char* names[] = {"SALU (s_add+s_xor)", "VALU (2 v_fma)", "MIX (2 SALU + 2 VALU)", "v_readlane x2",
                           "v_writelane x2"};
    for (int wps : {8, 2}) {  // waves per SIMD: blocks of 4 waves, wps blocks per CU
        const int grid = cus * wps;
        float ms[5] = {run<0>(d, grid, iters), run<1>(d, grid, iters), run<2>(d, grid, iters),
                       run<3>(d, grid, iters), run<4>(d, grid, iters)};
        for (int kind = 0; kind < 5; ++kind) {
            // instructions per SIMD: wps waves x iters x CH chains x 2 (x2 again for MIX)
            const double per_simd = double(wps) * iters * CH * 2 * (kind == 2 ? 2 : 1);
            const double cyc = ms[kind] * 1e-3 * 2.4e9;
            printf("{\"waves_per_simd\": %d, \"kind\": \"%s\", \"ms\": %.4f, \"cycles_per_instr_per_simd\": %.3f, "
                   "\"instr_per_cycle_per_cu\": %.3f}\n",
                   wps, names[kind], ms[kind], cyc / per_simd, 4.0 * per_simd / cyc);
        }
    }
    (void)hipFree(d);
    return 0;
}
