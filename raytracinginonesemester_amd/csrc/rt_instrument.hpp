// rt_instrument.hpp — instrumentation of the render kernels for variant builds only
// (scripts/build_variant.sh <name> -DRT_STATS / -DRT_FRAME_SPAN / -DRT_WAVE_TIMES /
// -DRT_LANE_ITERS; scripts/stats.py, frame_span.py, wave_times.py, lane_iters.py read them
// through rt_debug_*).  The product build compiles none of it: every hook below is empty.
// Part of rt_device.hip's translation unit, included inside its anonymous namespace after the wave primitives (rt_wave.hpp).
#pragma once

// ---- traversal statistics (instrumented variant builds only: -DRT_STATS) -----------------
#ifdef RT_STATS
__device__ unsigned long long g_rt_stats[24];
#define RT_STAT(i, n) do { if (lane_id() == 0) atomicAdd(&g_rt_stats[(i)], (unsigned long long)(n)); } while (0)
#else
#define RT_STAT(i, n) do { } while (0)
#endif
// 0/1 traversals (primary/shadow), 2/3 pops, 4/5 pops after a mask test passed, 6/7 pop-time
// re-tests, 8/9 internal nodes, 10/11 leaves, 12 ambiguous box tests (wave-level), 13 lanes
// active at traversal start (primary), 14 (shadow), 15 primary traversals with no lane hitting,
// 16 their pops, 17 primary traversals whose root test no lane passes

#ifdef RT_FRAME_SPAN  // instrumented variant builds only: per render launch (drain_tag % 256) the first
// wave's start and the last wave's end (wall clock, 100 MHz), and the pre-passes' first start
__device__ unsigned long long* g_frame_span;
#endif
#ifdef RT_WAVE_TIMES  // instrumented variant builds only: per-wave start / end (wall clock, 100 MHz),
// per-wave phase ends (primary traversal, whole sample) and per tile the number of cut boxes
// its rays may meet (tile_cut_kernel)
__device__ unsigned long long* g_wave_times;
__device__ uint32_t* g_wave_meta;  // per item: block << 8 | XCC << 4 | first item << 2 | wave in block
__device__ unsigned long long* g_wave_phase;
__device__ int* g_cut_counts;
#define RT_PHASE(P, x, y, k)                                                                           \
    do {                                                                                               \
        if (g_wave_phase && lane_id() == 0)                                                            \
            g_wave_phase[(((size_t)((y) / (P).tile_h) * (P).tiles_x + (x) / (P).tile_w) * 4 + threadIdx.x / 64) * 2 + (k)] = \
                wall_clock64();                                                                        \
    } while (0)
#else
#define RT_PHASE(P, x, y, k) do { } while (0)
#endif

#ifdef RT_LANE_ITERS  // instrumented variant builds only (with RT_WAVE_TIMES): per work item, the
// loop iterations (record visits) of the per-lane traversals of its bounce and bounce-shadow
// rays: [0] sum over the wave's traversal calls of its longest lane's iterations, [1] the longest
// lane's total over all calls, [2] all lanes' total, [3] calls.  [0] is what the wave waits for
// when lanes meet after every traversal; [1] what it would wait for if they did not.
__device__ uint32_t* g_lane_iters;
__device__ uint32_t* g_lane_acc;  // per thread slot of the grid: 4 running words
#endif

#ifdef RT_LANE_ITERS
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off));
    return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    for (int off = 32; off > 0; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off);
    return v;
}
// every lane of the wave calls it after a per-lane traversal
__device__ __forceinline__ void lane_iters_note(uint32_t it) {
    if (g_lane_acc == nullptr) return;
    uint32_t* a = g_lane_acc + 4 * ((size_t)blockIdx.x * 256 + threadIdx.x);
    a[1] += it;
    const uint32_t m = wave_max_u32(it);
    if ((threadIdx.x & 63) == 0) {
        a[0] += m;
        a[3] += 1;
    }
}
#define RT_LI_ZERO(hs) ((hs).iters = 0)
#define RT_LI_STEP(hs) (++(hs).iters)
#else
#define RT_LI_ZERO(hs) do { } while (0)
#define RT_LI_STEP(hs) do { } while (0)
#endif

// Hooks of render_tiles_body's item loop (rt_device.hip): the frame span's first start / last
// end, a work item's start, and at its end the wave's times, lane iterations and XCC.
#ifdef RT_FRAME_SPAN
#define RT_HOOK_FRAME_FIRST(first, lane, RG)                                                              \
    do {                                                                                                   \
        if ((first) && (lane) == 0 && g_frame_span)                                                        \
            atomicMin(&g_frame_span[4 * ((RG).drain_tag & 255u)], wall_clock64());                         \
    } while (0)
#define RT_HOOK_FRAME_LAST(lane, RG)                                                                       \
    do {                                                                                                   \
        if ((lane) == 0 && g_frame_span) atomicMax(&g_frame_span[4 * ((RG).drain_tag & 255u) + 1], wall_clock64()); \
    } while (0)
#else
#define RT_HOOK_FRAME_FIRST(first, lane, RG) do { } while (0)
#define RT_HOOK_FRAME_LAST(lane, RG) do { } while (0)
#endif

#ifdef RT_LANE_ITERS
__device__ __forceinline__ void lane_iters_reset() {
    if (g_lane_acc) {
        uint32_t* a = g_lane_acc + 4 * ((size_t)blockIdx.x * 256 + threadIdx.x);
        a[0] = a[1] = a[2] = a[3] = 0;
    }
}
#endif
#ifdef RT_WAVE_TIMES
#ifdef RT_LANE_ITERS
#define RT_HOOK_ITEM_START(wt0)                                                                            \
    const unsigned long long wt0 = wall_clock64();                                                         \
    lane_iters_reset()
#else
#define RT_HOOK_ITEM_START(wt0) const unsigned long long wt0 = wall_clock64()
#endif
// the item's wave times (and, with RT_LANE_ITERS, its lane iterations) and its block / XCC
__device__ __forceinline__ void item_times_note(unsigned long long wt0, int tile, int wpt, uint32_t qw, uint32_t bx,
                                                bool first, uint32_t wv) {
#ifdef RT_LANE_ITERS
    if (g_lane_iters) {
        const uint32_t* a = g_lane_acc + 4 * ((size_t)blockIdx.x * 256 + threadIdx.x);
        const uint32_t mx = wave_max_u32(a[1]), sm = wave_sum_u32(a[1]);
        if ((threadIdx.x & 63) == 0) {
            g_lane_iters[((size_t)tile * wpt + qw) * 4 + 1] = mx;
            g_lane_iters[((size_t)tile * wpt + qw) * 4 + 2] = sm;
        }
    }
#endif
    if (g_wave_times && fresh_lane_id() == 0) {
        const size_t k = ((size_t)tile * wpt + qw) * 2;
        g_wave_times[k] = wt0;
        g_wave_times[k + 1] = wall_clock64();
#ifdef RT_LANE_ITERS
        if (g_lane_iters) {
            const uint32_t* a = g_lane_acc + 4 * ((size_t)blockIdx.x * 256 + threadIdx.x);
            g_lane_iters[((size_t)tile * wpt + qw) * 4 + 0] = a[0];
            g_lane_iters[((size_t)tile * wpt + qw) * 4 + 3] = a[3];
        }
#endif
        if (g_wave_meta) {
            const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u;  // HW_REG_XCC_ID
            g_wave_meta[(size_t)tile * wpt + qw] = bx << 8 | xcc << 4 | (first ? 4u : 0u) | wv;
        }
    }
}
#define RT_HOOK_ITEM_END(wt0, tile, wpt, qw, bx, first, wv) item_times_note(wt0, tile, wpt, qw, bx, first, wv)
#else
#ifdef RT_LANE_ITERS
#define RT_HOOK_ITEM_START(wt0) lane_iters_reset()
#else
#define RT_HOOK_ITEM_START(wt0) do { } while (0)
#endif
#define RT_HOOK_ITEM_END(wt0, tile, wpt, qw, bx, first, wv) do { } while (0)
#endif

