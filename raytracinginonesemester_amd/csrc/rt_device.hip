// rt_device.hip — the hot path on gfx950: camera ray -> BVH traversal -> Möller–Trumbore
// -> Lambert/Blinn-Phong with hard shadow rays (-> optional bounces), and the C-ABI
// entry points that own device memory.
//
// Reference path (G/ = HW2/HW2/GPUandCPU): render() CPU branch include/query.cu:130-166,
// TraceRayIterative query.h:156-220, SearchBVH query.h:224-311, ShadeDirect/IsInShadow
// shader.h:44-110, EvaluateBRDF brdf.h:12-40, Camera::get_ray camera.h:49-53.
//
// Device layout (built from the reference arrays by rt_scene_create):
//   inode[i]  64 B  children's AABBs + child refs of internal node i   (4 x float4)
//   ibox[i]   32 B  internal node i's own AABB (pop-time re-tests)      (2 x float4)
//   leaf[j]   64 B  v0, e1, e2, triangle index and the leaf's own AABB  (4 x float4)
//   tnorm[t]  48 B  n0, n1, n2 of triangle t (read once per hit)        (3 x float4)
// AABBs are stored as per-axis (min, max) pairs (BoxP), one packed FMA per axis.
// A child ref is an internal index, LEAF_BIT | leaf index, or NO_REF.
//
// Two traversal kernels, both bit-exact against the reference order:
//  * WAVE: one DFS per wavefront over a shared stack held in four VGPRs (entry k in lane
//    k, pushed with v_writelane, popped with v_readlane); each entry carries the 64-bit
//    mask of lanes that pushed it.  The reference's order (push left then right, pop
//    right first) is the same for every ray, so each lane sees exactly its own DFS as a
//    subsequence and makes every box/triangle decision with the same bestT the reference
//    would.  Node records are wave-uniform and come in through the scalar cache.
//  * LANE: one private stack per lane (the reference's structure, kept for A/B).
// Pop-time box re-tests are skipped when no lane's bestT changed since the push (the
// re-test would repeat the push-time computation with the same inputs).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <functional>
#include <memory>
#include <new>
#include <string>
#include <array>
#include <vector>

#include "rt_common.hpp"
#include "rt_hip_host.hpp"
#include "rt_math.hpp"
#include "rt_ppm.hpp"

using namespace rtd;

namespace {

constexpr uint32_t LEAF_BIT = 0x80000000u;
constexpr uint32_t NO_REF = 0xFFFFFFFFu;
// traverse_frustum's stack: two VGPRs, entry k in lane k of the first, 64 + k of the second
constexpr int FRUSTUM_STACK = 128;
constexpr uint32_t RT_FAULT_FRUSTUM_STACK = 1u;  // rt_scene_faults bit 0
constexpr uint32_t VER_FORCE = 0xFFFFFFFFu;   // pop must re-test (root)
constexpr int STACK_CAP = 64;                 // one entry per lane of the wave stack
constexpr int LANE_LDS_CAP = 32;              // traverse_lane_lds: per-lane stack entries in LDS (frog needs 18)
constexpr int BLOCK = 256;
// Kernel instantiation flag on top of RT_KERNEL_WAVE: traverse the 4-ary records (SceneView::wide).
// A compile-time choice, so each kernel holds one traversal loop per ray kind.
constexpr int MODE_WIDE = 16;
constexpr int MODE_PK = 32;  // the wave traversal's box tests in packed FMAs (box_ends_pk): depth-1 kernels
// Trees whose DFS needs more than STACK_CAP entries: SearchBVH literally, per lane, with the
// reference's 512-entry stack, its overflow rule and brute-force completion (traverse_deep).
constexpr int MODE_DEEP = 64;
// The depth-1 kernels' one-light form: the scene has exactly one light, so shade_d1 has no light
// loop (whose loop-carried values spilled in the big-scene 8-wave build).
constexpr int MODE_1L = 128;
// The big-scene kernels' frustum traversal over the quantised records (qent/qhdr: 16 B per entry
// instead of 32; build_quant_records)
constexpr int MODE_QR = 256;
constexpr int REF_STACK = 512;                // query.h:245
constexpr uint32_t INV_LEAF = 0xFFFFFFFEu;    // deep stack entry: a leaf naming no triangle (query.h:263)
constexpr uint32_t BRUTE_BIT = 0x40000000u;   // HitState::slot of a brute-force hit: BRUTE_BIT | triangle
constexpr float kRayTMin = 1e-4f;             // query.h:233
constexpr float RT_EPS = 1e-3f;               // shader.h:22

struct DevMaterial {  // rt_material, read through a 4-byte aligned pointer
    float albedo[3], kd, spec[3], ks, shininess, kr, emission[3];
};
struct DevLight {
    float pos[3], color[3];
    int32_t intensity;
};

struct SceneView {
    const float4* __restrict__ inode;
    const float4* __restrict__ wnode;  // 4-ary records (8 x float4) by internal index, if wide
    const float* __restrict__ fnode;   // 2^f_log2-ary records (8 x 2^f_log2 floats) of traverse_frustum, or null
    int32_t f_log2;                    // 3..5 with fnode; 2: traverse_frustum takes wnode
    const uint4* __restrict__ qent;    // fnode's records quantised (MODE_QR kernels): 2^f_log2 x 16 B each
    const float4* __restrict__ qhdr;   // their grids: (origin xyz, step x | step yz, -, -) per record
    const float4* __restrict__ ibox;
    const float4* __restrict__ rootb;  // the root's box, pairs (x | y, z), after ibox's entries
    const float4* __restrict__ leaf;
    const float4* __restrict__ tnorm;
    const int32_t* __restrict__ objids;
    const DevMaterial* __restrict__ mats;
    const DevLight* __restrict__ lights;
    int32_t num_tris, num_mats, num_lights;
    uint32_t root_ref;
    float root_box[6];
    float bmax[3];  // per axis max |coordinate| over every AABB of the scene (make_ray)
    int32_t wide;
    int32_t lane_stack;  // the binary DFS fits LANE_LDS_CAP entries: bounce rays take traverse_lane_lds
    int32_t lane_wide;   // ... and the 4-ary DFS fits them too: traverse_lane_lds_wide
    const float* __restrict__ cut;  // tile culling: boxes of a cut of the tree (6 floats each)
    int32_t ncut;
    const float* __restrict__ cut2;  // 2^cut_sub_log2 boxes of a cut of each cut box's subtree
    int32_t cut_sub_log2;            // 0: no second level
    const float4* __restrict__ tri;  // deep trees: v0 | e1, e2.x | e2.y, e2.z by triangle index (brute force)
    uint32_t* fault;  // RT_FAULT_* bits the kernels OR in (rt_scene_faults)
};

__device__ __forceinline__ f3 scene_bmax(const SceneView& sc) { return mk(sc.bmax[0], sc.bmax[1], sc.bmax[2]); }

struct RenderParams {
    SceneView sc;
    f3 cam_center, cam_p00, cam_du, cam_dv;
    int32_t W, H, spp, max_depth, diffuse_bounce;
    f3 miss;
    const float* __restrict__ jitter;  // 2*spp (device)
    int32_t band_rows, band_index, band_count, rows;  // rows = local rows rendered
    int32_t tile_w, tile_h, tiles_x, tiles_total;     // pixel tile per block
    int32_t lane_samples;                             // 1: one sample per lane; else pixel loop
    int32_t half_waves;                               // samples kernel: lanes >= 64 >> half_waves idle
    int32_t paired_only;                              // multi-bounce, half waves, one light: LS = 3 kernels
    int32_t tile_order;                               // RT_TILES_*
    int32_t spp_log2, tile_w_log2;                    // samples kernel: both powers of two
    int32_t cull;                                     // tile culling against the root box
    f3 miss_pixel;                                    // pixel value when all spp samples miss
    uint32_t* live_count;                             // [k * COUNTER_STRIDE], tile_cull_kernel
    int32_t* live_tiles;                              // nqueues lists of queue_cap entries
    int32_t* cut_tiles;   // tile_cut_kernel's survivors (not culled, not heavy), per list (sc.ncut > 0)
    uint32_t* next_count; // the counter set of the frame after next, zeroed by tile_cull_kernel
    int32_t cut_force;    // test every candidate in tile_cut_kernel (no pass-through)
    int32_t nqueues;
    int32_t queue_cap;
    float* __restrict__ rgb;
    int32_t* __restrict__ hit_idx;
    float* __restrict__ hit_t;
    uint8_t* __restrict__ p6;  // optional: write_p6-default samples of the pixels (rows*W*3 bytes)
    uint8_t miss_p6[4];        // the culled pixels' samples
    // Heavy-first dispatch (speed only, an approximate longest-first schedule): render waves
    // record their duration per tile (tile_cost, 4 x u16 per tile, 10 ns ticks); the next frame's
    // cut pass moves tiles whose last cost is >= heavy_ticks[c] (descending) to list q's class-c
    // heavy list (heavy_tiles, heavy_cap entries per (class, list), lengths in counter slots
    // heavy_counter(c, q)).  Each work queue hands out its list's heavy entries first, heaviest
    // class first, so the longest tiles start first (render_tiles_kernel).  heavy_cap == 0: off.
    uint16_t* __restrict__ tile_cost;
    int32_t* heavy_tiles;
    int32_t heavy_cap;
    uint32_t heavy_ticks[8];  // NCLASS thresholds, descending
    // rt_count_rays only (LANE and DEEP kernels; null otherwise): [1] shadow rays cast, [2]
    // bounce rays traced, the classes of the oracle's orc_stats.rays ([0], camera rays, is
    // W*H*spp by definition and counted on the host), [3] camera rays of the tiles the culling
    // passes left to the render kernel (the camera rays that are actually traversed)
    unsigned long long* ray_count;
    // The pre-pass gate (RT_TUNE_PREPASS_GATE): the first waves to find their queue drained
    // store drain_tag into this host word, and the next frame's pre-passes wait for it on the
    // prep stream (hipStreamWaitValue32), so they take wave slots in this kernel's tail instead
    // of racing its grid for them at its start.  Null: no gate.
    uint32_t* drained;
    uint32_t drain_tag;
    int32_t gate_q8;  // the gate opens when a queue has handed out gate_q8/256 of its items (256: drained)
};

// ---- wave primitives ------------------------------------------------------------------
__device__ __forceinline__ uint32_t lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
// A lane id the compiler cannot merge with any other (mbcnt of an opaque zero): one kept for a
// whole loop of items is live across all of them (and spills).
__device__ __forceinline__ uint32_t fresh_lane_id() {
    uint32_t z = 0;
    asm volatile("" : "+s"(z));
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, z));
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
// This lane's bit of a wave-uniform mask, the inverse of ballot: one v_cndmask on the SGPR pair
// (`(m >> lane_id()) & 1` keeps a 64-bit lane bit live across the traversal loop, which the
// compiler spills to scratch and reloads at every leaf pop).
__device__ __forceinline__ bool lane_in(uint64_t m) {
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, 0, 1, %1" : "=v"(r) : "s"(m));
    return r != 0;
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}
// v_writelane_b32 (the LLVM intrinsic; clang has no builtin for it on this toolchain): lane l
// takes v.  v and l are wave-uniform at every call.
extern "C" __device__ int rt_llvm_writelane(int, int, int) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ uint32_t wrlane(uint32_t v, uint32_t l, uint32_t old) {
    return (uint32_t)rt_llvm_writelane((int)v, (int)l, (int)old);
}
// Wave-wide max / min of a float over all 64 lanes (callers pass the identity on lanes that do
// not take part), wave-uniform result: DPP steps within quads, half rows, rows, then the row
// broadcasts; lane 63 ends with the whole wave's.
template <bool MAX, int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_step(float x) {
    const float id = MAX ? -INFINITY : INFINITY;
    const float y =
        __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(id), __float_as_int(x), CTRL, ROW_MASK, 0xF, false));
    return MAX ? fmaxf(x, y) : fminf(x, y);
}
template <bool MAX>
__device__ __forceinline__ float wave_reduce_f(float v) {
    v = dpp_step<MAX, 0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
    v = dpp_step<MAX, 0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
    v = dpp_step<MAX, 0x141, 0xF>(v);  // row_half_mirror
    v = dpp_step<MAX, 0x140, 0xF>(v);  // row_mirror
    v = dpp_step<MAX, 0x142, 0xA>(v);  // row_bcast:15 into rows 1, 3
    v = dpp_step<MAX, 0x143, 0xC>(v);  // row_bcast:31 into rows 2, 3
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

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

// ---- node accessors ---------------------------------------------------------------------
// Scene arrays are immutable while a frame renders: read them through the constant address
// space, so wave-uniform node addresses become scalar loads even inside loops that also
// store (the compiler cannot otherwise prove the stores do not clobber them).
typedef float __attribute__((ext_vector_type(4))) vf4;
typedef uint32_t __attribute__((ext_vector_type(4))) vu4;
__device__ __forceinline__ float4 ldc(const float4* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    const vf4 v = *(const __attribute__((address_space(4))) vf4*)p;
    return make_float4(v.x, v.y, v.z, v.w);
#else
    return *p;
#endif
}
__device__ __forceinline__ vf4 ldc_v(const float4* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return *(const __attribute__((address_space(4))) vf4*)p;
#else
    return *reinterpret_cast<const vf4*>(p);
#endif
}
__device__ __forceinline__ uint4 ldc_u(const float4* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    const vu4 v = *(const __attribute__((address_space(4))) vu4*)p;
    return make_uint4(v.x, v.y, v.z, v.w);
#else
    return *reinterpret_cast<const uint4*>(p);
#endif
}

__device__ __forceinline__ uint32_t ldc_u32(const uint32_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return *(const __attribute__((address_space(4))) uint32_t*)p;
#else
    return *p;
#endif
}
__device__ __forceinline__ v2f lo2(float4 q) { return (v2f){q.x, q.y}; }
__device__ __forceinline__ v2f hi2(float4 q) { return (v2f){q.z, q.w}; }

// Box of a node for the pop-time re-test: the root's from rootb, a leaf's from
// its record, an internal node's from ibox.
__device__ __forceinline__ BoxP own_box(const SceneView& sc, uint32_t ref, bool is_root) {
    BoxP b;
    if (is_root) {
        const float4 p = ldc(sc.rootb), q = ldc(sc.rootb + 1);
        b.x = lo2(p);
        b.y = hi2(p);
        b.z = lo2(q);
    } else if (ref & LEAF_BIT) {
        const float4* L = sc.leaf + 4 * (size_t)(ref & ~LEAF_BIT);
        const float4 c = ldc(L + 2), d = ldc(L + 3);
        b.x = hi2(c);
        b.y = lo2(d);
        b.z = hi2(d);
    } else {
        const float4* B = sc.ibox + 2 * (size_t)ref;
        const float4 p = ldc(B), q = ldc(B + 1);
        b.x = lo2(p);
        b.y = hi2(p);
        b.z = lo2(q);
    }
    return b;
}

// A node's 64-byte record (inode or leaf array), wave-uniform.
struct NodeRec {
    float4 a, b, c;
    uint4 d;
};

__device__ __forceinline__ NodeRec load_rec(const SceneView& sc, uint32_t ref) {
    const float4* p = (ref & LEAF_BIT) ? sc.leaf + 4 * (size_t)(ref & ~LEAF_BIT) : sc.inode + 4 * (size_t)ref;
    return NodeRec{ldc(p), ldc(p + 1), ldc(p + 2), ldc_u(p + 3)};
}

__device__ __forceinline__ BoxP leaf_box(const NodeRec& r) {
    return BoxP{hi2(r.c), (v2f){__uint_as_float(r.d.x), __uint_as_float(r.d.y)},
                (v2f){__uint_as_float(r.d.z), __uint_as_float(r.d.w)}};
}

// box_hit for the lanes in `act` (a wave mask; all lanes call it), as the mask of lanes that
// pass: the float pre-classification for everyone, the exact double test only behind a
// wave-uniform branch taken when some lane is ambiguous.
template <bool PK = false, bool XL = false>
__device__ __forceinline__ uint64_t box_hit_mask(const RayPre& r, const BoxP& b, float tmax, uint64_t act) {
    AxisEnds e;
    if constexpr (PK) e = box_ends_pk(r, b);
    else e = box_ends(r, b);
    const BoxEnds c = box_lc_hc(e, kRayTMin, tmax);
    uint64_t hit = ballot(box_sure_hit1(r, c)) & act;
    uint64_t amb = act & ~(hit | ballot(box_miss(c)));
    if (amb == 0) return hit;
    const uint64_t h2 = ballot(box_sure_hit2(r, e, kRayTMin, tmax)) & amb;
    hit |= h2;
    amb &= ~h2;
    if (amb == 0) return hit;
    RT_STAT(12, 1);
    // double(tmin), double(FLT_MAX): made here (RT_KF64), not hoisted into spilled VGPR pairs
    RT_KF64(tmin_d, (double)kRayTMin)
    RT_KF64(fltmax_d, (double)FLT_MAX)
    const double tmax_d = tmax == FLT_MAX ? fltmax_d : (double)tmax;
    return hit | (ballot(box_hit_exact<XL>(r, b, tmin_d, tmax_d)) & amb);
}

// rt_count_rays: one wave-aggregated add of the lanes where `c` holds into ray class `cls`.
// Compiled into the LANE and DEEP kernels only (the WAVE kernels' code is unchanged); every
// lane of the wave calls it (converged control flow).
template <int MODE>
__device__ __forceinline__ void count_rays(unsigned long long* rc, int cls, bool c) {
    if constexpr (MODE == RT_KERNEL_LANE || (MODE & MODE_DEEP) != 0) {
        if (rc != nullptr) {
            const uint64_t b = ballot(c);
            if (lane_id() == 0 && b != 0) atomicAdd(rc + cls, (unsigned long long)__popcll(b));
        }
    }
}

// Result of one closest-hit query.
struct HitState {
    float bestT;
    int32_t slot;  // leaf index of the current best, -1 = none
#ifdef RT_STATS
    uint32_t pops;
#endif
#ifdef RT_LANE_ITERS
    uint32_t iters;
#endif
};

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

// ---- WAVE traversal ---------------------------------------------------------------------
// One DFS per wavefront over a shared stack held in three VGPRs (entry k in lane k: node ref
// and the 64-bit mask of the lanes that pushed it; push = v_writelane, pop = v_readlane).  The
// reference's order (push left then right, pop right first) does not depend on the ray, so
// every lane's sequence of tests is a subsequence of the wave's, made with exactly the bestT the
// reference would hold.  Every lane of the wave must call this (uniform control flow); `active`
// selects the lanes that own a ray.  any_hit: shadow query, a lane stops as soon as its bestT <
// any_hit_dist (bestT only decreases, so the reference's final `hit && t < dist` is decided).
// The per-CU scalar unit (which also issues v_readlane / v_writelane) is the kernel's busiest
// pipe, so the loop is written for few scalar instructions per entry:
// - the entry in hand: after an internal record, the last entry it would push (the one the
//   reference pops next) stays in SGPRs and is processed at once, skipping its push and pop.
//   Nothing runs between its test and its processing, so it needs no re-test;
// - a stale watermark instead of a per-entry version lane: entries [0, stale) were pushed
//   before the latest bestT change of some lane and take the pop-time re-test.  A hit sets
//   stale = sp, and a re-tested pop at index sp lowers it to sp, so stale <= sp and what is
//   pushed next is fresh (pop-time re-tests are skipped while no lane's bestT has changed
//   since the push: the re-test would repeat the push-time computation with the same inputs);
// - records addressed by 32-bit byte offsets, which the scalar loads take as their SGPR offset
//   (rt_scene_create sends larger trees to MODE_DEEP);
// - the camera ray's query skips the `alive` AND (only a shadow query's lanes leave early).
template <bool WIDE, bool PK = false, bool XL = false>
__device__ __forceinline__ void traverse_wave_split(const SceneView& sc, const RayPre& r, bool active,
                                                  bool any_hit, float any_hit_dist, HitState& hs) {
    uint64_t alive = ballot(active);
    hs.bestT = FLT_MAX;
    hs.slot = -1;
#ifdef RT_STATS
    hs.pops = 0;
#endif
    if (alive == 0) return;
    [[maybe_unused]] const int so = any_hit ? 1 : 0;
    RT_STAT(0 + so, 1);
    RT_STAT(13 + so, __popcll(alive));
    // The root's pop-time test (SearchBVH tests every popped node, query.h:252-254) is made
    // here with the initial bestT; the root is then the first entry in hand.
    uint64_t mask = box_hit_mask<PK, XL>(r, own_box(sc, sc.root_ref, true), hs.bestT, alive);
    if (mask == 0) {
        if (!any_hit) RT_STAT(17, 1);
        return;
    }
    uint32_t ref = sc.root_ref;
    uint32_t st_ref = 0, st_mlo = 0, st_mhi = 0;  // lane k holds entry k
    int sp = 0;
    int stale = 0;  // entries [0, stale) take the pop-time re-test
    // The record arrays' bases (the compiler re-reads them from the kernel arguments at every
    // pop; holding them in SGPRs measured no faster).
    const char* leaf_b = reinterpret_cast<const char*>(sc.leaf);
    const char* wnode_b = reinterpret_cast<const char*>(sc.wnode);
    const char* ibox_b = reinterpret_cast<const char*>(sc.ibox);
    while (true) {
        RT_STAT(2 + so, 1);
#ifdef RT_STATS
        ++hs.pops;
#endif
        uint32_t pref = 0;
        uint64_t pmask = 0;  // the entry to hold next (0: pop)
        if (mask != 0) {
            RT_STAT(4 + so, 1);
            if (ref & LEAF_BIT) {
                RT_STAT(10 + so, 1);
                const uint32_t slot = ref & ~LEAF_BIT;
                const float4* L = reinterpret_cast<const float4*>(leaf_b + (slot << 6));
                const bool act = lane_in(mask);
                const float4 a = ldc(L), b = ldc(L + 1), c = ldc(L + 2);
                float t, u, v;
                const bool h = act && mt_g(r, mk(a.x, a.y, a.z), mk(b.x, b.y, b.z), mk(b.w, c.x, c.y), kRayTMin,
                                           hs.bestT, t, u, v);
                if (h) {
                    hs.bestT = t;
                    hs.slot = (int32_t)slot;
                }
                const uint64_t hm = ballot(h);
                if (hm != 0) {
                    stale = sp;
                    if (any_hit) alive &= ~ballot(h && t < any_hit_dist);
                }
            } else {
                RT_STAT(8 + so, 1);
                if constexpr (WIDE) {
                    // 4-ary record in one round trip: the seven 16-byte scalar loads are issued
                    // together and waited for once (the empty asm keeps the compiler from sinking
                    // each load next to its entry's test), addressed by 32-bit byte offset
                    const float4* W = reinterpret_cast<const float4*>(wnode_b + (ref << 7));
                    vf4 wq[7];
#pragma unroll
                    for (int k = 0; k < 7; ++k) wq[k] = ldc_v(W + k);
                    asm volatile("" ::"s"(wq[0]), "s"(wq[1]), "s"(wq[2]), "s"(wq[3]), "s"(wq[4]), "s"(wq[5]), "s"(wq[6]));
                    const uint32_t refs[4] = {__float_as_uint(wq[6].x), __float_as_uint(wq[6].y),
                                              __float_as_uint(wq[6].z), __float_as_uint(wq[6].w)};
                    float4 wv[6];
#pragma unroll
                    for (int k = 0; k < 6; ++k) wv[k] = make_float4(wq[k].x, wq[k].y, wq[k].z, wq[k].w);
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        if (refs[k] == NO_REF) continue;
                        const float4 p = wv[(3 * k) / 2], q = wv[(3 * k) / 2 + 1];
                        const BoxP bk = (k & 1) ? BoxP{hi2(p), lo2(q), hi2(q)} : BoxP{lo2(p), hi2(p), lo2(q)};
                        const uint64_t mk_ = box_hit_mask<PK, XL>(r, bk, hs.bestT, mask);
                        if (mk_ != 0) {
                            if (pmask != 0) {  // the previous passing entry goes to the stack
                                st_ref = wrlane(pref, sp, st_ref);
                                st_mlo = wrlane((uint32_t)pmask, sp, st_mlo);
                                st_mhi = wrlane((uint32_t)(pmask >> 32), sp, st_mhi);
                                ++sp;
                            }
                            pref = refs[k];
                            pmask = mk_;
                        }
                    }
                } else {
                    const float4* N = sc.inode + 4 * (size_t)ref;
                    const float4 q0 = ldc(N), q1 = ldc(N + 1), q2 = ldc(N + 2);
                    const uint4 q3 = ldc_u(N + 3);
                    const uint32_t lref = q3.x, rref = q3.y;
                    if (lref != NO_REF) {
                        const uint64_t ml = box_hit_mask<PK, XL>(r, BoxP{lo2(q0), hi2(q0), lo2(q1)}, hs.bestT, mask);
                        if (ml != 0) {
                            pref = lref;
                            pmask = ml;
                        }
                    }
                    if (rref != NO_REF) {
                        const uint64_t mr = box_hit_mask<PK, XL>(r, BoxP{hi2(q1), lo2(q2), hi2(q2)}, hs.bestT, mask);
                        if (mr != 0) {
                            if (pmask != 0) {
                                st_ref = wrlane(pref, sp, st_ref);
                                st_mlo = wrlane((uint32_t)pmask, sp, st_mlo);
                                st_mhi = wrlane((uint32_t)(pmask >> 32), sp, st_mhi);
                                ++sp;
                            }
                            pref = rref;
                            pmask = mr;
                        }
                    }
                }
            }
        }
        if (pmask != 0) {  // hold the last pushed entry: the next one the reference pops
            ref = pref;
            mask = pmask;
        } else {
            if (sp == 0) break;
            --sp;
            ref = rdlane(st_ref, sp);
            mask = ((uint64_t)rdlane(st_mhi, sp) << 32) | rdlane(st_mlo, sp);
            // only a shadow query's lanes leave early (alive shrinks); any_hit is a constant at
            // each inlined call
            if (any_hit) mask &= alive;
            if (sp < stale) {  // re-test (and lower the watermark to this slot)
                stale = sp;
                RT_STAT(6 + so, 1);
                BoxP ob;
                if (ref & LEAF_BIT) {
                    const float4* L = reinterpret_cast<const float4*>(leaf_b + ((ref & ~LEAF_BIT) << 6));
                    const float4 c = ldc(L + 2), d = ldc(L + 3);
                    ob = BoxP{hi2(c), lo2(d), hi2(d)};
                } else {
                    const float4* B = reinterpret_cast<const float4*>(ibox_b + (ref << 5));
                    const float4 p = ldc(B), q = ldc(B + 1);
                    ob = BoxP{lo2(p), hi2(p), lo2(q)};
                }
                mask = box_hit_mask<PK, XL>(r, ob, hs.bestT, mask);
            }
        }
    }
}

// ---- FRUSTUM traversal (camera rays over 16-ary records) ---------------------------------
// The camera rays of a wave share their origin, and their directions lie in a narrow cone.
// traverse_wave_split tests every pushed entry for every lane (per-lane slab tests of four boxes
// per record, 64-bit lane masks on the stack, pop-time re-tests after hits); here an internal
// entry is tested once for the whole wave against the family of directions instead, and only
// leaves take the per-lane test:
// - the family: per axis the interval [dl, dh] of the live lanes' direction components.  For a
//   box and a direction d in the family, the slab parameters (b - o)/d of an axis lie between
//   the values at d = dl and d = dh (linear in 1/d, and 1/d is monotone on an interval of one
//   sign), so min / max over the four products (min - o, max - o) x (1/dl, 1/dh) bound every
//   lane's near / far end of that axis; an axis whose interval reaches |d| < 1e-8 (where the
//   reference's test is an inside test) or crosses 0 gets the one-sided bound of the "loose axes"
//   below (an axis of coordinates near the float range gets none: 1/dl, 1/dh = -inf, +inf, the
//   products are +-inf or NaN, which the min / max drop).  The wave passes a box when
//   max(tmin, max near) <= min(tmax_w, min far), widened by 2^-19 relative (the float rounding
//   of (b - o), 1/d and the product is < 2^-22 relative; the reference's double ends are within
//   2^-52), with tmax_w the largest bestT over the live lanes.  So the wave test passes whenever
//   some live lane's exact test (intersectAABB, bvh.h:81-129) passes with that lane's bestT;
// - the DFS is the reference's order (SearchBVH, query.h:224-311): entries pushed in record
//   order, the last passing one held (popped next).  At a leaf, each lane makes the reference's
//   pop-time test of the leaf's own box with its own bestT (box_hit_mask, exact), then
//   Moller-Trumbore.  Exactness: leaves are reached in the reference's order, so a lane holds
//   the reference's bestT at each of them; the reference reaches a leaf for a lane iff the leaf's
//   own pop-time test and every ancestor's test (made earlier, with bestT no smaller) pass, and
//   since every internal box contains its children's boxes (checked at scene build, wide_ok) and
//   slab tests are monotone in the box and in tmax, the ancestors' tests are implied by the
//   leaf's own.  The wave reaches every leaf a lane's reference DFS reaches (the wave test is
//   conservative), and at leaves it does not, the lane's own test fails.  The root's pop-time
//   test is made per lane first (the root box need not contain its children's);
// - records: one wave-level test costs the same for 4 entries as for 16 (lane k tests entry k),
//   so the records hold an internal node's descendants four levels down (fnode, rt_scene_create):
//   a DFS over them makes about half the internal pops of the 4-ary one, each a dependent
//   round trip to memory.  Lane k loads entry k's box and ref (vector loads); the stack holds
//   refs only (entry k in lane k).  Scenes whose 16-ary DFS would need more than STACK_CAP
//   entries take the 4-ary records the same way.
// Scenes whose coordinates come within 1e30 of the float range give no bound on those axes
// (products stay finite: |b - o| < 1e30, |1/d| <= 1e8).
// - loose axes (round 6): a wave whose direction interval on an axis reaches |d| < 1e-8 (a 2x2
//   pixel quad on the camera's own axis plane: any camera off a symmetric position has one such
//   line of quads across the image) got no bound on that axis, so its family passed every box
//   its other two axes allowed, a whole slice of the scene (c3 with the camera moved 0.5 mm in x:
//   0.43 vs 0.13 ms, profiles/r06/exp/loose_axis_*.log).  Such an axis still bounds the near
//   end from one side: with db = (min - o, max - o), a box with db.lo > 0 is reached only by
//   lanes with d > 1e-8 (d <= 0 never reaches it; |d| < 1e-8 is the reference's inside test,
//   which fails), each at t >= db.lo / d >= db.lo / dh; a box with db.hi < 0 only by lanes with
//   d < -1e-8, at t >= db.hi / dl; a box across the plane gets no bound.  So near =
//   max(db.lo * ihp, db.hi * iln) with ihp = 1/dh (dh > 0; +inf otherwise: no lane reaches the
//   box) and iln = 1/dl (dl < 0; -inf otherwise), <= 0 for a box across the plane, and far = +inf.
//   Waves with a loose axis take a copy of the loop that computes it (LOOSE): the others' loop is
//   unchanged.
template <bool PK, bool XL, bool QR, bool LOOSE>
__device__ __forceinline__ void frustum_loop(const SceneView& sc, const RayPre& r, bool live, HitState& hs,
                                             const float* o, const v2f* U);
template <bool PK = false, bool XL = false, bool QR = false>
__device__ __forceinline__ void traverse_frustum(const SceneView& sc, const RayPre& r, bool active, HitState& hs) {
    hs.bestT = FLT_MAX;
    hs.slot = -1;
#ifdef RT_STATS
    hs.pops = 0;
#endif
    uint64_t alive = ballot(active);
    if (alive == 0) return;
    RT_STAT(0, 1);
    RT_STAT(13, __popcll(alive));
    alive = box_hit_mask<PK, XL>(r, own_box(sc, sc.root_ref, true), FLT_MAX, alive);  // the root's pop-time test
    if (alive == 0) {
        RT_STAT(17, 1);
        return;
    }
    const bool live = lane_in(alive);
    // the family: the shared origin and per axis (1/dl, 1/dh), wave-uniform
    const float o[3] = {__int_as_float(uni(__float_as_int(r.o.x))), __int_as_float(uni(__float_as_int(r.o.y))),
                        __int_as_float(uni(__float_as_int(r.o.z)))};
    // per axis [dl, dh], the live lanes' range (two wave reductions: the tight interval matters, the
    // frog's triangles are about a pixel wide; one reduction of |d - c| around one lane's c, an
    // interval up to twice as wide, took c3 from 0.157 to 0.477 ms).  The reciprocals are
    // v_rcp_f32 (1 ulp; inside the 2^-19 widening below).
    const float dd[3] = {r.d.x, r.d.y, r.d.z};
    v2f U[3];
    bool loose = false;  // a loose axis (see above); U = (ihp, iln) on it: U.x > 0 > U.y, which no
                         // other axis has (bounded: one sign; no bound: -inf, +inf)
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float dl = wave_reduce_f<false>(live ? dd[a] : INFINITY);
        const float dh = wave_reduce_f<true>(live ? dd[a] : -INFINITY);
        const bool fin = sc.bmax[a] + fabsf(o[a]) < 1e30f;
        const bool ok = (dl >= 1e-8f || dh <= -1e-8f) && fin;
        const bool lz = !ok && fin;
        loose = loose || lz;
        // (made SGPRs: wave-uniform values the VALU computed stay in VGPRs otherwise)
        const float u0 = ok ? rcp_approx(dl) : lz ? (dh > 0.0f ? rcp_approx(dh) : INFINITY) : -INFINITY;
        const float u1 = ok ? rcp_approx(dh) : lz ? (dl < 0.0f ? rcp_approx(dl) : -INFINITY) : INFINITY;
        U[a] = (v2f){__int_as_float(uni(__float_as_int(u0))), __int_as_float(uni(__float_as_int(u1)))};
    }
    if (__builtin_amdgcn_readfirstlane((int)loose) != 0) frustum_loop<PK, XL, QR, true>(sc, r, live, hs, o, U);
    else frustum_loop<PK, XL, QR, false>(sc, r, live, hs, o, U);
}

// traverse_frustum's DFS over the records (LOOSE: the wave has a loose axis).
template <bool PK, bool XL, bool QR, bool LOOSE>
__device__ __forceinline__ void frustum_loop(const SceneView& sc, const RayPre& r, bool live, HitState& hs,
                                             const float* o, const v2f* U) {
    const float kW = 1.0f / 524288.0f;  // 2^-19
    float tmax_w = FLT_MAX;
    uint32_t ref = sc.root_ref;
    uint32_t st_ref = 0, st_hi = 0;  // lane k holds entry k, st_hi entries 64 + k (FRUSTUM_STACK)
    int sp = 0;
    // A push past FRUSTUM_STACK (records whose DFS bound exceeds it: rt_scene_create never
    // builds them; RT_TUNE_FRUSTUM_STACK_CAP can, for the test of this guard) drops the entry
    // instead of wrapping a lane index over live ones; the wave's answers are then poisoned
    // (no hit) and RT_FAULT_FRUSTUM_STACK is raised for rt_render to report.
    bool ovf = false;
    const char* leaf_b = reinterpret_cast<const char*>(sc.leaf);
    // the wide records (fnode) when the scene has them, else the 4-ary ones (wnode): lane k
    // (mod the arity A = 2^f_log2) tests entry k; a record is 8A floats, refs at float 6A
    const uint32_t lg = (uint32_t)sc.f_log2;
    const char* rec_b = sc.fnode != nullptr ? reinterpret_cast<const char*>(sc.fnode) : reinterpret_cast<const char*>(sc.wnode);
    const uint32_t rec_shift = 5u + lg;
    const uint32_t ent_mask = (uint32_t)((1ull << (1u << lg)) - 1ull);
    // (a fresh lane id: lane_id() merged with the kernel's own was kept live across the item loop)
    const uint32_t kl = fresh_lane_id() & ((1u << lg) - 1u);
    const uint32_t k6 = 6u * kl, kref = (6u << lg) + kl;  // this lane's entry, in floats
    while (true) {
        RT_STAT(2, 1);
#ifdef RT_STATS
        ++hs.pops;
#endif
        uint32_t next = NO_REF;
        if (ref & LEAF_BIT) {
            RT_STAT(10, 1);
            const uint32_t slot = ref & ~LEAF_BIT;
            const float4* L = reinterpret_cast<const float4*>(leaf_b + (slot << 6));
            const float4 a = ldc(L), b = ldc(L + 1), c = ldc(L + 2), d = ldc(L + 3);
            // Moller-Trumbore first, for every live lane; the leaf's pop-time box test (which the
            // reference makes before it) only for lanes whose triangle test would change their
            // state: the same outcome, and most leaf pops change no lane's bestT
            float t, u, v;
            const bool hm = live && mt_g(r, mk(a.x, a.y, a.z), mk(b.x, b.y, b.z), mk(b.w, c.x, c.y),
                                                  kRayTMin, hs.bestT, t, u, v);
            const uint64_t mh = ballot(hm);
            if (mh != 0) {
                RT_STAT(4, 1);
                const uint64_t m = box_hit_mask<PK, XL>(r, BoxP{hi2(c), lo2(d), hi2(d)}, hs.bestT, mh);
                if (m != 0) {
                    if (lane_in(m)) {
                        hs.bestT = t;
                        hs.slot = (int32_t)slot;
                    }
                    tmax_w = wave_reduce_f<true>(live ? hs.bestT : 0.0f);
                }
            }
        } else {
            RT_STAT(8, 1);
            v2f bb[3];
            uint32_t rk;
            if constexpr (QR) {
                // entry k: (x lo | x hi, y lo | y hi, z lo | z hi) 16-bit grid steps and the ref, one
                // 16 B load; the record's grid (scalar loads) maps step q to fma(q, step, origin),
                // which the host checked lies at or below the entry's min (lo) and at or above its
                // max (hi): a box containing the entry's own, so the family test stays conservative
                const vf4 g0 = ldc_v(sc.qhdr + 2 * ref), g1 = ldc_v(sc.qhdr + 2 * ref + 1);
                const uint4 e = sc.qent[((size_t)ref << lg) + kl];
                const float og[3] = {g0.x, g0.y, g0.z}, st[3] = {g0.w, g1.x, g1.y};
                const uint32_t qw[3] = {e.x, e.y, e.z};
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    const v2f q = {(float)(qw[a] & 0xFFFFu), (float)(qw[a] >> 16)};
                    bb[a] = __builtin_elementwise_fma(q, (v2f){st[a], st[a]}, (v2f){og[a], og[a]});
                }
                rk = e.w;
            } else {
                const float* W = reinterpret_cast<const float*>(rec_b + ((size_t)ref << rec_shift));
                const v2f* B = reinterpret_cast<const v2f*>(W + k6);
                bb[0] = B[0];
                bb[1] = B[1];
                bb[2] = B[2];
                rk = reinterpret_cast<const uint32_t*>(W)[kref];
            }
            float nr[3], fr[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const v2f db = bb[a] - (v2f){o[a], o[a]};
                const v2f p = (v2f){db.x, db.x} * U[a], q = (v2f){db.y, db.y} * U[a];
                nr[a] = fminf(fminf(p.x, p.y), fminf(q.x, q.y));
                fr[a] = fmaxf(fmaxf(p.x, p.y), fmaxf(q.x, q.y));
                if constexpr (LOOSE) {  // U[a] = (ihp, iln) on a loose axis
                    if (U[a].x > 0.0f && U[a].y < 0.0f) {
                        nr[a] = fmaxf(p.x, q.y);
                        fr[a] = INFINITY;
                    }
                }
            }
            float Lc = fmaxf(fmaxf(nr[0], nr[1]), nr[2]);
            float Hc = fminf(fminf(fr[0], fr[1]), fr[2]);
            Lc = __builtin_fmaf(fabsf(Lc), -kW, Lc);
            Hc = __builtin_fmaf(fabsf(Hc), kW, Hc);
            const uint32_t m =
                (uint32_t)ballot(rk != NO_REF && fmaxf(Lc, kRayTMin) <= fminf(Hc, tmax_w)) & ent_mask;
            if (m != 0) {
                RT_STAT(4, 1);
                // push the passing entries in record order, hold the last (the reference pops it next)
                const uint32_t hold = 31u - __builtin_clz(m);
                next = rdlane(rk, hold);
                for (uint32_t rest = m & ~(1u << hold); rest != 0; rest &= rest - 1u) {
                    const uint32_t e = rdlane(rk, __builtin_ctz(rest));
                    if (sp < 64) {
                        st_ref = wrlane(e, sp, st_ref);
                    } else if (sp < FRUSTUM_STACK) {
                        st_hi = wrlane(e, sp - 64, st_hi);
                    } else {  // never with records built for this stack (the host bound)
                        ovf = true;
                        continue;
                    }
                    ++sp;
                }
            }
        }
        if (next != NO_REF) {
            ref = next;
            continue;
        }
        if (sp == 0) break;
        --sp;
        ref = sp < 64 ? rdlane(st_ref, sp) : rdlane(st_hi, sp - 64);
    }
    if (ovf) {
        if (fresh_lane_id() == 0) atomicOr(sc.fault, RT_FAULT_FRUSTUM_STACK);
        hs.bestT = __int_as_float(0x7fc00000);
        hs.slot = -1;
    }
}

// ---- LANE traversal (private stack per lane; the reference's shape) ---------------------
__device__ __forceinline__ void traverse_lane(const SceneView& sc, const RayPre& r, bool active,
                                              bool any_hit, float any_hit_dist, HitState& hs) {
    hs.bestT = FLT_MAX;
    hs.slot = -1;
    if (!active) return;
    uint32_t st_ref[STACK_CAP];
    uint32_t st_ver[STACK_CAP];
    int sp = 0;
    uint32_t ver = 0;
    st_ref[0] = sc.root_ref;
    st_ver[0] = VER_FORCE;
    sp = 1;
    while (sp > 0) {
        --sp;
        const uint32_t ref = st_ref[sp];
        const uint32_t pv = st_ver[sp];
        if (pv != ver) {
            if (!box_hit(r, own_box(sc, ref, pv == VER_FORCE), kRayTMin, hs.bestT)) continue;
        }
        if (ref & LEAF_BIT) {
            const uint32_t slot = ref & ~LEAF_BIT;
            const float4* L = sc.leaf + 4 * (size_t)slot;
            const float4 a = ldc(L), b = ldc(L + 1), c = ldc(L + 2);
            float t, u, v;
            if (mt_g(r, mk(a.x, a.y, a.z), mk(b.x, b.y, b.z), mk(b.w, c.x, c.y), kRayTMin, hs.bestT, t, u, v)) {
                hs.bestT = t;
                hs.slot = (int32_t)slot;
                ++ver;
                if (any_hit && t < any_hit_dist) return;
            }
            continue;
        }
        const float4* N = sc.inode + 4 * (size_t)ref;
        const float4 q0 = ldc(N), q1 = ldc(N + 1), q2 = ldc(N + 2);
        const uint4 q3 = ldc_u(N + 3);
        if (q3.x != NO_REF && box_hit(r, BoxP{lo2(q0), hi2(q0), lo2(q1)}, kRayTMin, hs.bestT)) {
            st_ref[sp] = q3.x;
            st_ver[sp] = ver;
            ++sp;
        }
        if (q3.y != NO_REF && box_hit(r, BoxP{hi2(q1), lo2(q2), hi2(q2)}, kRayTMin, hs.bestT)) {
            st_ref[sp] = q3.y;
            st_ver[sp] = ver;
            ++sp;
        }
    }
}

// ---- DEEP traversal: SearchBVH (G/include/query.h:224-311) as written, per lane ---------
// For trees whose DFS may need more than STACK_CAP entries.  A 512-entry private stack; the
// root is pushed unconditionally (:249); every pop tests the node's own box with the current
// bestT (:255); a leaf naming no triangle still occupies its stack entry (it was pushed after
// its box passed, :263); an internal node pushes left then right when the child's box passes,
// or sets the overflow flag when the stack is full (:277-295); after the loop an overflow is
// completed by every triangle in index order with t <= bestT (:298-308).  A shadow query stops
// once bestT < dist (bestT only decreases afterwards, so `hit && t < dist` is decided).
__device__ void traverse_deep(const SceneView& sc, const RayPre& r, bool active, bool any_hit, float any_hit_dist,
                              HitState& hs) {
    hs.bestT = FLT_MAX;
    hs.slot = -1;
    if (!active) return;
    uint32_t st[REF_STACK];
    int sp = 0;
    bool overflow = false;
    st[sp++] = sc.root_ref;
    while (sp > 0) {
        const uint32_t ref = st[--sp];
        if (ref == INV_LEAF) continue;  // its box test decides nothing
        if (!box_hit(r, own_box(sc, ref, false), kRayTMin, hs.bestT)) continue;
        if (ref & LEAF_BIT) {
            const uint32_t slot = ref & ~LEAF_BIT;
            const float4* L = sc.leaf + 4 * (size_t)slot;
            const float4 a = ldc(L), b = ldc(L + 1), c = ldc(L + 2);
            float t, u, v;
            if (mt_g(r, mk(a.x, a.y, a.z), mk(b.x, b.y, b.z), mk(b.w, c.x, c.y), kRayTMin, hs.bestT, t, u, v)) {
                hs.bestT = t;
                hs.slot = (int32_t)slot;
                if (any_hit && t < any_hit_dist) return;
            }
            continue;
        }
        const float4* N = sc.inode + 4 * (size_t)ref;
        const float4 q0 = ldc(N), q1 = ldc(N + 1), q2 = ldc(N + 2);
        const uint4 q3 = ldc_u(N + 3);  // left ref, right ref, invalid-leaf flags (bit 0 left, bit 1 right)
        if ((q3.x != NO_REF || (q3.z & 1u)) && box_hit(r, BoxP{lo2(q0), hi2(q0), lo2(q1)}, kRayTMin, hs.bestT)) {
            if (sp < REF_STACK) st[sp++] = (q3.z & 1u) ? INV_LEAF : q3.x;
            else overflow = true;
        }
        if ((q3.y != NO_REF || (q3.z & 2u)) && box_hit(r, BoxP{hi2(q1), lo2(q2), hi2(q2)}, kRayTMin, hs.bestT)) {
            if (sp < REF_STACK) st[sp++] = (q3.z & 2u) ? INV_LEAF : q3.y;
            else overflow = true;
        }
    }
    if (overflow) {
        for (int i = 0; i < sc.num_tris; ++i) {
            const float4* T = sc.tri + 3 * (size_t)i;
            const float4 a = ldc(T), b = ldc(T + 1), c = ldc(T + 2);
            float t, u, v;
            if (mt_g(r, mk(a.x, a.y, a.z), mk(b.x, b.y, b.z), mk(b.w, c.x, c.y), kRayTMin, hs.bestT, t, u, v)) {
                hs.bestT = t;
                hs.slot = (int32_t)(BRUTE_BIT | (uint32_t)i);
                if (any_hit && t < any_hit_dist) return;
            }
        }
    }
}

// ---- LANE traversal with its stack in LDS (incoherent rays: bounce rays, their shadow rays) --
// A wave-shared DFS visits the union of its lanes' paths: fine for the coherent camera rays of a
// 2x2-pixel quad and their shadow rays toward one light, but 64 diffuse bounce rays leave the
// surface in 64 directions, and the union of their paths is most of the tree (c3b, frog.json's
// own 8 bounces: 10.9 ms per frame with wave-shared bounce traversals).  Here each lane runs
// SearchBVH's DFS over the binary records on its own: the wave's time is its longest path, not
// the union.  The stack holds LANE_LDS_CAP entries per lane in LDS (stride BLOCK; trees whose
// DFS needs more take the wave traversal); as in the wave traversal, the last entry an internal
// node would push is held and processed at once (its pop-time test would repeat the push-time
// one with the same bestT), and a stale watermark selects the entries that were pushed before
// the latest bestT change: only those take the pop-time re-test.  Same tests, same order, same
// bestT at every test as the reference: exact.
__device__ __forceinline__ void traverse_lane_lds(const SceneView& sc, const RayPre& r, bool active, bool any_hit,
                                                  float any_hit_dist, HitState& hs, uint32_t* stk) {
    hs.bestT = FLT_MAX;
    hs.slot = -1;
    RT_LI_ZERO(hs);
    if (!active) return;
    if (!box_hit(r, own_box(sc, sc.root_ref, true), kRayTMin, hs.bestT)) return;  // the root's pop-time test
    uint32_t ref = sc.root_ref;
    int sp = 0, stale = 0;
    while (true) {
        RT_LI_STEP(hs);
        uint32_t next = NO_REF;  // the entry to hold
        if (ref & LEAF_BIT) {
            const uint32_t slot = ref & ~LEAF_BIT;
            const float4* L = sc.leaf + 4 * (size_t)slot;
            const float4 a = L[0], b = L[1], c = L[2];
            float t, u, v;
            if (mt_g(r, mk(a.x, a.y, a.z), mk(b.x, b.y, b.z), mk(b.w, c.x, c.y), kRayTMin, hs.bestT, t, u, v)) {
                hs.bestT = t;
                hs.slot = (int32_t)slot;
                stale = sp;
                if (any_hit && t < any_hit_dist) return;
            }
        } else {
            const float4* N = sc.inode + 4 * (size_t)ref;
            const float4 q0 = N[0], q1 = N[1], q2 = N[2];
            const uint4 q3 = *reinterpret_cast<const uint4*>(N + 3);
            const bool hl = q3.x != NO_REF && box_hit(r, BoxP{lo2(q0), hi2(q0), lo2(q1)}, kRayTMin, hs.bestT);
            const bool hr = q3.y != NO_REF && box_hit(r, BoxP{hi2(q1), lo2(q2), hi2(q2)}, kRayTMin, hs.bestT);
            if (hl && hr) {
                stk[sp * BLOCK] = q3.x;
                ++sp;
            }
            next = hr ? q3.y : (hl ? q3.x : NO_REF);
        }
        if (next != NO_REF) {
            ref = next;
            continue;
        }
        bool found = false;
        while (sp > 0) {
            --sp;
            ref = stk[sp * BLOCK];
            if (sp < stale) {  // pushed before the latest bestT change: the pop-time re-test
                stale = sp;
                if (!box_hit(r, own_box(sc, ref, false), kRayTMin, hs.bestT)) continue;
            }
            found = true;
            break;
        }
        if (!found) return;
    }
}

// traverse_lane_lds over the 4-ary records: a record holds an internal node's grandchildren in
// the reference's push order, so one visit tests what the reference reaches in
// two and the lane's chain of dependent record loads is about half as long (the bounce paths of
// c3b are latency-bound: a wave's longest path sets the kernel's tail).  The entries that pass
// are pushed in record order except the last, which is held (the entry the reference pops
// next); the same stale watermark.  Exact for the same reason as the wave traversal's 4-ary
// records.
__device__ __forceinline__ void traverse_lane_lds_wide(const SceneView& sc, const RayPre& r, bool active, bool any_hit,
                                                       float any_hit_dist, HitState& hs, uint32_t* stk) {
    hs.bestT = FLT_MAX;
    hs.slot = -1;
    RT_LI_ZERO(hs);
    if (!active) return;
    if (!box_hit(r, own_box(sc, sc.root_ref, true), kRayTMin, hs.bestT)) return;  // the root's pop-time test
    uint32_t ref = sc.root_ref;
    bool retest = false;  // the entry in ref was popped and takes the pop-time re-test first
    int sp = 0, stale = 0;
    // One batch of loads per iteration and lane: the entry's record (a leaf's 64 bytes, which
    // hold its own box, or a 4-ary record) and, for a popped internal entry that takes the
    // re-test, its box.  The lanes of a wave sit at leaves and internal entries at once; with
    // the loads inside the leaf and internal branches, and the re-test's inside the pop loop,
    // an iteration waited for up to three memory round trips one after another.
    while (true) {
        RT_LI_STEP(hs);
        const bool leaf = (ref & LEAF_BIT) != 0;
        const uint32_t idx = ref & ~LEAF_BIT;
        const float4* R = leaf ? sc.leaf + 4 * (size_t)idx : sc.wnode + 8 * (size_t)idx;
        const float4 w0 = R[0], w1 = R[1], w2 = R[2], w3 = R[3];
        // (defaults that do not read w0: a copy of a loaded value waits for the load)
        float4 w4 = make_float4(0.f, 0.f, 0.f, 0.f), w5 = w4, w6 = w4;
        if (!leaf) {
            w4 = R[4];
            w5 = R[5];
            w6 = R[6];
        }
        // own_box's six floats are consecutive in both layouts: a leaf's at word 10 of its
        // record, an internal node's at the start of its ibox entry; loaded as such (a select
        // between loaded values would wait for the record before the other loads are issued)
        const float* bp = leaf ? reinterpret_cast<const float*>(R + 2) + 2 : reinterpret_cast<const float*>(sc.ibox + 2 * (size_t)idx);
        v2f bx = {0.f, 0.f}, by = bx, bz = bx;
        if (retest) {
            bx = *reinterpret_cast<const v2f*>(bp);
            by = *reinterpret_cast<const v2f*>(bp + 2);
            bz = *reinterpret_cast<const v2f*>(bp + 4);
        }
        // pushed before the latest bestT change: the pop-time re-test
        const bool go = !retest || box_hit(r, BoxP{bx, by, bz}, kRayTMin, hs.bestT);
        uint32_t next = NO_REF;  // the entry to hold
        if (go) {
            if (leaf) {
                float t, u, v;
                if (mt_g(r, mk(w0.x, w0.y, w0.z), mk(w1.x, w1.y, w1.z), mk(w1.w, w2.x, w2.y), kRayTMin, hs.bestT, t, u,
                         v)) {
                    hs.bestT = t;
                    hs.slot = (int32_t)idx;
                    stale = sp;
                    if (any_hit && t < any_hit_dist) return;
                }
            } else {
                const float4 wv[7] = {w0, w1, w2, w3, w4, w5, w6};
                const uint32_t refs[4] = {__float_as_uint(w6.x), __float_as_uint(w6.y), __float_as_uint(w6.z),
                                          __float_as_uint(w6.w)};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (refs[k] == NO_REF) continue;
                    const float4 p = wv[(3 * k) / 2], q = wv[(3 * k) / 2 + 1];
                    const BoxP bk = (k & 1) ? BoxP{hi2(p), lo2(q), hi2(q)} : BoxP{lo2(p), hi2(p), lo2(q)};
                    if (box_hit(r, bk, kRayTMin, hs.bestT)) {
                        if (next != NO_REF) {
                            stk[sp * BLOCK] = next;
                            ++sp;
                        }
                        next = refs[k];
                    }
                }
            }
        }
        if (next != NO_REF) {
            ref = next;
            retest = false;
            continue;
        }
        if (sp == 0) return;
        --sp;
        ref = stk[sp * BLOCK];
        retest = sp < stale;
        if (retest) stale = sp;
    }
}

// The per-lane traversal of an incoherent ray over the kernel's records (4-ary in MODE_WIDE
// kernels, binary otherwise).
template <bool WIDE>
__device__ __forceinline__ void traverse_lane(const SceneView& sc, const RayPre& r, bool active, bool any_hit,
                                              float any_hit_dist, HitState& hs, uint32_t* stk) {
    if constexpr (WIDE) traverse_lane_lds_wide(sc, r, active, any_hit, any_hit_dist, hs, stk);
    else traverse_lane_lds(sc, r, active, any_hit, any_hit_dist, hs, stk);
}
// The scene's per-lane stacks fit the LDS stack for these records.
template <bool WIDE>
__device__ __forceinline__ bool lane_ok(const SceneView& sc) {
    return WIDE ? sc.lane_wide != 0 : sc.lane_stack != 0;
}

// any_hit (wave-uniform): shadow query, stop a lane once bestT < any_hit_dist.
template <int MODE>
__device__ __forceinline__ void traverse(const SceneView& sc, const RayPre& r, bool active, bool any_hit,
                                         float any_hit_dist, HitState& hs) {
    if constexpr ((MODE & MODE_DEEP) != 0) traverse_deep(sc, r, active, any_hit, any_hit_dist, hs);
    else if constexpr (MODE == RT_KERNEL_LANE) traverse_lane(sc, r, active, any_hit, any_hit_dist, hs);
    else traverse_wave_split<(MODE & MODE_WIDE) != 0, (MODE & MODE_PK) != 0, (MODE & MODE_PK) != 0 && (MODE & MODE_1L) == 0>(
        sc, r, active, any_hit, any_hit_dist, hs);
}

// A camera ray's closest-hit query (all lanes share the origin): the frustum traversal in the
// 4-ary WAVE kernels, the kernel's own traversal otherwise.
template <int MODE>
__device__ __forceinline__ void traverse_camera(const SceneView& sc, const RayPre& r, bool active, HitState& hs) {
#ifndef RT_NO_FRUSTUM
    if constexpr (MODE != RT_KERNEL_LANE && (MODE & MODE_DEEP) == 0 && (MODE & MODE_WIDE) != 0) {
        traverse_frustum<(MODE & MODE_PK) != 0, (MODE & MODE_PK) != 0 && (MODE & MODE_1L) == 0, (MODE & MODE_QR) != 0>(
            sc, r, active, hs);
        return;
    }
#endif
    traverse<MODE>(sc, r, active, false, 0.0f, hs);
}

// The traversal of a ray at bounce depth `depth` (wave-uniform): camera rays (depth 0) and their
// shadow rays are coherent and take the kernel's traversal; in the WAVE kernels the bounce rays
// and their shadow rays take traverse_lane_lds when the tree's DFS fits its LDS stack.
template <int MODE>
__device__ __forceinline__ void traverse_at(const SceneView& sc, int depth, const RayPre& r, bool active, bool any_hit,
                                            float any_hit_dist, HitState& hs, float* lds) {
    if constexpr (MODE != RT_KERNEL_LANE && (MODE & MODE_DEEP) == 0) {
        constexpr bool W = (MODE & MODE_WIDE) != 0;
        if (depth > 0 && lane_ok<W>(sc)) {
            traverse_lane<W>(sc, r, active, any_hit, any_hit_dist, hs, reinterpret_cast<uint32_t*>(lds));
#ifdef RT_LANE_ITERS
            lane_iters_note(active ? hs.iters : 0u);
#endif
            return;
        }
    }
    traverse<MODE>(sc, r, active, any_hit, any_hit_dist, hs);
}

// Triangle index of a hit (the primary-hit AOV): the leaf's, or (DEEP kernels) the triangle a
// brute-force completion accepted.
template <bool DEEP = false>
__device__ __forceinline__ int32_t leaf_tri(const SceneView& sc, int32_t slot) {
    if constexpr (DEEP) {
        if ((uint32_t)slot & BRUTE_BIT) return (int32_t)((uint32_t)slot & ~BRUTE_BIT);
    }
    return __float_as_int(sc.leaf[4 * (size_t)slot].w);
}

struct SurfHit {
    f3 p, n;
    int32_t tri;
};

// Full hit record of the winning triangle (intersectTriangle's tail, query.h:110-130).
template <bool DEEP = false>
__device__ __forceinline__ SurfHit resolve_hit(const SceneView& sc, const RayPre& r, int32_t slot) {
    const float4* L = sc.leaf + 4 * (size_t)slot;
    bool brute = false;
    if constexpr (DEEP) {
        brute = ((uint32_t)slot & BRUTE_BIT) != 0;
        if (brute) L = sc.tri + 3 * (size_t)((uint32_t)slot & ~BRUTE_BIT);
    }
    const float4 a = L[0], b = L[1], c = L[2];
    const f3 v0 = mk(a.x, a.y, a.z), e1 = mk(b.x, b.y, b.z), e2 = mk(b.w, c.x, c.y);
    float t = 0.f, u = 0.f, v = 0.f;
    mt_g(r, v0, e1, e2, -FLT_MAX, FLT_MAX, t, u, v);  // same t/u/v as the accepting test
    SurfHit s;
    s.tri = brute ? (int32_t)((uint32_t)slot & ~BRUTE_BIT) : __float_as_int(a.w);
    const float4* Nn = sc.tnorm + 3 * (size_t)s.tri;
    const float4 n0 = Nn[0], n1 = Nn[1], n2 = Nn[2];
    hit_frame(r, e1, e2, mk(n0.x, n0.y, n0.z), mk(n1.x, n1.y, n1.z), mk(n2.x, n2.y, n2.z), t, u, v, s.p, s.n);
    return s;
}

__device__ __forceinline__ DevMaterial material_of(const SceneView& sc, int32_t tri) {
    // assignMaterialToHit (query.h:134-153) over Material() defaults (material.h:8-19)
    DevMaterial m = {{0.8f, 0.8f, 0.8f}, 1.0f, {0.04f, 0.04f, 0.04f}, 0.0f, 32.0f, 0.0f, {0.f, 0.f, 0.f}};
    if (sc.objids != nullptr && sc.mats != nullptr && tri >= 0 && tri < sc.num_tris) {
        const int oid = sc.objids[tri];
        if (oid >= 0 && oid < sc.num_mats) m = sc.mats[oid];
    }
    return m;
}

// EvaluateBRDF (brdf.h:12-40)
__device__ __forceinline__ f3 eval_brdf(const DevMaterial& m, f3 N, f3 V, f3 L) {
    const float NdotL = fmaxf(dot(N, L), 0.0f);
    const float NdotV = fmaxf(dot(N, V), 0.0f);
    if (NdotL <= 0.f || NdotV <= 0.f) return mk(0.f, 0.f, 0.f);
    const float invPi = 0.31830988618f;
    const f3 fd = scale(mk(m.albedo[0], m.albedo[1], m.albedo[2]), m.kd * invPi);
    const f3 Hh = unit(add(L, V));
    const float NdotH = fmaxf(dot(N, Hh), 0.0f);
    const float inv2Pi = 0.15915494309f;
    const float specNorm = (m.shininess + 2.0f) * inv2Pi;
    const float specLobe = specNorm * ref_powf(NdotH, m.shininess);
    const f3 fs = scale(scale(mk(m.spec[0], m.spec[1], m.spec[2]), m.ks), specLobe);
    return add(fd, fs);
}

// Camera::get_ray(float, float) (camera.h:49-53) with the jittered_samples offsets.
__device__ __forceinline__ RayPre camera_ray(const RenderParams& P, bool valid, int x, int y, int s) {
    const float jx = valid ? P.jitter[2 * s] : 0.f;
    const float jy = valid ? P.jitter[2 * s + 1] : 0.f;
    const float px = (float)x + jx, py = (float)y + jy;
    const f3 pix = add(add(P.cam_p00, scale(P.cam_du, px)), scale(P.cam_dv, py));
    return make_ray(P.cam_center, cam_unit(sub(pix, P.cam_center)), scene_bmax(P.sc));
}

// The rest of TraceRayIterative at maxDepth 1 once the camera ray's closest hit is known:
// missColor on a miss (query.h:181-183), else ShadeDirect (shader.h:65-110) with one shadow
// ray per light; the bounce has no effect at depth 1 and is not traced.  All lanes of a wave
// call it (the shadow traversals are wave-wide).
// Per-lane state parked in LDS across a shadow traversal (PARK_SLOTS floats per lane, struct
// of arrays with stride BLOCK): the traversal needs every VGPR the kernel's occupancy allows, and
// values kept live across it were spilled to scratch (private memory through L2/HBM); LDS is a
// few tens of cycles away and otherwise unused by the render kernels.
constexpr int PARK_SLOTS = 14;
struct Park {
    // the wave's slot 0 (LDS, wave-uniform); a lane's slot is found afresh at every access (a
    // per-lane pointer kept across the traversals was itself spilled in the 64-VGPR build)
    float* p;
    __device__ __forceinline__ uint32_t lane() const {
        uint32_t z = 0;
        asm volatile("" : "+s"(z));
        return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, z));
    }
    __device__ __forceinline__ void put(int k, float v) const { p[k * BLOCK + lane()] = v; }
    __device__ __forceinline__ float get(int k) const { return p[k * BLOCK + lane()]; }
    // The traversal between put and get writes no LDS, so without this the compiler would
    // forward the stored values and keep them in registers after all.
    __device__ __forceinline__ static void fence() { asm volatile("" ::: "memory"); }
};

template <int MODE>
__device__ __forceinline__ f3 shade_d1(const RenderParams& P, bool valid_in, const RayPre& ray, const HitState& hs,
                                       float* park_wave) {
    const SceneView& sc = P.sc;
    const Park pk{park_wave};
    bool valid = valid_in;
    bool hit = valid && hs.slot >= 0;
    // radiance = 0 + (1,1,1) * missColor on a miss (query.h:181-183), 0 + (1,1,1) * Lo on a hit:
    // made once the lights are done, so nothing but Lo is live across the shadow traversals
    auto radiance_of = [&](f3 Lo) {
        f3 radiance = mk(0.f, 0.f, 0.f);
        if (valid && !hit) radiance = add(radiance, mul(mk(1.f, 1.f, 1.f), P.miss));
        if (hit) radiance = add(radiance, mul(mk(1.f, 1.f, 1.f), Lo));
        return clamp01(radiance);
    };
    if (ballot(hit) == 0) return radiance_of(mk(0.f, 0.f, 0.f));
    int32_t slot = hs.slot;
    // valid and hit go to LDS at once (slot 10; lit, known later, to slot 11): kept live
    // across the shading, the lane's valid bit was spilled to scratch in the 64-VGPR build
    pk.put(10, __int_as_float((valid ? 1 : 0) | (hit ? 2 : 0)));
    // The camera ray's origin is the (uniform) camera centre; only its direction is per lane.
    RayPre cray;
    cray.o = ray.o;
    cray.d = ray.d;
    f3 Lo = mk(0.f, 0.f, 0.f);
    if (hit) {
        const DevMaterial m = material_of(sc, leaf_tri<(MODE & MODE_DEEP) != 0>(sc, slot));
        Lo = add(Lo, scale(mk(m.albedo[0], m.albedo[1], m.albedo[2]), 0.05f));
        Lo = add(Lo, mk(m.emission[0], m.emission[1], m.emission[2]));
    }
    // One light (frog, sphere scenes): the body straight, no loop -- as a loop, values the
    // compiler carried between iterations (the unset shadow ray of lanes without one) spilled.
    auto light = [&](int li) {
        const DevLight& lt = sc.lights[li];
        const f3 lpos = mk(lt.pos[0], lt.pos[1], lt.pos[2]);
        float dist = 0.f;
        bool need = false, lit = false;
        f3 Lo_lit = Lo;
        // Lanes without a shadow ray leave sray unset: the traversal masks them out (their
        // results are never read), and copying the camera ray in would keep it live.
        RayPre sray;
        if (hit) {
            // The hit record (point, normals, material) is rebuilt per light from the leaf and
            // the camera ray (the accepting test's own t/u/v), so none of it stays live across the
            // shadow traversal.
            const SurfHit sh = resolve_hit<(MODE & MODE_DEEP) != 0>(sc, cray, slot);
            const f3 N = unit(sh.n);
            const f3 V = unit(sub(cray.o, sh.p));
            const f3 L = unit(sub(lpos, sh.p));
            const float NdotL = fmaxf(dot(N, L), 0.0f);
            if (NdotL > 0.0f) {
                const DevMaterial m = material_of(sc, sh.tri);
                const f3 f = eval_brdf(m, sh.n, V, L);
                const f3 rad = scale(mk(lt.color[0], lt.color[1], lt.color[2]), (float)lt.intensity);
                // Lo + contrib, taken below if the shadow ray is clear (the same single add)
                Lo_lit = add(Lo, scale(mul(rad, f), NdotL));
                lit = true;
                // IsInShadow (shader.h:44-62)
                const f3 toL = sub(lpos, sh.p);
                dist = sqrtf(dot(toL, toL));
                if (dist > 0.0f) {
                    need = true;
                    sray = make_ray(add(sh.p, scale(N, RT_EPS)), divf(toL, dist), scene_bmax(sc));
                }
            }
        }
        pk.put(0, cray.d.x);
        pk.put(1, cray.d.y);
        pk.put(2, cray.d.z);
        pk.put(3, __int_as_float(slot));
        pk.put(4, Lo.x);
        pk.put(5, Lo.y);
        pk.put(6, Lo.z);
        pk.put(7, Lo_lit.x);
        pk.put(8, Lo_lit.y);
        pk.put(9, Lo_lit.z);
        pk.put(11, lit ? 1.0f : 0.0f);
        Park::fence();
        HitState shs;
        count_rays<MODE>(P.ray_count, 1, need);
        traverse<MODE>(sc, sray, need, true, dist, shs);
        const bool occluded = need && shs.slot >= 0 && shs.bestT < dist;
        Park::fence();
        const int fl = __float_as_int(pk.get(10));
        valid = (fl & 1) != 0;
        hit = (fl & 2) != 0;
        lit = pk.get(11) != 0.0f;
        const bool take = lit && !occluded;
        Lo = take ? mk(pk.get(7), pk.get(8), pk.get(9)) : mk(pk.get(4), pk.get(5), pk.get(6));
        slot = __float_as_int(pk.get(3));
        cray.d = mk(pk.get(0), pk.get(1), pk.get(2));
    };
    if ((MODE & MODE_1L) != 0) {
        light(0);
    } else if (sc.num_lights == 1) {
        light(0);
    } else {
        for (int li = 0; li < sc.num_lights; ++li) light(li);
    }
    return radiance_of(Lo);
}


// The paired-only kernels resume their per-lane traversals across calls (paired_bounces_resume;
// c3b 1.425 vs 1.467 ms and 1.422 vs 1.501 in one process, frames identical).  -DRT_NO_RESUME
// builds the plain paired loop into them for A/B.
#ifndef RT_NO_RESUME
#define RT_RESUME 1
#endif
#ifdef RT_RESUME
#ifndef RT_RESUME_SHIFT
#define RT_RESUME_SHIFT 2
#endif
// A per-lane DFS over the 4-ary records that a call can leave with lanes still
// mid-traversal: their state stays in LaneDfs (and the LDS stack) and the next call resumes it.
struct LaneDfs {
    uint32_t ref;
    int sp, stale;
    bool retest, run;
};
__device__ __forceinline__ void dfs_start(const SceneView& sc, const RayPre& r, bool go, HitState& hs, LaneDfs& d) {
    if (go) {
        hs.bestT = FLT_MAX;
        hs.slot = -1;
        d.run = box_hit(r, own_box(sc, sc.root_ref, true), kRayTMin, FLT_MAX);  // the root's pop-time test
        d.ref = sc.root_ref;
        d.sp = 0;
        d.stale = 0;
        d.retest = false;
    }
}
// Runs the lanes with d.run until at most `quota` of them still run (traverse_lane_lds_wide's
// visits, one load batch each; the same tests in the same order: exact).  The guard only ends a
// call, never a traversal: lanes still running resume in the caller's next call.
__device__ __forceinline__ void dfs_run(const SceneView& sc, const RayPre& r, bool any_hit, float any_hit_dist,
                                        HitState& hs, LaneDfs& d, uint32_t* stk, uint32_t quota) {
    for (uint32_t guard = 0; guard < (1u << 22); ++guard) {
        if ((uint32_t)__popcll(ballot(d.run)) <= quota) break;
        if (d.run) {
            RT_LI_STEP(hs);
            const uint32_t ref = d.ref;
            const bool leaf = (ref & LEAF_BIT) != 0;
            const uint32_t idx = ref & ~LEAF_BIT;
            const float4* R = leaf ? sc.leaf + 4 * (size_t)idx : sc.wnode + 8 * (size_t)idx;
            const float4 w0 = R[0], w1 = R[1], w2 = R[2], w3 = R[3];
            float4 w4 = make_float4(0.f, 0.f, 0.f, 0.f), w5 = w4, w6 = w4;
            if (!leaf) {
                w4 = R[4];
                w5 = R[5];
                w6 = R[6];
            }
            const float* bp = leaf ? reinterpret_cast<const float*>(R + 2) + 2 : reinterpret_cast<const float*>(sc.ibox + 2 * (size_t)idx);
            v2f bx = {0.f, 0.f}, by = bx, bz = bx;
            if (d.retest) {
                bx = *reinterpret_cast<const v2f*>(bp);
                by = *reinterpret_cast<const v2f*>(bp + 2);
                bz = *reinterpret_cast<const v2f*>(bp + 4);
            }
            const bool go = !d.retest || box_hit(r, BoxP{bx, by, bz}, kRayTMin, hs.bestT);
            uint32_t next = NO_REF;
            bool stop = false;
            if (go) {
                if (leaf) {
                    float t, u, v;
                    if (mt_g(r, mk(w0.x, w0.y, w0.z), mk(w1.x, w1.y, w1.z), mk(w1.w, w2.x, w2.y), kRayTMin, hs.bestT, t, u,
                             v)) {
                        hs.bestT = t;
                        hs.slot = (int32_t)idx;
                        d.stale = d.sp;
                        if (any_hit && t < any_hit_dist) stop = true;
                    }
                } else {
                    const float4 wv[7] = {w0, w1, w2, w3, w4, w5, w6};
                    const uint32_t refs[4] = {__float_as_uint(w6.x), __float_as_uint(w6.y), __float_as_uint(w6.z),
                                              __float_as_uint(w6.w)};
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        if (refs[k] == NO_REF) continue;
                        const float4 p = wv[(3 * k) / 2], q = wv[(3 * k) / 2 + 1];
                        const BoxP bk = (k & 1) ? BoxP{hi2(p), lo2(q), hi2(q)} : BoxP{lo2(p), hi2(p), lo2(q)};
                        if (box_hit(r, bk, kRayTMin, hs.bestT)) {
                            if (next != NO_REF) {
                                stk[d.sp * BLOCK] = next;
                                ++d.sp;
                            }
                            next = refs[k];
                        }
                    }
                }
            }
            if (stop) {
                d.run = false;
            } else if (next != NO_REF) {
                d.ref = next;
                d.retest = false;
            } else if (d.sp == 0) {
                d.run = false;
            } else {
                --d.sp;
                d.ref = stk[d.sp * BLOCK];
                d.retest = d.sp < d.stale;
                if (d.retest) d.stale = d.sp;
            }
        }
    }
}

// paired_bounces with resumable per-lane traversals: a call returns once three quarters of its
// running lanes are done; a pair (path lane l, shadow lane l + 32) whose two traversals have
// ended is shaded and sent on at once, while the others resume in the next call.  Per sample the
// same rays, tests, arithmetic and order of radiance adds as paired_bounces: exact.
template <int MODE>
__device__ __forceinline__ void paired_bounces_resume(const RenderParams& P, RayPre& ray, bool alive, f3& thr,
                                                      f3& radiance, uint32_t& rng, float* park, HitState hs) {
    const SceneView& sc = P.sc;
    const bool upper = lane_id() >= 32;
    const int max_depth = P.max_depth;
    uint32_t* stk = reinterpret_cast<uint32_t*>(park);
    LaneDfs d;
    d.run = false;
    d.ref = 0;
    d.sp = d.stale = 0;
    d.retest = false;
    int depth = 0;                   // lower lanes: the depth of the path result in hs
    bool unproc = !upper;            // lower lanes: hs holds a path result not yet shaded
    bool need_up = false;            // upper lanes: tracing (or holding the answer of) a shadow ray
    float dist_up = 0.f;
    bool pend = false, lit_p = false;
    f3 thr_p = mk(0.f, 0.f, 0.f), Lo_p = thr_p, Lo_lit_p = thr_p;
    // Every call ends at least one lane's traversal and a path has at most max_depth rays, so
    // the loop ends long before the guard; should the guard ever run out, the sample is
    // poisoned (NaN) rather than silently truncated, so no parity test can pass over it.
    bool finished = false;
    for (uint32_t guard = 0; guard < (1u << 16); ++guard) {
        const uint64_t runm = ballot(d.run);
        const bool ready = !upper && !d.run && !lane_in(runm >> 32);
        const uint64_t readym = ballot(ready);
        const bool pready = upper && lane_in(readym << 32);
        // IsInShadow's answer (shader.h:44-62) of the upper lanes whose pair is ready
        const uint64_t occ = ballot(pready && need_up && hs.slot >= 0 && hs.bestT < dist_up);
        if (ready && pend) {
            const bool occluded = lane_in(occ >> 32);
            radiance = add(radiance, mul(thr_p, (lit_p && !occluded) ? Lo_lit_p : Lo_p));
            pend = false;
        }
        if (pready) need_up = false;
        bool need = false;
        float dist = 0.f;
        f3 so = mk(0.f, 0.f, 0.f), sd = so;
        bool launch = false;  // lower lanes: a new path ray to trace
        if (ready && unproc) {
            unproc = false;
            const bool hit = alive && hs.slot >= 0;
            if (alive && !hit) {
                radiance = add(radiance, mul(thr, P.miss));
                alive = false;
            }
            if (hit) {
                const SurfHit sh = resolve_hit<false>(sc, ray, hs.slot);
                const DevMaterial m = material_of(sc, sh.tri);
                const f3 N = unit(sh.n);
                const f3 V = unit(sub(ray.o, sh.p));
                f3 Lo = mk(0.f, 0.f, 0.f);
                Lo = add(Lo, scale(mk(m.albedo[0], m.albedo[1], m.albedo[2]), 0.05f));
                Lo = add(Lo, mk(m.emission[0], m.emission[1], m.emission[2]));
                const DevLight& lt = sc.lights[0];
                const f3 lpos = mk(lt.pos[0], lt.pos[1], lt.pos[2]);
                f3 contrib = mk(0.f, 0.f, 0.f);
                bool lit = false;
                const f3 L = unit(sub(lpos, sh.p));
                const float NdotL = fmaxf(dot(N, L), 0.0f);
                if (NdotL > 0.0f) {
                    const f3 f = eval_brdf(m, sh.n, V, L);
                    const f3 rad = scale(mk(lt.color[0], lt.color[1], lt.color[2]), (float)lt.intensity);
                    contrib = scale(mul(rad, f), NdotL);
                    lit = true;
                    const f3 toL = sub(lpos, sh.p);
                    dist = sqrtf(dot(toL, toL));
                    if (dist > 0.0f) {
                        need = true;
                        so = add(sh.p, scale(N, RT_EPS));
                        sd = divf(toL, dist);
                    }
                }
                thr_p = thr;
                Lo_p = Lo;
                Lo_lit_p = add(Lo, contrib);
                lit_p = lit;
                pend = true;
                if (depth + 1 < max_depth) {
                    const float kd = m.kd, kr = m.kr, total = kd + kr;
                    if (total <= 0.0f) {
                        alive = false;
                    } else {
                        const f3 Nb = unit(sh.n);
                        const float xi = rng_next(rng);
                        if (P.diffuse_bounce && xi < kd / total) {
                            f3 dd = random_unit_vector(rng);
                            if (!(dot(dd, Nb) > 0.0f)) dd = mk(-dd.x, -dd.y, -dd.z);
                            ray = make_ray(add(sh.p, scale(Nb, RT_EPS)), dd, scene_bmax(sc));
                            const float nl = fmaxf(dot(Nb, dd), 0.0f);
                            thr = mul(thr, scale(mk(m.albedo[0], m.albedo[1], m.albedo[2]), 2.0f * nl));
                        } else {
                            const f3 I = unit(ray.d);
                            const f3 refl = sub(I, scale(Nb, 2.0f * dot(I, Nb)));
                            ray = make_ray(add(sh.p, scale(Nb, RT_EPS)), refl, scene_bmax(sc));
                            thr = mul(thr, scale(mk(m.spec[0], m.spec[1], m.spec[2]), kr));
                        }
                        if (thr.x < 1e-4f && thr.y < 1e-4f && thr.z < 1e-4f) alive = false;
                    }
                    ++depth;
                } else {
                    alive = false;
                }
            }
            launch = alive;
        }
        const uint64_t needm = ballot(need);
        const float ox = __shfl_xor(so.x, 32), oy = __shfl_xor(so.y, 32), oz = __shfl_xor(so.z, 32);
        const float dx = __shfl_xor(sd.x, 32), dy = __shfl_xor(sd.y, 32), dz = __shfl_xor(sd.z, 32);
        const float dd = __shfl_xor(dist, 32);
        bool go = launch;
        if (pready) {
            need_up = lane_in(needm << 32);
            dist_up = dd;
            if (need_up) ray = make_ray(mk(ox, oy, oz), mk(dx, dy, dz), scene_bmax(sc));
            go = need_up;
        }
        dfs_start(sc, ray, go, hs, d);
        if (launch) unproc = true;
        if (ballot(d.run || pend || unproc) == 0) {
            finished = true;
            break;
        }
        const uint32_t quota = (uint32_t)__popcll(ballot(d.run)) >> RT_RESUME_SHIFT;
        dfs_run(sc, ray, upper, dist_up, hs, d, stk, quota);
    }
    if (!finished) radiance = mk(__int_as_float(0x7fc00000), 0.f, 0.f);
}
#endif

// TraceRayIterative (query.h:156-220) from the camera ray's hit on, for half waves over one
// light, the lanes in pairs: a sample's path lives in lane l < 32 (the lanes that trace in a half
// wave), and lane l + 32, otherwise idle, traces that path's shadow rays.  The bounce direction
// does not depend on the shadow ray's answer (ShadeDirect draws no random numbers;
// shader.h:65-110), so the shadow ray of depth d and the bounce ray of depth d + 1 are traced by
// one per-lane traversal call, and depth d's `radiance += throughput * Lo` waits for that call:
// the adds keep their order.  Each call's time is its longest lane's, so a wave's path time
// drops from two calls per depth to one (c3b: the longest waves bound the kernel, DESIGN.md
// §4.10).  Same tests, same arithmetic and same order per sample as the unpaired loop: exact.
template <int MODE>
__device__ __forceinline__ void paired_bounces(const RenderParams& P, RayPre& ray, bool alive, f3& thr, f3& radiance,
                                               uint32_t& rng, float* park, HitState hs) {
    constexpr bool W = (MODE & MODE_WIDE) != 0;
    const SceneView& sc = P.sc;
    const bool upper = lane_id() >= 32;
    const int max_depth = P.max_depth;
    bool need_up = false;  // upper lanes: `ray` holds the shadow ray to trace
    float dist_up = 0.f;
    bool pend = false, lit_p = false;  // lower lanes: a depth's Lo awaits its shadow ray
    f3 thr_p = mk(0.f, 0.f, 0.f), Lo_p = thr_p, Lo_lit_p = thr_p;
    // hs: the closest hit of the path ray of `depth` (depth 0: the camera ray's, wave traversal)
    for (int depth = 0;; ++depth) {
        need_up = false;
        const bool hit = alive && hs.slot >= 0;
        if (alive && !hit) {
            radiance = add(radiance, mul(thr, P.miss));
            alive = false;
        }
        bool need = false;
        float dist = 0.f;
        f3 so = mk(0.f, 0.f, 0.f), sd = so;
        if (hit) {
            const SurfHit sh = resolve_hit<false>(sc, ray, hs.slot);
            const DevMaterial m = material_of(sc, sh.tri);
            // ShadeDirect (shader.h:65-110) over the one light
            const f3 N = unit(sh.n);
            const f3 V = unit(sub(ray.o, sh.p));
            f3 Lo = mk(0.f, 0.f, 0.f);
            Lo = add(Lo, scale(mk(m.albedo[0], m.albedo[1], m.albedo[2]), 0.05f));
            Lo = add(Lo, mk(m.emission[0], m.emission[1], m.emission[2]));
            const DevLight& lt = sc.lights[0];
            const f3 lpos = mk(lt.pos[0], lt.pos[1], lt.pos[2]);
            f3 contrib = mk(0.f, 0.f, 0.f);
            bool lit = false;
            const f3 L = unit(sub(lpos, sh.p));
            const float NdotL = fmaxf(dot(N, L), 0.0f);
            if (NdotL > 0.0f) {
                const f3 f = eval_brdf(m, sh.n, V, L);
                const f3 rad = scale(mk(lt.color[0], lt.color[1], lt.color[2]), (float)lt.intensity);
                contrib = scale(mul(rad, f), NdotL);
                lit = true;
                const f3 toL = sub(lpos, sh.p);
                dist = sqrtf(dot(toL, toL));
                if (dist > 0.0f) {
                    need = true;
                    so = add(sh.p, scale(N, RT_EPS));
                    sd = divf(toL, dist);
                }
            }
            thr_p = thr;
            Lo_p = Lo;
            Lo_lit_p = add(Lo, contrib);
            lit_p = lit;
            pend = true;
            // bounce (query.h:193-216)
            if (depth + 1 < max_depth) {
                const float kd = m.kd, kr = m.kr, total = kd + kr;
                if (total <= 0.0f) {
                    alive = false;
                } else {
                    const f3 Nb = unit(sh.n);
                    const float xi = rng_next(rng);
                    if (P.diffuse_bounce && xi < kd / total) {
                        f3 dd = random_unit_vector(rng);
                        if (!(dot(dd, Nb) > 0.0f)) dd = mk(-dd.x, -dd.y, -dd.z);
                        ray = make_ray(add(sh.p, scale(Nb, RT_EPS)), dd, scene_bmax(sc));
                        const float nl = fmaxf(dot(Nb, dd), 0.0f);
                        thr = mul(thr, scale(mk(m.albedo[0], m.albedo[1], m.albedo[2]), 2.0f * nl));
                    } else {
                        const f3 I = unit(ray.d);
                        const f3 refl = sub(I, scale(Nb, 2.0f * dot(I, Nb)));
                        ray = make_ray(add(sh.p, scale(Nb, RT_EPS)), refl, scene_bmax(sc));
                        thr = mul(thr, scale(mk(m.spec[0], m.spec[1], m.spec[2]), kr));
                    }
                    if (thr.x < 1e-4f && thr.y < 1e-4f && thr.z < 1e-4f) alive = false;
                }
            } else {
                alive = false;
            }
        }
        // the shadow ray to the partner lane (every lane shuffles: converged)
        const uint64_t needm = ballot(need);
        const float ox = __shfl_xor(so.x, 32), oy = __shfl_xor(so.y, 32), oz = __shfl_xor(so.z, 32);
        const float dx = __shfl_xor(sd.x, 32), dy = __shfl_xor(sd.y, 32), dz = __shfl_xor(sd.z, 32);
        const float dd = __shfl_xor(dist, 32);
        if (upper) {
            need_up = lane_in(needm << 32);
            dist_up = dd;
            if (need_up) ray = make_ray(mk(ox, oy, oz), mk(dx, dy, dz), scene_bmax(sc));
        }
        // (a depth's Lo may wait with no shadow ray to trace: NdotL <= 0 or a zero distance)
        if (ballot(alive || need_up || pend) == 0) break;
        traverse_lane<W>(sc, ray, alive || need_up, upper, dist_up, hs, reinterpret_cast<uint32_t*>(park));
#ifdef RT_LANE_ITERS
        lane_iters_note((alive || need_up) ? hs.iters : 0u);
#endif
        // IsInShadow's answer (shader.h:44-62) of the upper lanes, read by their lower partners
        const uint64_t occ = ballot(need_up && hs.slot >= 0 && hs.bestT < dist_up);
        if (pend) {
            const bool occluded = lane_in(occ >> 32);
            radiance = add(radiance, mul(thr_p, (lit_p && !occluded) ? Lo_lit_p : Lo_p));
            pend = false;
        }
    }
}

// One camera sample through TraceRayIterative (query.h:156-220) + ShadeDirect (shader.h).
// All lanes of a wave call it; `valid` marks lanes owning a sample.  D1: max_depth == 1 (no
// bounce; the configuration the benchmarks run).
template <int MODE, bool D1, int PAIR = 0>
// The primary-hit AOV (P.hit_idx / P.hit_t at element aov, when aov >= 0) is written as soon as
// the camera ray's traversal ends, so nothing of it stays live across the shading.
// park: the lane's own LDS slot (slot k of the lane at park[k * BLOCK]).
// PAIR (half waves): 1, the camera ray's shading on in paired_bounces when the scene has one
// light; 2, always (the paired-only kernels, LS = 3: no unpaired loop in the kernel).
__device__ __forceinline__ f3 trace_sample(const RenderParams& P, bool valid, int x, int y, int s, int64_t aov,
                                          float* park, float* park_wave) {
    const SceneView& sc = P.sc;
    RayPre ray = camera_ray(P, valid, x, y, s);
    count_rays<MODE>(P.ray_count, 3, valid && P.max_depth > 0);  // camera rays that reach traversal
    if constexpr (D1) {
        // the AOV index waits in LDS across the traversal (PARK slots 12-13; kept in registers
        // it was spilled to scratch in the 64-VGPR build)
        const Park pk{park_wave};
        pk.put(12, __int_as_float((int32_t)aov));
        pk.put(13, __int_as_float((int32_t)(aov >> 32)));
        Park::fence();
        HitState hs;
        traverse_camera<MODE>(sc, ray, valid, hs);
        Park::fence();
        aov = (int64_t)(uint32_t)__float_as_int(pk.get(12)) | ((int64_t)__float_as_int(pk.get(13)) << 32);
        RT_PHASE(P, x, y, 0);
#ifdef RT_STATS
        if constexpr (MODE != RT_KERNEL_LANE && (MODE & MODE_DEEP) == 0) {
            if (ballot(valid) != 0 && ballot(valid && hs.slot >= 0) == 0) {
                RT_STAT(15, 1);
                RT_STAT(16, hs.pops);
            }
        }
#endif
        if (valid) {
            if (aov >= 0) {
                P.hit_idx[aov] = hs.slot >= 0 ? leaf_tri<(MODE & MODE_DEEP) != 0>(sc, hs.slot) : -1;
                P.hit_t[aov] = hs.slot >= 0 ? hs.bestT : -1.0f;
            }
        }
        return shade_d1<MODE>(P, valid, ray, hs, park_wave);
    }
    uint32_t rng = make_rng_seed(x, y, s);

    f3 radiance = mk(0.f, 0.f, 0.f);
    f3 thr = mk(1.f, 1.f, 1.f);
    const int max_depth = P.max_depth;
    bool alive = valid && max_depth > 0;
    bool paired = PAIR == 2;
    if constexpr (PAIR == 1 && MODE != RT_KERNEL_LANE && (MODE & MODE_DEEP) == 0)
        paired = sc.num_lights == 1 && lane_ok<(MODE & MODE_WIDE) != 0>(sc);
    if constexpr (PAIR != 0 && MODE != RT_KERNEL_LANE && (MODE & MODE_DEEP) == 0) {
        if (PAIR == 2 || paired) {
            // depth 0's camera ray takes the wave traversal; its shadow ray and every later ray
            // go to paired_bounces' per-lane traversals
            HitState hs;
            traverse_camera<MODE>(sc, ray, alive, hs);
            if (valid && aov >= 0) {
                const bool hit = alive && hs.slot >= 0;
                P.hit_idx[aov] = hit ? leaf_tri<false>(sc, hs.slot) : -1;
                P.hit_t[aov] = hit ? hs.bestT : -1.0f;
            }
#ifdef RT_RESUME
            if constexpr ((MODE & MODE_WIDE) != 0 && PAIR == 2)
                paired_bounces_resume<MODE>(P, ray, alive, thr, radiance, rng, park, hs);
            else
#endif
                paired_bounces<MODE>(P, ray, alive, thr, radiance, rng, park, hs);
            return clamp01(radiance);
        }
    }
    for (int depth = 0; depth < max_depth; ++depth) {
        if (ballot(alive) == 0) break;
        HitState hs;
        if (depth > 0) count_rays<MODE>(P.ray_count, 2, alive);
        if (depth == 0) traverse_camera<MODE>(sc, ray, alive, hs);
        else traverse_at<MODE>(sc, depth, ray, alive, false, 0.0f, hs, park);
        const bool hit = alive && hs.slot >= 0;
        SurfHit sh;
        sh.tri = -1;
        if (hit) sh = resolve_hit<(MODE & MODE_DEEP) != 0>(sc, ray, hs.slot);
        if (depth == 0 && valid) {
            if (aov >= 0) {
                P.hit_idx[aov] = hit ? sh.tri : -1;
                P.hit_t[aov] = hit ? hs.bestT : -1.0f;
            }
        }
        if (alive && !hit) {
            radiance = add(radiance, mul(thr, P.miss));
            alive = false;
        }
        // ShadeDirect (shader.h:65-110)
        f3 N = mk(0.f, 0.f, 1.f), V = N, Lo = mk(0.f, 0.f, 0.f);
        if (hit) {
            const DevMaterial m = material_of(sc, sh.tri);
            N = unit(sh.n);
            V = unit(sub(ray.o, sh.p));
            Lo = add(Lo, scale(mk(m.albedo[0], m.albedo[1], m.albedo[2]), 0.05f));
            Lo = add(Lo, mk(m.emission[0], m.emission[1], m.emission[2]));
        }
        for (int li = 0; li < sc.num_lights; ++li) {
            const DevLight& lt = sc.lights[li];
            const f3 lpos = mk(lt.pos[0], lt.pos[1], lt.pos[2]);
            float dist = 0.f;
            bool need = false, lit = false;
            f3 contrib = mk(0.f, 0.f, 0.f);
            RayPre sray;  // unset for lanes without a shadow ray (masked out by the traversal)
            if (hit) {
                const f3 L = unit(sub(lpos, sh.p));
                const float NdotL = fmaxf(dot(N, L), 0.0f);
                if (NdotL > 0.0f) {
                    // The light's term, added below if the shadow ray is clear (the material is
                    // re-read per light so it is not live across the traversal).
                    const DevMaterial m = material_of(sc, sh.tri);
                    const f3 f = eval_brdf(m, sh.n, V, L);
                    const f3 rad = scale(mk(lt.color[0], lt.color[1], lt.color[2]), (float)lt.intensity);
                    contrib = scale(mul(rad, f), NdotL);
                    lit = true;
                    // IsInShadow (shader.h:44-62)
                    const f3 toL = sub(lpos, sh.p);
                    dist = sqrtf(dot(toL, toL));
                    if (dist > 0.0f) {
                        need = true;
                        sray = make_ray(add(sh.p, scale(N, RT_EPS)), divf(toL, dist), scene_bmax(sc));
                    }
                }
            }
            HitState shs;
            count_rays<MODE>(P.ray_count, 1, need);
            traverse_at<MODE>(sc, depth, sray, need, true, dist, shs, park);
            const bool occluded = need && shs.slot >= 0 && shs.bestT < dist;
            if (lit && !occluded) Lo = add(Lo, contrib);
        }
        if (hit) {
            radiance = add(radiance, mul(thr, Lo));
            // bounce (query.h:193-216); skipped after the last depth where it has no effect
            if (depth + 1 < max_depth) {
                const DevMaterial m = material_of(sc, sh.tri);
                const float kd = m.kd, kr = m.kr, total = kd + kr;
                if (total <= 0.0f) {
                    alive = false;
                } else {
                    const f3 Nb = unit(sh.n);
                    const float xi = rng_next(rng);
                    if (P.diffuse_bounce && xi < kd / total) {
                        f3 dd = random_unit_vector(rng);
                        if (!(dot(dd, Nb) > 0.0f)) dd = mk(-dd.x, -dd.y, -dd.z);
                        ray = make_ray(add(sh.p, scale(Nb, RT_EPS)), dd, scene_bmax(sc));
                        const float nl = fmaxf(dot(Nb, dd), 0.0f);
                        thr = mul(thr, scale(mk(m.albedo[0], m.albedo[1], m.albedo[2]), 2.0f * nl));
                    } else {
                        const f3 I = unit(ray.d);
                        const f3 refl = sub(I, scale(Nb, 2.0f * dot(I, Nb)));
                        ray = make_ray(add(sh.p, scale(Nb, RT_EPS)), refl, scene_bmax(sc));
                        thr = mul(thr, scale(mk(m.spec[0], m.spec[1], m.spec[2]), kr));
                    }
                    if (thr.x < 1e-4f && thr.y < 1e-4f && thr.z < 1e-4f) alive = false;
                }
            } else {
                alive = false;
            }
        }
    }
    return clamp01(radiance);
}

// ---- tile culling ---------------------------------------------------------------------
// A tile is culled only if every camera ray of pixels [x0,x1] x rows [y0,y1] provably fails
// intersectAABB(ray, B, 1e-4, FLT_MAX) (bvh.h:81-129) for every box B of a cut of the tree (a
// set of nodes holding every leaf exactly once: the root alone, or the cut the scene keeps in
// sc.cut).  SearchBVH only tests a triangle after its ancestors' box tests passed, with tmax =
// bestT <= FLT_MAX (a smaller tmax only fails more), so such a ray tests no triangle: a miss.
// Ray directions are positive multiples of D(px,py) = pixel00 + px*du + py*dv - center with
// px in [x0-0.5, x1+0.5) (jitter), an affine map: its per-component range over the
// (1-pixel-padded) tile comes from the corners, widened by 1e-5*|D| plus 8 float ulps of every
// term to cover the float rounding of the per-sample computation (pixel position, difference,
// cam_unit).  Scaling d by k > 0 scales every slab parameter by 1/k, so "some axis's entry >
// another axis's exit" is scale-free.  An axis whose component can come near 0
// (|d_a| < 1e-6 |d|, far above the 1e-8 parallel threshold) is ignored (no constraint):
// conservative.  A box is missed iff, with 1e-9 relative slack (the reference's doubles carry
// ~1e-15; the reciprocals below add ~1e-16), some axis's smallest entry exceeds some axis's
// largest exit, or some axis's largest exit is < 0 (< tmin).  The camera inside a padded box
// never culls.
struct TileDirs {
    double c[3], Dl[3], Dh[3], iDl[3], iDh[3], scale;
    bool usable;
};
__device__ __forceinline__ TileDirs tile_dirs(const RenderParams& P, int x0, int x1, int y0, int y1) {
    TileDirs T;
    const double p0[3] = {P.cam_p00.x, P.cam_p00.y, P.cam_p00.z};
    const double du[3] = {P.cam_du.x, P.cam_du.y, P.cam_du.z};
    const double dv[3] = {P.cam_dv.x, P.cam_dv.y, P.cam_dv.z};
    T.c[0] = P.cam_center.x;
    T.c[1] = P.cam_center.y;
    T.c[2] = P.cam_center.z;
    const double pxl = x0 - 1.0, pxh = x1 + 1.0, pyl = y0 - 1.0, pyh = y1 + 1.0;
    const double pxm = fmax(fabs(pxl), fabs(pxh)), pym = fmax(fabs(pyl), fabs(pyh));
    T.scale = 0.0;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double base = p0[a] - T.c[a];
        const double u0 = pxl * du[a], u1 = pxh * du[a], v0 = pyl * dv[a], v1 = pyh * dv[a];
        const double ulp = 8.0 * 1.1920928955078125e-7 * (fabs(T.c[a]) + fabs(p0[a]) + pxm * fabs(du[a]) + pym * fabs(dv[a]));
        T.Dl[a] = base + fmin(u0, u1) + fmin(v0, v1) - ulp;
        T.Dh[a] = base + fmax(u0, u1) + fmax(v0, v1) + ulp;
        T.scale = fmax(T.scale, fmax(fabs(T.Dl[a]), fabs(T.Dh[a])));
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        T.Dl[a] -= 1e-5 * T.scale;
        T.Dh[a] += 1e-5 * T.scale;
        T.iDl[a] = 1.0 / T.Dl[a];
        T.iDh[a] = 1.0 / T.Dh[a];
    }
    T.usable = T.scale > 0.0;
    return T;
}

__device__ __forceinline__ bool tile_misses_box(const TileDirs& T, const float* bx) {
    const double mn[3] = {bx[0], bx[1], bx[2]}, mx[3] = {bx[3], bx[4], bx[5]};
    bool inside = true;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double tol = 1e-6 * (fabs(mn[a]) + fabs(mx[a]) + fabs(T.c[a])) + 1e-30;
        inside = inside && T.c[a] >= mn[a] - tol && T.c[a] <= mx[a] + tol;
    }
    if (inside || !T.usable || !(mn[0] <= mx[0] && mn[1] <= mx[1] && mn[2] <= mx[2])) return false;
    double entry_min = -INFINITY, exit_max = INFINITY;  // max over axes of min entry; min of max exit
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        if (!(T.Dl[a] > 1e-6 * T.scale || T.Dh[a] < -1e-6 * T.scale)) continue;  // may be ~parallel
        const double nA = mn[a] - T.c[a], xA = mx[a] - T.c[a];
        // d > 0: entry (mn-c)/d, exit (mx-c)/d; d < 0: swapped.  Over d in [Dl, Dh] each
        // quotient is monotone in d, so its range sits at the endpoints.
        const double ne = T.Dl[a] > 0 ? nA : xA, nx = T.Dl[a] > 0 ? xA : nA;
        const double e0 = ne * T.iDl[a], e1 = ne * T.iDh[a];
        const double f0 = nx * T.iDl[a], f1 = nx * T.iDh[a];
        entry_min = fmax(entry_min, fmin(e0, e1));
        exit_max = fmin(exit_max, fmax(f0, f1));
    }
    if (!(exit_max == exit_max) || !(entry_min == entry_min)) return false;
    if (exit_max < -1e-9 * fabs(exit_max) - 1e-30) return true;
    return entry_min - exit_max > 1e-9 * (fabs(entry_min) + fabs(exit_max)) + 1e-30;
}

// Float form of tile_dirs / tile_misses_box for tile_cut_kernel (a wave-uniform computation
// per tile, made 64 times more often than the root test).  Every bound carries its own float
// rounding on top of the double version's margins: the tile corners are padded by twice the
// per-sample ulp term (the corner sums are themselves float), and the miss decisions keep a
// 1e-4 relative slack (the float entry/exit bounds are within ~5 float ulps of the exact
// quotients), so a culled tile is still one whose every ray fails the reference's double test.
struct TileDirsF {
    float c[3], Dl[3], Dh[3], iDl[3], iDh[3], scale;
    bool usable;
};
__device__ __forceinline__ TileDirsF tile_dirs_f(const RenderParams& P, int x0, int x1, int y0, int y1) {
    TileDirsF T;
    const float p0[3] = {P.cam_p00.x, P.cam_p00.y, P.cam_p00.z};
    const float du[3] = {P.cam_du.x, P.cam_du.y, P.cam_du.z};
    const float dv[3] = {P.cam_dv.x, P.cam_dv.y, P.cam_dv.z};
    T.c[0] = P.cam_center.x;
    T.c[1] = P.cam_center.y;
    T.c[2] = P.cam_center.z;
    const float pxl = (float)x0 - 1.0f, pxh = (float)x1 + 1.0f, pyl = (float)y0 - 1.0f, pyh = (float)y1 + 1.0f;
    const float pxm = fmaxf(fabsf(pxl), fabsf(pxh)), pym = fmaxf(fabsf(pyl), fabsf(pyh));
    T.scale = 0.0f;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float base = p0[a] - T.c[a];
        const float u0 = pxl * du[a], u1 = pxh * du[a], v0 = pyl * dv[a], v1 = pyh * dv[a];
        const float ulp = 16.0f * 1.1920928955078125e-7f * (fabsf(T.c[a]) + fabsf(p0[a]) + pxm * fabsf(du[a]) + pym * fabsf(dv[a]));
        T.Dl[a] = base + fminf(u0, u1) + fminf(v0, v1) - ulp;
        T.Dh[a] = base + fmaxf(u0, u1) + fmaxf(v0, v1) + ulp;
        T.scale = fmaxf(T.scale, fmaxf(fabsf(T.Dl[a]), fabsf(T.Dh[a])));
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        T.Dl[a] -= 1.1e-5f * T.scale;
        T.Dh[a] += 1.1e-5f * T.scale;
        // v_rcp_f32 (1 ulp): far inside the 1e-4 decision slack, and ~10x cheaper than the
        // correctly rounded division
        T.iDl[a] = rcp_approx(T.Dl[a]);
        T.iDh[a] = rcp_approx(T.Dh[a]);
    }
    T.usable = T.scale > 0.0f && T.scale < 1e30f;
    return T;
}

__device__ __forceinline__ bool tile_misses_box_f(const TileDirsF& T, const float* bx) {
    const float mn[3] = {bx[0], bx[1], bx[2]}, mx[3] = {bx[3], bx[4], bx[5]};
    bool inside = true;
    float mag = 0.0f, imax = 0.0f;  // magnitude of the subtraction operands, largest |1/D|
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float tol = 1e-4f * (fabsf(mn[a]) + fabsf(mx[a]) + fabsf(T.c[a])) + 1e-30f;
        inside = inside && T.c[a] >= mn[a] - tol && T.c[a] <= mx[a] + tol;
        mag = fmaxf(mag, fabsf(mn[a]) + fabsf(mx[a]) + fabsf(T.c[a]));
    }
    if (inside || !T.usable || !(mn[0] <= mx[0] && mn[1] <= mx[1] && mn[2] <= mx[2]) || !(mag < 1e30f)) return false;
    float entry_min = -INFINITY, exit_max = INFINITY;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        if (!(T.Dl[a] > 1e-6f * T.scale || T.Dh[a] < -1e-6f * T.scale)) continue;  // may be ~parallel
        imax = fmaxf(imax, fmaxf(fabsf(T.iDl[a]), fabsf(T.iDh[a])));
        const float nA = mn[a] - T.c[a], xA = mx[a] - T.c[a];
        const float ne = T.Dl[a] > 0.0f ? nA : xA, nx = T.Dl[a] > 0.0f ? xA : nA;
        const float e0 = ne * T.iDl[a], e1 = ne * T.iDh[a];
        const float f0 = nx * T.iDl[a], f1 = nx * T.iDh[a];
        entry_min = fmaxf(entry_min, fminf(e0, e1));
        exit_max = fminf(exit_max, fmaxf(f0, f1));
    }
    if (!(exit_max == exit_max) || !(entry_min == entry_min)) return false;
    const float abs_slack = 1e-4f * mag * imax + 1e-30f;
    if (!(abs_slack < 1e30f)) return false;
    if (exit_max < -1e-4f * fabsf(exit_max) - abs_slack) return true;
    return entry_min - exit_max > 1e-4f * (fabsf(entry_min) + fabsf(exit_max)) + abs_slack;
}

// The root test of tile_cull_kernel, one lane per tile: the float form (its bounds carry their
// own rounding, see tile_dirs_f; 2x cheaper than the double form on the 129,600 c3 tiles).
__device__ __forceinline__ bool tile_misses_root(const RenderParams& P, int x0, int x1, int y0, int y1) {
    return tile_misses_box_f(tile_dirs_f(P, x0, x1, y0, y1), P.sc.root_box);
}

// What a sample that misses the root returns: clamp(0 + (1,1,1) * missColor) (query.h:181-183),
// or 0 when max_depth <= 0 (query.h:172).
__device__ __forceinline__ f3 miss_sample_color(const RenderParams& P) {
    if (P.max_depth <= 0) return mk(0.f, 0.f, 0.f);
    return clamp01(add(mk(0.f, 0.f, 0.f), mul(mk(1.f, 1.f, 1.f), P.miss)));
}

// Local row -> image row for the band sharding of rt_render_opts.
__device__ __forceinline__ int global_row(const RenderParams& P, int r) {
    if (P.band_count <= 1) return r;
    const int k = r / P.band_rows, within = r - k * P.band_rows;
    return (P.band_index + k * P.band_count) * P.band_rows + within;
}

// ---- tile work lists ---------------------------------------------------------------------
// Pre-pass, one lane per pixel tile: a tile whose every ray provably misses the root box gets
// its pixels written here (P.miss_pixel = the reference's sum of spp miss samples / spp; hit
// AOV -1), every other tile is appended to a live list the render kernels dequeue.
// There are P.nqueues lists.  Workgroups are dealt round-robin over the 8 XCDs, so with 8
// lists the render kernel's queue blockIdx % 8 runs on one XCD: RT_TILES_ROWS gives it the tile rows k, k+8,
// ... (neighbouring tiles share an L2, the work spreads evenly); RT_TILES_XCD_CHUNK gives it
// a contiguous 1/8 of the frame.
// RT_TILES_LINEAR is one list in raster order.  The order is a speed property only.
// The lists' length counters sit 256 B apart (separate channels) so the appends do not
// serialise.
constexpr int COUNTER_STRIDE = 64;
// Heavy cost classes: 5, of which depth-1 frames use the first 3 (c3 0.1835 ms with 3 vs
// 0.1859 with 4 and 0.1862 with 5) and multi-bounce frames all 5 (c3b 1.768 vs 1.898 ms with 3:
// their waves' durations spread wider; profiles/r03/exp/heavy_classes_ab_*.log).
#ifndef RT_NCLASS
#define RT_NCLASS 5
#endif
constexpr int NCLASS = RT_NCLASS;                // (<= 8)
constexpr int NCLASS_D1 = 3;
// A counter set: 9 list counters COUNTER_STRIDE apart (8 live lists + a spare), then the
// heavy list lengths packed (class-major, 8 per class), the 8 cut survivor lengths and the 8
// work-queue heads, each in its own slot.
constexpr int HEAVY_SLOT0 = 9;
constexpr int CUT_SLOT0 = HEAVY_SLOT0 + 8 * NCLASS;  // then 8: lengths of the cut pass's survivor lists
constexpr int HEAD_SLOT0 = CUT_SLOT0 + 8;  // then 8: the render kernel's work-queue heads (one per XCD)
constexpr int COUNTER_SLOTS = HEAD_SLOT0 + 8;
constexpr int COUNTER_SET_U32 = COUNTER_SLOTS * COUNTER_STRIDE;
__host__ __device__ constexpr int heavy_counter(int k, int q) { return (HEAVY_SLOT0 + 8 * k + q) * COUNTER_STRIDE; }
__device__ __forceinline__ int queue_of_tile(const RenderParams& P, int tile) {
    if (P.nqueues == 1) return 0;
    if (P.tile_order == RT_TILES_XCD_CHUNK) return (int)((int64_t)tile * 8 / P.tiles_total);
    return (tile / P.tiles_x) & 7;
}

// Miss pixels (and hit AOV -1) of a culled tile, written by the lanes of `lanes` threads
// starting at `first` (one lane per tile in tile_cull_kernel, a whole wave in tile_cut_kernel).
__device__ __forceinline__ void write_culled_tile(const RenderParams& P, int tile, int first, int lanes) {
    const int tx = tile % P.tiles_x, ty = tile / P.tiles_x;
    const int xa = tx * P.tile_w, ra = ty * P.tile_h;
    const int tw = min(xa + P.tile_w, P.W) - xa, th = min(ra + P.tile_h, P.rows) - ra;
    const float mp[3] = {P.miss_pixel.x, P.miss_pixel.y, P.miss_pixel.z};
    if (lanes == 1 && tw == 4 && (xa & 3) == 0 && (P.W & 3) == 0 && ((uintptr_t)P.rgb & 15) == 0 &&
        ((uintptr_t)P.p6 & 3) == 0) {
        // 4-pixel rows (the common tile width): 48 B of floats as three 16-byte stores and 12 B
        // of samples as three 4-byte stores per row (W and x multiples of 4: aligned)
        const float4 f0 = make_float4(mp[0], mp[1], mp[2], mp[0]), f1 = make_float4(mp[1], mp[2], mp[0], mp[1]),
                     f2 = make_float4(mp[2], mp[0], mp[1], mp[2]);
        const uint32_t b0 = P.miss_p6[0], b1 = P.miss_p6[1], b2 = P.miss_p6[2];
        const uint32_t w0 = b0 | b1 << 8 | b2 << 16 | b0 << 24, w1 = b1 | b2 << 8 | b0 << 16 | b1 << 24,
                       w2 = b2 | b0 << 8 | b1 << 16 | b2 << 24;
        for (int r = ra; r < ra + th; ++r) {
            if (P.rgb) {
                float4* o = reinterpret_cast<float4*>(P.rgb + ((size_t)r * P.W + xa) * 3);
                o[0] = f0;
                o[1] = f1;
                o[2] = f2;
            }
            if (P.p6) {
                uint32_t* q = reinterpret_cast<uint32_t*>(P.p6 + ((size_t)r * P.W + xa) * 3);
                q[0] = w0;
                q[1] = w1;
                q[2] = w2;
            }
        }
    } else {
        for (int i = first; i < tw * th * 3; i += lanes) {
            const int px = i / 3, c = i - 3 * px;
            const int r = ra + px / tw, x = xa + px % tw;
            // component c by selects (an array indexed by c would live in scratch)
            if (P.rgb) P.rgb[((size_t)r * P.W + x) * 3 + c] = c == 0 ? mp[0] : c == 1 ? mp[1] : mp[2];
            if (P.p6) P.p6[((size_t)r * P.W + x) * 3 + c] = c == 0 ? P.miss_p6[0] : c == 1 ? P.miss_p6[1] : P.miss_p6[2];
        }
    }
    if (P.hit_idx) {
        for (int i = first; i < tw * th * P.spp; i += lanes) {
            const int px = i / P.spp, smp = i - P.spp * px;
            const int r = ra + px / tw, x = xa + px % tw;
            const size_t k = ((size_t)r * P.W + x) * (size_t)P.spp + smp;
            P.hit_idx[k] = -1;
            P.hit_t[k] = -1.0f;
        }
    }
}

// Wave-aggregated append of the lanes with `live` to the live list of their tile: one atomic
// per (wave, list).
__device__ __forceinline__ void append_live(const RenderParams& P, bool live, int tile) {
    const int q = live ? queue_of_tile(P, tile) : 0;
    const uint32_t lane = lane_id();
    uint64_t pending = ballot(live);
    while (pending != 0) {
        const uint32_t leader = (uint32_t)__builtin_ctzll(pending);
        const int lq = rdlane(q, leader);
        const uint64_t m = pending & ballot(q == lq);
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&P.live_count[lq * COUNTER_STRIDE], (uint32_t)__popcll(m));
        base = rdlane(base, leader);
        if ((m >> lane) & 1ull)
            P.live_tiles[(size_t)lq * P.queue_cap + base + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = tile;
        pending &= ~m;
    }
}

// The root test of one tile per lane (tiles past the end: no-ops); survivors to the live lists.
__device__ __forceinline__ void cull_tiles(const RenderParams& P, int tile) {
    bool live = false;
    if (tile < P.tiles_total) {
        const int tx = tile % P.tiles_x, ty = tile / P.tiles_x;
        const int xa = tx * P.tile_w, ra = ty * P.tile_h;
        const int xb = min(xa + P.tile_w, P.W) - 1, rb = min(ra + P.tile_h, P.rows) - 1;
        const bool culled = P.cull && tile_misses_root(P, xa, xb, global_row(P, ra), global_row(P, rb));
        if (culled) write_culled_tile(P, tile, 0, 1);
        else live = true;
    }
    append_live(P, live, tile);
}

// Pass 1, one lane per tile: the root test; the survivors go to the live lists.
__global__ __launch_bounds__(BLOCK) void tile_cull_kernel(RenderParams P) {
    __builtin_amdgcn_s_setprio(3);  // ahead of the previous frame's render waves (see Launch)
    // Counter sets rotate over six frames (no reset launch): this frame's set was zeroed by the
    // pass of the frame two before it; zero the set of the frame two after it (its last user,
    // frame k-4, has finished: the scene's prep stream waited for it).
    if (blockIdx.x == 0 && threadIdx.x < COUNTER_SLOTS) P.next_count[threadIdx.x * COUNTER_STRIDE] = 0u;
#ifdef RT_FRAME_SPAN
    if (threadIdx.x == 0 && g_frame_span) atomicMin(&g_frame_span[4 * (P.drain_tag & 255u) + 2], wall_clock64());
#endif
    cull_tiles(P, (int)(blockIdx.x * BLOCK + threadIdx.x));
}

// Pass 2 (sc.ncut > 0), one wave per CUT_GROUP consecutive slots of a live list, one lane
// per box of the cut (sc.cut, <= 64 boxes that hold every leaf exactly once): a tile is culled
// when every lane proves its box missed by every ray of the tile (tile_misses_box_f; the tile
// bounds are wave-uniform).  A culled tile gets its miss pixels here; the others go to list q's
// heavy lists (below) or its survivor list, one atomic per (wave, list): the render kernel's
// blocks then find only real tiles (a block for a culled or moved slot that leaves at once still
// cost its launch and loads).  The pass runs on the scene's prep stream, overlapping the
// previous frame's render kernel, so its atomics are off the critical path.
#ifndef RT_CUT_GROUP
#define RT_CUT_GROUP 8
#endif
constexpr int CUT_GROUP = RT_CUT_GROUP;
// The cut pass's test condition and this lane's box of the cut (loaded once per wave).
__device__ __forceinline__ bool cut_setup(const RenderParams& P, uint32_t lane, float* box, int& max_len) {
    int n = 0;
    max_len = 0;
    for (int k = 0; k < P.nqueues; ++k) {
        const int l = (int)ldc_u32(&P.live_count[k * COUNTER_STRIDE]);
        n += l;
        max_len = max(max_len, l);
    }
    // When the root test already keeps more than a quarter of the tiles the scene fills the
    // view and the cut rarely removes one (c5's heightfield: none of 739,248): flags 0, no
    // tests (a speed choice only: keeping a tile is always exact).
    const bool test = P.cut_force || 4 * (int64_t)n <= (int64_t)P.tiles_total;
    if (test && (int)lane < P.sc.ncut) {
#pragma unroll
        for (int i = 0; i < 6; ++i) box[i] = P.sc.cut[6 * (size_t)lane + i];
    }
    return test;
}

// The cut's second level for one tile: hm = the cut boxes some ray of the tile may reach (a
// wave-uniform mask).  Their sub-boxes (sc.cut2: S = 2^cut_sub_log2 per cut box, a cut of its
// subtree) are tested 64 at a time, 64 / S cut boxes per pass, lane l taking sub-box l % S of
// the (l / S)-th remaining box of hm.  True when a sub-box may be reached; false when every one
// is provably missed by every ray of the tile, which, with the cut boxes outside hm, proves that
// no ray reaches any leaf (each leaf has an ancestor-or-self among the tested boxes, and
// SearchBVH reaches a triangle only after every ancestor's box test passed).
__device__ __forceinline__ bool tile_cut_sub(const RenderParams& P, const TileDirsF& T, uint64_t hm, uint32_t lane) {
    const int sl = P.sc.cut_sub_log2;
    const int per = 64 >> sl;
    const int gi = (int)(lane >> sl);
    const uint32_t c = lane & ((1u << sl) - 1u);
    while (hm != 0) {
        int mine = -1;
        for (int k = 0; k < per && hm != 0; ++k) {
            const int b = __builtin_ctzll(hm);
            if (gi == k) mine = b;
            hm &= hm - 1;
        }
        bool reach = false;
        if (mine >= 0) {
            const float* p = P.sc.cut2 + 6 * (((size_t)mine << sl) | c);
            const float bx[6] = {p[0], p[1], p[2], p[3], p[4], p[5]};
            reach = !tile_misses_box_f(T, bx);
        }
        if (ballot(reach) != 0) return true;
    }
    return false;
}

// One unit of the cut pass: group g (CUT_GROUP consecutive slots) of live list q; false when
// the group is past the list's end.
__device__ __forceinline__ bool cut_unit(const RenderParams& P, uint32_t lane, int q, int g, bool test,
                                         const float* box) {
    const int len = (int)ldc_u32(&P.live_count[q * COUNTER_STRIDE]);
    if (CUT_GROUP * g >= len) return false;
    const int m = min(CUT_GROUP, len - CUT_GROUP * g);
    const size_t slot0 = (size_t)q * P.queue_cap + (size_t)(CUT_GROUP * g);
    const int my_tile = (int)lane < m ? P.live_tiles[slot0 + lane] : -1;
    // the tile's last render cost, loaded before the tests so the load overlaps them
    uint2 cost = make_uint2(0u, 0u);
    if (P.heavy_cap > 0 && (int)lane < m) cost = *reinterpret_cast<const uint2*>(P.tile_cost + 4 * (size_t)my_tile);
    uint64_t culled = 0;
    for (int j = 0; test && j < m; ++j) {
        const int tile = (int)rdlane((uint32_t)my_tile, (uint32_t)j);
        const int tx = tile % P.tiles_x, ty = tile / P.tiles_x;
        const int xa = tx * P.tile_w, ra = ty * P.tile_h;
        const int xb = min(xa + P.tile_w, P.W) - 1, rb = min(ra + P.tile_h, P.rows) - 1;
        const TileDirsF T = tile_dirs_f(P, xa, xb, global_row(P, ra), global_row(P, rb));
        const bool hit = (int)lane < P.sc.ncut && !tile_misses_box_f(T, box);
#ifdef RT_WAVE_TIMES
        {
            const uint64_t hm = ballot(hit);
            if (g_cut_counts && lane == 0) g_cut_counts[tile] = __popcll(hm);
        }
#endif
        const uint64_t hm = ballot(hit);
        if (hm == 0 || (P.sc.cut_sub_log2 > 0 && !tile_cut_sub(P, T, hm, lane))) {
            write_culled_tile(P, tile, (int)lane, 64);
            culled |= 1ull << j;
        }
    }
    // Heavy-first: a surviving tile whose last render took >= heavy_ticks[c] goes to list q's
    // class-c heavy list, the others to its survivor list (the render kernel's normal part).
    // The appends take one vector atomic, lane k adding class k's count (lane NCLASS the
    // survivors'), so a group pays one round trip for them.
    int cls = -1;  // -1: no tile, or culled
    if ((int)lane < m && !((culled >> lane) & 1ull)) {
        cls = NCLASS;
        if (P.heavy_cap > 0) {
            const uint32_t mx = max(max(cost.x & 0xffffu, cost.x >> 16), max(cost.y & 0xffffu, cost.y >> 16));
            for (int k = NCLASS - 1; k >= 0; --k)
                if (mx >= P.heavy_ticks[k]) cls = k;
        }
    }
    uint64_t cm[NCLASS + 1];
    uint32_t add = 0;
#pragma unroll
    for (int k = 0; k <= NCLASS; ++k) {
        cm[k] = ballot(cls == k);
        if ((int)lane == k) add = (uint32_t)__popcll(cm[k]);
    }
    const uint64_t below = (1ull << lane) - 1;
    if (ballot(add != 0) != 0) {
        uint32_t base = 0;
        if ((int)lane <= NCLASS && add != 0)
            base = atomicAdd(&P.live_count[(int)lane < NCLASS ? heavy_counter((int)lane, q) : (CUT_SLOT0 + q) * COUNTER_STRIDE], add);
        bool spill = false;  // a heavy tile past its list's capacity goes to the survivor list
#pragma unroll
        for (int k = 0; k <= NCLASS; ++k) {
            const uint32_t idx = rdlane(base, (uint32_t)k) + (uint32_t)__popcll(cm[k] & below);
            if (cls == k) {
                if (k == NCLASS) P.cut_tiles[(size_t)q * P.queue_cap + idx] = my_tile;
                else if (idx < (uint32_t)P.heavy_cap) P.heavy_tiles[((size_t)k * 8 + q) * P.heavy_cap + idx] = my_tile;
                else spill = true;
            }
        }
        const uint64_t sm = ballot(spill);
        if (sm != 0) {  // rare: a full heavy list
            const uint32_t leader = (uint32_t)__builtin_ctzll(sm);
            uint32_t b2 = 0;
            if (lane == leader) b2 = atomicAdd(&P.live_count[(CUT_SLOT0 + q) * COUNTER_STRIDE], (uint32_t)__popcll(sm));
            if (spill) P.cut_tiles[(size_t)q * P.queue_cap + rdlane(b2, leader) + (uint32_t)__popcll(sm & below)] = my_tile;
        }
    }
    return true;
}

__global__ __launch_bounds__(BLOCK) void tile_cut_kernel(RenderParams P) {
    __builtin_amdgcn_s_setprio(3);
    const uint32_t lane = lane_id();
    const int waves = (int)(gridDim.x * (BLOCK / 64));
    float box[6] = {0.f, 0.f, 0.f, -1.f, -1.f, -1.f};
    int max_len;
    const bool test = cut_setup(P, lane, box, max_len);
    // (list q, group g) pairs, lists interleaved, each wave from its own index on
    for (int p = (int)(blockIdx.x * (BLOCK / 64) + threadIdx.x / 64);; p += waves) {
        const int q = p % P.nqueues, g = p / P.nqueues;
        if (CUT_GROUP * g >= max_len) break;
        (void)cut_unit(P, lane, q, g, test, box);
    }
#ifdef RT_FRAME_SPAN
    if (lane == 0 && g_frame_span) atomicMax(&g_frame_span[4 * (P.drain_tag & 255u) + 3], wall_clock64());
#endif
}

// The render kernel's work: list q's entries, its heavy lists' first (classes in order,
// heaviest first; each capped at heavy_cap), then its survivors (the cut pass's list, or the
// cull pass's live list when there is no cut).  The lists are immutable while the render
// kernel runs, so their lengths and entries are read through the constant address space
// (scalar loads).
__device__ __forceinline__ int work_length(const RenderParams& P, int q, int& heavy) {
    heavy = 0;
    if (P.heavy_cap > 0)
        for (int k = 0; k < NCLASS; ++k) heavy += min((int)ldc_u32(P.live_count + heavy_counter(k, q)), P.heavy_cap);
    const int slot = P.sc.ncut > 0 ? CUT_SLOT0 + q : q;
    return heavy + (int)ldc_u32(&P.live_count[slot * COUNTER_STRIDE]);
}

// cls: the entry's heavy class (0 heaviest), NCLASS for a survivor.
__device__ __forceinline__ int work_tile(const RenderParams& P, int q, int e, int heavy, int& cls) {
    const uint32_t* list;
    cls = NCLASS;
    if (e < heavy) {
        int k = 0;
        for (; k < NCLASS - 1; ++k) {
            const int n = min((int)ldc_u32(P.live_count + heavy_counter(k, q)), P.heavy_cap);
            if (e < n) break;
            e -= n;
        }
        list = reinterpret_cast<const uint32_t*>(P.heavy_tiles) + ((size_t)k * 8 + q) * P.heavy_cap;
        cls = k;
    } else {
        e -= heavy;
        list = reinterpret_cast<const uint32_t*>(P.sc.ncut > 0 ? P.cut_tiles : P.live_tiles) + (size_t)q * P.queue_cap;
    }
    return (int)ldc_u32(list + e);
}

// The next work item of a queue: one returning device-scope atomic from lane 0 (a vector
// atomic), the value made wave-uniform.
__device__ __forceinline__ uint32_t dequeue(uint32_t* head, uint32_t lane) {
    uint32_t v = 0;
    if (lane == 0) v = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return uni(v);
}

// One sample per lane: a block covers a tile_w x tile_h pixel tile x spp samples (spp a power
// of two <= 256, tile_w*tile_h*spp == BLOCK); per-pixel sums run in sample order from LDS.
template <int MODE, bool D1, int LS = 0>
// qw: the wave's quarter of the tile (its work item); LDS is indexed by the thread's own slot,
// t (the thread index, made afresh for each item).
__device__ __forceinline__ void samples_tile(const RenderParams& P, int tile, uint32_t qw, int t, float* col,
                                             int* kpix, float* park, const int* lds_zero) {
    const uint32_t wv = uni((uint32_t)t) >> 6;  // the wave's index in the block (an SGPR)
    // LS = 1, half waves (band shards of a multi-GPU frame, spp <= 32; the bounce kernels'
    // unpaired loop): each wave traces 32
    // samples in its low lanes, so a tile's longest wave, which bounds a short kernel, has half
    // the rays' path union; lt is the sample's index in the (half-size) tile.  A template
    // parameter: a run-time flag here cost the full-wave c3 kernel 0.8 % (register allocation).
    constexpr int wl = LS != 0 ? 32 : 64;  // lanes that trace
    const bool on = (t & 63) < wl;
    const int lt = ((int)qw * wl) | (t & (wl - 1));
    {
        const int s = lt & (P.spp - 1);  // spp and tile_w are powers of two here
        const int pit = lt >> P.spp_log2;
        const int tx = tile % P.tiles_x, ty = tile / P.tiles_x;
#ifndef RT_ROW_PIXELS
        // Pixels in Z order inside a square tile (a wave's pixels form a square: 2x2 at 16 spp,
        // more coherent rays than a row of 4); row-major otherwise.  Any order gives the same
        // image: each sample is independent and each pixel's samples stay consecutive lanes.
        int px, py;
        if (P.tile_w == P.tile_h) {
            px = (pit & 1) | ((pit >> 1) & 2) | ((pit >> 2) & 4) | ((pit >> 3) & 8);
            py = ((pit >> 1) & 1) | ((pit >> 2) & 2) | ((pit >> 3) & 4) | ((pit >> 4) & 8);
        } else {
            px = pit & (P.tile_w - 1);
            py = pit >> P.tile_w_log2;
        }
#else
        const int px = pit & (P.tile_w - 1), py = pit >> P.tile_w_log2;
#endif
        const int x = tx * P.tile_w + px;
        const int r = ty * P.tile_h + py;
        const bool valid = on && x < P.W && r < P.rows;
        const int y = valid ? global_row(P, r) : 0;
        const int pix = valid ? r * P.W + x : -1;
        // The pixel's index goes through LDS (read back below), so the compiler does not keep
        // it, or addresses made from it, live (and spilled) across the shading.
        if (s == 0) kpix[t >> P.spp_log2] = pix;
        const int64_t aov = valid && P.hit_idx ? (int64_t)pix * P.spp + s : -1;
        const f3 c = trace_sample<MODE, D1, LS == 3 ? 2 : 0>(P, valid, x, y, s, aov, park + t,
                                                                             park + (wv << 6));
        RT_PHASE(P, x, r, 1);
        // The thread index again, from the wave's index and a lane id the compiler cannot
        // merge with the first one (mbcnt of a zero read back from LDS): keeping t itself live
        // across the traversals cost a 4-byte scratch spill per lane (c3: ~8 MB of writes per
        // launch).
        const int te = (int)((wv << 6) | __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(
                                                  ~0u, (uint32_t)*(const volatile int*)lds_zero)));
        col[3 * te] = c.x;
        col[3 * te + 1] = c.y;
        col[3 * te + 2] = c.z;
    }
    const int t2 = (int)((wv << 6) | __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(
                                             ~0u, (uint32_t)*(const volatile int*)lds_zero)));
    if (P.spp <= 64) {
        // A pixel's samples are consecutive lanes of one wave: only this wave's LDS writes are
        // read below, so the wave synchronises alone (its siblings in the block may still be
        // tracing; a block barrier here cost 13 % of the waves' time on c3).
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        __syncthreads();
    }
    if ((t2 & (P.spp - 1)) == 0) {
        const int pix = kpix[t2 >> P.spp_log2];
        if (pix >= 0) {
            // col = col + TraceRayIterative(...) in sample order, then col / float(spp)
            f3 acc = mk(0.f, 0.f, 0.f);
            for (int k = 0; k < P.spp; ++k)
                acc = add(acc, mk(col[3 * (t2 + k)], col[3 * (t2 + k) + 1], col[3 * (t2 + k) + 2]));
            // x / 2^k and x * 2^-k are the same correctly rounded value (the exact quotients
            // are equal), so the power-of-two divide is a multiply here.
            const float rs = 1.0f / (float)P.spp;
            const size_t k = (size_t)pix * 3;
            const f3 px = mk(acc.x * rs, acc.y * rs, acc.z * rs);
            if (P.rgb) {
                P.rgb[k] = px.x;
                P.rgb[k + 1] = px.y;
                P.rgb[k + 2] = px.z;
            }
            if (P.p6) {  // the frame epilogue fused in (write_p6 defaults)
                P.p6[k] = rtp::p6_default_sample(px.x);
                P.p6[k + 1] = rtp::p6_default_sample(px.y);
                P.p6[k + 2] = rtp::p6_default_sample(px.z);
            }
        }
    }
}

// General spp: one pixel per lane looping over its samples in order (query.cu:146-163).
template <int MODE, bool D1>
__device__ __forceinline__ void pixels_tile(const RenderParams& P, int tile, uint32_t qw, int tid, float* park) {
    const int t = (int)((qw << 6) | (tid & 63));
    const int tx = tile % P.tiles_x, ty = tile / P.tiles_x;
    const int x = tx * P.tile_w + t % P.tile_w;
    const int r = ty * P.tile_h + t / P.tile_w;
    const bool valid = x < P.W && r < P.rows;
    const int y = valid ? global_row(P, r) : 0;
    f3 acc = mk(0.f, 0.f, 0.f);
    for (int s = 0; s < P.spp; ++s) {
        const int64_t aov = valid && P.hit_idx ? ((int64_t)r * P.W + x) * P.spp + s : -1;
        acc = add(acc, trace_sample<MODE, D1>(P, valid, x, y, s, aov, park + tid, park + (uni((uint32_t)tid) & ~63u)));
    }
    if (valid) {
        const float fs = (float)P.spp;
        const size_t k = ((size_t)r * P.W + x) * 3;
        const f3 px = mk(acc.x / fs, acc.y / fs, acc.z / fs);
        if (P.rgb) {
            P.rgb[k] = px.x;
            P.rgb[k + 1] = px.y;
            P.rgb[k + 2] = px.z;
        }
        if (P.p6) {
            P.p6[k] = rtp::p6_default_sample(px.x);
            P.p6[k + 1] = rtp::p6_default_sample(px.y);
            P.p6[k + 2] = rtp::p6_default_sample(px.z);
        }
    }
}

// A persistent grid (the blocks one dispatch keeps resident) over per-XCD work queues: block b
// serves queue g = b % 8 (dispatch deals blocks round-robin over the XCDs, so queue g is served
// on XCD g and list g's tiles share an L2).  With 8 lists queue g is list g; with one list
// (RT_TILES_LINEAR) queue g takes the list's entries g, g+8, ....  Each wave dequeues its own
// item, a quarter of a tile (BLOCK / 64 waves per tile), so a wave that finishes early takes
// the next quarter at once; with spp > 64 a pixel's samples span the block's waves and the
// block takes whole tiles.  (One block per live-list slot of a frame-sized virtual grid, empty
// blocks leaving at once, cost c3 0.207 ms vs 0.183 for a grid sized exactly to the lists read
// back on the host: the ~10^5 empty blocks' dispatch is not free; the queues need neither.)
#ifndef RT_RENDER_WAVES
#define RT_RENDER_WAVES 7
#endif
// The multi-bounce kernels (D1 false): the bounce loop keeps more state live than the depth-1
// shading (RNG, throughput, the ray, two rays' RayPre, the 4-ary record in the lane traversal).
// c3b with the lane traversal over 4-ary records: 2.26 ms at 3 waves (167 VGPRs, no scratch)
// vs 2.81 at 4 (164 B scratch); binary records at 4 waves 3.20 (profiles/r03/exp/).
#ifndef RT_BOUNCE_WAVES
#define RT_BOUNCE_WAVES 3
#endif
// Scenes whose data (records, leaves, normals) exceed kBigSceneBytes do not stay in the L2s and
// MALL: their depth-1 wave kernels run 8 waves per SIMD (64 VGPRs, a few spills outside the
// traversal loops), more waves to hide the record loads' latency (c5, 345 MB: DESIGN.md §4.2).
// RT_TUNE_BIG_SCENE_BYTES (rt_tuning_set) overrides the threshold (A/B).
// The paired-only bounce kernels (one light, half waves: paired_bounces and nothing else).
#ifndef RT_PAIRED_WAVES
#define RT_PAIRED_WAVES 4
#endif
#ifndef RT_RENDER_WAVES_BIG
#define RT_RENDER_WAVES_BIG 8
#endif
constexpr size_t kBigSceneBytes = size_t(64) << 20;
// Two frames in one launch (RT_TUNE_PAIR_FRAMES, rt_renderer_submit_pair): frame A's parameters,
// then frame B's, one kernel argument.
struct PairParams {
    RenderParams f[2];
};

// Two frames in one render launch (render_pair_kernel) take their pre-passes in one launch
// each too: four dependent launches in the previous pair kernel's tail measured 51 us between
// pair kernels (profiles/r05/exp/pair_timeline_c3.log).  The frames' counter sets and lists are
// disjoint (a cull pass zeroes the set two frames ahead, rt_scene::kSets).
// tile_cull_kernel over both frames: frame A's blocks, then frame B's.
__global__ __launch_bounds__(BLOCK) void tile_cull_pair_kernel(PairParams PP) {
    __builtin_amdgcn_s_setprio(3);
    const int nba = (PP.f[0].tiles_total + BLOCK - 1) / BLOCK;
    const bool b = (int)blockIdx.x >= nba;
    const RenderParams& P = b ? PP.f[1] : PP.f[0];
    const int bx = b ? (int)blockIdx.x - nba : (int)blockIdx.x;
    if (bx == 0 && threadIdx.x < COUNTER_SLOTS) P.next_count[threadIdx.x * COUNTER_STRIDE] = 0u;
    cull_tiles(P, bx * BLOCK + (int)threadIdx.x);
}

// tile_cut_kernel over both frames: every wave takes its (list, group) units of frame A, then
// of frame B.
__global__ __launch_bounds__(BLOCK) void tile_cut_pair_kernel(PairParams PP) {
    __builtin_amdgcn_s_setprio(3);
    const uint32_t lane = lane_id();
    const int waves = (int)(gridDim.x * (BLOCK / 64));
    for (int f = 0; f < 2; ++f) {
        const RenderParams& P = f ? PP.f[1] : PP.f[0];
        float box[6] = {0.f, 0.f, 0.f, -1.f, -1.f, -1.f};
        int max_len;
        const bool test = cut_setup(P, lane, box, max_len);
        for (int p = (int)(blockIdx.x * (BLOCK / 64) + threadIdx.x / 64);; p += waves) {
            const int q = p % P.nqueues, g = p / P.nqueues;
            if (CUT_GROUP * g >= max_len) break;
            (void)cut_unit(P, lane, q, g, test, box);
        }
    }
}

// The pair kernel's item e of queue q: the two frames' heavy lists class by class (A's class k,
// then B's, so the heaviest items of both start first), then A's survivors, then B's.  which:
// the frame; returns the tile, cls its class as work_tile's.
__device__ __forceinline__ int pair_tile(const RenderParams& A, const RenderParams& B, int q, int e, int& which,
                                         int& cls) {
    for (int k = 0; k < NCLASS; ++k) {
        const int na = A.heavy_cap > 0 ? min((int)ldc_u32(A.live_count + heavy_counter(k, q)), A.heavy_cap) : 0;
        if (e < na) {
            which = 0;
            cls = k;
            return (int)ldc_u32(reinterpret_cast<const uint32_t*>(A.heavy_tiles) + ((size_t)k * 8 + q) * A.heavy_cap + e);
        }
        e -= na;
        const int nb = B.heavy_cap > 0 ? min((int)ldc_u32(B.live_count + heavy_counter(k, q)), B.heavy_cap) : 0;
        if (e < nb) {
            which = 1;
            cls = k;
            return (int)ldc_u32(reinterpret_cast<const uint32_t*>(B.heavy_tiles) + ((size_t)k * 8 + q) * B.heavy_cap + e);
        }
        e -= nb;
    }
    cls = NCLASS;
    const int ra = (int)ldc_u32(&A.live_count[(A.sc.ncut > 0 ? CUT_SLOT0 + q : q) * COUNTER_STRIDE]);
    which = e < ra ? 0 : 1;
    const RenderParams& X = e < ra ? A : B;
    if (e >= ra) e -= ra;
    return (int)ldc_u32(reinterpret_cast<const uint32_t*>(X.sc.ncut > 0 ? X.cut_tiles : X.live_tiles) +
                        (size_t)q * X.queue_cap + e);
}

// Heavy-first dispatch: the queues hand out the heavy lists first; the waves record their
// items' costs.  PAIR: the kernel argument is a PairParams; the items of both frames come from
// frame A's queue heads (pair_tile), and frame B's parameters carry the pre-pass gate.
template <int MODE, bool SAMPLES, bool D1, int WAVES, int LS, bool PAIR>
__device__ __forceinline__ void render_tiles_body() {
    constexpr int WPT = BLOCK / 64;  // waves per tile
    __shared__ float col[SAMPLES ? BLOCK * 3 : 1];
    __shared__ int kpix[SAMPLES ? BLOCK : 1];
    // D1: shade_d1's state across shadow rays; else (WAVE kernels) traverse_lane_lds's stacks
    __shared__ float park[D1 ? PARK_SLOTS * BLOCK
                             : (MODE == RT_KERNEL_LANE || (MODE & MODE_DEEP) != 0 ? 1 : LANE_LDS_CAP * BLOCK)];
    // the wave's item start time goes through LDS (an SGPR pair live across the whole tile spilled)
    __shared__ uint32_t t_start[WPT], t_item[WPT];
    __shared__ int lds_zero;  // 0, written by every lane (samples_tile's fresh lane id)
    __shared__ uint32_t block_item;  // spp > 64: the block's item
    if constexpr (SAMPLES) lds_zero = 0;
    // the wave's index in the block as a uniform value (threadIdx.x itself, kept live to the
    // tile-cost write at the end, was spilled to scratch)
    const uint32_t wv = uni((uint32_t)threadIdx.x) >> 6;
    // The first item of each wave (block) is its place in the grid, the rest come from the
    // queue after those: 900 dequeues per head at once when the grid starts took ~10 us to serve.
    for (bool first = true;; first = false) {
        // Everything the item needs is derived inside the loop from a laundered block index and
        // parameter pointer (the kernel's argument segment): hoisted out of the loop, the
        // parameters' loads and the values made from them stay live across every item and spill.
        typedef const __attribute__((address_space(4))) RenderParams* KernargP;
        KernargP pp = (KernargP)__builtin_amdgcn_kernarg_segment_ptr();
        uint32_t bx = blockIdx.x;
        asm volatile("" : "+s"(pp), "+s"(bx));
        const RenderParams& R0 = *(const RenderParams*)pp;
        const RenderParams& RG = PAIR ? *(const RenderParams*)(pp + 1) : R0;  // the gate's frame
        const int g = (int)(bx & 7);
        const int q = R0.nqueues == 1 ? 0 : g;
        uint32_t* head = R0.live_count + (HEAD_SLOT0 + g) * COUNTER_STRIDE;
        const bool blockwise = SAMPLES && R0.spp > 64;
        const uint32_t lane = fresh_lane_id();
#ifdef RT_FRAME_SPAN
        if (first && lane == 0 && g_frame_span) atomicMin(&g_frame_span[4 * (RG.drain_tag & 255u)], wall_clock64());
#endif
        const int tid = (int)((wv << 6) | lane);
        const uint32_t per_queue = (gridDim.x >> 3) * (blockwise ? 1u : (uint32_t)WPT);  // first items
        uint32_t j;
        if (first) {
            j = (bx >> 3) * (blockwise ? 1u : (uint32_t)WPT) + (blockwise ? 0u : wv);
        } else if (blockwise) {
            // one barrier per item: the previous item's LDS reads finished at samples_tile's
            // own barrier, before thread 0 overwrites block_item
            if (tid == 0) block_item = dequeue(head, lane);
            __syncthreads();
            j = per_queue + uni(block_item);
        } else {
            j = per_queue + dequeue(head, lane);
        }
        int heavy;
        int n = work_length(R0, q, heavy);
        if constexpr (PAIR) {
            int hb;
            n += work_length(RG, q, hb);
        }
        const int e = (R0.nqueues == 1 ? g : 0) + (R0.nqueues == 1 ? 8 : 1) * (int)(blockwise ? j : j / WPT);
        // the waves at the queue's gate item (its items are handed out in order, so every queue
        // has them; gate_q8 = 256: the first waves past its end) open the next frame's
        // pre-passes (a vector store to host memory)
        if (RG.drained && lane == 0) {
            const int ge = (int)(((int64_t)n * RG.gate_q8) >> 8);
            if (e >= ge && e < ge + (R0.nqueues == 1 ? 8 : 1))
                __hip_atomic_store(RG.drained, RG.drain_tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (e >= n) {
#ifdef RT_FRAME_SPAN
            if (lane == 0 && g_frame_span) atomicMax(&g_frame_span[4 * (RG.drain_tag & 255u) + 1], wall_clock64());
#endif
            break;
        }
        const uint32_t qw = blockwise ? wv : j % WPT;
        int cls;
        KernargP pr = pp;  // the item's frame
        int tile;
        if constexpr (PAIR) {
            int which;
            tile = pair_tile(R0, RG, q, e, which, cls);
            pr = pp + which;
        } else {
            tile = work_tile(R0, q, e, heavy, cls);
        }
        const RenderParams& R = *(const RenderParams*)pr;
        // Issue priority by cost class: every SIMD keeps all its wave slots busy until the queues
        // drain, so the heaviest items (the kernel's critical path, started first) would share
        // their SIMD with six other waves throughout; ahead of the rest they finish sooner
        // (c3 0.182 vs 0.210 ms without priorities, 0.199 with class 0 alone raised).
        if (cls == 0) __builtin_amdgcn_s_setprio(3);
        else if (cls == 1) __builtin_amdgcn_s_setprio(2);
        else if (cls == 2) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
#ifdef RT_WAVE_TIMES
        const unsigned long long wt0 = wall_clock64();
#endif
#ifdef RT_LANE_ITERS
        if (g_lane_acc) {
            uint32_t* a = g_lane_acc + 4 * ((size_t)blockIdx.x * 256 + threadIdx.x);
            a[0] = a[1] = a[2] = a[3] = 0;
        }
#endif
        if (R.tile_cost && lane == 0) {
            t_start[wv] = (uint32_t)wall_clock64();
            t_item[wv] = (uint32_t)tile * WPT + qw;
        }
        if constexpr (SAMPLES) samples_tile<MODE, D1, LS>(R, tile, qw, tid, col, kpix, park, &lds_zero);
        else pixels_tile<MODE, D1>(R, tile, qw, tid, park);
        if (R.tile_cost && fresh_lane_id() == 0) {  // this wave's duration, for the next frame's heavy lists
            asm volatile("" ::: "memory");
            const uint32_t d = (uint32_t)wall_clock64() - t_start[wv];
            R.tile_cost[t_item[wv]] = (uint16_t)(d < 0xffffu ? d : 0xffffu);
        }
#if defined(RT_WAVE_TIMES) && defined(RT_LANE_ITERS)
        if (g_lane_iters) {
            const uint32_t* a = g_lane_acc + 4 * ((size_t)blockIdx.x * 256 + threadIdx.x);
            const uint32_t mx = wave_max_u32(a[1]), sm = wave_sum_u32(a[1]);
            if ((threadIdx.x & 63) == 0) {
                g_lane_iters[((size_t)tile * WPT + qw) * 4 + 1] = mx;
                g_lane_iters[((size_t)tile * WPT + qw) * 4 + 2] = sm;
            }
        }
#endif
#ifdef RT_WAVE_TIMES
        if (g_wave_times && fresh_lane_id() == 0) {
            const size_t k = ((size_t)tile * WPT + qw) * 2;
            g_wave_times[k] = wt0;
            g_wave_times[k + 1] = wall_clock64();
#ifdef RT_LANE_ITERS
            if (g_lane_iters) {
                const uint32_t* a = g_lane_acc + 4 * ((size_t)blockIdx.x * 256 + threadIdx.x);
                g_lane_iters[((size_t)tile * WPT + qw) * 4 + 0] = a[0];
                g_lane_iters[((size_t)tile * WPT + qw) * 4 + 3] = a[3];
            }
#endif
            if (g_wave_meta) {
                const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u;  // HW_REG_XCC_ID
                g_wave_meta[(size_t)tile * WPT + qw] = bx << 8 | xcc << 4 | (first ? 4u : 0u) | wv;
            }
        }
#endif
    }
}

template <int MODE, bool SAMPLES, bool D1, int WAVES = RT_RENDER_WAVES, int LS = 0>
__global__ __launch_bounds__(BLOCK, WAVES) void render_tiles_kernel(RenderParams P) {
    render_tiles_body<MODE, SAMPLES, D1, WAVES, LS, false>();
}

template <int MODE, bool SAMPLES, bool D1, int WAVES = RT_RENDER_WAVES, int LS = 0>
__global__ __launch_bounds__(BLOCK, WAVES) void render_pair_kernel(PairParams P) {
    render_tiles_body<MODE, SAMPLES, D1, WAVES, LS, true>();
}

// ---- HW1 brute force (HW1/src/render.cpp:72-116) ----------------------------------------
struct Hw1Params {
    const float4* __restrict__ tri;   // 3 float4 per triangle: v0, e1, e2
    const float4* __restrict__ nrm;   // 3 float4 per triangle: n0, n1, n2
    const int4* __restrict__ rects;   // binned path: per triangle (ix_lo, iy_lo, ix_hi, iy_hi)
    const uint32_t* __restrict__ bin_count;   // binned path: per wave tile, triangles listed
    const uint32_t* __restrict__ bin_offset;  // exclusive prefix sum of bin_count
    const uint32_t* __restrict__ bin_list;    // triangle indices, per tile (any order)
    int32_t num_tris;
    f3 center, p00, du, dv;
    int32_t W, H, spp;
    f3 lpos, lcol;
    const float* __restrict__ jitter;
    float* __restrict__ rgb;          // optional (W*H*3 floats)
    int32_t* __restrict__ hit_idx;
    float* __restrict__ hit_t;
    uint8_t* __restrict__ p6;         // optional: write_p6-default samples (W*H*3 bytes)
    uint32_t list_cap;                // binned path: entries bin_list holds; a tile whose list would
                                      // reach past it takes the brute-force loop (exact, slower)
    // chunked path (rt_render_hw1_device): work items of at most HW1_CHUNK list entries
    const uint32_t* __restrict__ chunk_tile;   // per chunk: its tile
    const uint32_t* __restrict__ chunk_first;  // per tile: its first chunk (exclusive prefix; [ntiles] = total)
    uint32_t chunk_cap;                         // chunk_tile's entries
    unsigned long long* __restrict__ keys;      // per (pixel, sample): min over chunks of (t bits << 32 | index)
    uint32_t* __restrict__ zero_counts;         // resolve: counts + cursor (2 * ntiles) zeroed for the next frame
    int32_t ntiles;
};

// HW1 shade (HW1/include/raytracer.h:21-48), material hard-coded at ray.h:111-114.
__device__ __forceinline__ f3 shade_hw1(f3 o, f3 d, bool hit, f3 p, f3 n, f3 lpos, f3 lcol) {
    if (!hit) {
        const f3 ud = unit(d);
        const float t = 0.5f * (ud.z + 1.0f);
        return add(scale(mk(1.f, 1.f, 1.f), 1.0f - t), scale(mk(0.5f, 0.7f, 1.0f), t));
    }
    const f3 albedo = mk(0.8f, 0.2f, 0.2f);
    const f3 ambient = scale(albedo, 0.1f);
    const f3 lightDir = unit(sub(lpos, p));
    const float diff = fmaxf(dot(n, lightDir), 0.0f);
    const f3 diffuse = scale(mul(albedo, lcol), diff);
    const f3 viewDir = unit(sub(o, p));
    const f3 halfDir = unit(add(lightDir, viewDir));
    const float spec = ref_powf(fmaxf(dot(n, halfDir), 0.0f), 64.0f);
    f3 c = add(add(ambient, diffuse), scale(lcol, spec));
    if (c.x > 1.0f) c.x = 1.0f;
    if (c.y > 1.0f) c.y = 1.0f;
    if (c.z > 1.0f) c.z = 1.0f;
    return c;
}

// The pixel: the sample sum / float(spp) (HW1/src/render.cpp:113-115), as floats and/or as
// write_p6-default samples (the frame epilogue fused in).
__device__ __forceinline__ void hw1_write_pixel(const Hw1Params& P, int x, int y, f3 acc) {
    const float fs = (float)P.spp;
    const f3 px = mk(acc.x / fs, acc.y / fs, acc.z / fs);
    const size_t k = ((size_t)y * P.W + x) * 3;
    if (P.rgb) {
        P.rgb[k] = px.x;
        P.rgb[k + 1] = px.y;
        P.rgb[k + 2] = px.z;
    }
    if (P.p6) {
        P.p6[k] = rtp::p6_default_sample(px.x);
        P.p6[k + 1] = rtp::p6_default_sample(px.y);
        P.p6[k + 2] = rtp::p6_default_sample(px.z);
    }
}

__global__ __launch_bounds__(BLOCK) void render_hw1_kernel(Hw1Params P) {
    const int tiles_x = (P.W + 15) / 16;
    const int tile = (int)blockIdx.x;
    const int x = (tile % tiles_x) * 16 + (int)threadIdx.x % 16;
    const int y = (tile / tiles_x) * 16 + (int)threadIdx.x / 16;
    const bool valid = x < P.W && y < P.H;
    f3 acc = mk(0.f, 0.f, 0.f);
    for (int s = 0; s < P.spp; ++s) {
        const float px = (float)x + P.jitter[2 * s];
        const float py = (float)y + P.jitter[2 * s + 1];
        const int ix = (int)px, iy = (int)py;  // get_pixel_position(int, int) truncates
        const f3 pix = add(add(P.p00, scale(P.du, (float)ix)), scale(P.dv, (float)iy));
        const f3 d = unit(sub(pix, P.center));  // HW1 Ray normalises (ray.h:25)
        const f3 o = P.center;
        float best = FLT_MAX;
        int32_t besti = -1;
        for (int k = 0; k < P.num_tris; ++k) {  // wave-uniform: triangle data via the scalar cache
            const float4* T = P.tri + 3 * (size_t)k;
            const float4 a = T[0], b = T[1], c = T[2];
            float t, u, v;
            if (valid && mt_hw1(o, d, mk(a.x, a.y, a.z), mk(b.x, b.y, b.z), mk(c.x, c.y, c.z), t, u, v)) {
                if (t < best) {  // rec.t < prev.t: the first index wins ties
                    best = t;
                    besti = k;
                }
            }
        }
        f3 p = mk(0.f, 0.f, 0.f), n = p;
        const bool hit = besti >= 0;
        if (hit) {
            const float4* T = P.tri + 3 * (size_t)besti;
            const float4 a = T[0], b = T[1], c = T[2];
            float t, u, v;
            mt_hw1(o, d, mk(a.x, a.y, a.z), mk(b.x, b.y, b.z), mk(c.x, c.y, c.z), t, u, v);
            p = add(o, scale(d, t));
            const float4* N = P.nrm + 3 * (size_t)besti;
            const float w = 1.0f - u - v;
            n = add(add(scale(mk(N[0].x, N[0].y, N[0].z), w), scale(mk(N[1].x, N[1].y, N[1].z), u)),
                    scale(mk(N[2].x, N[2].y, N[2].z), v));
        }
        acc = add(acc, shade_hw1(o, d, hit, p, n, P.lpos, P.lcol));
        if (valid && P.hit_idx) {
            const size_t kk = ((size_t)y * P.W + x) * (size_t)P.spp + (size_t)s;
            P.hit_idx[kk] = besti;
            P.hit_t[kk] = hit ? best : -1.0f;
        }
    }
    if (valid) hw1_write_pixel(P, x, y, acc);
}

// ---- HW1 binned (rt_render_hw1 default; same output as render_hw1_kernel) ---------------
// The brute-force loop's answer is the first index among the triangles ray_intersection
// (mt_hw1) accepts with the smallest t.  Skipping triangles that provably cannot be accepted
// for a ray, and visiting the rest in index order with the same strict `<`, gives that answer
// bit for bit.  hw1_rect (hw1_rect_count_kernel) bounds, per triangle, the integer pixel positions (ix, iy)
// whose camera ray mt_hw1 may accept; the render kernel gives each 16x16-pixel block the
// triangles whose rectangle meets it, in index order.
//
// Why the rectangle is conservative.  With tvec = o - v0 and qvec = tvec x e1 (float, exactly
// as mt_hw1 computes them, both ray-independent), mt_hw1's float quantities are
//   det = d.(e2 x e1) + Ed,   U = d.(e2 x tvec) + Eu,   V = d.qvec + Ev,   tnum = e2.qvec,
// u = U * (1/det), v = V * (1/det), t = tnum * (1/det), with |Ed|, |Eu|, |Ev| bounded by the
// standard dot/cross rounding bounds (|d_j| <= 1).  When |tnum| is not tiny its sign s must
// be det's (else t < 0), so acceptance needs four linear inequalities in d:
//   s U >= 0,  s V >= 0,  s (det - U - V) >= -(4u|det| rounding of u + v and the divisions),
//   s det >= FLT_EPSILON,
// each relaxed by its error bound and by the rounding of unit() (d = D/|D| (1 + 3u)).  With
// D = pixel00 + ix du + iy dv - center (exact, widened per axis by the tile-cull padding
// for its float evaluation) and |D| in [Nmin, Nmax] over the image, every inequality becomes
// a half-plane in (ix, iy); the rectangle is the bounding box (+1 pixel) of the padded image
// rectangle clipped by the four half-planes.  Degenerate cases (tiny tnum, huge magnitudes,
// an image whose directions reach 0) get the whole image.
__device__ __forceinline__ void hw1_cross_d(const double a[3], const double b[3], double r[3]) {
    r[0] = a[1] * b[2] - a[2] * b[1];
    r[1] = a[2] * b[0] - a[0] * b[2];
    r[2] = a[0] * b[1] - a[1] * b[0];
}

__device__ int4 hw1_rect(const Hw1Params& P, int k) {
    const int X0 = -2, X1 = P.W + 1, Y0 = -2, Y1 = P.H + 1;  // ix in [x, x+1] (truncation)
    const int4 all = make_int4(X0, Y0, X1, Y1), none = make_int4(1, 1, 0, 0);
    const float4 A = P.tri[3 * (size_t)k], B = P.tri[3 * (size_t)k + 1], Cq = P.tri[3 * (size_t)k + 2];
    const f3 v0 = mk(A.x, A.y, A.z), e1 = mk(B.x, B.y, B.z), e2 = mk(Cq.x, Cq.y, Cq.z);
    const f3 tvec = sub(P.center, v0);  // mt_hw1's own float values
    const f3 qvec = cross(tvec, e1);
    const float tnum = dot(e2, qvec);
    double mag = 0.0;
    const float mv[15] = {v0.x, v0.y, v0.z, e1.x, e1.y, e1.z, e2.x, e2.y, e2.z, tvec.x, tvec.y, tvec.z,
                          qvec.x, qvec.y, qvec.z};
    for (int i = 0; i < 15; ++i) mag = fmax(mag, fabs((double)mv[i]));
    if (!(mag < 1e15) || !(fabsf(tnum) >= 1e-20f)) {
        return all;
    }
    const double sg = tnum > 0.0f ? 1.0 : -1.0;
    const double tv[3] = {tvec.x, tvec.y, tvec.z}, ea[3] = {e1.x, e1.y, e1.z}, eb[3] = {e2.x, e2.y, e2.z},
                 qv[3] = {qvec.x, qvec.y, qvec.z};
    double au[3], ad[3];
    hw1_cross_d(eb, tv, au);  // U = tvec.(d x e2) = d.(e2 x tvec)
    hw1_cross_d(eb, ea, ad);  // det = (d x e2).e1 = d.(e2 x e1)
    const double uu = 0x1p-24, dm = 1.0001;
    const double pb[3] = {fabs(eb[2]) + fabs(eb[1]), fabs(eb[0]) + fabs(eb[2]), fabs(eb[1]) + fabs(eb[0])};
    double Eu = 0, Ed = 0, Ev = 0, dmax = 0;
    for (int i = 0; i < 3; ++i) {
        Eu += fabs(tv[i]) * pb[i];
        Ed += fabs(ea[i]) * pb[i];
        Ev += fabs(qv[i]);
        dmax += fabs(ad[i]);
    }
    Eu *= 8 * uu * dm;
    Ed *= 8 * uu * dm;
    Ev *= 4 * uu * dm;
    dmax = dmax * dm + Ed;
    if (!(dmax < 1e10)) {  // keeps |t| = |tnum / det| >= 1e-30: a wrong-sign t stays negative
        return all;
    }
    const double tiny = 1e-30;
    double c[4][3], w[4];
    for (int i = 0; i < 3; ++i) {
        c[0][i] = sg * au[i];
        c[1][i] = sg * qv[i];
        c[2][i] = sg * (ad[i] - au[i] - qv[i]);
        c[3][i] = sg * ad[i];
    }
    w[0] = -(Eu + tiny);
    w[1] = -(Ev + tiny);
    w[2] = -(4 * uu * dmax + Eu + Ev + Ed + tiny);
    w[3] = (double)FLT_EPSILON - Ed;
    // D over the image, per axis, padded as in tile_dirs
    const double cc[3] = {P.center.x, P.center.y, P.center.z}, p0[3] = {P.p00.x, P.p00.y, P.p00.z},
                 du[3] = {P.du.x, P.du.y, P.du.z}, dv[3] = {P.dv.x, P.dv.y, P.dv.z};
    const double xm = fmax(fabs((double)X0), fabs((double)X1)), ym = fmax(fabs((double)Y0), fabs((double)Y1));
    double D00[3], Dl[3], Dh[3], pad[3], scale = 0.0;
    for (int a = 0; a < 3; ++a) {
        D00[a] = p0[a] - cc[a];
        const double u0 = X0 * du[a], u1 = X1 * du[a], w0 = Y0 * dv[a], w1 = Y1 * dv[a];
        Dl[a] = D00[a] + fmin(u0, u1) + fmin(w0, w1);
        Dh[a] = D00[a] + fmax(u0, u1) + fmax(w0, w1);
        pad[a] = 8.0 * 0x1p-23 * (fabs(cc[a]) + fabs(p0[a]) + xm * fabs(du[a]) + ym * fabs(dv[a]));
        scale = fmax(scale, fmax(fabs(Dl[a]), fabs(Dh[a])));
    }
    double nmin2 = 0.0, nmax2 = 0.0;
    for (int a = 0; a < 3; ++a) {
        pad[a] += 1e-5 * scale;
        Dl[a] -= pad[a];
        Dh[a] += pad[a];
        const double near = Dl[a] > 0 ? Dl[a] : (Dh[a] < 0 ? Dh[a] : 0.0);
        const double far = fmax(fabs(Dl[a]), fabs(Dh[a]));
        nmin2 += near * near;
        nmax2 += far * far;
    }
    const double nmin = sqrt(nmin2) * (1 - 1e-12), nmax = sqrt(nmax2) * (1 + 1e-12);
    if (!(nmin > 0.0) || !(nmax < 1e300)) {
        return all;
    }
    double px[8 + 4], py[8 + 4];
    int n = 4;
    px[0] = X0; py[0] = Y0;
    px[1] = X1; py[1] = Y0;
    px[2] = X1; py[2] = Y1;
    px[3] = X0; py[3] = Y1;
    for (int i = 0; i < 4 && n > 0; ++i) {
        double cs = 0.0, cdm = 0.0, cpad = 0.0, cD00 = 0.0, al = 0.0, be = 0.0;
        for (int a = 0; a < 3; ++a) {
            cs += fabs(c[i][a]);
            cdm += fabs(c[i][a]) * fmax(fabs(Dl[a]), fabs(Dh[a]));
            cpad += fabs(c[i][a]) * pad[a];
            cD00 += c[i][a] * D00[a];
            al += c[i][a] * du[a];
            be += c[i][a] * dv[a];
        }
        const double w1 = w[i] - 4 * uu * dm * cs;              // unit() rounding of d
        const double g = fmin(w1 * nmin, w1 * nmax);            // c.D >= w1 |D|
        const double ga = g - cpad - 1e-9 * cdm - tiny - cD00;  // al ix + be iy >= ga
        if (!(fabs(al) < 1e300 && fabs(be) < 1e300 && fabs(ga) < 1e300)) {
            return all;
        }
        double qx[12], qy[12];
        int m = 0;
        for (int j = 0; j < n; ++j) {
            const int jn = (j + 1) % n;
            const double fc = al * px[j] + be * py[j] - ga, fn = al * px[jn] + be * py[jn] - ga;
            if (fc >= 0) {
                qx[m] = px[j];
                qy[m] = py[j];
                ++m;
            }
            if ((fc >= 0) != (fn >= 0)) {
                const double tt = fc / (fc - fn);
                qx[m] = px[j] + tt * (px[jn] - px[j]);
                qy[m] = py[j] + tt * (py[jn] - py[j]);
                ++m;
            }
        }
        n = m;
        for (int j = 0; j < n; ++j) {
            px[j] = qx[j];
            py[j] = qy[j];
        }
    }
    if (n == 0) {
        return none;
    }
    double lx = px[0], hx = px[0], ly = py[0], hy = py[0];
    for (int j = 1; j < n; ++j) {
        lx = fmin(lx, px[j]);
        hx = fmax(hx, px[j]);
        ly = fmin(ly, py[j]);
        hy = fmax(hy, py[j]);
    }
    return make_int4(max(X0, (int)floor(lx) - 1), max(Y0, (int)floor(ly) - 1), min(X1, (int)ceil(hx) + 1),
                     min(Y1, (int)ceil(hy) + 1));
}

// Binning (a tiled rasterizer's): hw1_rect_count_kernel counts, per 16x4-pixel wave tile, the
// triangles whose rectangle meets the tile's (ix, iy) range (pixel x uses ix in {x, x+1});
// hw1_scan_chunks_kernel turns the counts into offsets; hw1_fill_kernel writes the lists.  A list's
// order is whatever the atomics give, so the render kernel keeps the lexicographic minimum of
// (t, index): the smallest t, the smallest index among equal t — exactly the brute-force
// loop's winner (it keeps the first index whose t is strictly below every earlier one), and
// independent of the visiting order.  (A NaN t is never below or equal to anything, in
// either form.)
constexpr int HW1_TW = 16, HW1_TH = 4;  // wave tile: 16 x 4 pixels
__device__ __forceinline__ bool hw1_tile_range(const Hw1Params& P, int4 r, int& tx0, int& tx1, int& ty0, int& ty1) {
    const int tiles_x = (P.W + HW1_TW - 1) / HW1_TW, tiles_y = (P.H + HW1_TH - 1) / HW1_TH;
    if (r.x > r.z || r.y > r.w) return false;
    tx0 = max(0, r.x - 1) / HW1_TW;
    ty0 = max(0, r.y - 1) / HW1_TH;
    tx1 = min(tiles_x - 1, r.z / HW1_TW);
    ty1 = min(tiles_y - 1, r.w / HW1_TH);
    return r.z >= 0 && r.w >= 0 && tx0 <= tx1 && ty0 <= ty1;
}

// The (triangle, tile) pairs of a wave's 64 triangles, 64 at a time over the wave's lanes: a
// triangle covering many tiles no longer keeps one lane looping while the others wait (c2: 30 and
// 25 us for the two passes with a lane per triangle).  Lane l's triangle covers cnt tiles from
// (tx0, ty0), w per row; fn(tx, ty, triangle) runs once per pair.  Every lane of the wave calls
// this (the shuffles read every lane).
template <typename F>
__device__ __forceinline__ void hw1_wave_pairs(uint32_t lane, int k, uint32_t cnt, int tx0, int ty0, int w, F&& fn) {
    uint32_t incl = cnt;  // inclusive prefix sum over the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t v = (uint32_t)__shfl_up((int)incl, d);
        if ((int)lane >= d) incl += v;
    }
    const uint32_t excl = incl - cnt;
    const uint32_t total = uni((uint32_t)__shfl((int)incl, 63));
    for (uint32_t base = 0; base < total; base += 64) {
        const uint32_t p = base + lane;
        // the pair's lane: the last one whose range starts at or before p (lanes without pairs
        // start where the next lane does, so the last such lane has pairs)
        int o = 0;
#pragma unroll
        for (int step = 32; step > 0; step >>= 1) {
            const uint32_t e = (uint32_t)__shfl((int)excl, o + step);
            if (e <= p) o += step;
        }
        const uint32_t local = p - (uint32_t)__shfl((int)excl, o);
        const int ow = __shfl(w, o);
        const int tx = __shfl(tx0, o) + (int)(local % (uint32_t)max(ow, 1));
        const int ty = __shfl(ty0, o) + (int)(local / (uint32_t)max(ow, 1));
        const int tri = __shfl(k, o);
        if (p < total) fn(tx, ty, tri);
    }
}

// Pass 1: each triangle's rectangle (kept for pass 2) and its count in every tile it meets.
// (Launched with 64-thread blocks: one wave each.)
__global__ __launch_bounds__(64) void hw1_rect_count_kernel(Hw1Params P, int4* __restrict__ rects,
                                                            uint32_t* __restrict__ counts) {
    const uint32_t lane = lane_id();
    const int k = (int)(blockIdx.x * 64 + lane);
    const int tiles_x = (P.W + HW1_TW - 1) / HW1_TW;
    int tx0 = 0, tx1 = -1, ty0 = 0, ty1 = -1;
    if (k < P.num_tris) {
        const int4 r = hw1_rect(P, k);
        rects[k] = r;
        if (!hw1_tile_range(P, r, tx0, tx1, ty0, ty1)) tx1 = tx0 - 1;
    }
    const uint32_t cnt = tx1 >= tx0 && ty1 >= ty0 ? (uint32_t)((tx1 - tx0 + 1) * (ty1 - ty0 + 1)) : 0u;
    hw1_wave_pairs(lane, k, cnt, tx0, ty0, tx1 - tx0 + 1,
                   [&](int tx, int ty, int) { atomicAdd(&counts[ty * tiles_x + tx], 1u); });
}

// Pass 2: the lists.  A tile whose list would reach past list_cap is not written; the render
// kernel gives that tile the brute-force loop instead.
__global__ __launch_bounds__(64) void hw1_fill_kernel(Hw1Params P, uint32_t* __restrict__ cursor,
                                                      uint32_t* __restrict__ list) {
    const uint32_t lane = lane_id();
    const int k = (int)(blockIdx.x * 64 + lane);
    const int tiles_x = (P.W + HW1_TW - 1) / HW1_TW;
    int tx0 = 0, tx1 = -1, ty0 = 0, ty1 = -1;
    if (k < P.num_tris && !hw1_tile_range(P, P.rects[k], tx0, tx1, ty0, ty1)) tx1 = tx0 - 1;
    const uint32_t cnt = tx1 >= tx0 && ty1 >= ty0 ? (uint32_t)((tx1 - tx0 + 1) * (ty1 - ty0 + 1)) : 0u;
    hw1_wave_pairs(lane, k, cnt, tx0, ty0, tx1 - tx0 + 1, [&](int tx, int ty, int tri) {
        const int t = ty * tiles_x + tx;
        if (P.bin_offset[t + 1] <= P.list_cap) list[P.bin_offset[t] + atomicAdd(&cursor[t], 1u)] = (uint32_t)tri;
    });
}

// The chunked pass: a tile's list is cut into work items of at most HW1_CHUNK entries (a tile
// whose list does not fit the capacity is one item over every triangle), so a long list no
// longer makes one wave the kernel's tail.
constexpr uint32_t HW1_CHUNK = 64;

// Exclusive prefix sum of n counts in one workgroup (n is the number of wave tiles, small);
// offsets[n] = total.  With chunk_first: the same over the tiles' chunk counts, and every
// chunk's tile in chunk_tile (at most chunk_cap; chunks past it are not written, the total in
// chunk_first[n] says how many there were).
__global__ __launch_bounds__(1024) void hw1_scan_chunks_kernel(const uint32_t* __restrict__ counts,
                                                               uint32_t* __restrict__ offsets, int n, uint32_t list_cap,
                                                               uint32_t* __restrict__ chunk_first,
                                                               uint32_t* __restrict__ chunk_tile, uint32_t chunk_cap) {
    __shared__ uint32_t part[1024], cpart[1024];
    const int t = (int)threadIdx.x;
    const int per = (n + 1023) / 1024;
    const int lo = min(n, t * per), hi = min(n, lo + per);
    uint32_t sum = 0;
    for (int i = lo; i < hi; ++i) sum += counts[i];
    part[t] = sum;
    __syncthreads();
    for (int st = 1; st < 1024; st <<= 1) {  // Hillis-Steele inclusive scan
        const uint32_t v = t >= st ? part[t - st] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    // the tiles' chunk counts need the tiles' offsets (a list past the capacity: one chunk)
    uint32_t run = part[t] - sum, csum = 0;
    for (int i = lo; i < hi; ++i) {
        offsets[i] = run;
        const uint32_t c = counts[i];
        csum += run + c > list_cap ? 1u : (c + HW1_CHUNK - 1) / HW1_CHUNK;
        run += c;
    }
    if (t == 1023) offsets[n] = part[1023];
    cpart[t] = csum;
    __syncthreads();
    for (int st = 1; st < 1024; st <<= 1) {
        const uint32_t v = t >= st ? cpart[t - st] : 0u;
        __syncthreads();
        cpart[t] += v;
        __syncthreads();
    }
    uint32_t crun = cpart[t] - csum;
    run = part[t] - sum;
    for (int i = lo; i < hi; ++i) {
        chunk_first[i] = crun;
        const uint32_t c = counts[i];
        const uint32_t nc = run + c > list_cap ? 1u : (c + HW1_CHUNK - 1) / HW1_CHUNK;
        for (uint32_t k = 0; k < nc; ++k)
            if (crun + k < chunk_cap) chunk_tile[crun + k] = (uint32_t)i;
        crun += nc;
        run += c;
    }
    if (t == 1023) chunk_first[n] = cpart[1023];
}

// One wave per chunk, grid-stride over the frame's chunks: the tile's 64 pixel lanes run mt_hw1
// over the chunk's entries and fold each sample's winner into keys with a 64-bit atomicMin of
// (t bits << 32 | index).  t >= 0 and never -0 (t + 0.0f), so its bits order like its value; the
// minimum over the chunks is the lexicographic (t, index) minimum of the whole list -- the
// brute-force loop's winner (rec.t < prev.t keeps the first index).
__global__ __launch_bounds__(BLOCK) void render_hw1_chunks_kernel(Hw1Params P) {
    const uint32_t total = uni(P.chunk_first[P.ntiles]);
    const uint32_t nchunks = total < P.chunk_cap ? total : P.chunk_cap;
    const int tiles_x = (P.W + HW1_TW - 1) / HW1_TW;
    const uint32_t lane = lane_id();
    const uint32_t waves = gridDim.x * (BLOCK / 64);
    for (uint32_t j = blockIdx.x * (BLOCK / 64) + threadIdx.x / 64; j < nchunks; j += waves) {
        const uint32_t tidx = uni(P.chunk_tile[uni(j)]);
        const uint32_t c = j - uni(P.chunk_first[tidx]);
        const uint32_t cnt = uni(P.bin_count[tidx]);
        const uint32_t off = uni(P.bin_offset[tidx]);
        const bool all = off + cnt > P.list_cap;  // the list was not written: every triangle, in order
        const uint32_t b = all ? 0u : c * HW1_CHUNK;
        const uint32_t e = all ? (uint32_t)P.num_tris : min(cnt, b + HW1_CHUNK);
        const int x = (int)(tidx % tiles_x) * HW1_TW + (int)(lane % HW1_TW);
        const int y = (int)(tidx / tiles_x) * HW1_TH + (int)(lane / HW1_TW);
        const bool valid = x < P.W && y < P.H;
        for (int s = 0; s < P.spp; ++s) {
            const float pxs = (float)x + P.jitter[2 * s];
            const float pys = (float)y + P.jitter[2 * s + 1];
            const int ix = (int)pxs, iy = (int)pys;  // get_pixel_position(int, int) truncates
            const f3 pix = add(add(P.p00, scale(P.du, (float)ix)), scale(P.dv, (float)iy));
            const f3 d = unit(sub(pix, P.center));  // HW1 Ray normalises (ray.h:25)
            const f3 o = P.center;
            unsigned long long best = ~0ull;
            for (uint32_t i = b; i < e; i += 4) {
                int kk[4];
                float4 tq[12];
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    kk[q] = i + q < e ? (all ? (int)(i + q) : (int)ldc_u32(P.bin_list + off + i + q)) : -1;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4* T = P.tri + 3 * (size_t)(kk[q] < 0 ? kk[0] : kk[q]);
                    tq[3 * q] = ldc(T);
                    tq[3 * q + 1] = ldc(T + 1);
                    tq[3 * q + 2] = ldc(T + 2);
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 a = tq[3 * q], bq = tq[3 * q + 1], cq = tq[3 * q + 2];
                    float t, u, v;
                    // (t < FLT_MAX: the loop's `t < best` from best = FLT_MAX never takes FLT_MAX,
                    // +inf or NaN)
                    if (valid && kk[q] >= 0 &&
                        mt_hw1(o, d, mk(a.x, a.y, a.z), mk(bq.x, bq.y, bq.z), mk(cq.x, cq.y, cq.z), t, u, v) &&
                        t < FLT_MAX) {
                        const unsigned long long key =
                            (unsigned long long)__float_as_uint(t + 0.0f) << 32 | (uint32_t)kk[q];
                        best = key < best ? key : best;
                    }
                }
            }
            if (valid && best != ~0ull) atomicMin(&P.keys[((size_t)y * P.W + x) * (size_t)P.spp + (size_t)s], best);
        }
    }
}

// Per pixel: each sample's winner from keys (then reset for the next frame), HW1 shade, the
// average, AOVs; the first threads also zero the bin counters for the next frame.
__global__ __launch_bounds__(BLOCK) void hw1_resolve_kernel(Hw1Params P) {
    const int gid = (int)(blockIdx.x * BLOCK + threadIdx.x);
    if (gid < 2 * P.ntiles) P.zero_counts[gid] = 0u;
    if (gid >= P.W * P.H) return;
    const int x = gid % P.W, y = gid / P.W;
    f3 acc = mk(0.f, 0.f, 0.f);
    for (int s = 0; s < P.spp; ++s) {
        const float pxs = (float)x + P.jitter[2 * s];
        const float pys = (float)y + P.jitter[2 * s + 1];
        const int ix = (int)pxs, iy = (int)pys;
        const f3 pix = add(add(P.p00, scale(P.du, (float)ix)), scale(P.dv, (float)iy));
        const f3 d = unit(sub(pix, P.center));
        const f3 o = P.center;
        const size_t kk = (size_t)gid * (size_t)P.spp + (size_t)s;
        const unsigned long long key = P.keys[kk];
        P.keys[kk] = ~0ull;
        const bool hit = key != ~0ull;
        const int32_t besti = hit ? (int32_t)(uint32_t)key : -1;
        f3 p = mk(0.f, 0.f, 0.f), n = p;
        float best = FLT_MAX;
        if (hit) {  // the accepting test's own t, u, v
            const float4* T = P.tri + 3 * (size_t)besti;
            const float4 a = T[0], b = T[1], cq = T[2];
            float t, u, v;
            mt_hw1(o, d, mk(a.x, a.y, a.z), mk(b.x, b.y, b.z), mk(cq.x, cq.y, cq.z), t, u, v);
            best = t;
            p = add(o, scale(d, t));
            const float4* N = P.nrm + 3 * (size_t)besti;
            const float wgt = 1.0f - u - v;
            n = add(add(scale(mk(N[0].x, N[0].y, N[0].z), wgt), scale(mk(N[1].x, N[1].y, N[1].z), u)),
                    scale(mk(N[2].x, N[2].y, N[2].z), v));
        }
        acc = add(acc, shade_hw1(o, d, hit, p, n, P.lpos, P.lcol));
        if (P.hit_idx) {
            P.hit_idx[kk] = besti;
            P.hit_t[kk] = hit ? best : -1.0f;
        }
    }
    hw1_write_pixel(P, x, y, acc);
}

__global__ __launch_bounds__(BLOCK) void powf_kernel(const float* __restrict__ x, const float* __restrict__ y, int n,
                                                     float* __restrict__ out) {
    const int i = (int)(blockIdx.x * BLOCK + threadIdx.x);
    if (i < n) out[i] = ref_powf(x[i], y[i]);
}

// Batched ray-triangle queries (KAT path): one lane per ray.
__global__ __launch_bounds__(BLOCK) void intersect_kernel(f3 v0, f3 e1, f3 e2, f3 o, const float* __restrict__ dirs,
                                                          int n, int hw1, float tmin, float tmax,
                                                          int32_t* __restrict__ hit, float* __restrict__ tout) {
    const int i = (int)(blockIdx.x * BLOCK + threadIdx.x);
    if (i >= n) return;
    f3 d = mk(dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2]);
    float t = 0.f, u = 0.f, v = 0.f;
    bool h;
    if (hw1) {
        d = unit(d);
        h = mt_hw1(o, d, v0, e1, e2, t, u, v);
    } else {
        const RayPre r = make_ray_mt(o, d);
        h = mt_g(r, v0, e1, e2, tmin, tmax, t, u, v);
    }
    hit[i] = h ? 1 : 0;
    tout[i] = h ? t : -1.0f;
}

}  // namespace

// =========================================================================================
// Host side
// =========================================================================================
using rt::set_error;
using rt::hip_msg;
using rt::DevBuf;
using rt::check_device;
using rt::DeviceGuard;

struct rt_scene {
    int device = 0;
    const char* last_kernel = nullptr;  // the render kernel instantiation of the latest frame
    size_t P = 0;
    int nmat = 0, nlights = 0;
    uint32_t root_ref = 0;
    float root_box[6] = {0, 0, 0, 0, 0, 0};
    float bmax[3] = {0, 0, 0};
    DevBuf inode, wnode, ibox, leaf, tnorm, objids, mats, lights, jitter;
    DevBuf fnode;    // 2^f_log2-ary records of the frustum traversal (empty: it takes wnode's 4-ary ones)
    int f_log2 = 2;
    int f_bound = 0;  // their DFS stack bound (<= FRUSTUM_STACK unless RT_TUNE_FRUSTUM_STACK_CAP raised it)
    DevBuf qent, qhdr;  // fnode quantised (build_quant_records): the big-scene kernels' records
    DevBuf fault;     // one word: RT_FAULT_* bits the kernels OR in (rt_scene_faults)
    DevBuf cut;  // tile culling: boxes of a cut of the tree (6 floats each)
    int ncut = 0;
    DevBuf cut2;  // 2^cut_sub_log2 boxes below each cut box (tile_cut_sub), 6 floats each
    int cut_sub_log2 = 0;
    bool deep = false;  // the DFS may need more than STACK_CAP entries: MODE_DEEP kernels
    DevBuf tri;         // deep: triangles by index (brute-force completion)
    bool wide = false;
    bool lane_stack = false;  // binary DFS stack <= LANE_LDS_CAP (traverse_lane_lds)
    bool lane_wide = false;   // 4-ary records whose DFS stack <= LANE_LDS_CAP (traverse_lane_lds_wide)
    DevBuf work;  // kSets counter sets, then kSets x (live lists | cut survivor lists | heavy lists)
    int64_t last_tiles_total = 0;
    int cus = 256;
    // heavy-first dispatch: per-tile wave durations of the last frames (4 x u16 per tile) for
    // the tile geometry cost_key, and the latest finished frame's render-kernel time
    DevBuf cost;
    uint64_t cost_key = 0;
    float kernel_ms_est = 0.f;
    int last_heavy_cap = 0;
    int jitter_spp = -1;
    std::vector<float> jitter_host;
    // Ring of HIP events per frame.  A frame's pre-passes (tile_cull_kernel, tile_cut_kernel)
    // run on the scene's own high-priority `prep` stream, its render kernel on the caller's:
    //   prep:   [wait ev1 of frame k-2 (k-1 too if the outputs overlap)] ev0 | cull | cut | pdone
    //   caller: [wait pdone] evm | render kernel | ev1
    // so frame k's pre-passes overlap frame k-1's render kernel (its tail leaves CUs idle).
    static constexpr int kRing = 256;
    hipEvent_t ev0[kRing] = {}, evm[kRing] = {}, ev1[kRing] = {}, pdone[kRing] = {};
    // evm is recorded (the render kernel's start timestamp) only for timed frames: a start event
    // holds the kernel's dispatch until the previous kernel has completed and its timestamp is
    // written, ~5 us between back-to-back kernels (scripts/micro/kernel_gap.hip); the
    // renderer's frames time one in RT_TUNE_KERNEL_TIMING_EVERY
    bool timed[kRing] = {};
    // frames of the slot's render launch: 2 for the frames of a pair (rt::render_pair; frame A's
    // events bracket the pair kernel, frame B's ev1 is recorded after it), else 1
    uint8_t span[kRing] = {};
    // evq: recorded on the caller's stream at the start of a frame; the prep stream waits for it
    // so the pre-passes (which write the culled tiles' pixels into the caller's buffers) come
    // after everything the caller queued on that stream before the call.  A caller that orders
    // its buffer reuse itself on the host (rt_renderer) sets caller_ordered and skips it.
    hipEvent_t evq[kRing] = {};
    bool caller_ordered = false;
    hipStream_t prep = nullptr;
    // RT_TUNE_OVERLAP_FRAMES (caller-ordered frames only): render kernels alternate over these
    // two streams, so frame k+1's kernel takes the wave slots frame k's tail leaves
    hipStream_t rstream[2] = {};
    uint64_t launches = 0;
    // the pre-pass gate's host word (RenderParams::drained) and the frame whose render kernel
    // last stored into it (~0: none)
    uint32_t* drain = nullptr;
    uint64_t drain_frame = ~0ull;
    uint64_t est_next = 0;  // the oldest frame not yet seen finished (heavy-threshold estimate)
    size_t bytes = 0;
    // Work buffers rotate over kSets per frame (frame k: set k % 6; its cull pass zeroes the
    // counters of set k+2, last used by frame k-4, so the two frames of a pair never touch each
    // other's sets and their pre-passes run side by side).  Six sets: the two frames of a
    // running pair kernel, the next pair's two, whose pre-passes run in its tail, and the two
    // sets those zero.  A frame launched on another stream than the previous one first waits for
    // that frame.  A frame whose launches failed part-way leaves the counter sets unknown: the
    // next frame zeroes them all.
    static constexpr int kSets = 6;
    hipStream_t last_stream = nullptr;
    bool counters_dirty = false;
    // the previous frame's output ranges (device byte ranges): overlapping outputs serialise
    struct Range { uintptr_t lo = 0, hi = 0; };
    Range prev_out[4];
    size_t set_bytes = 0;  // bytes of one set of lists for the current geometry
    ~rt_scene() {
        if (prep) (void)hipStreamSynchronize(prep);
        for (int i = 0; i < kRing; ++i) {
            if (ev0[i]) (void)hipEventDestroy(ev0[i]);
            if (evm[i]) (void)hipEventDestroy(evm[i]);
            if (ev1[i]) (void)hipEventDestroy(ev1[i]);
            if (pdone[i]) (void)hipEventDestroy(pdone[i]);
            if (evq[i]) (void)hipEventDestroy(evq[i]);
        }
        for (hipStream_t r : rstream)
            if (r) {
                (void)hipStreamSynchronize(r);
                (void)hipStreamDestroy(r);
            }
        if (prep) (void)hipStreamDestroy(prep);
        if (drain) (void)hipHostFree(drain);
    }
    int create_sync() {  // streams and events (rt_scene_create / rt_scene_clone)
        int lo = 0, hi = 0;
        HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIP_TRY(hipStreamCreateWithPriority(&prep, hipStreamNonBlocking, hi));
        for (hipStream_t& r : rstream) HIP_TRY(hipStreamCreateWithFlags(&r, hipStreamNonBlocking));
        if (int rc = fault.alloc(sizeof(uint32_t)); rc != RT_OK) return rc;
        HIP_TRY(hipMemset(fault.p, 0, sizeof(uint32_t)));
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&drain), sizeof(uint32_t), hipHostMallocCoherent));
        *drain = 0;
        for (int i = 0; i < kRing; ++i) {
            HIP_TRY(hipEventCreate(&ev0[i]));
            HIP_TRY(hipEventCreate(&evm[i]));
            HIP_TRY(hipEventCreate(&ev1[i]));
            HIP_TRY(hipEventCreate(&pdone[i]));
            HIP_TRY(hipEventCreateWithFlags(&evq[i], hipEventDisableTiming));
        }
        return RT_OK;
    }
};

extern "C" int rt_device_count(int* n) {
    if (!n) return set_error(RT_ERR_ARG, "null");
    *n = 0;
    hipError_t e = hipGetDeviceCount(n);
    if (e != hipSuccess) { *n = 0; return set_error(RT_ERR_NODEVICE, hip_msg(e, "hipGetDeviceCount")); }
    return RT_OK;
}

// Wide records for the camera rays' frustum traversal (traverse_frustum): an internal node's
// descendants D levels down in SearchBVH's push order, for the root and, in turn, every internal
// entry of a record; A = 2^D entries.  A leaf stands for itself and a child naming no valid
// triangle is skipped, as in the 4-ary records.  Records by their own index (an internal entry's
// ref is its record's), 8A floats: A x (x pair, y pair, z pair) | A refs (NO_REF pads) | unused.
// Exact for the reason the 4-ary records are (every internal box contains its children's,
// wide_ok).  The largest A in {32, 16, 8} (at most 2^dmax) whose DFS needs at most `cap` stack
// entries (FRUSTUM_STACK = 128: frog 32, bound 91; the c5 heightfield 32, bound 126); log2 = 2
// when none fits (the frustum traversal then takes the 4-ary records, wnode).
// cid: compact ids as rt_scene_create makes them (LEAF_BIT | slot, internal index, or NO_REF).
// (Leaf-pair entries, an internal node with two leaf children tested in one pop, measured no
// faster: c3 0.1517 vs 0.1517 ms, c5 48.2 vs 45.9; profiles/r04/exp/pairs_stack128_ab_*.log.)
// Valid leaves under each node (the greedy record rules' weights): a post-order walk from the
// root over the nodes rt_scene_create gave ids (cid: NO_REF for nodes naming no valid triangle).
static std::vector<uint32_t> subtree_leaves(const rt_bvh_node* nodes, size_t NN, const uint32_t* cid) {
    std::vector<uint32_t> leaves(NN, 0u);
    std::vector<uint8_t> seen(NN, 0);  // each node expanded once (the tree is checked elsewhere)
    auto ref_of0 = [&](uint32_t n) -> uint32_t { return n == NO_REF || n >= NN ? NO_REF : cid[n]; };
    std::vector<std::pair<uint32_t, bool>> st{{0u, false}};
    while (!st.empty()) {
        auto [v, post] = st.back();
        st.pop_back();
        if (ref_of0(v) == NO_REF) continue;
        if (ref_of0(v) & LEAF_BIT) {
            leaves[v] = 1;
            continue;
        }
        if (!post) {
            if (seen[v]) continue;
            seen[v] = 1;
            st.push_back({v, true});
            for (uint32_t c : {nodes[v].left_idx, nodes[v].right_idx})
                if (c != NO_REF) st.push_back({c, false});
        } else {
            uint32_t sum = 0;
            for (uint32_t c : {nodes[v].left_idx, nodes[v].right_idx})
                if (c != NO_REF && ref_of0(c) != NO_REF) sum += leaves[c];
            leaves[v] = sum;
        }
    }
    return leaves;
}

struct FrustumRecords {
    int log2 = 2;
    int bound = 0;  // the DFS stack bound of the records (root record)
    size_t nrec = 0;
    std::vector<float> rec;
};
static FrustumRecords build_frustum_records(const rt_bvh_node* nodes, size_t NN, const uint32_t* cid,
                                            const rt_aabb* aabbs, int dmax, int cap) {
    FrustumRecords out;
    auto ref_of0 = [&](uint32_t n) -> uint32_t { return n == NO_REF ? NO_REF : cid[n]; };
    // RT_TUNE_RECORD_GREEDY: a record's entries are grown from its node's children by expanding,
    // in place (the DFS order stays the reference's), the internal entry of largest weight until
    // A entries: 2 (default) surface area x sqrt(valid leaves below), 1 surface area (3: x
    // log2(leaves + 1), 4: x leaves); 0: every path to the same depth.  Larger boxes are the ones
    // rays reach: c3 0.1412 vs 0.1452 ms, c5 41.0 vs 42.9 with the area (frog 3,416 records vs
    // 3,854, bound 94 vs 91; profiles/r05/exp/record_greedy_ab_c*.log); the leaf weight: c5
    // 39.3-39.9 vs 40.8-41.1, c3 within noise (record_rules_ab.log)
    const int greedy_rule = int(rt::tuning(RT_TUNE_RECORD_GREEDY, 2.0) + 0.5);
    const bool greedy = greedy_rule > 0;
    const std::vector<uint32_t> leaves = greedy_rule >= 2 ? subtree_leaves(nodes, NN, cid) : std::vector<uint32_t>();
    auto area = [&](uint32_t n) {
        const rt_aabb& b = aabbs[n];
        const double dx = std::max(0.0, double(b.max_corner.x) - b.min_corner.x);
        const double dy = std::max(0.0, double(b.max_corner.y) - b.min_corner.y);
        const double dz = std::max(0.0, double(b.max_corner.z) - b.min_corner.z);
        double a = dx * dy + dy * dz + dz * dx;
        if (greedy_rule == 2) a *= std::sqrt(double(leaves[n]));
        if (greedy_rule == 3) a *= std::log2(double(leaves[n]) + 1.0);
        if (greedy_rule == 4) a *= double(leaves[n]);
        return std::isfinite(a) ? a : 1e300;
    };
    for (int D = std::min(dmax, 5); D >= 3; --D) {
        const int A = 1 << D;
        auto expand = [&](auto&& self, uint32_t n, int d, uint32_t* e, int& k) -> void {
            if (ref_of0(n) == NO_REF) return;
            if (d == 0 || (ref_of0(n) & LEAF_BIT)) {
                e[k++] = n;
                return;
            }
            self(self, nodes[n].left_idx, d - 1, e, k);
            self(self, nodes[n].right_idx, d - 1, e, k);
        };
        std::vector<uint32_t> recs{0u};  // binary node of each record, breadth first
        std::vector<uint32_t> fid(NN, NO_REF);
        fid[0] = 0;
        std::vector<std::array<uint32_t, 32>> ents;
        std::vector<int> nent;
        for (size_t r = 0; r < recs.size(); ++r) {
            std::array<uint32_t, 32> e;
            int k = 0;
            if (greedy) {
                std::vector<uint32_t> fr;
                for (uint32_t c : {nodes[recs[r]].left_idx, nodes[recs[r]].right_idx})
                    if (ref_of0(c) != NO_REF) fr.push_back(c);
                while ((int)fr.size() < A) {
                    int best = -1;
                    double ba = -1.0;
                    for (int i = 0; i < (int)fr.size(); ++i) {
                        if (ref_of0(fr[i]) & LEAF_BIT) continue;
                        const double a = area(fr[i]);
                        if (a > ba) {
                            ba = a;
                            best = i;
                        }
                    }
                    if (best < 0) break;
                    std::vector<uint32_t> kids;
                    for (uint32_t c : {nodes[fr[best]].left_idx, nodes[fr[best]].right_idx})
                        if (ref_of0(c) != NO_REF) kids.push_back(c);
                    fr.erase(fr.begin() + best);
                    fr.insert(fr.begin() + best, kids.begin(), kids.end());
                }
                for (uint32_t n : fr) e[k++] = n;
            } else {
                expand(expand, nodes[recs[r]].left_idx, D - 1, e.data(), k);
                expand(expand, nodes[recs[r]].right_idx, D - 1, e.data(), k);
            }
            for (int i = 0; i < k; ++i)
                if (!(ref_of0(e[i]) & LEAF_BIT) && fid[e[i]] == NO_REF) {
                    fid[e[i]] = uint32_t(recs.size());
                    recs.push_back(e[i]);
                }
            ents.push_back(e);
            nent.push_back(k);
        }
        // DFS stack bound: entry i of a record is processed with entries 0..i-1 on the stack
        std::vector<int> SF(recs.size(), 0);
        for (size_t r = recs.size(); r-- > 0;) {
            int sf = nent[r];
            for (int i = 0; i < nent[r]; ++i)
                if (!(ref_of0(ents[r][i]) & LEAF_BIT)) sf = std::max(sf, i + SF[fid[ents[r][i]]]);
            SF[r] = sf;
        }
        if (SF[0] > cap) continue;
        out.rec.assign(size_t(8 * A) * recs.size(), 0.f);
        for (size_t r = 0; r < recs.size(); ++r) {
            float* w = &out.rec[size_t(8 * A) * r];
            for (int i = 0; i < A; ++i) {
                uint32_t wr = NO_REF;
                if (i < nent[r]) {
                    const uint32_t n = ents[r][i];
                    const rt_aabb& bb = aabbs[n];
                    const float v6[6] = {bb.min_corner.x, bb.max_corner.x, bb.min_corner.y,
                                         bb.max_corner.y, bb.min_corner.z, bb.max_corner.z};
                    std::memcpy(&w[6 * i], v6, sizeof(v6));
                    wr = (ref_of0(n) & LEAF_BIT) ? ref_of0(n) : fid[n];
                }
                std::memcpy(&w[6 * A + i], &wr, 4);
            }
        }
        out.log2 = D;
        out.bound = SF[0];
        out.nrec = recs.size();
        return out;
    }
    return out;
}

// The frustum records quantised (MODE_QR kernels: the big scenes, whose 1 KB records do not stay
// in the L2s): per record a grid over the union of its entries' boxes, origin o = the union's
// min and per axis a step h >= extent / 65534; entry bounds become 16-bit steps q_lo = the
// largest q with fma(q, h, o) <= min and q_hi = the smallest with fma(q, h, o) >= max, evaluated
// in float as the kernel does (fmaf, one rounding), so the dequantised box contains the entry's.
// The family test only decides what is pushed (leaves are tested exactly at pop), so looser
// boxes cost pops, never a different hit.  qent: A x (x lo | x hi << 16, y, z, ref) per record;
// qhdr: (o.x, o.y, o.z, h.x), (h.y, h.z, 0, 0).  False (no quantised records) when a bound is not
// finite, an extent exceeds 1e30 or a step would be subnormal.
static bool build_quant_records(const FrustumRecords& fr, std::vector<uint32_t>& qent, std::vector<float>& qhdr) {
    const int A = 1 << fr.log2;
    qent.assign(size_t(4 * A) * fr.nrec, 0u);
    qhdr.assign(size_t(8) * fr.nrec, 0.f);
    for (size_t r = 0; r < fr.nrec; ++r) {
        const float* w = &fr.rec[size_t(8 * A) * r];
        uint32_t* qe = &qent[size_t(4 * A) * r];
        float* qh = &qhdr[8 * r];
        for (int a = 0; a < 3; ++a) {
            float lo = INFINITY, hi = -INFINITY;
            for (int i = 0; i < A; ++i) {
                uint32_t ref;
                std::memcpy(&ref, &w[6 * A + i], 4);
                if (ref == NO_REF) continue;
                lo = std::min(lo, w[6 * i + 2 * a]);
                hi = std::max(hi, w[6 * i + 2 * a + 1]);
            }
            if (lo > hi) lo = hi = 0.f;  // a record without entries (not built, kept total)
            if (!std::isfinite(lo) || !std::isfinite(hi) || double(hi) - double(lo) > 1e30) return false;
            float h = float((double(hi) - double(lo)) / 65534.0);
            if (double(h) * 65534.0 < double(hi) - double(lo)) h = std::nextafter(h, INFINITY);
            if (h != 0.f && !(h >= 1e-30f)) return false;
            (a == 0 ? qh[3] : qh[3 + a]) = h;
            qh[a] = lo;
            for (int i = 0; i < A; ++i) {
                uint32_t ref;
                std::memcpy(&ref, &w[6 * A + i], 4);
                if (ref == NO_REF) continue;
                const float mn = w[6 * i + 2 * a], mx = w[6 * i + 2 * a + 1];
                uint32_t ql = 0, qh16 = 0;
                if (h > 0.f) {
                    double fl = std::floor((double(mn) - double(lo)) / double(h));
                    double fh = std::ceil((double(mx) - double(lo)) / double(h));
                    ql = uint32_t(std::clamp(fl, 0.0, 65535.0));
                    qh16 = uint32_t(std::clamp(fh, 0.0, 65535.0));
                    while (ql > 0 && std::fmaf(float(ql), h, lo) > mn) --ql;
                    while (qh16 < 65535 && std::fmaf(float(qh16), h, lo) < mx) ++qh16;
                }
                if (std::fmaf(float(ql), h, lo) > mn || std::fmaf(float(qh16), h, lo) < mx) return false;
                qe[4 * i + a] = ql | (qh16 << 16);
            }
        }
        for (int i = 0; i < A; ++i) std::memcpy(&qe[4 * i + 3], &w[6 * A + i], 4);
    }
    return true;
}

// Host-only view of build_frustum_records for the CPU tests (no device), with the ids as
// rt_scene_create makes them.  info: log2, bound, record count.  rec: copied when rec_cap
// (floats) suffices.
extern "C" int rt_debug_frustum_records(size_t P, const rt_bvh_node* nodes, const rt_aabb* aabbs, int max_log2,
                                        int stack_cap, int64_t* info, float* rec, size_t rec_cap) {
    if (P == 0 || !nodes || !aabbs || !info) return set_error(RT_ERR_ARG, "rt_debug_frustum_records: null argument");
    if (P > 0x3FFFFFFFull) return set_error(RT_ERR_UNSUPPORTED, "more than 2^30 triangles");
    const size_t NN = 2 * P - 1;
    // the caller's arrays are checked as rt_scene_create checks them: children in range and no
    // cycle reachable from the root (tests/test_host_fuzz.py)
    {
        std::vector<uint8_t> state(NN, 0);  // 0 new, 1 on the path, 2 done
        std::vector<std::pair<uint32_t, bool>> st{{0u, false}};
        while (!st.empty()) {
            auto [v, post] = st.back();
            st.pop_back();
            if (post) {
                state[v] = 2;
                continue;
            }
            if (state[v] == 1) return set_error(RT_ERR_ARG, "BVH contains a cycle");
            if (state[v] == 2) continue;
            state[v] = 1;
            st.push_back({v, true});
            const rt_bvh_node& nd = nodes[v];
            if (nd.object_idx != 0xFFFFFFFFu) continue;
            for (const uint32_t c : {nd.left_idx, nd.right_idx}) {
                if (c == NO_REF) continue;
                if (c >= NN) return set_error(RT_ERR_ARG, "BVH child index out of range");
                st.push_back({c, false});
            }
        }
    }
    std::vector<uint32_t> cid(NN, NO_REF);
    size_t n_int = 0, n_leaf = 0;
    for (size_t n = 0; n < NN; ++n) {
        if (nodes[n].object_idx == 0xFFFFFFFFu) cid[n] = uint32_t(n_int++);
        else if (nodes[n].object_idx < P) cid[n] = LEAF_BIT | uint32_t(n_leaf++);
    }
    if (nodes[0].object_idx != 0xFFFFFFFFu) {  // a leaf root: no records (rt_scene_create makes none)
        info[0] = 2;
        info[1] = 0;
        info[2] = 0;
        return RT_OK;
    }
    const FrustumRecords fr = build_frustum_records(nodes, NN, cid.data(), aabbs, std::clamp(max_log2, 2, 5), stack_cap);
    info[0] = fr.log2;
    info[1] = fr.bound;
    info[2] = (int64_t)fr.nrec;
    if (rec && rec_cap >= fr.rec.size() && !fr.rec.empty()) std::memcpy(rec, fr.rec.data(), fr.rec.size() * sizeof(float));
    return RT_OK;
}

extern "C" int rt_scene_create(int device, size_t P, const rt_bvh_node* nodes, const rt_aabb* aabbs,
                               const rt_triangle* tris, const int32_t* objids, const rt_material* mats,
                               int nmat, const rt_light* lights, int nlights, rt_scene** out) {
    if (!out) return set_error(RT_ERR_ARG, "rt_scene_create: null out");
    *out = nullptr;
    if (P == 0 || !nodes || !aabbs || !tris) return set_error(RT_ERR_ARG, "rt_scene_create: empty scene");
    if (P > 0x3FFFFFFFull) return set_error(RT_ERR_UNSUPPORTED, "more than 2^30 triangles");
    if (nmat < 0 || nlights < 0 || (nmat > 0 && !mats) || (nlights > 0 && !lights))
        return set_error(RT_ERR_ARG, "rt_scene_create: bad material/light arrays");
    const size_t NN = 2 * P - 1;
    // Classify nodes, give internal/leaf nodes compact ids, and check the reachable graph is
    // a finite tree; a tree whose DFS may need more than the 64-entry wave stack (SearchBVH's
    // push/pop order) is rendered by the MODE_DEEP kernels (the reference's 512-entry stack).
    std::vector<uint32_t> cid(NN, NO_REF);
    size_t n_int = 0, n_leaf = 0;
    for (size_t n = 0; n < NN; ++n) {
        const rt_bvh_node& nd = nodes[n];
        if (nd.object_idx == 0xFFFFFFFFu) {
            if ((nd.left_idx != NO_REF && nd.left_idx >= NN) || (nd.right_idx != NO_REF && nd.right_idx >= NN))
                return set_error(RT_ERR_ARG, "BVH child index out of range");
            cid[n] = uint32_t(n_int++);
        } else if (nd.object_idx < P) {
            cid[n] = LEAF_BIT | uint32_t(n_leaf++);
        }  // leaves naming no valid triangle are skipped by SearchBVH (query.h:263): NO_REF
    }
    // Wide (4-ary) records: internal node n lists the children of its children in SearchBVH's
    // push order (a leaf child stands for itself), so one visit tests and pushes what the
    // reference reaches in two.  The result is the same provided every internal child's box
    // contains its children's boxes (the pass the skipped test would give is then implied,
    // slab tests being monotone in the box), checked here; the wave path falls back to the
    // binary records otherwise, or when the 4-ary DFS stack would exceed 64 entries.
    auto ref_of0 = [&](uint32_t n) -> uint32_t { return n == NO_REF ? NO_REF : cid[n]; };
    // RT_TUNE_WIDE4_GREEDY (default 1): the 4-ary records' entries grown from the node's children
    // by expanding, in place, the internal entry of largest surface area (up to 4 entries); 0:
    // the grandchildren.  Exact for the reasons the grandchildren are (every box contains its
    // children's, checked below for every parent-child pair; the DFS order is SearchBVH's; no
    // leaf is tested between an expanded node's pop and its children's in the reference).
    // c3 0.1390 vs 0.1419 ms, c3b 1.2455 vs 1.2986, c5 40.35 vs 40.82
    // (profiles/r05/exp/wide4_greedy_ab.log)
    const int wide4_rule = int(rt::tuning(RT_TUNE_WIDE4_GREEDY, 1.0) + 0.5);
    const bool wide4_greedy = wide4_rule > 0;
    const std::vector<uint32_t> wleaves = wide4_rule == 2 ? subtree_leaves(nodes, NN, cid.data()) : std::vector<uint32_t>();
    auto box_area = [&](uint32_t n) {
        const rt_aabb& b = aabbs[n];
        const double dx = std::max(0.0, double(b.max_corner.x) - b.min_corner.x);
        const double dy = std::max(0.0, double(b.max_corner.y) - b.min_corner.y);
        const double dz = std::max(0.0, double(b.max_corner.z) - b.min_corner.z);
        double a = dx * dy + dy * dz + dz * dx;
        if (wide4_rule == 2) a *= std::sqrt(double(wleaves[n]));
        return std::isfinite(a) ? a : 1e300;
    };
    auto wide_entries = [&](const rt_bvh_node& nd, uint32_t* e) {
        int k = 0;
        if (wide4_greedy) {
            for (const uint32_t c : {nd.left_idx, nd.right_idx})
                if (ref_of0(c) != NO_REF) e[k++] = c;
            while (k < 4) {
                int best = -1;
                double ba = -1.0;
                for (int i = 0; i < k; ++i) {
                    if (ref_of0(e[i]) & LEAF_BIT) continue;
                    const double a = box_area(e[i]);
                    if (a > ba) {
                        ba = a;
                        best = i;
                    }
                }
                if (best < 0) break;
                uint32_t kids[2];
                int nk = 0;
                for (const uint32_t g : {nodes[e[best]].left_idx, nodes[e[best]].right_idx})
                    if (ref_of0(g) != NO_REF) kids[nk++] = g;
                uint32_t grown[4];
                int t = 0;
                for (int i = 0; i < k; ++i) {
                    if (i != best) grown[t++] = e[i];
                    else
                        for (int j = 0; j < nk; ++j) grown[t++] = kids[j];
                }
                for (int i = 0; i < t; ++i) e[i] = grown[i];
                k = t;
            }
            return k;
        }
        for (const uint32_t c : {nd.left_idx, nd.right_idx}) {
            if (ref_of0(c) == NO_REF) continue;
            if (ref_of0(c) & LEAF_BIT) {
                e[k++] = c;
                continue;
            }
            const rt_bvh_node& cn = nodes[c];
            if (ref_of0(cn.left_idx) != NO_REF) e[k++] = cn.left_idx;
            if (ref_of0(cn.right_idx) != NO_REF) e[k++] = cn.right_idx;
        }
        return k;
    };
    auto contains = [](const rt_aabb& o, const rt_aabb& i) {
        return o.min_corner.x <= i.min_corner.x && o.min_corner.y <= i.min_corner.y &&
               o.min_corner.z <= i.min_corner.z && o.max_corner.x >= i.max_corner.x &&
               o.max_corner.y >= i.max_corner.y && o.max_corner.z >= i.max_corner.z;
    };
    bool wide_ok = true, deep = false;
    int binary_stack = 0, wide_stack = 0;
    {
        std::vector<uint8_t> state(NN, 0);  // 0 new, 1 on path, 2 done
        std::vector<int> S(NN, 0), SW(NN, 0);
        std::vector<std::pair<uint32_t, bool>> st{{0u, false}};
        while (!st.empty()) {
            auto [v, post] = st.back();
            st.pop_back();
            const rt_bvh_node& nd = nodes[v];
            const bool internal = nd.object_idx == 0xFFFFFFFFu;
            if (!post) {
                if (state[v] == 1) return set_error(RT_ERR_ARG, "BVH contains a cycle");
                if (state[v] == 2) continue;
                state[v] = 1;
                st.push_back({v, true});
                if (internal) {
                    if (nd.left_idx != NO_REF) st.push_back({nd.left_idx, false});
                    if (nd.right_idx != NO_REF) st.push_back({nd.right_idx, false});
                }
            } else {
                state[v] = 2;
                if (internal) {
                    const int sl = nd.left_idx != NO_REF ? S[nd.left_idx] : 0;
                    const int sr = nd.right_idx != NO_REF ? S[nd.right_idx] : 0;
                    const int pushes = (nd.left_idx != NO_REF) + (nd.right_idx != NO_REF);
                    int s = pushes;
                    if (nd.right_idx != NO_REF) s = std::max(s, (nd.left_idx != NO_REF ? 1 : 0) + sr);
                    if (nd.left_idx != NO_REF) s = std::max(s, sl);
                    S[v] = s;
                    for (const uint32_t c : {nd.left_idx, nd.right_idx}) {
                        if (c == NO_REF || nodes[c].object_idx != 0xFFFFFFFFu) continue;
                        for (const uint32_t g : {nodes[c].left_idx, nodes[c].right_idx})
                            if (g != NO_REF && !contains(aabbs[c], aabbs[g])) wide_ok = false;
                    }
                    uint32_t e[4];
                    const int k = wide_entries(nd, e);
                    int sw = k;
                    for (int i = 0; i < k; ++i)
                        if (!(ref_of0(e[i]) & LEAF_BIT)) sw = std::max(sw, i + SW[e[i]]);
                    SW[v] = sw;
                }
            }
        }
        deep = std::max(1, S[0]) > STACK_CAP;
        binary_stack = std::max(1, S[0]);
        wide_stack = std::max(1, SW[0]);
        // traverse_wave_split addresses records by 32-bit byte offsets (ref << 7 into the 4-ary
        // array, << 5 into ibox, slot << 6 into the leaves): larger trees take the MODE_DEEP
        // kernels, which are exact for any tree.
        if (n_int >= (size_t(1) << 25) || n_leaf >= (size_t(1) << 26)) deep = true;
        if (deep || std::max(1, SW[0]) > STACK_CAP) wide_ok = false;
    }
    std::vector<float4> hin(4 * std::max<size_t>(n_int, 1)), hib(2 * std::max<size_t>(n_int, 1));
    std::vector<float4> hwn(wide_ok ? 8 * std::max<size_t>(n_int, 1) : 0);
    std::vector<float4> hlf(4 * std::max<size_t>(n_leaf, 1)), hnm(3 * P);
    auto ref_of = [&](uint32_t n) -> uint32_t { return n == NO_REF ? NO_REF : cid[n]; };
    for (size_t n = 0; n < NN; ++n) {
        const uint32_t c = cid[n];
        if (c == NO_REF) continue;
        const rt_bvh_node& nd = nodes[n];
        if (!(c & LEAF_BIT)) {
            const rt_aabb lb = nd.left_idx != NO_REF ? aabbs[nd.left_idx] : rt_aabb{};
            const rt_aabb rb = nd.right_idx != NO_REF ? aabbs[nd.right_idx] : rt_aabb{};
            float4* q = &hin[4 * c];  // per axis (min, max) pairs: left x y | left z, right x | right y z
            q[0] = make_float4(lb.min_corner.x, lb.max_corner.x, lb.min_corner.y, lb.max_corner.y);
            q[1] = make_float4(lb.min_corner.z, lb.max_corner.z, rb.min_corner.x, rb.max_corner.x);
            q[2] = make_float4(rb.min_corner.y, rb.max_corner.y, rb.min_corner.z, rb.max_corner.z);
            // z: children that are leaves naming no triangle (pushed by SearchBVH all the same:
            // the deep kernels keep their stack entries)
            const uint32_t inv = (nd.left_idx != NO_REF && ref_of(nd.left_idx) == NO_REF ? 1u : 0u) |
                                 (nd.right_idx != NO_REF && ref_of(nd.right_idx) == NO_REF ? 2u : 0u);
            uint32_t refs[4] = {ref_of(nd.left_idx), ref_of(nd.right_idx), inv, 0u};
            std::memcpy(&q[3], refs, 16);
            const rt_aabb& ob = aabbs[n];
            hib[2 * c] = make_float4(ob.min_corner.x, ob.max_corner.x, ob.min_corner.y, ob.max_corner.y);
            hib[2 * c + 1] = make_float4(ob.min_corner.z, ob.max_corner.z, 0.f, 0.f);
            if (wide_ok) {  // 4 x (x pair, y pair, z pair) | 4 refs | unused
                float w[32] = {};
                uint32_t e[4], wr[4] = {NO_REF, NO_REF, NO_REF, NO_REF};
                const int k = wide_entries(nd, e);
                for (int i = 0; i < k; ++i) {
                    const rt_aabb& bb = aabbs[e[i]];
                    const float v6[6] = {bb.min_corner.x, bb.max_corner.x, bb.min_corner.y,
                                         bb.max_corner.y, bb.min_corner.z, bb.max_corner.z};
                    std::memcpy(&w[6 * i], v6, sizeof(v6));
                    wr[i] = ref_of(e[i]);
                }
                std::memcpy(&w[24], wr, sizeof(wr));
                std::memcpy(&hwn[8 * c], w, sizeof(w));
            }
        } else {
            const uint32_t j = c & ~LEAF_BIT;
            const rt_triangle& t = tris[nd.object_idx];
            const rt_aabb& ob = aabbs[n];
            float4* q = &hlf[4 * j];
            int32_t ti = int32_t(nd.object_idx);
            float tif;
            std::memcpy(&tif, &ti, 4);
            // e1 = v1 - v0, e2 = v2 - v0 exactly as intersectTriangle computes them
            // v0 | e1, e2.x | e2.y e2.z, box x pair | box y pair, box z pair
            q[0] = make_float4(t.v0.x, t.v0.y, t.v0.z, tif);
            q[1] = make_float4(t.v1.x - t.v0.x, t.v1.y - t.v0.y, t.v1.z - t.v0.z, t.v2.x - t.v0.x);
            q[2] = make_float4(t.v2.y - t.v0.y, t.v2.z - t.v0.z, ob.min_corner.x, ob.max_corner.x);
            q[3] = make_float4(ob.min_corner.y, ob.max_corner.y, ob.min_corner.z, ob.max_corner.z);
        }
    }
    for (size_t t = 0; t < P; ++t) {
        hnm[3 * t] = make_float4(tris[t].n0.x, tris[t].n0.y, tris[t].n0.z, 0.f);
        hnm[3 * t + 1] = make_float4(tris[t].n1.x, tris[t].n1.y, tris[t].n1.z, 0.f);
        hnm[3 * t + 2] = make_float4(tris[t].n2.x, tris[t].n2.y, tris[t].n2.z, 0.f);
    }
    int rc = check_device(device);
    if (rc != RT_OK) return rc;
    DeviceGuard g(device);
    std::unique_ptr<rt_scene> s(new (std::nothrow) rt_scene());
    if (!s) return set_error(RT_ERR_NOMEM, "out of memory");
    s->device = device;
    s->P = P;
    s->nmat = nmat;
    s->nlights = nlights;
    s->root_ref = cid[0];
    if (s->root_ref == NO_REF) s->root_ref = LEAF_BIT | 0u;  // degenerate: unreachable leaf
    for (size_t n = 0; n < NN; ++n) {
        const rt_aabb& bb = aabbs[n];
        s->bmax[0] = std::max({s->bmax[0], std::fabs(bb.min_corner.x), std::fabs(bb.max_corner.x)});
        s->bmax[1] = std::max({s->bmax[1], std::fabs(bb.min_corner.y), std::fabs(bb.max_corner.y)});
        s->bmax[2] = std::max({s->bmax[2], std::fabs(bb.min_corner.z), std::fabs(bb.max_corner.z)});
    }
    // The pre-classification takes min <= max per axis (near/far bounds by the ray's sign); a
    // scene with an inverted, NaN or infinite box gets bmax = inf, which turns every float
    // classification ambiguous (make_ray: E = inf), so all its box tests take the exact path.
    bool sorted_boxes = true;
    for (size_t n = 0; n < NN; ++n) {
        const rt_aabb& bb = aabbs[n];
        sorted_boxes = sorted_boxes && bb.min_corner.x <= bb.max_corner.x && bb.min_corner.y <= bb.max_corner.y &&
                       bb.min_corner.z <= bb.max_corner.z;
    }
    for (float& v : s->bmax)
        if (!(v <= FLT_MAX) || !sorted_boxes) v = INFINITY;
    s->root_box[0] = aabbs[0].min_corner.x; s->root_box[1] = aabbs[0].min_corner.y; s->root_box[2] = aabbs[0].min_corner.z;
    s->root_box[3] = aabbs[0].max_corner.x; s->root_box[4] = aabbs[0].max_corner.y; s->root_box[5] = aabbs[0].max_corner.z;
    if (cid[0] == NO_REF) {  // root names no triangle: nothing can be hit; empty box
        s->root_box[0] = s->root_box[1] = s->root_box[2] = INFINITY;
        s->root_box[3] = s->root_box[4] = s->root_box[5] = -INFINITY;
    }
    // Tile-culling cut (tile_misses_scene): from the root, repeatedly replace the internal node
    // with the largest box (half surface area) by its children, up to kCut nodes.  Every leaf
    // keeps exactly one ancestor-or-self in the set; a missing child (NO_REF) holds no leaf.
    if (cid[0] != NO_REF && !(cid[0] & LEAF_BIT)) {
        // one box per lane of tile_cut_kernel (RT_TUNE_CULL_BOXES: fewer, for tests)
        const int kcut = int(std::clamp(rt::tuning(RT_TUNE_CULL_BOXES, 64.0), 0.0, 64.0));
        auto area = [&](uint32_t n) {
            const rt_aabb& bb = aabbs[n];
            const double dx = double(bb.max_corner.x) - bb.min_corner.x, dy = double(bb.max_corner.y) - bb.min_corner.y,
                         dz = double(bb.max_corner.z) - bb.min_corner.z;
            const double a = dx * dy + dy * dz + dz * dx;
            return a == a ? a : INFINITY;
        };
        std::vector<uint32_t> cutn{0u};
        while (int(cutn.size()) < kcut) {
            int best = -1;
            double ba = -1.0;
            for (int i = 0; i < int(cutn.size()); ++i) {
                if (cid[cutn[i]] & LEAF_BIT) continue;
                const double a = area(cutn[i]);
                if (a > ba) { ba = a; best = i; }
            }
            if (best < 0) break;
            const rt_bvh_node& nd = nodes[cutn[best]];
            cutn.erase(cutn.begin() + best);
            if (nd.left_idx != NO_REF && cid[nd.left_idx] != NO_REF) cutn.push_back(nd.left_idx);
            if (nd.right_idx != NO_REF && cid[nd.right_idx] != NO_REF) cutn.push_back(nd.right_idx);
        }
        if (kcut > 1) {
            std::vector<float> hc(6 * cutn.size());
            for (size_t i = 0; i < cutn.size(); ++i) {
                const rt_aabb& bb = aabbs[cutn[i]];
                const float v6[6] = {bb.min_corner.x, bb.min_corner.y, bb.min_corner.z,
                                     bb.max_corner.x, bb.max_corner.y, bb.max_corner.z};
                std::memcpy(&hc[6 * i], v6, sizeof(v6));
            }
            if ((rc = s->cut.upload(hc.data(), hc.size() * sizeof(float))) != RT_OK) return rc;
            s->ncut = int(cutn.size());
            // Second level (RT_TUNE_CUT_SUB sub-boxes per cut box, a power of two <= 64): the
            // same rule inside each cut node's subtree, so the tiles whose rays reach a cut box
            // are tested against the boxes below it (tile_cut_sub).  Unused slots repeat the
            // node's first sub-box: a duplicate changes no "every box missed" decision.
            const int sub = int(std::clamp(rt::tuning(RT_TUNE_CUT_SUB, 16.0), 0.0, 64.0));
            int sl = 0;
            while ((2 << sl) <= sub) ++sl;
            if (sub >= 2) {
                const int S = 1 << sl;
                std::vector<float> h2(size_t(6) * S * cutn.size());
                for (size_t i = 0; i < cutn.size(); ++i) {
                    std::vector<uint32_t> sn{cutn[i]};
                    while (int(sn.size()) < S) {
                        int best = -1;
                        double ba = -1.0;
                        for (int j = 0; j < int(sn.size()); ++j) {
                            if (cid[sn[j]] & LEAF_BIT) continue;
                            const double a = area(sn[j]);
                            if (a > ba) { ba = a; best = j; }
                        }
                        if (best < 0) break;
                        const rt_bvh_node& nd = nodes[sn[best]];
                        std::vector<uint32_t> kids;
                        if (nd.left_idx != NO_REF && cid[nd.left_idx] != NO_REF) kids.push_back(nd.left_idx);
                        if (nd.right_idx != NO_REF && cid[nd.right_idx] != NO_REF) kids.push_back(nd.right_idx);
                        if (int(sn.size()) - 1 + int(kids.size()) > S) break;
                        sn.erase(sn.begin() + best);
                        sn.insert(sn.end(), kids.begin(), kids.end());
                        if (sn.empty()) break;
                    }
                    if (sn.empty()) sn.push_back(cutn[i]);
                    for (int j = 0; j < S; ++j) {
                        const rt_aabb& bb = aabbs[sn[size_t(j) < sn.size() ? j : 0]];
                        const float v6[6] = {bb.min_corner.x, bb.min_corner.y, bb.min_corner.z,
                                             bb.max_corner.x, bb.max_corner.y, bb.max_corner.z};
                        std::memcpy(&h2[6 * (i * S + j)], v6, sizeof(v6));
                    }
                }
                if ((rc = s->cut2.upload(h2.data(), h2.size() * sizeof(float))) != RT_OK) return rc;
                s->cut_sub_log2 = sl;
            }
        }
    }
    if ((rc = s->inode.upload(hin.data(), hin.size() * sizeof(float4))) != RT_OK) return rc;
    if (wide_ok && (rc = s->wnode.upload(hwn.data(), hwn.size() * sizeof(float4))) != RT_OK) return rc;
    // the camera rays' frustum records (build_frustum_records), for the traversal's 128-entry stack
    // RT_TUNE_FRUSTUM_ARITY: the largest arity's log2 to try (tests; 2 = the 4-ary records)
    int fr_dmax = int(std::clamp(rt::tuning(RT_TUNE_FRUSTUM_ARITY, 5.0), 2.0, 5.0));
#ifdef RT_NO_F16  // (variant builds for A/B runs: the frustum traversal over the 4-ary records)
    fr_dmax = 2;
#endif
    const bool frustum = wide_ok && !(s->root_ref & LEAF_BIT) && fr_dmax > 2;
    if (frustum) {
        // RT_TUNE_FRUSTUM_STACK_CAP (test hook only): records whose DFS may outgrow the stack,
        // to exercise traverse_frustum's overflow guard
        const int cap = int(std::clamp(rt::tuning(RT_TUNE_FRUSTUM_STACK_CAP, double(FRUSTUM_STACK)), 1.0, 1e6));
        const FrustumRecords fr = build_frustum_records(nodes, NN, cid.data(), aabbs, fr_dmax, cap);
        if (fr.log2 > 2) {
            if ((rc = s->fnode.upload(fr.rec.data(), fr.rec.size() * sizeof(float))) != RT_OK) return rc;
            s->f_log2 = fr.log2;
            s->f_bound = fr.bound;
            // RT_TUNE_QUANT_RECORDS: 1 quantised records for every scene with frustum records,
            // -1 for scenes whose float records alone exceed the big-scene threshold's eighth
            // (c5: 34 MB; frog: 0.6 MB), 0 (default) none: c5 45.5 vs 42.4 ms with them, the
            // dequantisation's VALU costing more than the halved record lines save
            // (profiles/r05/exp/quant_records_ab_c5.log)
            const double qk = rt::tuning(RT_TUNE_QUANT_RECORDS, 0.0);
            const double big = rt::tuning(RT_TUNE_BIG_SCENE_BYTES, double(kBigSceneBytes));
            const bool want_q = qk > 0.5 || (qk < -0.5 && double(fr.rec.size() * sizeof(float)) > big / 8.0);
            std::vector<uint32_t> qe;
            std::vector<float> qh;
            if (want_q && build_quant_records(fr, qe, qh)) {
                if ((rc = s->qent.upload(qe.data(), qe.size() * sizeof(uint32_t))) != RT_OK) return rc;
                if ((rc = s->qhdr.upload(qh.data(), qh.size() * sizeof(float))) != RT_OK) return rc;
            }
        }
    }
    s->wide = wide_ok && !(s->root_ref & LEAF_BIT);
    s->lane_stack = !deep && binary_stack <= LANE_LDS_CAP;
    s->lane_wide = s->wide && s->lane_stack && wide_stack <= LANE_LDS_CAP;
    s->deep = deep;
    if (deep) {  // v0 | e1, e2.x | e2.y, e2.z by triangle index, e1/e2 as intersectTriangle computes them
        std::vector<float4> ht(3 * P);
        for (size_t t = 0; t < P; ++t) {
            const rt_triangle& tr = tris[t];
            ht[3 * t] = make_float4(tr.v0.x, tr.v0.y, tr.v0.z, 0.f);
            ht[3 * t + 1] = make_float4(tr.v1.x - tr.v0.x, tr.v1.y - tr.v0.y, tr.v1.z - tr.v0.z, tr.v2.x - tr.v0.x);
            ht[3 * t + 2] = make_float4(tr.v2.y - tr.v0.y, tr.v2.z - tr.v0.z, 0.f, 0.f);
        }
        if ((rc = s->tri.upload(ht.data(), ht.size() * sizeof(float4))) != RT_OK) return rc;
    }
    // the root's box (pair layout) after the internal boxes: the traversals' first test reads it
    // with scalar loads like any other box (SceneView::rootb)
    hib.push_back(make_float4(s->root_box[0], s->root_box[3], s->root_box[1], s->root_box[4]));
    hib.push_back(make_float4(s->root_box[2], s->root_box[5], 0.f, 0.f));
    if ((rc = s->ibox.upload(hib.data(), hib.size() * sizeof(float4))) != RT_OK) return rc;
    if ((rc = s->leaf.upload(hlf.data(), hlf.size() * sizeof(float4))) != RT_OK) return rc;
    if ((rc = s->tnorm.upload(hnm.data(), hnm.size() * sizeof(float4))) != RT_OK) return rc;
    if (objids && (rc = s->objids.upload(objids, P * sizeof(int32_t))) != RT_OK) return rc;
    if (nmat > 0 && (rc = s->mats.upload(mats, size_t(nmat) * sizeof(rt_material))) != RT_OK) return rc;
    if (nlights > 0 && (rc = s->lights.upload(lights, size_t(nlights) * sizeof(rt_light))) != RT_OK) return rc;
    if ((rc = s->create_sync()) != RT_OK) return rc;
    s->bytes = s->inode.n + s->wnode.n + s->fnode.n + s->ibox.n + s->leaf.n + s->tnorm.n + s->objids.n +
               s->mats.n + s->lights.n;
    *out = s.release();
    return RT_OK;
}

extern "C" int rt_scene_clone(const rt_scene* src, int device, rt_scene** out) {
    if (!src || !out) return set_error(RT_ERR_ARG, "rt_scene_clone: null argument");
    *out = nullptr;
    int rc = check_device(device);
    if (rc != RT_OK) return rc;
    DeviceGuard g(device);
    std::unique_ptr<rt_scene> s(new (std::nothrow) rt_scene());
    if (!s) return set_error(RT_ERR_NOMEM, "out of memory");
    s->device = device;
    s->P = src->P;
    s->nmat = src->nmat;
    s->nlights = src->nlights;
    s->root_ref = src->root_ref;
    std::memcpy(s->root_box, src->root_box, sizeof(s->root_box));
    std::memcpy(s->bmax, src->bmax, sizeof(s->bmax));
    s->ncut = src->ncut;
    s->cut_sub_log2 = src->cut_sub_log2;
    s->wide = src->wide;
    s->lane_stack = src->lane_stack;
    s->lane_wide = src->lane_wide;
    s->f_log2 = src->f_log2;
    s->f_bound = src->f_bound;
    s->deep = src->deep;
    s->cus = src->cus;
    s->bytes = src->bytes;
    // device-to-device copies of the packed arrays (over xGMI when the devices differ)
    const std::pair<DevBuf*, const DevBuf*> bufs[] = {{&s->inode, &src->inode}, {&s->wnode, &src->wnode},
                                                      {&s->fnode, &src->fnode},
                                                      {&s->qent, &src->qent},   {&s->qhdr, &src->qhdr},
                                                      {&s->ibox, &src->ibox},   {&s->leaf, &src->leaf},
                                                      {&s->tnorm, &src->tnorm}, {&s->objids, &src->objids},
                                                      {&s->mats, &src->mats},   {&s->lights, &src->lights},
                                                      {&s->cut, &src->cut},     {&s->cut2, &src->cut2},
                                                      {&s->tri, &src->tri}};
    for (const auto& [d, q] : bufs) {
        if ((rc = d->alloc(q->n)) != RT_OK) return rc;
        if (q->n) HIP_TRY(hipMemcpyPeer(d->p, device, q->p, src->device, q->n));
    }
    if ((rc = s->create_sync()) != RT_OK) return rc;
    *out = s.release();
    return RT_OK;
}

extern "C" void rt_scene_destroy(rt_scene* s) {
    if (!s) return;
    DeviceGuard g(s->device);
    delete s;
}
extern "C" int rt_scene_device(const rt_scene* s) { return s ? s->device : -1; }

extern "C" int rt_scene_traversal_info(const rt_scene* s, int64_t info[4]) {
    if (!s || !info) return set_error(RT_ERR_ARG, "rt_scene_traversal_info: null argument");
    const bool frustum = s->wide && !s->deep;
    info[0] = frustum ? s->f_log2 : 0;
    info[1] = frustum && s->f_log2 > 2 ? s->f_bound : 0;
    info[2] = s->wide ? 1 : 0;
    info[3] = s->deep ? 1 : 0;
    return RT_OK;
}

extern "C" int rt_scene_faults(rt_scene* s, uint32_t* flags, int clear) {
    if (!s || !flags) return set_error(RT_ERR_ARG, "rt_scene_faults: null argument");
    DeviceGuard g(s->device);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(flags, s->fault.p, sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (clear) HIP_TRY(hipMemset(s->fault.p, 0, sizeof(uint32_t)));
    return RT_OK;
}
extern "C" size_t rt_scene_device_bytes(const rt_scene* s) { return s ? s->bytes : 0; }

extern "C" void rt_render_opts_default(rt_render_opts* o) {
    o->max_depth = 1;
    o->spp = 1;
    o->diffuse_bounce = 1;
    o->miss_color = rt_vec3{0.f, 0.f, 0.f};
    o->jitter = nullptr;
    o->band_rows = 8;
    o->band_index = 0;
    o->band_count = 1;
    o->kernel = RT_KERNEL_AUTO;
    o->tile_order = RT_TILES_AUTO;
    o->flags = 0;
}

extern "C" int rt_shard_rows(int H, int band_rows, int band_index, int band_count) {
    if (H <= 0) return 0;
    if (band_count <= 1) return H;
    if (band_rows <= 0 || band_index < 0 || band_index >= band_count) return -1;
    const int nbands = (H + band_rows - 1) / band_rows;
    int rows = 0;
    for (int b = band_index; b < nbands; b += band_count) rows += std::min(band_rows, H - b * band_rows);
    return rows;
}

namespace {

int prepare_jitter(rt_scene* s, const rt_render_opts* o) {
    std::vector<float> tab(2 * size_t(o->spp));
    if (o->jitter) std::memcpy(tab.data(), o->jitter, tab.size() * sizeof(float));
    else {
        int rc = rt_jittered_samples(o->spp, 42u, 1, tab.data());
        if (rc != RT_OK) return rc;
    }
    if (s->jitter_spp == o->spp && s->jitter_host == tab) return RT_OK;
    int rc = s->jitter.upload(tab.data(), tab.size() * sizeof(float));
    if (rc != RT_OK) return rc;
    s->jitter_host = tab;
    s->jitter_spp = o->spp;
    return RT_OK;
}

// The render kernel's persistent grid: the blocks of it one dispatch keeps resident on every CU
// (the occupancy the kernel was compiled for, LDS permitting), a multiple of 8 (one share per
// XCD queue), at most one block per tile.  Blocks beyond residency would only find the queues
// empty.  The render kernel's start / end events (rt_kernel_times) go into its dispatch
// (hipExtLaunchKernel): no separate event packets on the stream between the frames' kernels.
struct Launch {
    hipStream_t st;
    hipEvent_t start, stop;
    int cus;
    bool big;  // scene data beyond kBigSceneBytes: the depth-1 wave kernels at RT_RENDER_WAVES_BIG
    bool qr;   // ... over the quantised frustum records (MODE_QR), which the scene has
    const char** name;  // out: the launched instantiation, as rocprofv3 names it (rt_scene_kernel_name)
};
template <int MODE, bool SAMPLES, bool D1, int WAVES = RT_RENDER_WAVES, int LS = 0>
void launch_render(const RenderParams& P, const Launch& L) {
    constexpr auto KERNEL = render_tiles_kernel<MODE, SAMPLES, D1, WAVES, LS>;
    static const int per_cu = [] {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, KERNEL, BLOCK, 0) != hipSuccess || n < 1) n = 1;
        return n;
    }();
    static const std::string name = "render_tiles_kernel<" + std::to_string(MODE) + (SAMPLES ? ", true" : ", false") +
                                    (D1 ? ", true, " : ", false, ") + std::to_string(WAVES) + ", " +
                                    std::to_string(LS) + ">";
    if (L.name) *L.name = name.c_str();
    const int tiles8 = (P.tiles_total + 7) / 8 * 8;
    const dim3 grid((unsigned)std::max(8, std::min(tiles8, L.cus * per_cu / 8 * 8)));
    hipExtLaunchKernelGGL(KERNEL, grid, dim3(BLOCK), 0, L.st, L.start, L.stop, 0, P);
}

// Two frames, one persistent grid (render_pair_kernel): the grid launch_render gives one frame,
// at most one block per tile of the two.
template <int MODE, bool SAMPLES, bool D1, int WAVES = RT_RENDER_WAVES, int LS = 0>
void launch_render_pair(const RenderParams& A, const RenderParams& B, const Launch& L, double reserve_default) {
    constexpr auto KERNEL = render_pair_kernel<MODE, SAMPLES, D1, WAVES, LS>;
    static const int per_cu = [] {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, KERNEL, BLOCK, 0) != hipSuccess || n < 1) n = 1;
        return n;
    }();
    static const std::string name = "render_pair_kernel<" + std::to_string(MODE) + (SAMPLES ? ", true" : ", false") +
                                    (D1 ? ", true, " : ", false, ") + std::to_string(WAVES) + ", " +
                                    std::to_string(LS) + ">";
    if (L.name) *L.name = name.c_str();
    const int tiles8 = (A.tiles_total + B.tiles_total + 7) / 8 * 8;
    // RT_TUNE_PAIR_RESERVE: block slots per CU left to the next pair's pre-passes, which then run
    // beside this kernel instead of after it (c3: 0.148 ms per delivered frame vs 0.151 with
    // none and 0.157 with two, profiles/r05/exp/pair_knobs_c3.log; fractions: that many slots
    // per CU on average).  The bounce kernels' pairs reserve none by default: a 1.2 ms kernel
    // hides its pre-passes anyway, and a slot is a quarter of their 4 waves per SIMD (c3b 1.53
    // ms per frame with one, 1.13 with none, profiles/r05/exp/pair_c3b.log).
    const double reserve = std::clamp(rt::tuning(RT_TUNE_PAIR_RESERVE, reserve_default), 0.0, double(per_cu - 1));
    const int blocks = L.cus * per_cu - int(std::lround(reserve * L.cus));
    const dim3 grid((unsigned)std::max(8, std::min(tiles8, blocks / 8 * 8)));
    PairParams PP;
    PP.f[0] = A;
    PP.f[1] = B;
    hipExtLaunchKernelGGL(KERNEL, grid, dim3(BLOCK), 0, L.st, L.start, L.stop, 0, PP);
}

// The frames a pair kernel is instantiated for: depth-1 sample kernels of the 4-ary-record wave
// traversal on a scene within kBigSceneBytes, full or half waves (c3 and its band shards).
// Anything else renders a pair as two launches.
// Multi-bounce frames take it too where launch_mode picks the paired-only bounce kernels (one
// light, half waves, LS = 3: c3b): their longest items bound a launch, and a pair overlaps two
// frames' longest items.
bool pair_kernel_fits(const RenderParams& P, bool samples, bool wave_wide, bool big) {
    const bool d1 = P.max_depth == 1;
    const bool bounce = P.max_depth > 1 && P.half_waves && P.paired_only;
    return samples && wave_wide && !big && (d1 || bounce) && P.nqueues == 8 && P.spp <= 64 && !P.ray_count &&
           P.lane_samples == 1;
}
void launch_pair(const RenderParams& A, const RenderParams& B, const Launch& L) {
    constexpr int M = RT_KERNEL_WAVE | MODE_WIDE | MODE_PK;  // launch_mode's D1_MODE for these
    if (A.max_depth > 1) launch_render_pair<RT_KERNEL_WAVE | MODE_WIDE, true, false, RT_PAIRED_WAVES, 3>(A, B, L, 0.0);
    else if (A.half_waves) launch_render_pair<M, true, true, RT_RENDER_WAVES, 1>(A, B, L, 1.0);
    else launch_render_pair<M, true, true>(A, B, L, 1.0);
}

template <int MODE, bool SAMPLES>
void launch_mode(const RenderParams& P, const Launch& L) {
    // depth-1 kernels of the wave traversal: packed box tests (box_ends_pk)
    constexpr int D1_MODE = (MODE & (MODE_DEEP | RT_KERNEL_LANE)) == 0 ? (MODE | MODE_PK) : MODE;
    if (P.max_depth == 1) {
        if constexpr (SAMPLES) {
            if (P.half_waves) {
                launch_render<D1_MODE, SAMPLES, true, RT_RENDER_WAVES, 1>(P, L);
                return;
            }
        }
        if constexpr ((MODE & (MODE_DEEP | RT_KERNEL_LANE)) == 0) {
            if (L.big) {
                if constexpr ((MODE & MODE_WIDE) != 0) {
                    if (L.qr) {
                        if (P.sc.num_lights == 1)
                            launch_render<D1_MODE | MODE_1L | MODE_QR, SAMPLES, true, RT_RENDER_WAVES_BIG>(P, L);
                        else launch_render<D1_MODE | MODE_QR, SAMPLES, true, RT_RENDER_WAVES_BIG>(P, L);
                        return;
                    }
                }
                if (P.sc.num_lights == 1) launch_render<D1_MODE | MODE_1L, SAMPLES, true, RT_RENDER_WAVES_BIG>(P, L);
                else launch_render<D1_MODE, SAMPLES, true, RT_RENDER_WAVES_BIG>(P, L);
                return;
            }
        }
        launch_render<D1_MODE, SAMPLES, true>(P, L);
    } else {
        if constexpr (SAMPLES && (MODE & (MODE_DEEP | RT_KERNEL_LANE)) == 0) {
            if (P.half_waves && P.paired_only) {
                launch_render<MODE, SAMPLES, false, RT_PAIRED_WAVES, 3>(P, L);
                return;
            }
        }
        if constexpr (SAMPLES) {
            if (P.half_waves) {
                // the unpaired loop alone (one-light scenes whose lanes can pair take LS = 3 above;
                // carrying paired_bounces here as well cost 84 B of scratch per lane: cornell 7.94
                // vs 7.06 ms, profiles/r04/exp/ls2_ab_cornell.log)
                launch_render<MODE, SAMPLES, false, RT_BOUNCE_WAVES, 1>(P, L);
                return;
            }
        }
        launch_render<MODE, SAMPLES, false, RT_BOUNCE_WAVES>(P, L);
    }
}

template <int MODE>
void launch(const RenderParams& P, bool samples, const Launch& L) {
    if (samples) launch_mode<MODE, true>(P, L);
    else launch_mode<MODE, false>(P, L);
}

// Host restatement of a pixel whose spp samples all miss the root: each sample is
// clamp(0 + (1,1,1) * missColor) (query.h:181-183), or 0 when max_depth <= 0 (query.h:172);
// col accumulates them in order and is divided by float(spp) (query.cu:146-163).
f3 miss_pixel_value(const rt_render_opts* o) {
    f3 c = mk(0.f, 0.f, 0.f);
    if (o->max_depth > 0)
        c = clamp01(add(mk(0.f, 0.f, 0.f), mul(mk(1.f, 1.f, 1.f), f3{o->miss_color.x, o->miss_color.y, o->miss_color.z})));
    f3 acc = mk(0.f, 0.f, 0.f);
    for (int k = 0; k < o->spp; ++k) acc = add(acc, c);
    const float fs = (float)o->spp;
    return f3{acc.x / fs, acc.y / fs, acc.z / fs};
}

}  // namespace

namespace {
// Fraction of the image covered by the bounding rectangle of the root box's projected corners
// (1 when a corner is not in front of the camera).  The tree-cut culling pass (tile_cut_kernel)
// is launched only when this is small: a scene that fills the view gains no culled tiles from
// it and pays for the pass (a speed choice; culling or not gives the same image).
double root_box_coverage(const float* rb, const rt_camera* cam) {
    const double c[3] = {cam->center.x, cam->center.y, cam->center.z};
    const double b0[3] = {cam->pixel00_loc.x - c[0], cam->pixel00_loc.y - c[1], cam->pixel00_loc.z - c[2]};
    const double du[3] = {cam->pixel_delta_u.x, cam->pixel_delta_u.y, cam->pixel_delta_u.z};
    const double dv[3] = {cam->pixel_delta_v.x, cam->pixel_delta_v.y, cam->pixel_delta_v.z};
    // solve s*b0 + a*du + b*dv = corner - c (Cramer); pixel = (a/s, b/s)
    auto det3 = [](const double* x, const double* y, const double* z) {
        return x[0] * (y[1] * z[2] - y[2] * z[1]) - y[0] * (x[1] * z[2] - x[2] * z[1]) + z[0] * (x[1] * y[2] - x[2] * y[1]);
    };
    const double D = det3(b0, du, dv);
    if (!(std::fabs(D) > 0.0) || !(rb[0] <= rb[3] && rb[1] <= rb[4] && rb[2] <= rb[5])) return 1.0;
    double x0 = INFINITY, x1 = -INFINITY, y0 = INFINITY, y1 = -INFINITY;
    for (int k = 0; k < 8; ++k) {
        const double p[3] = {double(rb[(k & 1) ? 3 : 0]) - c[0], double(rb[(k & 2) ? 4 : 1]) - c[1],
                             double(rb[(k & 4) ? 5 : 2]) - c[2]};
        const double sx = det3(p, du, dv) / D, a = det3(b0, p, dv) / D, b = det3(b0, du, p) / D;
        if (!(sx > 0.0)) return 1.0;
        x0 = std::min(x0, a / sx);
        x1 = std::max(x1, a / sx);
        y0 = std::min(y0, b / sx);
        y1 = std::max(y1, b / sx);
    }
    const double W = cam->pixel_width, H = cam->pixel_height;
    const double w = std::max(0.0, std::min(W, x1) - std::max(0.0, x0)), h = std::max(0.0, std::min(H, y1) - std::max(0.0, y0));
    return w * h / (W * H);
}
}  // namespace

// Set by rt_count_rays around its one render (the calling thread's frame only).
thread_local unsigned long long* t_ray_count = nullptr;

extern "C" int rt_render_device(rt_scene* s, const rt_camera* cam, const rt_render_opts* o, float* rgb,
                                int32_t* hit_idx, float* hit_t, void* stream) {
    return rt_render_device_p6(s, cam, o, rgb, hit_idx, hit_t, nullptr, stream);
}

namespace {
// Two frames in one render launch (rt::render_pair).  Frame A's call runs its pre-passes and,
// when the pair kernel fits it (pair_kernel_fits, RT_TUNE_PAIR_FRAMES on), keeps its parameters
// here instead of launching; frame B's call runs its pre-passes and launches both.  A frame B
// that cannot join (another tile geometry or cut, a failed call) launches A on its own first.
struct PairStage {
    int phase = 0;          // 0: frame A's call, 1: frame B's
    bool deferred = false;  // frame A's render launch is held here
    RenderParams A;
    Launch LA{};
    uint64_t kA = 0;
    hipStream_t stream = nullptr;
};

// A frame's pre-passes on the scene's prep stream; ev0 / pdone: their start and end, recorded
// by the dispatches themselves.
int launch_prepasses(rt_scene* s, const RenderParams& P, int slot) {
    const bool cut = P.cull && P.sc.ncut > 0;
    hipExtLaunchKernelGGL(tile_cull_kernel, dim3((P.tiles_total + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s->prep,
                          s->ev0[slot], cut ? nullptr : s->pdone[slot], 0, P);
    HIP_TRY(hipGetLastError());
    if (cut) {
        // 16 waves per CU; each takes (list, group) pairs grid-stride (c3: about one each)
        const int cut_blocks = 4 * s->cus;
        hipExtLaunchKernelGGL(tile_cut_kernel, dim3(cut_blocks), dim3(BLOCK), 0, s->prep, nullptr, s->pdone[slot], 0, P);
        HIP_TRY(hipGetLastError());
    }
    return RT_OK;
}

int flush_pair_a(rt_scene* s, PairStage& ps) {
    if (!ps.deferred) return RT_OK;
    ps.deferred = false;
    const int slot = int(ps.kA % rt_scene::kRing);
    s->span[slot] = 1;
    if (int rc = launch_prepasses(s, ps.A, slot); rc != RT_OK) return rc;
    HIP_TRY(hipStreamWaitEvent(ps.LA.st, s->pdone[slot], 0));
    launch<RT_KERNEL_WAVE | MODE_WIDE>(ps.A, true, ps.LA);
    HIP_TRY(hipGetLastError());
    if (ps.A.drained) s->drain_frame = ps.kA;
    return RT_OK;
}

int render_frame(rt_scene* s, const rt_camera* cam, const rt_render_opts* o, float* rgb, int32_t* hit_idx,
                 float* hit_t, uint8_t* p6, void* stream, PairStage* ps);
}  // namespace

extern "C" int rt_render_device_p6(rt_scene* s, const rt_camera* cam, const rt_render_opts* o, float* rgb,
                                   int32_t* hit_idx, float* hit_t, uint8_t* p6, void* stream) {
    return render_frame(s, cam, o, rgb, hit_idx, hit_t, p6, stream, nullptr);
}

extern "C" int rt_render_device_pair(rt_scene* s, const rt_camera* cam_a, const rt_camera* cam_b,
                                     const rt_render_opts* o, float* rgb_a, uint8_t* p6_a, float* rgb_b,
                                     uint8_t* p6_b, void* stream) {
    if (!s || !cam_a || !cam_b || !o || (!rgb_a && !p6_a) || (!rgb_b && !p6_b))
        return set_error(RT_ERR_ARG, "rt_render_device_pair: null argument");
    PairStage ps;
    int rc = render_frame(s, cam_a, o, rgb_a, nullptr, nullptr, p6_a, stream, &ps);
    if (rc != RT_OK) return rc;
    ps.phase = 1;
    rc = render_frame(s, cam_b, o, rgb_b, nullptr, nullptr, p6_b, stream, &ps);
    if (ps.deferred) {  // frame B failed before its launch: frame A still renders
        DeviceGuard g(s->device);
        const int rc2 = flush_pair_a(s, ps);
        if (rc == RT_OK) rc = rc2;
    }
    return rc;
}

namespace {
int render_frame(rt_scene* s, const rt_camera* cam, const rt_render_opts* o, float* rgb, int32_t* hit_idx,
                 float* hit_t, uint8_t* p6, void* stream, PairStage* ps) {
    if (!s || !cam || !o || (!rgb && !p6)) return set_error(RT_ERR_ARG, "rt_render_device: null argument");
    if (o->spp < 1) return set_error(RT_ERR_ARG, "spp must be >= 1");
    if ((hit_idx == nullptr) != (hit_t == nullptr)) return set_error(RT_ERR_ARG, "hit_idx and hit_t go together");
    const int W = cam->pixel_width, H = cam->pixel_height;
    if (W < 1 || H < 1) return set_error(RT_ERR_ARG, "camera has no pixels");
    const int rows = rt_shard_rows(H, o->band_rows, o->band_index, o->band_count);
    if (rows < 0) return set_error(RT_ERR_ARG, "bad band sharding parameters");
    DeviceGuard g(s->device);
    int rc = prepare_jitter(s, o);
    if (rc != RT_OK) return rc;
    if (rows == 0) return RT_OK;

    RenderParams P;
    std::memset(&P, 0, sizeof(P));
    P.sc.inode = static_cast<const float4*>(s->inode.p);
    P.sc.wnode = static_cast<const float4*>(s->wnode.p);
    P.sc.fnode = static_cast<const float*>(s->fnode.p);
    P.sc.f_log2 = s->fnode.p ? s->f_log2 : 2;
    P.sc.qent = static_cast<const uint4*>(s->qent.p);
    P.sc.qhdr = static_cast<const float4*>(s->qhdr.p);
    P.sc.wide = s->wide && !(o->flags & RT_FLAG_BINARY) ? 1 : 0;
    P.sc.lane_stack = s->lane_stack ? 1 : 0;
    P.sc.lane_wide = s->lane_wide ? 1 : 0;
    P.sc.ibox = static_cast<const float4*>(s->ibox.p);
    P.sc.rootb = static_cast<const float4*>(s->ibox.p) + s->ibox.n / sizeof(float4) - 2;
    P.sc.leaf = static_cast<const float4*>(s->leaf.p);
    P.sc.tnorm = static_cast<const float4*>(s->tnorm.p);
    P.sc.objids = static_cast<const int32_t*>(s->objids.p);
    P.sc.mats = static_cast<const DevMaterial*>(s->mats.p);
    P.sc.lights = static_cast<const DevLight*>(s->lights.p);
    P.sc.num_tris = int32_t(s->P);
    P.sc.num_mats = s->nmat;
    P.sc.num_lights = s->nlights;
    P.sc.root_ref = s->root_ref;
    std::memcpy(P.sc.root_box, s->root_box, sizeof(P.sc.root_box));
    P.sc.cut = static_cast<const float*>(s->cut.p);
    P.sc.cut2 = static_cast<const float*>(s->cut2.p);
    P.sc.cut_sub_log2 = s->cut2.p ? s->cut_sub_log2 : 0;
    P.sc.tri = static_cast<const float4*>(s->tri.p);
    P.sc.fault = static_cast<uint32_t*>(s->fault.p);
    // RT_TUNE_CULL_COVERAGE: tests force the cut pass on (>= 1: always, untested candidates none)
    const double max_cov = rt::tuning(RT_TUNE_CULL_COVERAGE, 0.3);
    P.sc.ncut = s->ncut > 0 && root_box_coverage(s->root_box, cam) <= max_cov ? s->ncut : 0;
    P.cut_force = max_cov >= 1.0 ? 1 : 0;
    std::memcpy(P.sc.bmax, s->bmax, sizeof(P.sc.bmax));
    P.cam_center = f3{cam->center.x, cam->center.y, cam->center.z};
    P.cam_p00 = f3{cam->pixel00_loc.x, cam->pixel00_loc.y, cam->pixel00_loc.z};
    P.cam_du = f3{cam->pixel_delta_u.x, cam->pixel_delta_u.y, cam->pixel_delta_u.z};
    P.cam_dv = f3{cam->pixel_delta_v.x, cam->pixel_delta_v.y, cam->pixel_delta_v.z};
    P.W = W;
    P.H = H;
    P.spp = o->spp;
    P.max_depth = o->max_depth;
    P.diffuse_bounce = o->diffuse_bounce ? 1 : 0;
    P.miss = f3{o->miss_color.x, o->miss_color.y, o->miss_color.z};
    P.jitter = static_cast<const float*>(s->jitter.p);
    P.band_rows = o->band_count <= 1 ? H : o->band_rows;
    P.band_index = o->band_count <= 1 ? 0 : o->band_index;
    P.band_count = o->band_count <= 1 ? 1 : o->band_count;
    P.rows = rows;
    P.rgb = rgb;
    P.hit_idx = hit_idx;
    P.hit_t = hit_t;
    P.p6 = p6;
    P.ray_count = t_ray_count;
    {
        const f3 mp = miss_pixel_value(o);
        P.miss_p6[0] = rtp::p6_default_sample(mp.x);
        P.miss_p6[1] = rtp::p6_default_sample(mp.y);
        P.miss_p6[2] = rtp::p6_default_sample(mp.z);
        P.miss_p6[3] = 0;
    }
    const bool samples = o->kernel != RT_KERNEL_WAVE_PIXELS && o->spp <= BLOCK && (o->spp & (o->spp - 1)) == 0;
    // Half waves (32 samples per wave) for the shards of an 8-way split: a shard's kernel is then
    // bound by its longest waves, and halving their rays shortens them (c3 band shards on one
    // GPU, max over the 8: kernel 0.101 -> 0.095 ms, frame 0.122 -> 0.116; at 4 and fewer shards
    // the doubled wave count costs more: N = 4 0.106 -> 0.116, N = 1 0.211 -> 0.373;
    // scripts/half_waves_ab.py).  RT_TUNE_HALF_WAVES = 0/1 overrides.  (Quarter waves,
    // 16 samples, measured slower at N = 8 and were dropped.)
    // The multi-bounce kernels take half waves at any split: a wave's bounce paths end with its
    // longest lane's, and the longest waves bound the kernel (c3b 1.96 vs 2.37 ms per frame).
    // (With the frustum traversal, profiles/r04/exp/half_waves_ab_c3.log: N = 8 max kernel 0.0758
    // vs 0.0867 ms, N = 4 0.0831 vs 0.0857, N = 2 0.140 vs 0.097: half waves from 4 shards.)
    int half = o->band_count >= 4 || o->max_depth > 1 ? 1 : 0;
    if (const double h = rt::tuning(RT_TUNE_HALF_WAVES, -1.0); h >= 0.0) half = h >= 1.0 ? 1 : 0;
    if (!samples || o->spp > (64 >> half)) half = 0;
    P.half_waves = half;
    // One light and a tree whose DFS fits the per-lane LDS stacks: the bounce kernels that hold
    // only the paired loop (paired_bounces), fewer live registers than the kernels that also
    // carry the unpaired one.  RT_PAIRED_ONLY=0 turns them off (A/B: the unpaired loop on half waves).
    P.paired_only = half && o->max_depth > 1 && s->nlights == 1 && !s->deep && o->kernel != RT_KERNEL_LANE &&
                            (P.sc.wide ? s->lane_wide : s->lane_stack)
                        ? 1
                        : 0;
    P.paired_only = P.paired_only && rt::tuning(RT_TUNE_PAIRED_ONLY, 1.0) != 0.0;
    int ppb = samples ? (BLOCK >> half) / o->spp : BLOCK;  // pixels per block
    int tw = 1;
    while (tw * tw < ppb) tw <<= 1;                // square-ish power-of-two tile
    int th = ppb / tw;
    P.tile_w = tw;
    P.tile_h = th;
    P.tile_w_log2 = __builtin_ctz(unsigned(tw));
    P.spp_log2 = samples ? __builtin_ctz(unsigned(o->spp)) : 0;
    P.tiles_x = (W + tw - 1) / tw;
    const int tiles_y = (rows + th - 1) / th;
    P.tiles_total = P.tiles_x * tiles_y;
    P.lane_samples = samples ? 1 : 0;
    P.tile_order = o->tile_order == RT_TILES_AUTO ? RT_TILES_ROWS : o->tile_order;
    P.cull = (o->flags & RT_FLAG_NO_CULL) ? 0 : 1;
    if (!P.cull) P.sc.ncut = 0;  // the render kernel reads the cut pass's lists only when it ran
    P.miss_pixel = miss_pixel_value(o);
    P.nqueues = P.tile_order == RT_TILES_LINEAR ? 1 : 8;
    // a list holds at most tiles_x * ceil(tiles_y / 8) tiles (RT_TILES_ROWS) or ceil(tiles / 8)
    // (RT_TILES_XCD_CHUNK): tiles_x * ceil(tiles_y / 8) bounds both
    P.queue_cap = P.tile_order == RT_TILES_LINEAR ? P.tiles_total : P.tiles_x * ((tiles_y + 7) / 8);
    // Heavy-first dispatch needs the cut pass (it builds the heavy lists) and the 8 lists.
    // RT_TUNE_HEAVY_FRAC (speed experiments): a tile is in heavy class c when one of its waves took
    // at least 2^(2-c) times this fraction of the latest finished frame's render kernel
    // (0: off).
    // c3 (frustum traversal, profiles/r04/exp/heavy_frac_ab_c3*.log): 0.05 0.153, 0.06 0.149,
    // 0.08 0.148, 0.10 0.147, 0.12 0.150, 0.18 0.151, 0.25 0.158 ms, off 0.187
    const double heavy_frac = rt::tuning(RT_TUNE_HEAVY_FRAC, 0.10);
    const int mode = o->kernel == RT_KERNEL_LANE ? RT_KERNEL_LANE : RT_KERNEL_WAVE;
    const bool costs = P.cull && P.sc.ncut > 0 && P.nqueues == 8 && heavy_frac > 0.0;
    // RT_TUNE_HEAVY_CAP: entries per (class, list) (speed experiments)
    const int heavy_cap = int(std::clamp(rt::tuning(RT_TUNE_HEAVY_CAP, 512.0), 1.0, 1e9));
    P.heavy_cap = costs ? std::min(P.queue_cap, heavy_cap) : 0;
    // kSets counter sets (8 live lists, one spare, 8 heavy lists each) at fixed offsets, then
    // kSets x (live lists | cut survivor lists | heavy lists) sized for this geometry; rotating by frame
    constexpr size_t kCounterBytes = COUNTER_SET_U32 * sizeof(uint32_t);
    const size_t list_bytes = size_t(P.nqueues) * size_t(P.queue_cap) * sizeof(int32_t);
    const size_t cut_bytes = P.sc.ncut > 0 ? list_bytes : 0;
    const size_t heavy_bytes = size_t(8 * NCLASS) * size_t(P.heavy_cap) * sizeof(int32_t);
    const size_t set_bytes = list_bytes + cut_bytes + heavy_bytes;
    const size_t work_bytes = rt_scene::kSets * (kCounterBytes + set_bytes);
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint64_t k = s->launches;
    auto ev1_of = [&](uint64_t f) { return s->ev1[f % rt_scene::kRing]; };
    // The latest finished frame's render-kernel time sets the heavy threshold (non-blocking
    // queries; none finished yet: the previous estimate, or no heavy lists).  The frames are
    // scanned forward from the oldest one not yet seen finished (amortised one query per
    // frame), so a caller that submits many frames ahead of the GPU still gets an estimate once
    // its first frames finish (a look-back over the last three frames found none: all in flight).
    // frame B of a pair whose frame A waits in ps: its tiles and cut must be A's
    bool pair_b = ps && ps->phase == 1 && ps->deferred;
    if (pair_b) {
        const RenderParams& A = ps->A;
        const bool same = A.tiles_total == P.tiles_total && A.tiles_x == P.tiles_x && A.W == P.W && A.rows == P.rows &&
                          A.spp == P.spp && A.half_waves == P.half_waves && A.sc.ncut == P.sc.ncut && A.cull == P.cull &&
                          A.heavy_cap == P.heavy_cap && A.queue_cap == P.queue_cap && A.nqueues == P.nqueues &&
                          A.max_depth == P.max_depth && A.paired_only == P.paired_only && A.band_index == P.band_index &&
                          A.band_count == P.band_count && ps->stream == static_cast<hipStream_t>(stream);
        if (!same) {
            pair_b = false;
            if ((rc = flush_pair_a(s, *ps)) != RT_OK) return rc;
        }
    }
    bool cost_reset = false;
    if (costs) {
        uint64_t f = std::max<uint64_t>(s->est_next, k >= uint64_t(rt_scene::kRing) ? k - (rt_scene::kRing - 1) : 0);
        int64_t last = -1;
        const uint64_t f_end = ps && ps->deferred ? k - 1 : k;  // frame A's events are not recorded yet
        for (; f < f_end; ++f) {
            if (hipEventQuery(s->ev1[f % rt_scene::kRing]) != hipSuccess) break;
            last = int64_t(f);
        }
        s->est_next = f;
        if (last >= 0) {
            const int fl = int(uint64_t(last) % rt_scene::kRing);
            // the render kernel's time, or the frame period when shorter (overlapping frames:
            // RT_FLAG_OVERLAP starts a kernel while the previous one still runs); a pair
            // kernel's time per frame
            float ms = 0.f, period = 0.f;
            if (s->timed[fl] && hipEventElapsedTime(&ms, s->evm[fl], s->ev1[fl]) == hipSuccess) {
                const int f0 = int(uint64_t(last - 1) % rt_scene::kRing);
                if (s->span[fl] > 1) ms /= float(s->span[fl]);
                else if (last >= 1 && s->span[f0] == 1 &&
                         hipEventElapsedTime(&period, s->ev1[f0], s->ev1[fl]) == hipSuccess && period > 0.f)
                    ms = std::min(ms, period);
                s->kernel_ms_est = ms;
            }
        }
        (void)hipGetLastError();  // a not-ready query is not an error of this call
        // 10 ns ticks (wall_clock64 runs at 100 MHz)
        for (int c = 0; c < NCLASS; ++c) {
            const double ticks = std::ldexp(heavy_frac, 2 - c) * double(s->kernel_ms_est) * 1e5;
            const bool used = c < (o->max_depth == 1 ? NCLASS_D1 : NCLASS);
            P.heavy_ticks[c] = s->kernel_ms_est > 0.f && used ? uint32_t(std::clamp(ticks, 1.0, 65535.0)) : 0xffffffffu;
        }
        // the costs are per tile of this geometry
        const uint64_t key = (uint64_t(uint32_t(P.tiles_total)) * 0x9E3779B97F4A7C15ull) ^
                             (uint64_t(uint32_t(P.tiles_x)) << 40) ^ (uint64_t(uint32_t(W)) << 20) ^
                             uint64_t(uint32_t(rows)) ^ (uint64_t(uint32_t(P.band_index)) << 52) ^
                             (uint64_t(uint32_t(P.band_count)) << 58) ^ (uint64_t(uint32_t(P.spp)) << 32);
        const size_t cost_bytes = size_t(P.tiles_total) * 4 * sizeof(uint16_t);
        if (s->cost.n < cost_bytes) {
            if (k > 0) {  // the old buffer may still be written
                HIP_TRY(hipStreamSynchronize(s->prep));
                HIP_TRY(hipEventSynchronize(ev1_of(k - 1)));
            }
            if ((rc = s->cost.alloc(cost_bytes)) != RT_OK) return rc;
            s->cost_key = ~key;
        }
        cost_reset = s->cost_key != key;
        s->cost_key = key;
        P.tile_cost = static_cast<uint16_t*>(s->cost.p);
    }
    s->last_heavy_cap = P.heavy_cap;
    if (s->work.n < work_bytes) {
        if (k > 0) {  // the old buffers may still be read
            HIP_TRY(hipStreamSynchronize(s->prep));
            HIP_TRY(hipEventSynchronize(ev1_of(k - 1)));
        }
        if ((rc = s->work.alloc(work_bytes)) != RT_OK) return rc;
        s->counters_dirty = true;
    }
    // This frame's outputs against the previous frame's: overlapping ranges (a caller reusing
    // one buffer) make the pre-passes, which write the culled tiles' pixels, wait for the
    // previous render kernel; distinct buffers (rt_renderer's frame slots) let them overlap it.
    const size_t npx = size_t(rows) * size_t(W);
    const rt_scene::Range out_now[4] = {
        {uintptr_t(rgb), uintptr_t(rgb) + (rgb ? npx * 3 * sizeof(float) : 0)},
        {uintptr_t(p6), uintptr_t(p6) + (p6 ? npx * 3 : 0)},
        {uintptr_t(hit_idx), uintptr_t(hit_idx) + (hit_idx ? npx * size_t(o->spp) * sizeof(int32_t) : 0)},
        {uintptr_t(hit_t), uintptr_t(hit_t) + (hit_t ? npx * size_t(o->spp) * sizeof(float) : 0)}};
    // a new list layout may place this frame's lists over the previous frame's: serialise too
    bool overlap = s->set_bytes != set_bytes || cost_reset;
    for (const auto& a : out_now)
        for (const auto& b : s->prev_out)
            overlap = overlap || (a.lo < a.hi && b.lo < b.hi && a.lo < b.hi && b.lo < a.hi);
    if (pair_b && overlap) {  // frame B writes over frame A: A renders first, on its own
        pair_b = false;
        if ((rc = flush_pair_a(s, *ps)) != RT_OK) return rc;
    }
    const size_t big_bytes = size_t(std::max(0.0, rt::tuning(RT_TUNE_BIG_SCENE_BYTES, double(kBigSceneBytes))));
    const bool ovl = s->caller_ordered && rt::tuning(RT_TUNE_OVERLAP_FRAMES, 0.0) > 0.5;
    // frame A of a pair: its launch waits for frame B's call (PairStage)
    const bool pair_a = ps && ps->phase == 0 && rt::tuning(RT_TUNE_PAIR_FRAMES, 1.0) > 0.5 && !ovl &&
                        pair_kernel_fits(P, samples, !s->deep && mode == RT_KERNEL_WAVE && P.sc.wide != 0,
                                         s->bytes > big_bytes);
    // the previous frame of this scene ran on another stream: wait for it.  (Letting two frames'
    // render kernels overlap on two streams, the next filling the CUs the last waves of the
    // previous one leave idle, measured slower for rt_renderer: 0.257 vs 0.246 ms per c3 frame.)
    if (k > 0 && st != s->last_stream) {
        HIP_TRY(hipStreamWaitEvent(st, ev1_of(k - 1), 0));
        // (overlapping frames, RT_TUNE_OVERLAP_FRAMES: the one before may finish last)
        if (k > 1) HIP_TRY(hipStreamWaitEvent(st, ev1_of(k - 2), 0));
    }
    s->last_stream = st;
    const int set = int(k % rt_scene::kSets), nset = int((k + 2) % rt_scene::kSets);
    char* base = static_cast<char*>(s->work.p);
    char* lists = base + rt_scene::kSets * kCounterBytes + set * set_bytes;
    P.live_count = reinterpret_cast<uint32_t*>(base + set * kCounterBytes);
    P.next_count = reinterpret_cast<uint32_t*>(base + nset * kCounterBytes);
    s->last_tiles_total = P.tiles_total;
    P.live_tiles = reinterpret_cast<int32_t*>(lists);
    P.cut_tiles = reinterpret_cast<int32_t*>(lists + list_bytes);
    P.heavy_tiles = reinterpret_cast<int32_t*>(lists + list_bytes + cut_bytes);
    const int slot = int(k % rt_scene::kRing);
    // From the cull launch on, a failure leaves the counter sets unknown (counters_dirty).
    auto frame = [&]() -> int {
        hipStream_t pp = s->prep;
        P.drain_tag = uint32_t(k + 1);
        // set k was last read by frame k-6, set k+2 (zeroed by this cull pass) by frame k-4: a
        // frame waits for frame k-2 (the render kernel before the one its pre-passes overlap).
        // Frame A of a pair, k, waits for frame k-3 (the pair before the one running: frames
        // up to k-3 used the sets the pair reads and zeroes) and covers frame B: the pair's
        // pre-passes are launched together, after B's call has set B up.
        if (pair_a) {
            if (k >= 3) HIP_TRY(hipStreamWaitEvent(pp, ev1_of(k - 3), 0));
        } else if (!pair_b && k >= 2) {
            HIP_TRY(hipStreamWaitEvent(pp, ev1_of(k - 2), 0));
        }
        if (k >= 1 && overlap) HIP_TRY(hipStreamWaitEvent(pp, ev1_of(k - 1), 0));
        // the pre-pass gate: frame k-1's render kernel opens it when its first queue drains
        if (k >= 1 && s->drain_frame == k - 1)
            HIP_TRY(hipStreamWaitValue32(pp, s->drain, uint32_t(k), hipStreamWaitValueGte, 0xFFFFFFFFu));
        if (!s->caller_ordered) {  // stream order for the caller's buffers (see rt_scene::evq)
            HIP_TRY(hipEventRecord(s->evq[slot], st));
            HIP_TRY(hipStreamWaitEvent(pp, s->evq[slot], 0));
        }
        if (s->counters_dirty) {
            HIP_TRY(hipMemsetAsync(base, 0, rt_scene::kSets * kCounterBytes, pp));
            s->counters_dirty = false;
        }
        if (cost_reset) HIP_TRY(hipMemsetAsync(s->cost.p, 0, s->cost.n, pp));  // no heavy tiles yet
        // frame A of a pair: its pre-passes go out with frame B's (pair_b below, or flush_pair_a)
        if (pair_b) {
            // both frames' passes in one cull and one cut launch (the same cut: the pair's tile
            // geometry check); frame A's events bracket them, frame B's follow
            const int slot_a = int(ps->kA % rt_scene::kRing);
            PairParams PP;
            PP.f[0] = ps->A;
            PP.f[1] = P;
            // (frame B's pdone is the last launch's own end event: the render stream waits for it)
            const bool cut = P.cull && P.sc.ncut > 0;
            HIP_TRY(hipEventRecord(s->ev0[slot], pp));  // both frames' pre-pass times span the pair's
            hipExtLaunchKernelGGL(tile_cull_pair_kernel,
                                  dim3((ps->A.tiles_total + BLOCK - 1) / BLOCK + (P.tiles_total + BLOCK - 1) / BLOCK),
                                  dim3(BLOCK), 0, pp, s->ev0[slot_a], cut ? nullptr : s->pdone[slot], 0, PP);
            HIP_TRY(hipGetLastError());
            if (cut) {
                // 32 waves per CU (the cut kernel's occupancy): the pair's cut mostly runs after
                // the previous pair kernel has left the GPU, latency-bound per unit
                hipExtLaunchKernelGGL(tile_cut_pair_kernel, dim3(8 * s->cus), dim3(BLOCK), 0, pp, nullptr,
                                      s->pdone[slot], 0, PP);
                HIP_TRY(hipGetLastError());
            }
            HIP_TRY(hipEventRecord(s->pdone[slot_a], pp));
        } else if (!pair_a) {
            if ((rc = launch_prepasses(s, P, slot)) != RT_OK) return rc;
        }
        // RT_TUNE_OVERLAP_FRAMES: the render kernel on one of the scene's two render streams (the
        // caller orders its buffers itself; its stream then waits for the kernel), else on the
        // caller's stream
        const hipStream_t rs = ovl ? s->rstream[k & 1] : st;
        // (frame A of a pair: frame B's pdone, later on the same prep stream, covers both)
        if (!pair_a) HIP_TRY(hipStreamWaitEvent(rs, s->pdone[slot], 0));
        const bool qr = P.sc.qent != nullptr && P.sc.f_log2 > 2;
        // RT_TUNE_KERNEL_TIMING_EVERY: the caller-ordered (rt_renderer) frames record the render
        // kernel's start event in one frame of this many (direct calls: every frame); a pair
        // kernel's start is frame A's (frame B's slot is never timed)
        const uint64_t every = uint64_t(std::clamp(rt::tuning(RT_TUNE_KERNEL_TIMING_EVERY, 4.0), 1.0, 256.0));
        s->timed[slot] = !pair_b && (!s->caller_ordered || k % every == 0 || (pair_a && (k + 1) % every == 0));
        s->span[slot] = pair_a || pair_b ? 2 : 1;
        const Launch L{rs, s->timed[slot] ? s->evm[slot] : nullptr, s->ev1[slot], s->cus, s->bytes > big_bytes, qr,
                       &s->last_kernel};
        // RT_TUNE_PREPASS_GATE f in (0, 1]: this kernel opens the next frame's pre-passes when
        // its first queue has handed out the fraction f of its items (0.5 default; 1: drained);
        // 0 they start once the frame before this one has finished
        // (0.5: c3 0.1557-0.157 ms per delivered frame vs 0.1587-0.1593 at 1.0, the pre-passes
        // then finishing well before this kernel does; profiles/r05/exp/prepass_gate_frac_c3.log)
        // The gate word takes plain stores, so it needs one writer kernel at a time: with
        // overlapping frames (ovl: two render streams) a late store of frame k-2's kernel could
        // overwrite frame k-1's tag after frame k had started waiting for it, so ovl runs ungated.
        const double gate_f = ovl ? 0.0 : rt::tuning(RT_TUNE_PREPASS_GATE, 0.5);
        const bool gate = gate_f > 0.0;
        P.drained = gate ? s->drain : nullptr;
        P.drain_tag = uint32_t(k + 1);
        P.gate_q8 = int(std::clamp(gate_f, 0.0, 1.0) * 256.0 + 0.5);
        if (pair_a) {  // held for frame B's call
            ps->A = P;
            ps->LA = L;
            ps->kA = k;
            ps->stream = st;
            ps->deferred = true;
            return RT_OK;
        }
        if (pair_b) {
            // one grid over both frames: frame A's events bracket it (its start event when A is a
            // timed frame), frame B's end event follows; frame B's parameters carry the gate
            const int slot_a = int(ps->kA % rt_scene::kRing);
            RenderParams A = ps->A;
            A.drained = nullptr;
            const Launch LP{rs, s->timed[slot_a] ? s->evm[slot_a] : nullptr, s->ev1[slot_a], s->cus, false, false,
                            &s->last_kernel};
            ps->deferred = false;
            launch_pair(A, P, LP);
            HIP_TRY(hipGetLastError());
            HIP_TRY(hipEventRecord(s->ev1[slot], rs));
            if (gate) s->drain_frame = k;
            return RT_OK;
        }
        if (s->deep) launch<MODE_DEEP>(P, samples, L);
        else if (mode == RT_KERNEL_LANE) launch<RT_KERNEL_LANE>(P, samples, L);
        else if (P.sc.wide) launch<RT_KERNEL_WAVE | MODE_WIDE>(P, samples, L);
        else launch<RT_KERNEL_WAVE>(P, samples, L);
        HIP_TRY(hipGetLastError());
        if (ovl) HIP_TRY(hipStreamWaitEvent(st, s->ev1[slot], 0));
        if (gate) s->drain_frame = k;
        return RT_OK;
    };
    std::copy(std::begin(out_now), std::end(out_now), std::begin(s->prev_out));
    s->set_bytes = set_bytes;
    rc = frame();
    s->launches++;  // the events of this slot belong to this frame even when it failed
    if (rc != RT_OK) s->counters_dirty = true;
    return rc;
}
}  // namespace

void rt::scene_set_caller_ordered(rt_scene* s, bool on) {
    if (s) s->caller_ordered = on;
}

void rt::scene_frame_events(const rt_scene* s, hipEvent_t* first, hipEvent_t* last, int back) {
    hipEvent_t a = nullptr, b = nullptr;
    if (s && s->launches > uint64_t(back)) {
        const int slot = int((s->launches - 1 - uint64_t(back)) % rt_scene::kRing);
        a = s->ev0[slot];
        b = s->ev1[slot];
    }
    if (first) *first = a;
    if (last) *last = b;
}

namespace {
// what: 0 render kernel (evm -> ev1), 1 pre-passes (ev0 -> pdone), 2 both (the frame's device
// work: its pre-passes overlap the previous frame's render kernel, so the span ev0 -> ev1 would
// include the wait for it)
int event_times(const rt_scene* s, int what, float* ms_out, int max, int* n_out) {
    if (!s || max < 0 || (max > 0 && !ms_out)) return set_error(RT_ERR_ARG, "kernel times: bad args");
    DeviceGuard g(s->device);
    const uint64_t have = std::min<uint64_t>(s->launches, uint64_t(rt_scene::kRing));
    // the most recent frames with a kernel start event (all of them unless the renderer samples,
    // RT_TUNE_KERNEL_TIMING_EVERY), at most max, oldest first; pre-pass times need no sampling
    std::vector<int> slots;
    for (uint64_t b = 1; b <= have && (int)slots.size() < max; ++b) {
        const int slot = int((s->launches - b) % rt_scene::kRing);
        if (what == 1 || s->timed[slot]) slots.push_back(slot);
    }
    const int n = (int)slots.size();
    for (int k = 0; k < n; ++k) {
        const int slot = slots[size_t(n - 1 - k)];
        HIP_TRY(hipEventSynchronize(s->ev1[slot]));
        float kern = 0.f, prep = 0.f;
        if (what != 1) HIP_TRY(hipEventElapsedTime(&kern, s->evm[slot], s->ev1[slot]));
        if (what != 0) HIP_TRY(hipEventElapsedTime(&prep, s->ev0[slot], s->pdone[slot]));
        ms_out[k] = kern + prep;
    }
    if (n_out) *n_out = n;
    return RT_OK;
}
}  // namespace

namespace {
int live_tiles(const rt_scene* s, int64_t* live, int64_t* heavy, int64_t* total) {
    if (!s || !live || !total) return set_error(RT_ERR_ARG, "rt_live_tiles: null argument");
    *live = 0;
    *total = s->last_tiles_total;
    if (!s->work.p || s->launches == 0) return RT_OK;
    DeviceGuard g(s->device);
    const int slot = int((s->launches - 1) % rt_scene::kRing);
    HIP_TRY(hipEventSynchronize(s->ev1[slot]));
    uint32_t c[COUNTER_SET_U32];
    // the last frame's counter set (the sets sit at the start of the work buffer)
    const size_t counter_bytes = COUNTER_SET_U32 * sizeof(uint32_t);
    HIP_TRY(hipMemcpy(c, static_cast<const char*>(s->work.p) + ((s->launches - 1) % rt_scene::kSets) * counter_bytes, sizeof(c),
                      hipMemcpyDeviceToHost));
    for (int k = 0; k < 8; ++k) *live += c[k * COUNTER_STRIDE];
    if (heavy) {
        *heavy = 0;
        if (s->last_heavy_cap > 0)
            for (int k = 0; k < 8 * NCLASS; ++k)
                *heavy += std::min<int64_t>(c[(HEAVY_SLOT0 + k) * COUNTER_STRIDE], s->last_heavy_cap);
    }
    return RT_OK;
}
}  // namespace

extern "C" int rt_live_tiles(const rt_scene* s, int64_t* live, int64_t* total) {
    return live_tiles(s, live, nullptr, total);
}

extern "C" const char* rt_scene_kernel_name(const rt_scene* s) {
    return (s && s->last_kernel) ? s->last_kernel : "";
}

extern "C" int rt_heavy_tiles(const rt_scene* s, int64_t* heavy) {
    if (!heavy) return set_error(RT_ERR_ARG, "rt_heavy_tiles: null argument");
    int64_t live = 0, total = 0;
    *heavy = 0;
    return live_tiles(s, &live, heavy, &total);
}

#ifdef RT_STATS
extern "C" int rt_debug_stats(unsigned long long* out, int reset) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rt_stats), sizeof(g_rt_stats)));
    if (reset) {
        unsigned long long z[24] = {};
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_rt_stats), z, sizeof(z)));
    }
    return RT_OK;
}
#endif

#ifdef RT_WAVE_TIMES
extern "C" int rt_debug_wave_meta_set(void* dev_ptr) {
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_wave_meta), &dev_ptr, sizeof(dev_ptr)));
    return RT_OK;
}
extern "C" int rt_debug_wave_phase_set(void* dev_ptr) {
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_wave_phase), &dev_ptr, sizeof(dev_ptr)));
    return RT_OK;
}
#ifdef RT_LANE_ITERS
extern "C" int rt_debug_lane_iters_set(void* iters_ptr, void* acc_ptr) {
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_lane_iters), &iters_ptr, sizeof(iters_ptr)));
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_lane_acc), &acc_ptr, sizeof(acc_ptr)));
    return RT_OK;
}
#endif
extern "C" int rt_debug_wave_times_set(void* dev_ptr, void* cut_counts_ptr) {
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_wave_times), &dev_ptr, sizeof(dev_ptr)));
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_cut_counts), &cut_counts_ptr, sizeof(cut_counts_ptr)));
    return RT_OK;
}
#endif
#ifdef RT_FRAME_SPAN
extern "C" int rt_debug_frame_span_set(void* dev_ptr) {
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_frame_span), &dev_ptr, sizeof(dev_ptr)));
    return RT_OK;
}
#endif

extern "C" int rt_kernel_times(const rt_scene* s, float* ms_out, int max, int* n_out) {
    return event_times(s, 0, ms_out, max, n_out);
}

extern "C" int rt_frame_times(const rt_scene* s, float* ms_out, int max, int* n_out) {
    return event_times(s, 2, ms_out, max, n_out);
}

extern "C" int rt_prepass_times(const rt_scene* s, float* ms_out, int max, int* n_out) {
    return event_times(s, 1, ms_out, max, n_out);
}

extern "C" int rt_render(rt_scene* s, const rt_camera* cam, const rt_render_opts* o, float* rgb_host,
                         int32_t* hit_idx_host, float* hit_t_host) {
    if (!s || !cam || !o || !rgb_host) return set_error(RT_ERR_ARG, "rt_render: null argument");
    if ((hit_idx_host == nullptr) != (hit_t_host == nullptr)) return set_error(RT_ERR_ARG, "hit_idx and hit_t go together");
    const int rows = rt_shard_rows(cam->pixel_height, o->band_rows, o->band_index, o->band_count);
    if (rows < 0) return set_error(RT_ERR_ARG, "bad band sharding parameters");
    if (o->spp < 1) return set_error(RT_ERR_ARG, "spp must be >= 1");
    DeviceGuard g(s->device);
    const size_t npx = size_t(rows) * size_t(std::max(cam->pixel_width, 0));
    DevBuf rgb, hi, ht;
    int rc;
    if ((rc = rgb.alloc(npx * 3 * sizeof(float))) != RT_OK) return rc;
    if (hit_idx_host) {
        if ((rc = hi.alloc(npx * size_t(o->spp) * sizeof(int32_t))) != RT_OK) return rc;
        if ((rc = ht.alloc(npx * size_t(o->spp) * sizeof(float))) != RT_OK) return rc;
    }
    // the fault word belongs to this frame: earlier frames finish first, then it is cleared
    // (rt_scene_faults still sees what this frame raised)
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemset(s->fault.p, 0, sizeof(uint32_t)));
    rc = rt_render_device(s, cam, o, static_cast<float*>(rgb.p), static_cast<int32_t*>(hi.p),
                          static_cast<float*>(ht.p), nullptr);
    if (rc != RT_OK) return rc;
    HIP_TRY(hipDeviceSynchronize());
    if (npx) HIP_TRY(hipMemcpy(rgb_host, rgb.p, npx * 3 * sizeof(float), hipMemcpyDeviceToHost));
    if (hit_idx_host && npx) {
        HIP_TRY(hipMemcpy(hit_idx_host, hi.p, npx * size_t(o->spp) * sizeof(int32_t), hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(hit_t_host, ht.p, npx * size_t(o->spp) * sizeof(float), hipMemcpyDeviceToHost));
    }
    // a device-side guard fired (the frame's answers are poisoned where it did): loud, not silent
    uint32_t fault = 0;
    HIP_TRY(hipMemcpy(&fault, s->fault.p, sizeof(fault), hipMemcpyDeviceToHost));
    if (fault & RT_FAULT_FRUSTUM_STACK) return set_error(RT_ERR_INTERNAL, "frustum traversal stack overflow");
    return RT_OK;
}

// Rays one frame traces, by the oracle's classes (orc_stats.rays: camera, shadow, bounce).
// Camera rays are W*rows*spp whenever max_depth > 0 (TraceRayIterative traces every sample);
// shadow and bounce rays are counted on the device by one LANE-kernel render of the frame
// (wave-aggregated atomics; the frame itself is discarded).  Synchronous.
extern "C" int rt_count_rays(rt_scene* s, const rt_camera* cam, const rt_render_opts* o, uint64_t* counts) {
    if (!counts) return set_error(RT_ERR_ARG, "rt_count_rays: null argument");
    uint64_t c4[4];
    const int rc = rt_count_rays_ex(s, cam, o, c4);
    if (rc == RT_OK) std::memcpy(counts, c4, 3 * sizeof(uint64_t));
    return rc;
}

extern "C" int rt_count_rays_ex(rt_scene* s, const rt_camera* cam, const rt_render_opts* o, uint64_t* counts) {
    if (!s || !cam || !o || !counts) return set_error(RT_ERR_ARG, "rt_count_rays: null argument");
    const int rows = rt_shard_rows(cam->pixel_height, o->band_rows, o->band_index, o->band_count);
    if (rows < 0) return set_error(RT_ERR_ARG, "bad band sharding parameters");
    if (o->spp < 1) return set_error(RT_ERR_ARG, "spp must be >= 1");
    if (cam->pixel_width < 1 || cam->pixel_height < 1) return set_error(RT_ERR_ARG, "camera has no pixels");
    DeviceGuard g(s->device);
    const size_t npx = size_t(rows) * size_t(cam->pixel_width);
    DevBuf rgb, cnt;
    int rc;
    if ((rc = rgb.alloc(std::max<size_t>(npx * 3 * sizeof(float), 4))) != RT_OK) return rc;
    if ((rc = cnt.alloc(4 * sizeof(unsigned long long))) != RT_OK) return rc;
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemset(cnt.p, 0, 4 * sizeof(unsigned long long)));
    rt_render_opts lo = *o;
    lo.kernel = RT_KERNEL_LANE;  // deep trees take the DEEP kernels, which count too
    t_ray_count = static_cast<unsigned long long*>(cnt.p);
    rc = rt_render_device(s, cam, &lo, static_cast<float*>(rgb.p), nullptr, nullptr, nullptr);
    t_ray_count = nullptr;
    if (rc != RT_OK) return rc;
    HIP_TRY(hipDeviceSynchronize());
    unsigned long long h[4] = {0, 0, 0, 0};
    HIP_TRY(hipMemcpy(h, cnt.p, sizeof(h), hipMemcpyDeviceToHost));
    counts[0] = o->max_depth > 0 ? uint64_t(npx) * uint64_t(o->spp) : 0;
    counts[1] = h[1];
    counts[2] = h[2];
    counts[3] = h[3];
    return RT_OK;
}

extern "C" int rt_render_reference(size_t P, int W, int H, const rt_camera* cam, rt_vec3 miss, int max_depth,
                                   int spp, const rt_bvh_node* nodes, const rt_aabb* aabbs,
                                   const rt_triangle* tris, const int32_t* objids, const rt_material* mats,
                                   int nmat, const rt_light* lights, int nlights, int diffuse_bounce,
                                   rt_vec3* output) {
    // query.cu:131-133: a null scene/output array is a silent no-op in the reference CPU
    // branch; here it is reported.
    if (!cam || !output) return set_error(RT_ERR_ARG, "rt_render_reference: null argument");
    if (W != cam->pixel_width || H != cam->pixel_height)
        return set_error(RT_ERR_ARG, "W/H must match the camera's pixel dimensions");
    rt_scene* s = nullptr;
    int rc = rt_scene_create(0, P, nodes, aabbs, tris, objids, mats, nmat, lights, nlights, &s);
    if (rc != RT_OK) return rc;
    rt_render_opts o;
    rt_render_opts_default(&o);
    o.max_depth = max_depth;
    o.spp = spp;
    o.diffuse_bounce = diffuse_bounce;
    o.miss_color = miss;
    rc = rt_render(s, cam, &o, reinterpret_cast<float*>(output), nullptr, nullptr);
    rt_scene_destroy(s);
    return rc;
}

extern "C" int rt_render_hw1(int device, const rt_vec3* pos, const rt_vec3* nrm, const uint32_t* idx, size_t P,
                             const rt_camera* cam, rt_vec3 lpos, rt_vec3 lcol, int spp, const float* jitter,
                             float* rgb_host, int32_t* hit_idx_host, float* hit_t_host) {
    return rt_render_hw1_ex(device, pos, nrm, idx, P, cam, lpos, lcol, spp, jitter, 0, rgb_host, hit_idx_host,
                            hit_t_host, nullptr);
}

// ---- HW1 resident scene (the C2 configuration's device path) ---------------------------
// The mesh packed once (v0, e1, e2 as ray_intersection computes them, the three normals per
// triangle), the binning buffers kept across frames.  A frame is four launches on the caller's
// stream (counts zeroed, rect + count, scan, fill, render) and no host synchronisation: the
// bin list's capacity is checked on the device (a tile whose list would not fit takes the
// brute-force loop), and the host grows it from the latest finished frame's total.
struct rt_hw1_scene {
    int device = 0;
    size_t P = 0;
    DevBuf tri, nrm, rects, bins, list, jitter;
    DevBuf chunks;             // chunk_first (ntiles + 1) | chunk_tile (chunk_cap)
    DevBuf keys;               // per (pixel, sample): the chunked pass's winners, kept at ~0 between frames
    int bins_tiles = -1;       // tiles the bins buffer is laid out for
    size_t keys_n = 0;         // samples the keys buffer holds
    uint32_t list_cap = 0, chunk_cap = 0;
    int jitter_spp = -1;
    std::vector<float> jitter_host;
    static constexpr int kRing = 64;
    hipEvent_t e0[kRing] = {}, e1[kRing] = {};
    uint32_t* total_host = nullptr;  // pinned: the list total of frame f at [f % kRing]
    uint64_t frames = 0;
    hipStream_t last_stream = nullptr;
    const char* last_kernel = "";
    ~rt_hw1_scene() {
        for (int i = 0; i < kRing; ++i) {
            if (e0[i]) (void)hipEventSynchronize(e1[i]);
            if (e0[i]) (void)hipEventDestroy(e0[i]);
            if (e1[i]) (void)hipEventDestroy(e1[i]);
        }
        if (total_host) (void)hipHostFree(total_host);
    }
};

extern "C" int rt_hw1_scene_create(int device, const rt_vec3* pos, const rt_vec3* nrm, const uint32_t* idx, size_t P,
                                   rt_hw1_scene** out) {
    if (!out) return set_error(RT_ERR_ARG, "rt_hw1_scene_create: null out");
    *out = nullptr;
    if (!pos || !nrm || !idx || P == 0)
        return set_error(RT_ERR_ARG, "rt_hw1_scene_create: bad argument (HW1 requires per-vertex normals)");
    if (P > 0x7FFFFFFFull) return set_error(RT_ERR_UNSUPPORTED, "too many triangles");
    int rc = check_device(device);
    if (rc != RT_OK) return rc;
    DeviceGuard g(device);
    std::vector<float4> ht(3 * P), hn(3 * P);
    for (size_t k = 0; k < P; ++k) {
        const rt_vec3 a = pos[idx[3 * k]], b = pos[idx[3 * k + 1]], c = pos[idx[3 * k + 2]];
        // e1 = v1 - v0, e2 = v2 - v0 exactly as ray_intersection computes them (HW1/include/ray.h:71-72)
        ht[3 * k] = make_float4(a.x, a.y, a.z, 0.f);
        ht[3 * k + 1] = make_float4(b.x - a.x, b.y - a.y, b.z - a.z, 0.f);
        ht[3 * k + 2] = make_float4(c.x - a.x, c.y - a.y, c.z - a.z, 0.f);
        for (int j = 0; j < 3; ++j) {
            const rt_vec3 n = nrm[idx[3 * k + j]];
            hn[3 * k + j] = make_float4(n.x, n.y, n.z, 0.f);
        }
    }
    std::unique_ptr<rt_hw1_scene> s(new (std::nothrow) rt_hw1_scene());
    if (!s) return set_error(RT_ERR_NOMEM, "out of memory");
    s->device = device;
    s->P = P;
    if ((rc = s->tri.upload(ht.data(), ht.size() * sizeof(float4))) != RT_OK) return rc;
    if ((rc = s->nrm.upload(hn.data(), hn.size() * sizeof(float4))) != RT_OK) return rc;
    if ((rc = s->rects.alloc(P * sizeof(int4))) != RT_OK) return rc;
    // a first capacity: a few tiles per triangle (grown from the frames' totals)
    s->list_cap = uint32_t(std::min<size_t>(std::max<size_t>(4 * P, size_t(1) << 16), 0x7FFFFFFFull));
    if ((rc = s->list.alloc(size_t(s->list_cap) * sizeof(uint32_t))) != RT_OK) return rc;
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&s->total_host), rt_hw1_scene::kRing * sizeof(uint32_t),
                          hipHostMallocDefault));
    for (int i = 0; i < rt_hw1_scene::kRing; ++i) {
        s->total_host[i] = 0;
        HIP_TRY(hipEventCreate(&s->e0[i]));
        HIP_TRY(hipEventCreate(&s->e1[i]));
    }
    *out = s.release();
    return RT_OK;
}

extern "C" void rt_hw1_scene_destroy(rt_hw1_scene* s) {
    if (!s) return;
    DeviceGuard g(s->device);
    delete s;
}

extern "C" int rt_render_hw1_device(rt_hw1_scene* s, const rt_camera* cam, rt_vec3 lpos, rt_vec3 lcol, int spp,
                                    const float* jitter, int flags, float* rgb_dev, uint8_t* p6_dev,
                                    int32_t* hit_idx_dev, float* hit_t_dev, void* stream) {
    if (!s || !cam || spp < 1) return set_error(RT_ERR_ARG, "rt_render_hw1_device: bad argument");
    if ((hit_idx_dev == nullptr) != (hit_t_dev == nullptr)) return set_error(RT_ERR_ARG, "hit_idx and hit_t go together");
    const int W = cam->pixel_width, H = cam->pixel_height;
    if (W < 1 || H < 1) return set_error(RT_ERR_ARG, "camera has no pixels");
    DeviceGuard g(s->device);
    hipStream_t st = static_cast<hipStream_t>(stream);
    int rc;
    // jitter_samples(spp, 42u) offsets in [0,1) (HW1/include/antialias.h:12-27), or the caller's
    std::vector<float> tab(2 * size_t(spp));
    if (jitter) std::memcpy(tab.data(), jitter, tab.size() * sizeof(float));
    else if ((rc = rt_jittered_samples(spp, 42u, 0, tab.data())) != RT_OK) return rc;
    if (s->jitter_spp != spp || s->jitter_host != tab) {
        if (s->frames > 0) HIP_TRY(hipEventSynchronize(s->e1[(s->frames - 1) % rt_hw1_scene::kRing]));
        if ((rc = s->jitter.upload(tab.data(), tab.size() * sizeof(float))) != RT_OK) return rc;
        s->jitter_spp = spp;
        s->jitter_host = tab;
    }
    const bool brute = (flags & RT_HW1_BRUTE) != 0;
    const int ntiles = ((W + HW1_TW - 1) / HW1_TW) * ((H + HW1_TH - 1) / HW1_TH);
    // the latest finished frame's list total (frames are scanned back to front, non-blocking)
    for (uint64_t b = 1; b <= std::min<uint64_t>(s->frames, 4); ++b) {
        const int sl = int((s->frames - b) % rt_hw1_scene::kRing);
        if (hipEventQuery(s->e1[sl]) != hipSuccess) continue;
        const uint32_t tot = s->total_host[sl];
        if (tot > s->list_cap) {  // grow (the old list may still be read by frames in flight)
            HIP_TRY(hipEventSynchronize(s->e1[(s->frames - 1) % rt_hw1_scene::kRing]));
            s->list_cap = uint32_t(std::min<uint64_t>(uint64_t(tot) + tot / 4 + 1024, 0x7FFFFFFFull));
            if ((rc = s->list.alloc(size_t(s->list_cap) * sizeof(uint32_t))) != RT_OK) return rc;
            s->bins_tiles = -1;  // the chunk table follows the list's capacity
        }
        break;
    }
    (void)hipGetLastError();  // a not-ready query is not an error of this call
    const size_t nsamples = size_t(W) * size_t(H) * size_t(spp);
    if (!brute && (s->bins_tiles != ntiles || s->keys_n != nsamples)) {
        if (s->frames > 0) HIP_TRY(hipEventSynchronize(s->e1[(s->frames - 1) % rt_hw1_scene::kRing]));
        // counts | cursor | offsets (ntiles + 1): counts and cursor zeroed here, then by every
        // frame's resolve pass for the next
        if ((rc = s->bins.alloc(size_t(3 * ntiles + 1) * sizeof(uint32_t))) != RT_OK) return rc;
        HIP_TRY(hipMemset(s->bins.p, 0, size_t(2 * ntiles) * sizeof(uint32_t)));
        // chunks: at most one per HW1_CHUNK listed entries plus one per tile
        s->chunk_cap = uint32_t(std::min<uint64_t>(uint64_t(s->list_cap) / HW1_CHUNK + uint64_t(ntiles) + 1, 0x7FFFFFFFull));
        if ((rc = s->chunks.alloc((size_t(ntiles) + 1 + s->chunk_cap) * sizeof(uint32_t))) != RT_OK) return rc;
        if ((rc = s->keys.alloc(nsamples * sizeof(unsigned long long))) != RT_OK) return rc;
        HIP_TRY(hipMemset(s->keys.p, 0xFF, nsamples * sizeof(unsigned long long)));
        s->bins_tiles = ntiles;
        s->keys_n = nsamples;
    }
    Hw1Params hp;
    hp.tri = static_cast<const float4*>(s->tri.p);
    hp.nrm = static_cast<const float4*>(s->nrm.p);
    hp.num_tris = int32_t(s->P);
    hp.center = f3{cam->center.x, cam->center.y, cam->center.z};
    hp.p00 = f3{cam->pixel00_loc.x, cam->pixel00_loc.y, cam->pixel00_loc.z};
    hp.du = f3{cam->pixel_delta_u.x, cam->pixel_delta_u.y, cam->pixel_delta_u.z};
    hp.dv = f3{cam->pixel_delta_v.x, cam->pixel_delta_v.y, cam->pixel_delta_v.z};
    hp.W = W;
    hp.H = H;
    hp.spp = spp;
    hp.lpos = f3{lpos.x, lpos.y, lpos.z};
    hp.lcol = f3{lcol.x, lcol.y, lcol.z};
    hp.jitter = static_cast<const float*>(s->jitter.p);
    hp.rgb = rgb_dev;
    hp.hit_idx = hit_idx_dev;
    hp.hit_t = hit_t_dev;
    hp.p6 = p6_dev;
    hp.rects = static_cast<const int4*>(s->rects.p);
    hp.bin_count = hp.bin_offset = hp.bin_list = nullptr;
    hp.list_cap = s->list_cap;
    hp.chunk_first = hp.chunk_tile = nullptr;
    hp.chunk_cap = s->chunk_cap;
    hp.keys = static_cast<unsigned long long*>(s->keys.p);
    hp.zero_counts = static_cast<uint32_t*>(s->bins.p);
    hp.ntiles = ntiles;
    const int sl = int(s->frames % rt_hw1_scene::kRing);
    // the scene's buffers are shared by its frames: a frame on another stream waits for the last
    if (s->frames > 0 && st != s->last_stream)
        HIP_TRY(hipStreamWaitEvent(st, s->e1[(s->frames - 1) % rt_hw1_scene::kRing], 0));
    s->last_stream = st;
    HIP_TRY(hipEventRecord(s->e0[sl], st));
    const int blocks = ((W + 15) / 16) * ((H + 15) / 16);
    if (brute) {
        hipLaunchKernelGGL(render_hw1_kernel, dim3(blocks), dim3(BLOCK), 0, st, hp);
        s->last_kernel = "render_hw1_kernel";
    } else {
        // one wave per 64 triangles (a block each): the per-triangle passes spread over every CU
        // (256-thread blocks kept c2's 19,858 triangles on 78 CUs: 30 + 25 us)
        const dim3 tgrid(unsigned((s->P + 63) / 64));
        uint32_t* counts = static_cast<uint32_t*>(s->bins.p);  // zeroed by the previous frame's resolve
        uint32_t* cursor = counts + ntiles;
        uint32_t* offsets = cursor + ntiles;  // ntiles + 1 entries
        uint32_t* cfirst = static_cast<uint32_t*>(s->chunks.p);
        uint32_t* ctile = cfirst + ntiles + 1;
        hipLaunchKernelGGL(hw1_rect_count_kernel, tgrid, dim3(64), 0, st, hp, static_cast<int4*>(s->rects.p), counts);
        hipLaunchKernelGGL(hw1_scan_chunks_kernel, dim3(1), dim3(1024), 0, st, counts, offsets, ntiles, s->list_cap,
                           cfirst, ctile, s->chunk_cap);
        hp.bin_count = counts;
        hp.bin_offset = offsets;
        hp.bin_list = static_cast<const uint32_t*>(s->list.p);
        hp.chunk_first = cfirst;
        hp.chunk_tile = ctile;
        hipLaunchKernelGGL(hw1_fill_kernel, tgrid, dim3(64), 0, st, hp, cursor, static_cast<uint32_t*>(s->list.p));
        // chunks grid-stride over a grid of every CU's worth of waves (the count is on the device)
        hipLaunchKernelGGL(render_hw1_chunks_kernel, dim3(1024), dim3(BLOCK), 0, st, hp);
        const int rgrid = (std::max(W * H, 2 * ntiles) + BLOCK - 1) / BLOCK;
        hipLaunchKernelGGL(hw1_resolve_kernel, dim3(rgrid), dim3(BLOCK), 0, st, hp);
        s->last_kernel = "render_hw1_chunks_kernel";
        HIP_TRY(hipGetLastError());
        // this frame's total, for the capacity of the next ones
        HIP_TRY(hipMemcpyAsync(s->total_host + sl, offsets + ntiles, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(s->e1[sl], st));
    s->frames++;
    return RT_OK;
}

extern "C" int rt_hw1_kernel_times(const rt_hw1_scene* s, float* ms_out, int max, int* n_out) {
    if (!s || !ms_out || !n_out || max < 0) return set_error(RT_ERR_ARG, "rt_hw1_kernel_times: bad argument");
    DeviceGuard g(s->device);
    const int n = int(std::min<uint64_t>({uint64_t(max), s->frames, uint64_t(rt_hw1_scene::kRing)}));
    for (int i = 0; i < n; ++i) {
        const int sl = int((s->frames - uint64_t(n - i)) % rt_hw1_scene::kRing);
        HIP_TRY(hipEventSynchronize(s->e1[sl]));
        HIP_TRY(hipEventElapsedTime(&ms_out[i], s->e0[sl], s->e1[sl]));
    }
    *n_out = n;
    return RT_OK;
}

extern "C" const char* rt_hw1_kernel_name(const rt_hw1_scene* s) { return s ? s->last_kernel : ""; }

extern "C" int rt_hw1_list_info(const rt_hw1_scene* s, int64_t info[2]) {
    if (!s || !info) return set_error(RT_ERR_ARG, "rt_hw1_list_info: null argument");
    DeviceGuard g(s->device);
    info[0] = s->list_cap;
    info[1] = 0;
    if (s->frames > 0) {
        const int sl = int((s->frames - 1) % rt_hw1_scene::kRing);
        HIP_TRY(hipEventSynchronize(s->e1[sl]));
        info[1] = s->total_host[sl];
    }
    return RT_OK;
}

extern "C" int rt_render_hw1_ex(int device, const rt_vec3* pos, const rt_vec3* nrm, const uint32_t* idx, size_t P,
                                const rt_camera* cam, rt_vec3 lpos, rt_vec3 lcol, int spp, const float* jitter,
                                int flags, float* rgb_host, int32_t* hit_idx_host, float* hit_t_host,
                                float* kernel_ms) {
    if (!pos || !nrm || !idx || !cam || !rgb_host || spp < 1 || P == 0)
        return set_error(RT_ERR_ARG, "rt_render_hw1: bad argument (HW1 requires per-vertex normals)");
    if ((hit_idx_host == nullptr) != (hit_t_host == nullptr)) return set_error(RT_ERR_ARG, "hit_idx and hit_t go together");
    rt_hw1_scene* sp = nullptr;
    int rc = rt_hw1_scene_create(device, pos, nrm, idx, P, &sp);
    if (rc != RT_OK) return rc;
    std::unique_ptr<rt_hw1_scene, void (*)(rt_hw1_scene*)> s(sp, rt_hw1_scene_destroy);
    DeviceGuard g(device);
    const int W = cam->pixel_width, H = cam->pixel_height;
    const size_t npx = size_t(std::max(W, 0)) * size_t(std::max(H, 0));
    DevBuf drgb, dhi, dht;
    if ((rc = drgb.alloc(npx * 3 * sizeof(float))) != RT_OK) return rc;
    if (hit_idx_host) {
        if ((rc = dhi.alloc(npx * size_t(spp) * sizeof(int32_t))) != RT_OK) return rc;
        if ((rc = dht.alloc(npx * size_t(spp) * sizeof(float))) != RT_OK) return rc;
    }
    rc = rt_render_hw1_device(sp, cam, lpos, lcol, spp, jitter, flags, static_cast<float*>(drgb.p), nullptr,
                              static_cast<int32_t*>(dhi.p), static_cast<float*>(dht.p), nullptr);
    if (rc != RT_OK) return rc;
    HIP_TRY(hipDeviceSynchronize());
    if (kernel_ms) {
        int n = 0;
        if ((rc = rt_hw1_kernel_times(sp, kernel_ms, 1, &n)) != RT_OK) return rc;
    }
    HIP_TRY(hipMemcpy(rgb_host, drgb.p, npx * 3 * sizeof(float), hipMemcpyDeviceToHost));
    if (hit_idx_host) {
        HIP_TRY(hipMemcpy(hit_idx_host, dhi.p, npx * size_t(spp) * sizeof(int32_t), hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(hit_t_host, dht.p, npx * size_t(spp) * sizeof(float), hipMemcpyDeviceToHost));
    }
    return RT_OK;
}

extern "C" int rt_intersect_rays(int device, const rt_triangle* tri, const float origin[3], const float* dirs, int n,
                                 int hw1, float tmin, float tmax, int32_t* hit, float* t) {
    if (!tri || !origin || n < 0 || (n > 0 && (!dirs || !hit || !t))) return set_error(RT_ERR_ARG, "rt_intersect_rays: bad args");
    int rc = check_device(device);
    if (rc != RT_OK) return rc;
    if (n == 0) return RT_OK;
    DeviceGuard g(device);
    DevBuf dd, dh, dt;
    if ((rc = dd.upload(dirs, size_t(n) * 3 * sizeof(float))) != RT_OK) return rc;
    if ((rc = dh.alloc(size_t(n) * sizeof(int32_t))) != RT_OK) return rc;
    if ((rc = dt.alloc(size_t(n) * sizeof(float))) != RT_OK) return rc;
    const f3 v0{tri->v0.x, tri->v0.y, tri->v0.z};
    const f3 e1{tri->v1.x - tri->v0.x, tri->v1.y - tri->v0.y, tri->v1.z - tri->v0.z};
    const f3 e2{tri->v2.x - tri->v0.x, tri->v2.y - tri->v0.y, tri->v2.z - tri->v0.z};
    hipLaunchKernelGGL(intersect_kernel, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, nullptr, v0, e1, e2,
                       f3{origin[0], origin[1], origin[2]}, static_cast<const float*>(dd.p), n, hw1 ? 1 : 0, tmin,
                       tmax, static_cast<int32_t*>(dh.p), static_cast<float*>(dt.p));
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(hit, dh.p, size_t(n) * sizeof(int32_t), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(t, dt.p, size_t(n) * sizeof(float), hipMemcpyDeviceToHost));
    return RT_OK;
}

extern "C" float rt_powf_host(float x, float y) { return ref_powf(x, y); }

extern "C" int rt_powf_batch(int device, const float* x, const float* y, int n, float* out) {
    if (n < 0 || (n > 0 && (!x || !y || !out))) return set_error(RT_ERR_ARG, "rt_powf_batch: bad args");
    int rc = check_device(device);
    if (rc != RT_OK) return rc;
    if (n == 0) return RT_OK;
    DeviceGuard g(device);
    DevBuf dx, dy, dout;
    if ((rc = dx.upload(x, size_t(n) * sizeof(float))) != RT_OK) return rc;
    if ((rc = dy.upload(y, size_t(n) * sizeof(float))) != RT_OK) return rc;
    if ((rc = dout.alloc(size_t(n) * sizeof(float))) != RT_OK) return rc;
    hipLaunchKernelGGL(powf_kernel, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, nullptr,
                       static_cast<const float*>(dx.p), static_cast<const float*>(dy.p), n, static_cast<float*>(dout.p));
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(out, dout.p, size_t(n) * sizeof(float), hipMemcpyDeviceToHost));
    return RT_OK;
}

extern "C" int rt_box_test_host(const float* rays, const float* boxes, const float* tminmax, int n,
                                int32_t* out_fast, int32_t* out_exact, int32_t* out_class) {
    if (n < 0 || (n > 0 && (!rays || !boxes || !tminmax || !out_fast || !out_exact || !out_class)))
        return set_error(RT_ERR_ARG, "rt_box_test_host: bad args");
    for (int i = 0; i < n; ++i) {
        const float* R = rays + 6 * i;
        const float* B = boxes + 6 * i;
        f3 bm = mk(fmaxf(fabsf(B[0]), fabsf(B[3])), fmaxf(fabsf(B[1]), fabsf(B[4])), fmaxf(fabsf(B[2]), fabsf(B[5])));
        if (!(B[0] <= B[3] && B[1] <= B[4] && B[2] <= B[5])) bm = mk(INFINITY, INFINITY, INFINITY);  // as rt_scene_create
        const RayPre r = make_ray(mk(R[0], R[1], R[2]), mk(R[3], R[4], R[5]), bm);
        const BoxP b = {(v2f){B[0], B[3]}, (v2f){B[1], B[4]}, (v2f){B[2], B[5]}};
        out_class[i] = box_classify(r, b, tminmax[2 * i], tminmax[2 * i + 1]);
        out_fast[i] = box_hit(r, b, tminmax[2 * i], tminmax[2 * i + 1]) ? 1 : 0;
        out_exact[i] = box_hit_exact(r, b, (double)tminmax[2 * i], (double)tminmax[2 * i + 1]) ? 1 : 0;
    }
    return RT_OK;
}
