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
//
// Source layout (round 6): this translation unit holds the render kernels and their host side
// (scenes, launches, frames).  Its device code is read in sections, each included at its place
// inside the anonymous namespace below (device functions are force-inlined into the render
// kernels, so they share one translation unit; the build has no device-side linking):
//   rt_wave.hpp        wavefront primitives, constant-space loads (also used by rt_hw1.hip)
//   rt_instrument.hpp  RT_STATS / RT_FRAME_SPAN / RT_WAVE_TIMES / RT_LANE_ITERS hooks (variant builds)
//   rt_traverse.hpp    the traversals (wave DFS, frustum, lane, LDS, deep)
//   rt_shade.hpp       hit resolution, materials, camera ray, shading, bounces, trace_sample
//   rt_prepass.hpp     tile bounds, root and tree-cut culling passes, work lists
// Separate translation units: rt_records.cpp (host record builders), rt_hw1.hip (the HW1 path),
// rt_frame.hip, rt_lbvh.hip, rt_renderer.hip.

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
#include "rt_records.hpp"

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

#include "rt_wave.hpp"
#include "rt_instrument.hpp"
#include "rt_traverse.hpp"
#include "rt_shade.hpp"
#include "rt_prepass.hpp"

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
        RT_HOOK_FRAME_FIRST(first, lane, RG);
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
            RT_HOOK_FRAME_LAST(lane, RG);
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
        RT_HOOK_ITEM_START(wt0);
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
        RT_HOOK_ITEM_END(wt0, tile, WPT, qw, bx, first, wv);
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
using rt::FrustumRecords;
using rt::build_frustum_records;
using rt::build_quant_records;
using rt::subtree_leaves;
static_assert(LEAF_BIT == rt::kRecLeafBit && NO_REF == rt::kRecNoRef, "record ids follow the kernels' refs");
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
        HIP_TRY(hipDeviceSynchronize());  // (the frames run on non-blocking streams)
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

// The frustum and 4-ary record builders are host code of their own (rt_records.cpp).

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
    if (clear) {
        HIP_TRY(hipMemset(s->fault.p, 0, sizeof(uint32_t)));
        HIP_TRY(hipDeviceSynchronize());  // before any later frame on a non-blocking stream
    }
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
    HIP_TRY(hipDeviceSynchronize());  // (the frame runs on the scene's non-blocking streams)
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
    HIP_TRY(hipDeviceSynchronize());
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

// The HW1 path (rt_render_hw1*, rt_hw1_scene) is rt_hw1.hip.

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
