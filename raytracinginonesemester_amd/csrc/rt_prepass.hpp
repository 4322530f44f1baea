// rt_prepass.hpp — the frame's pre-passes: tile bounds, the root-box cull (tile_cull_kernel),
// the tree-cut cull with its second level (tile_cut_kernel, tile_cut_sub), the work lists and
// the heavy-first classes.  Exact: a tile is culled only when every ray of it provably misses
// a box SearchBVH must pass before any triangle below it.  DESIGN.md §4.1, §4.4, §4.16.
// Part of rt_device.hip's translation unit, included inside its anonymous namespace after rt_shade.hpp.
#pragma once

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
