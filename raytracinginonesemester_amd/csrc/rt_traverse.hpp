// rt_traverse.hpp — the BVH traversals of the G/ path (SearchBVH, G/include/query.h:224-311,
// with intersectAABB bvh.h:81-129 and intersectTriangle query.h:72-132): the wave DFS over
// per-lane masks, the camera rays' frustum traversal, the per-lane (LANE, LDS, DEEP) forms
// and the dispatch by kernel mode.  DESIGN.md §4.2, §4.10, §4.12.
// Part of rt_device.hip's translation unit, included inside its anonymous namespace after the scene and launch structs, rt_wave.hpp and rt_instrument.hpp.
#pragma once

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
// The direction family of the lanes with `member` (per axis the reciprocals of [dl, dh], or of
// the loose axis' one-sided form, see traverse_frustum), made wave-uniform; true when an axis
// is loose.  Per axis two wave reductions: the tight interval matters, the frog's triangles are
// about a pixel wide (one reduction of |d - c| around one lane's c, an interval up to twice as
// wide, took c3 from 0.157 to 0.477 ms).  The reciprocals are v_rcp_f32 (1 ulp; inside the
// 2^-19 widening of the family test).
__device__ __forceinline__ bool family_dirs(const SceneView& sc, const RayPre& r, bool member, const float* o, v2f* U) {
    const float dd[3] = {r.d.x, r.d.y, r.d.z};
    bool loose = false;  // a loose axis; U = (ihp, iln) on it: U.x > 0 > U.y, which no other axis
                         // has (bounded: one sign; no bound: -inf, +inf)
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float dl = wave_reduce_f<false>(member ? dd[a] : INFINITY);
        const float dh = wave_reduce_f<true>(member ? dd[a] : -INFINITY);
        const bool fin = sc.bmax[a] + fabsf(o[a]) < 1e30f;
        const bool ok = (dl >= 1e-8f || dh <= -1e-8f) && fin;
        const bool lz = !ok && fin;
        loose = loose || lz;
        // (made SGPRs: wave-uniform values the VALU computed stay in VGPRs otherwise)
        const float u0 = ok ? rcp_approx(dl) : lz ? (dh > 0.0f ? rcp_approx(dh) : INFINITY) : -INFINITY;
        const float u1 = ok ? rcp_approx(dh) : lz ? (dl < 0.0f ? rcp_approx(dl) : -INFINITY) : INFINITY;
        U[a] = (v2f){__int_as_float(uni(__float_as_int(u0))), __int_as_float(uni(__float_as_int(u1)))};
    }
    return loose;
}

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
    // per axis [dl, dh], the live lanes' range (family_dirs)
    v2f U[3];
    const bool loose = family_dirs(sc, r, live, o, U);
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
