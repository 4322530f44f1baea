// rt_shade.hpp — hit resolution, materials, the camera ray and the shading loop of a sample
// (assignMaterialToHit query.h:134-153, Camera::get_ray camera.h:49-53, ShadeDirect /
// IsInShadow / EvaluateBRDF shader.h:44-110 + brdf.h:12-40, TraceRayIterative
// query.h:156-220 with the bounce loops).  DESIGN.md §4.2, §4.10.
// Part of rt_device.hip's translation unit, included inside its anonymous namespace after rt_traverse.hpp.
#pragma once

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
