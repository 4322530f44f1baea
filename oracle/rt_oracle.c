/* oracle/rt_oracle.c — TEST INFRASTRUCTURE ONLY (see rt_oracle.h).
 *
 * CPU restatement of the reference's per-pixel ray path, written for readability, not
 * speed.  Every float expression keeps the reference's evaluation order and its
 * float/double mix; build flags (oracle/Makefile) forbid contraction.  Citations:
 *   G/   = /root/reference/HW2/HW2/GPUandCPU
 *   HW1/ = /root/reference/HW1
 */
#include "rt_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef orc_vec3 V;

/* ---- G/include/vec3.h:327-348 ------------------------------------------------------ */
static inline V v3(float x, float y, float z) { V r = {x, y, z}; return r; }
static inline V vadd(V a, V b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V vsub(V a, V b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V vneg(V a) { return v3(-a.x, -a.y, -a.z); }
static inline V vmul(V a, V b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline V vscale(V v, float t) { return v3(v.x * t, v.y * t, v.z * t); }
/* operator/(Vec3, double): double divide, rounded to float (vec3.h:334). */
static inline V vdivd(V a, double t) {
    return v3((float)((double)a.x / t), (float)((double)a.y / t), (float)((double)a.z / t));
}
static inline float vdot(V u, V v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
static inline V vcross(V u, V v) {
    return v3(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
static inline float vlength(V v) { return sqrtf(vdot(v, v)); }
/* normalize(v) = v / length(v) (vec3.h:343) */
static inline V vnormalize(V v) { return vdivd(v, (double)vlength(v)); }
/* unit_vector (vec3.h:345-348): float divide by sqrtf(x*x+y*y+z*z) */
static inline V vunit(V v) {
    float len = sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    return v3(v.x / len, v.y / len, v.z / len);
}
/* Camera::unit_vector with its 1e-12 fallback (G/include/camera.h:218-223). */
static inline V cam_unit(V v) {
    float len = sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    if ((double)len < 1e-12) return v3(0.0f, 0.0f, 1.0f);
    return vdivd(v, (double)len);
}

/* ---- jitter: std::mt19937 + uniform_real_distribution<float> (libstdc++) --------- */
typedef struct { uint32_t mt[624]; int i; } mt19937;
static void mt_seed(mt19937* g, uint32_t s) {
    g->mt[0] = s;
    for (int i = 1; i < 624; ++i)
        g->mt[i] = 1812433253u * (g->mt[i - 1] ^ (g->mt[i - 1] >> 30)) + (uint32_t)i;
    g->i = 624;
}
static uint32_t mt_next(mt19937* g) {
    if (g->i >= 624) {
        for (int k = 0; k < 624; ++k) {
            uint32_t y = (g->mt[k] & 0x80000000u) | (g->mt[(k + 1) % 624] & 0x7fffffffu);
            g->mt[k] = g->mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        g->i = 0;
    }
    uint32_t y = g->mt[g->i++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}
/* generate_canonical<float, 24>: one 32-bit draw, float(u) / 2^32, clamped below 1. */
static float mt_canonical(mt19937* g) {
    float sum = (float)mt_next(g) * 1.0f;
    float tmp = 4294967296.0f;
    float r = sum / tmp;
    if (r >= 1.0f) r = nextafterf(1.0f, 0.0f);
    return r;
}
void orc_jitter(int spp, uint32_t seed, int centered, float* out) {
    mt19937 g;
    mt_seed(&g, seed);
    for (int s = 0; s < spp; ++s) {
        float dx = mt_canonical(&g) * (1.0f - 0.0f) + 0.0f;
        float dy = mt_canonical(&g) * (1.0f - 0.0f) + 0.0f;
        if (centered) { dx = dx - 0.5f; dy = dy - 0.5f; }
        out[2 * s] = dx;
        out[2 * s + 1] = dy;
    }
}

/* ---- camera (G/include/camera.h:72-94 == HW1/include/camera.h:55-92) -------------- */
int orc_camera_init(orc_camera* cam, const float pos[3], const float look_at[3], const float up[3],
                    double focal_length_mm, double sensor_height_mm, int width, int height, int hw1) {
    if (hw1 && (width < 1 || height < 1)) return -1;  /* HW1 throws */
    if (width < 1) width = 1;                          /* G/ clamps (camera.h:73-74) */
    if (height < 1) height = 1;
    V center = v3(pos[0], pos[1], pos[2]);
    V look = v3(look_at[0], look_at[1], look_at[2]);
    V upv = v3(up[0], up[1], up[2]);
    V forward = cam_unit(vsub(look, center));
    V right = cam_unit(vcross(forward, upv));
    V up_corrected = vcross(right, forward);
    double focal_m = focal_length_mm / 1000.0;
    double sensor_m = sensor_height_mm / 1000.0;
    double vh = sensor_m;
    double vw = vh * ((double)width / (double)height);
    V vu = vscale(right, (float)vw);                /* double * Vec3 narrows the scalar */
    V vv = vscale(up_corrected, (float)(-vh));
    V du = vdivd(vu, (double)width);
    V dv = vdivd(vv, (double)height);
    V vcenter = vadd(center, vscale(forward, (float)focal_m));
    V vul = vsub(vsub(vcenter, vscale(vu, 0.5f)), vscale(vv, 0.5f));
    V p00 = vadd(vul, vscale(vadd(du, dv), 0.5f));
    cam->center = center;
    cam->pixel00 = p00;
    cam->du = du;
    cam->dv = dv;
    cam->width = width;
    cam->height = height;
    return 0;
}

/* ---- G/ traversal ------------------------------------------------------------------ */
typedef struct { V o, d; } Ray;
typedef struct {
    int tri; int hit; V p; V normal; double t; orc_material mat;
} Hit;

static const orc_material kDefaultMaterial = {  /* G/include/material.h:8-19 */
    {0.8f, 0.8f, 0.8f}, 1.0f, {0.04f, 0.04f, 0.04f}, 0.0f, 32.0f, 0.0f, {0.0f, 0.0f, 0.0f}};

/* G/include/bvh.h:81-129 — double-precision slabs */
static int intersect_aabb(const Ray* r, const orc_aabb* b, double tmin, double tmax) {
    const float eps = 1e-8f;
    double t0 = tmin, t1 = tmax;
    const float o[3] = {r->o.x, r->o.y, r->o.z}, d[3] = {r->d.x, r->d.y, r->d.z};
    const float mn[3] = {b->mn.x, b->mn.y, b->mn.z}, mx[3] = {b->mx.x, b->mx.y, b->mx.z};
    for (int a = 0; a < 3; ++a) {
        if (fabsf(d[a]) < eps) {
            if (o[a] < mn[a] || o[a] > mx[a]) return 0;
        } else {
            const double inv = 1.0 / (double)d[a];
            double tn = ((double)mn[a] - (double)o[a]) * inv;
            double tf = ((double)mx[a] - (double)o[a]) * inv;
            if (tn > tf) { double tmp = tn; tn = tf; tf = tmp; }
            if (tn > t0) t0 = tn;
            if (tf < t1) t1 = tf;
            if (t0 > t1) return 0;
        }
    }
    return 1;
}

/* G/include/query.h:72-132 */
static int intersect_tri(const Ray* r, const orc_tri* tri, float tmin, float tmax, Hit* rec) {
    rec->tri = -1;
    const V e1 = vsub(tri->v1, tri->v0);
    const V e2 = vsub(tri->v2, tri->v0);
    const V pvec = vcross(r->d, e2);
    const float det = vdot(e1, pvec);
    if (fabsf(det) < 1e-8f) { rec->hit = 0; return 0; }
    const float invDet = 1.0f / det;
    const V tvec = vsub(r->o, tri->v0);
    const float u = vdot(tvec, pvec) * invDet;
    if (u < 0.0f || u > 1.0f) { rec->hit = 0; return 0; }
    const V qvec = vcross(tvec, e1);
    const float v = vdot(r->d, qvec) * invDet;
    if (v < 0.0f || (u + v) > 1.0f) { rec->hit = 0; return 0; }
    const float t = vdot(e2, qvec) * invDet;
    if (t < tmin || t > tmax) { rec->hit = 0; return 0; }
    rec->hit = 1;
    rec->t = t;
    rec->p = vadd(r->o, vscale(r->d, t));
    V geomN = vnormalize(vcross(e1, e2));
    int front = vdot(r->d, geomN) < 0.0f;
    if (!front) geomN = vneg(geomN);
    const float w = 1.0f - u - v;
    V sN = vadd(vadd(vscale(tri->n0, w), vscale(tri->n1, u)), vscale(tri->n2, v));
    if (vdot(sN, sN) < 1e-12f) {
        sN = geomN;
    } else {
        sN = vnormalize(sN);
        if (vdot(sN, geomN) < 0.0f) sN = vneg(sN);
    }
    rec->normal = sN;
    rec->mat = kDefaultMaterial;
    return 1;
}

typedef struct { uint64_t pops, internal, leaf, max_pops; } TravCount;

/* G/include/query.h:224-311 */
static void search_bvh(int numTriangles, const Ray* ray, const orc_node* nodes,
                       const orc_aabb* aabbs, const orc_tri* tris, Hit* out, TravCount* tc) {
    const float tmin = 1e-4f;
    float bestT = FLT_MAX;
    Hit best;
    memset(&best, 0, sizeof(best));
    best.tri = -1;
    best.hit = 0;
    best.t = -1.0;
    best.mat = kDefaultMaterial;
    enum { CAP = 512 };
    uint32_t stack[CAP];
    int sp = 0, overflow = 0;
    uint64_t pops = 0;
    stack[sp++] = 0;
    while (sp > 0) {
        const uint32_t n = stack[--sp];
        ++pops;
        if (tc) tc->pops++;
        if (!intersect_aabb(ray, &aabbs[n], (double)tmin, (double)bestT)) continue;
        const orc_node node = nodes[n];
        if (node.object != 0xFFFFFFFFu) {
            if (tc) tc->leaf++;
            if (node.object < (uint32_t)numTriangles) {
                Hit rec;
                if (intersect_tri(ray, &tris[node.object], tmin, bestT, &rec)) {
                    rec.tri = (int)node.object;
                    bestT = (float)rec.t;
                    best = rec;
                }
            }
            continue;
        }
        if (tc) tc->internal++;
        if (node.left != 0xFFFFFFFFu && intersect_aabb(ray, &aabbs[node.left], (double)tmin, (double)bestT)) {
            if (sp < CAP) stack[sp++] = node.left; else overflow = 1;
        }
        if (node.right != 0xFFFFFFFFu && intersect_aabb(ray, &aabbs[node.right], (double)tmin, (double)bestT)) {
            if (sp < CAP) stack[sp++] = node.right; else overflow = 1;
        }
    }
    if (tc && pops > tc->max_pops) tc->max_pops = pops;
    if (overflow) {
        for (int i = 0; i < numTriangles; ++i) {
            Hit rec;
            if (intersect_tri(ray, &tris[i], tmin, bestT, &rec)) {
                rec.tri = i;
                bestT = (float)rec.t;
                best = rec;
            }
        }
    }
    *out = best;
}

int orc_search_bvh(size_t num_triangles, const float orig[3], const float dir[3],
                   const orc_node* nodes, const orc_aabb* aabbs, const orc_tri* tris, float* t_out) {
    Ray r = {v3(orig[0], orig[1], orig[2]), v3(dir[0], dir[1], dir[2])};
    Hit h;
    search_bvh((int)num_triangles, &r, nodes, aabbs, tris, &h, NULL);
    if (t_out) *t_out = h.hit ? (float)h.t : -1.0f;
    return h.hit ? h.tri : -1;
}

/* ---- shading (G/include/shader.h, brdf.h) ------------------------------------------ */
static const float RT_EPS = 1e-3f;  /* shader.h:22 */

static V clamp01v(V c) {  /* shader.h:24-32 */
    if (c.x > 1.0f) c.x = 1.0f;
    if (c.y > 1.0f) c.y = 1.0f;
    if (c.z > 1.0f) c.z = 1.0f;
    if (c.x < 0.0f) c.x = 0.0f;
    if (c.y < 0.0f) c.y = 0.0f;
    if (c.z < 0.0f) c.z = 0.0f;
    return c;
}

/* brdf.h:12-40 */
static V eval_brdf(const Hit* rec, V Vw, V L) {
    const orc_material* m = &rec->mat;
    const V N = rec->normal;
    const float NdotL = fmaxf(vdot(N, L), 0.0f);
    const float NdotV = fmaxf(vdot(N, Vw), 0.0f);
    if (NdotL <= 0.f || NdotV <= 0.f) return v3(0, 0, 0);
    const float invPi = 0.31830988618f;
    V fd = vscale(m->albedo, m->kd * invPi);
    V Hh = vunit(vadd(L, Vw));
    float NdotH = fmaxf(vdot(N, Hh), 0.0f);
    const float inv2Pi = 0.15915494309f;
    float specNorm = (m->shininess + 2.0f) * inv2Pi;
    float specLobe = specNorm * powf(NdotH, m->shininess);
    V fs = vscale(vscale(m->specular, m->ks), specLobe);
    return vadd(fd, fs);
}

typedef struct {
    int P; const orc_node* nodes; const orc_aabb* aabbs; const orc_tri* tris;
    const int32_t* objids; const orc_material* mats; int nmat;
    const orc_light* lights; int nlights;
    TravCount tc[3]; uint64_t rays[3], hits[3], occluded;
} Ctx;

/* shader.h:44-62 */
static int in_shadow(Ctx* c, V P, V N, const orc_light* light) {
    V toL = vsub(light->position, P);
    float dist = sqrtf(vdot(toL, toL));
    if (dist <= 0.0f) return 0;
    V Ldir = vdivd(toL, (double)dist);
    Ray sr = {vadd(P, vscale(N, RT_EPS)), Ldir};
    Hit sh;
    c->rays[1]++;
    search_bvh(c->P, &sr, c->nodes, c->aabbs, c->tris, &sh, &c->tc[1]);
    int occ = sh.hit && sh.t < (double)dist;
    if (sh.hit) c->hits[1]++;
    if (occ) c->occluded++;
    return occ;
}

/* shader.h:65-110 */
static V shade_direct(Ctx* c, const Ray* r, const Hit* rec) {
    V N = vunit(rec->normal);
    V Vw = vunit(vsub(r->o, rec->p));
    V Lo = v3(0, 0, 0);
    Lo = vadd(Lo, vscale(rec->mat.albedo, 0.05f));
    Lo = vadd(Lo, rec->mat.emission);
    for (int i = 0; i < c->nlights; ++i) {
        const orc_light* light = &c->lights[i];
        V L = vunit(vsub(light->position, rec->p));
        float NdotL = fmaxf(vdot(N, L), 0.0f);
        if (NdotL <= 0.0f) continue;
        if (in_shadow(c, rec->p, N, light)) continue;
        V f = eval_brdf(rec, Vw, L);
        V radiance = vscale(light->color, (float)light->intensity);
        V direct = vscale(vmul(radiance, f), NdotL);
        Lo = vadd(Lo, direct);
    }
    return Lo;
}

/* query.h:32-70 */
static float rng_next(uint32_t* state) {
    *state = *state * 1664525u + 1013904223u;
    uint32_t h = *state;
    h = (h ^ 61u) ^ (h >> 16u);
    h *= 9u;
    h ^= h >> 4u;
    h *= 0x27d4eb2du;
    h ^= h >> 15u;
    return (float)h / (float)0xFFFFFFFFu;
}
static uint32_t make_rng_seed(int x, int y, int s) {
    return (uint32_t)x * 73856093u ^ (uint32_t)y * 19349663u ^ (uint32_t)s * 83492791u;
}
static V random_unit_vector(uint32_t* st) {
    for (;;) {
        float x = 2.0f * rng_next(st) - 1.0f;
        float y = 2.0f * rng_next(st) - 1.0f;
        float z = 2.0f * rng_next(st) - 1.0f;
        float lensq = x * x + y * y + z * z;
        if (lensq > 1e-10f && lensq <= 1.0f) {
            float inv = 1.0f / sqrtf(lensq);
            return v3(x * inv, y * inv, z * inv);
        }
    }
}
static V random_on_hemisphere(V n, uint32_t* st) {
    V u = random_unit_vector(st);
    if (vdot(u, n) > 0.0f) return u;
    return v3(-u.x, -u.y, -u.z);
}

/* query.h:134-153 */
static void assign_material(Ctx* c, Hit* h) {
    if (!h->hit || c->objids == NULL || c->mats == NULL || h->tri < 0 || h->tri >= c->P) return;
    const int oid = c->objids[h->tri];
    if (oid >= 0 && oid < c->nmat) h->mat = c->mats[oid];
}

/* query.h:156-220 */
static V trace(Ctx* c, Ray ray, int maxDepth, V miss, uint32_t rng, int diffuse_bounce,
               int32_t* prim_idx, float* prim_t) {
    if (maxDepth <= 0) return v3(0, 0, 0);
    V radiance = v3(0, 0, 0);
    V thr = v3(1, 1, 1);
    for (int depth = 0; depth < maxDepth; ++depth) {
        Hit h;
        const int cls = depth == 0 ? 0 : 2;
        c->rays[cls]++;
        search_bvh(c->P, &ray, c->nodes, c->aabbs, c->tris, &h, &c->tc[cls]);
        if (depth == 0) {
            if (prim_idx) *prim_idx = h.hit ? h.tri : -1;
            if (prim_t) *prim_t = h.hit ? (float)h.t : -1.0f;
        }
        if (!h.hit) {
            radiance = vadd(radiance, vmul(thr, miss));
            break;
        }
        c->hits[cls]++;
        assign_material(c, &h);
        V direct = shade_direct(c, &ray, &h);
        radiance = vadd(radiance, vmul(thr, direct));
        const float kd = h.mat.kd, kr = h.mat.kr, total = kd + kr;
        if (total <= 0.0f) break;
        const V N = vnormalize(h.normal);
        const float xi = rng_next(&rng);
        if (diffuse_bounce && xi < kd / total) {
            V dd = random_on_hemisphere(N, &rng);
            ray.o = vadd(h.p, vscale(N, RT_EPS));
            ray.d = dd;
            float NdotL = fmaxf(vdot(N, dd), 0.0f);
            thr = vmul(thr, vscale(h.mat.albedo, 2.0f * NdotL));
        } else {
            V I = vunit(ray.d);
            V refl = vsub(I, vscale(N, 2.0f * vdot(I, N)));   /* shader.h:38-42 */
            ray.o = vadd(h.p, vscale(N, RT_EPS));
            ray.d = refl;
            thr = vmul(thr, vscale(h.mat.specular, kr));
        }
        if (thr.x < 1e-4f && thr.y < 1e-4f && thr.z < 1e-4f) break;
    }
    return clamp01v(radiance);
}

int orc_render_g(size_t num_triangles, int W, int H, const orc_camera* cam, orc_vec3 miss_color,
                 int max_depth, int spp, const orc_node* nodes, const orc_aabb* aabbs,
                 const orc_tri* tris, const int32_t* tri_obj_ids, const orc_material* mats,
                 int num_mats, const orc_light* lights, int num_lights, int diffuse_bounce,
                 const float* jitter, int rebuild_jitter_per_pixel, int y0, int y1, int threads,
                 float* out_rgb, int32_t* hit_idx, float* hit_t, orc_stats* stats) {
    if (!nodes || !aabbs || !tris || !out_rgb || spp < 1 || W < 1 || H < 1) return -1;
    if (y0 < 0) y0 = 0;
    if (y1 > H) y1 = H;
    float* tab = (float*)malloc(sizeof(float) * 2 * (size_t)spp);
    if (!tab) return -2;
    if (jitter) memcpy(tab, jitter, sizeof(float) * 2 * (size_t)spp);
    else orc_jitter(spp, 42u, 1, tab);
    orc_stats total;
    memset(&total, 0, sizeof(total));
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
#pragma omp parallel
    {
        Ctx c;
        memset(&c, 0, sizeof(c));
        c.P = (int)num_triangles; c.nodes = nodes; c.aabbs = aabbs; c.tris = tris;
        c.objids = tri_obj_ids; c.mats = mats; c.nmat = num_mats; c.lights = lights; c.nlights = num_lights;
        float* local = (float*)malloc(sizeof(float) * 2 * (size_t)spp);
#pragma omp for schedule(dynamic, 1)
        for (int y = y0; y < y1; ++y) {
            for (int x = 0; x < W; ++x) {
                const float* offs = tab;
                if (rebuild_jitter_per_pixel) {  /* query.cu:142 rebuilds the table per pixel */
                    orc_jitter(spp, 42u, 1, local);
                    offs = local;
                }
                V col = v3(0, 0, 0);
                for (int si = 0; si < spp; ++si) {
                    const float px = (float)x + offs[2 * si];
                    const float py = (float)y + offs[2 * si + 1];
                    /* Camera::get_ray(float, float), camera.h:49-53 */
                    V pix = vadd(vadd(cam->pixel00, vscale(cam->du, px)), vscale(cam->dv, py));
                    Ray r = {cam->center, cam_unit(vsub(pix, cam->center))};
                    const size_t k = ((size_t)y * W + x) * (size_t)spp + (size_t)si;
                    col = vadd(col, trace(&c, r, max_depth, miss_color, make_rng_seed(x, y, si),
                                          diffuse_bounce, hit_idx ? &hit_idx[k] : NULL,
                                          hit_t ? &hit_t[k] : NULL));
                }
                V o = vdivd(col, (double)(float)spp);
                float* dst = &out_rgb[((size_t)y * W + x) * 3];
                dst[0] = o.x; dst[1] = o.y; dst[2] = o.z;
            }
        }
        free(local);
#pragma omp critical
        {
            for (int k = 0; k < 3; ++k) {
                total.rays[k] += c.rays[k];
                total.pops[k] += c.tc[k].pops;
                total.internal_entered[k] += c.tc[k].internal;
                total.leaf_entered[k] += c.tc[k].leaf;
                if (c.tc[k].max_pops > total.max_pops[k]) total.max_pops[k] = c.tc[k].max_pops;
                total.hits[k] += c.hits[k];
            }
            total.occluded += c.occluded;
        }
    }
    free(tab);
    if (stats) *stats = total;
    return 0;
}

/* ---- HW1 (HW1/include/ray.h, raytracer.h; HW1/src/render.cpp) ---------------------- */
typedef struct { int hit; V p; V normal; double t; } Hit1;

/* ray.h:67-117 */
static void ray_intersection_hw1(const Ray* r, V v0, V v1, V v2, V n0, V n1, V n2, Hit1* rec) {
    const float eps = FLT_EPSILON;
    V e1 = vsub(v1, v0), e2 = vsub(v2, v0);
    V pvec = vcross(r->d, e2);
    float det = vdot(pvec, e1);
    if (fabsf(det) < eps) { rec->hit = 0; return; }
    float invDet = (float)(1.0 / (double)det);
    V tvec = vsub(r->o, v0);
    float u = vdot(tvec, pvec) * invDet;
    if ((double)u < 0.0 || (double)u > 1.0) { rec->hit = 0; return; }
    V qvec = vcross(tvec, e1);
    float v = vdot(r->d, qvec) * invDet;
    if ((double)v < 0.0 || (double)(u + v) > 1.0) { rec->hit = 0; return; }
    float t = vdot(e2, qvec) * invDet;
    if ((double)t < 0.0) { rec->hit = 0; return; }
    rec->hit = 1;
    rec->t = t;
    rec->p = vadd(r->o, vscale(r->d, (float)rec->t));   /* at(double t): t*dir narrows */
    const float w = 1.0f - u - v;
    rec->normal = vadd(vadd(vscale(n0, w), vscale(n1, u)), vscale(n2, v));
}

/* raytracer.h:21-48 (material hard-coded at ray.h:111-114) */
static V shade_hw1(const Ray* r, const Hit1* rec, V lpos, V lcol) {
    if (!rec->hit) {
        V ud = vunit(r->d);
        float t = 0.5f * (ud.z + 1.0f);
        return vadd(vscale(v3(1.0f, 1.0f, 1.0f), 1.0f - t), vscale(v3(0.5f, 0.7f, 1.0f), t));
    }
    const V albedo = v3(0.8f, 0.2f, 0.2f);
    V ambient = vscale(albedo, 0.1f);
    V lightDir = vunit(vsub(lpos, rec->p));
    float diff = fmaxf(vdot(rec->normal, lightDir), 0.0f);
    V diffuse = vscale(vmul(albedo, lcol), diff);
    V viewDir = vunit(vsub(r->o, rec->p));
    V halfDir = vunit(vadd(lightDir, viewDir));
    float spec = powf(fmaxf(vdot(rec->normal, halfDir), 0.0f), 64.0f);
    V specular = vscale(lcol, spec);
    V c = vadd(vadd(ambient, diffuse), specular);
    if ((double)c.x > 1.0) c.x = 1.0f;
    if ((double)c.y > 1.0) c.y = 1.0f;
    if ((double)c.z > 1.0) c.z = 1.0f;
    return c;
}

int orc_render_hw1(const orc_vec3* positions, const orc_vec3* normals, const uint32_t* indices,
                   size_t num_triangles, const orc_camera* cam, orc_vec3 light_pos,
                   orc_vec3 light_color, int spp, const float* jitter, int y0, int y1, int threads,
                   float* out_rgb, int32_t* hit_idx, float* hit_t) {
    if (!positions || !normals || !indices || !out_rgb || spp < 1) return -1;
    const int W = cam->width, H = cam->height;
    if (y0 < 0) y0 = 0;
    if (y1 > H) y1 = H;
    float* tab = (float*)malloc(sizeof(float) * 2 * (size_t)spp);
    if (!tab) return -2;
    if (jitter) memcpy(tab, jitter, sizeof(float) * 2 * (size_t)spp);
    else orc_jitter(spp, 42u, 0, tab);
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
#pragma omp parallel for schedule(dynamic, 1)
    for (int j = y0; j < y1; ++j) {
        for (int i = 0; i < W; ++i) {
            V acc = v3(0, 0, 0);
            for (int s = 0; s < spp; ++s) {
                float px = (float)i + tab[2 * s];
                float py = (float)j + tab[2 * s + 1];
                /* render.cpp:86: get_pixel_position(int, int) truncates px, py */
                const int pi = (int)px, pj = (int)py;
                V pix = vadd(vadd(cam->pixel00, vscale(cam->du, (float)(double)pi)),
                             vscale(cam->dv, (float)(double)pj));
                Ray r = {cam->center, vunit(vsub(pix, cam->center))};
                Hit1 prev;
                prev.hit = 0;
                prev.t = (double)FLT_MAX;
                V color = shade_hw1(&r, &prev, light_pos, light_color);
                int best = -1;
                for (size_t k = 0; k < num_triangles; ++k) {
                    const uint32_t a = indices[3 * k], b = indices[3 * k + 1], cc = indices[3 * k + 2];
                    Hit1 rec;
                    ray_intersection_hw1(&r, positions[a], positions[b], positions[cc],
                                         normals[a], normals[b], normals[cc], &rec);
                    if (rec.hit && rec.t < prev.t) {
                        color = shade_hw1(&r, &rec, light_pos, light_color);
                        prev = rec;
                        best = (int)k;
                    }
                }
                acc = vadd(acc, color);
                const size_t kk = ((size_t)j * W + i) * (size_t)spp + (size_t)s;
                if (hit_idx) hit_idx[kk] = best;
                if (hit_t) hit_t[kk] = best >= 0 ? (float)prev.t : -1.0f;
            }
            V o = vdivd(acc, (double)(float)spp);
            float* dst = &out_rgb[((size_t)j * W + i) * 3];
            dst[0] = o.x; dst[1] = o.y; dst[2] = o.z;
        }
    }
    free(tab);
    return 0;
}

void orc_kat_hw1(const orc_tri* tri, const float orig[3], const float* dirs, int n,
                 int32_t* hit, float* t) {
    for (int i = 0; i < n; ++i) {
        Ray r = {v3(orig[0], orig[1], orig[2]), vunit(v3(dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2]))};
        Hit1 rec;
        ray_intersection_hw1(&r, tri->v0, tri->v1, tri->v2, tri->n0, tri->n1, tri->n2, &rec);
        hit[i] = rec.hit;
        t[i] = rec.hit ? (float)rec.t : -1.0f;
    }
}

void orc_intersect_g(const orc_tri* tri, const float orig[3], const float* dirs, int n,
                     float tmin, float tmax, int32_t* hit, float* t) {
    for (int i = 0; i < n; ++i) {
        Ray r = {v3(orig[0], orig[1], orig[2]), v3(dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2])};
        Hit rec;
        hit[i] = intersect_tri(&r, tri, tmin, tmax, &rec);
        t[i] = hit[i] ? (float)rec.t : -1.0f;
    }
}

/* ppm_p6.cpp:137-155 */
void orc_ppm_quantize(const float* linear, size_t n, int maxval, int clamp, int gamma2, uint16_t* out) {
    for (size_t i = 0; i < n; ++i) {
        double l = (double)linear[i];
        if (gamma2) {
            if (l < 0.0) l = 0.0;
            l = sqrt(l);
        }
        if (clamp) {
            if (l < 0.0) l = 0.0;
            else if (l > 1.0) l = 1.0;
        }
        double scaled = l * (double)maxval;
        long rounded = lround(scaled);
        if (rounded < 0) rounded = 0;
        if (rounded > maxval) rounded = maxval;
        out[i] = (uint16_t)rounded;
    }
}
