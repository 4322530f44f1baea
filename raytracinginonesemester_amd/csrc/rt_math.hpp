// rt_math.hpp — device-side float/double math of the ray path, in the reference's exact
// evaluation order (G/include/vec3.h, bvh.h, query.h, shader.h, brdf.h, camera.h).
// The translation unit is compiled with -ffp-contract=off (no v_fma for a*b+c) and with
// HIP's default correctly-rounded f32 division and sqrt, so every helper below returns the
// bits the reference's x86-64 build returns; powf is the one libm call whose device
// implementation may differ in the last place ("Parity").
#pragma once

#include <hip/hip_runtime.h>
#include <cfloat>
#include <cstdint>

namespace rtd {

struct f3 {
    float x, y, z;
};

__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 neg(f3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ f3 mul(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ f3 scale(f3 v, float t) { return mk(v.x * t, v.y * t, v.z * t); }
__device__ __forceinline__ float dot(f3 u, f3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
__device__ __forceinline__ f3 cross(f3 u, f3 v) {
    return mk(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
// Vec3 / double(len) == correctly rounded f32 division (vec3.h:334).
__device__ __forceinline__ f3 divf(f3 v, float t) { return mk(v.x / t, v.y / t, v.z / t); }
// unit_vector (vec3.h:345-348) and normalize (vec3.h:343) round identically.
__device__ __forceinline__ f3 unit(f3 v) {
    const float len = sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    return divf(v, len);
}
// Camera::unit_vector with the 1e-12 fallback (camera.h:218-223).
__device__ __forceinline__ f3 cam_unit(f3 v) {
    const float len = sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    if ((double)len < 1e-12) return mk(0.0f, 0.0f, 1.0f);
    return divf(v, len);
}

// Per-ray constants of intersectAABB (bvh.h:81-129): the reference recomputes
// 1.0/double(dir) at every test; it depends on the ray only, so it is hoisted here
// (same double value, bit for bit).
struct RayPre {
    f3 o, d;
    double od[3];
    double inv[3];
    uint32_t par;  // bit a set: |dir[a]| < 1e-8f (slab degenerates to an inside test)
};

__device__ __forceinline__ RayPre make_ray(f3 o, f3 d) {
    RayPre r;
    r.o = o;
    r.d = d;
    r.od[0] = (double)o.x;
    r.od[1] = (double)o.y;
    r.od[2] = (double)o.z;
    const float eps = 1e-8f;
    r.par = 0;
    const float dd[3] = {d.x, d.y, d.z};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        if (fabsf(dd[a]) < eps) {
            r.par |= 1u << a;
            r.inv[a] = 0.0;
        } else {
            r.inv[a] = 1.0 / (double)dd[a];
        }
    }
    return r;
}

// intersectAABB(ray, box, tmin, tmax) — double slabs, reference compare/swap order.
__device__ __forceinline__ bool box_hit(const RayPre& r, float mnx, float mny, float mnz, float mxx,
                                        float mxy, float mxz, double tmin, double tmax) {
    double t0 = tmin, t1 = tmax;
    const float mn[3] = {mnx, mny, mnz}, mx[3] = {mxx, mxy, mxz};
    const float o[3] = {r.o.x, r.o.y, r.o.z};
    bool ok = true;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        if (r.par & (1u << a)) {
            ok = ok && !(o[a] < mn[a] || o[a] > mx[a]);
        } else {
            double tn = ((double)mn[a] - r.od[a]) * r.inv[a];
            double tf = ((double)mx[a] - r.od[a]) * r.inv[a];
            if (tn > tf) {
                const double tmp = tn;
                tn = tf;
                tf = tmp;
            }
            if (tn > t0) t0 = tn;
            if (tf < t1) t1 = tf;
            ok = ok && !(t0 > t1);  // monotone: an early return gives the same boolean
        }
    }
    return ok;
}

// Möller–Trumbore of intersectTriangle (query.h:72-108) with e1 = v1-v0, e2 = v2-v0
// precomputed on the host (same float subtraction).  Returns hit and t/u/v.
__device__ __forceinline__ bool mt_g(const RayPre& r, f3 v0, f3 e1, f3 e2, float tmin, float tmax,
                                     float& t_out, float& u_out, float& v_out) {
    const f3 pvec = cross(r.d, e2);
    const float det = dot(e1, pvec);
    if (fabsf(det) < 1e-8f) return false;
    const float invDet = 1.0f / det;
    const f3 tvec = sub(r.o, v0);
    const float u = dot(tvec, pvec) * invDet;
    if (u < 0.0f || u > 1.0f) return false;
    const f3 qvec = cross(tvec, e1);
    const float v = dot(r.d, qvec) * invDet;
    if (v < 0.0f || (u + v) > 1.0f) return false;
    const float t = dot(e2, qvec) * invDet;
    if (t < tmin || t > tmax) return false;
    t_out = t;
    u_out = u;
    v_out = v;
    return true;
}

// HW1 ray_intersection (HW1/include/ray.h:67-104): eps = FLT_EPSILON, t >= 0, no tmax.
__device__ __forceinline__ bool mt_hw1(f3 o, f3 d, f3 v0, f3 e1, f3 e2, float& t_out, float& u_out,
                                       float& v_out) {
    const f3 pvec = cross(d, e2);
    const float det = dot(pvec, e1);
    if (fabsf(det) < FLT_EPSILON) return false;
    const float invDet = 1.0f / det;  // == (float)(1.0 / (double)det)
    const f3 tvec = sub(o, v0);
    const float u = dot(tvec, pvec) * invDet;
    if (u < 0.0f || u > 1.0f) return false;
    const f3 qvec = cross(tvec, e1);
    const float v = dot(d, qvec) * invDet;
    if (v < 0.0f || (u + v) > 1.0f) return false;
    const float t = dot(e2, qvec) * invDet;
    if (t < 0.0f) return false;
    t_out = t;
    u_out = u;
    v_out = v;
    return true;
}

// Hit-record completion of intersectTriangle (query.h:110-127) for the winning triangle.
__device__ __forceinline__ void hit_frame(const RayPre& r, f3 e1, f3 e2, f3 n0, f3 n1, f3 n2, float t,
                                          float u, float v, f3& p, f3& shadingN) {
    p = add(r.o, scale(r.d, t));
    f3 geomN = unit(cross(e1, e2));
    const bool front = dot(r.d, geomN) < 0.0f;
    if (!front) geomN = neg(geomN);
    const float w = 1.0f - u - v;
    f3 sN = add(add(scale(n0, w), scale(n1, u)), scale(n2, v));
    if (dot(sN, sN) < 1e-12f) {
        sN = geomN;
    } else {
        sN = unit(sN);
        if (dot(sN, geomN) < 0.0f) sN = neg(sN);
    }
    shadingN = sN;
}

// G/include/query.h:32-48
__device__ __forceinline__ float rng_next(uint32_t& state) {
    state = state * 1664525u + 1013904223u;
    uint32_t h = state;
    h = (h ^ 61u) ^ (h >> 16u);
    h *= 9u;
    h ^= h >> 4u;
    h *= 0x27d4eb2du;
    h ^= h >> 15u;
    return (float)h / (float)0xFFFFFFFFu;
}
__device__ __forceinline__ uint32_t make_rng_seed(int x, int y, int s) {
    return (uint32_t)x * 73856093u ^ (uint32_t)y * 19349663u ^ (uint32_t)s * 83492791u;
}
__device__ __forceinline__ f3 random_unit_vector(uint32_t& st) {
    for (;;) {
        const float x = 2.0f * rng_next(st) - 1.0f;
        const float y = 2.0f * rng_next(st) - 1.0f;
        const float z = 2.0f * rng_next(st) - 1.0f;
        const float lensq = x * x + y * y + z * z;
        if (lensq > 1e-10f && lensq <= 1.0f) {
            const float inv = 1.0f / sqrtf(lensq);
            return mk(x * inv, y * inv, z * inv);
        }
    }
}

__device__ __forceinline__ f3 clamp01(f3 c) {  // shader.h:24-32
    if (c.x > 1.0f) c.x = 1.0f;
    if (c.y > 1.0f) c.y = 1.0f;
    if (c.z > 1.0f) c.z = 1.0f;
    if (c.x < 0.0f) c.x = 0.0f;
    if (c.y < 0.0f) c.y = 0.0f;
    if (c.z < 0.0f) c.z = 0.0f;
    return c;
}

}  // namespace rtd
