// rt_hw1.hip — the HW1 path on gfx950 (HW1/src/render.cpp:72-116: every triangle for every
// camera ray, the closest t >= 0 with the first index winning ties, HW1 shade
// HW1/include/raytracer.h:21-48; ray_intersection HW1/include/ray.h:67-117), and its C ABI:
// rt_render_hw1[_ex] (brute force or binned, synchronous), the resident rt_hw1_scene
// (rt_render_hw1_device: the C2 configuration's binned, chunked pipeline) and its
// pipelined host delivery (rt_render_hw1_deliver / rt_hw1_wait).  Split out of rt_device.hip in
// round 6; it shares only the wave primitives (rt_wave.hpp) with it.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>

#include "rt_common.hpp"
#include "rt_hip_host.hpp"
#include "rt_math.hpp"
#include "rt_ppm.hpp"
#include "rt_dma.hpp"

using namespace rtd;

namespace {

constexpr int BLOCK = 256;  // threads per block (rt_device.hip's render blocks are the same size)

#include "rt_wave.hpp"

// ---- HW1 brute force (HW1/src/render.cpp:72-116) ----------------------------------------
// The camera-only half of hw1_rect's bounds: the ray direction D = pixel00 + ix du + iy dv -
// center over the image's (ix, iy) range per axis, padded for its float evaluation, and |D|'s
// bounds.  The same for every triangle of a frame, so the host makes it once per frame; the same
// double operations in the same order (-ffp-contract=off on both sides) as the device made them
// per triangle before round 6.
struct Hw1Cam {
    double du[3], dv[3], D00[3], Dl[3], Dh[3], pad[3], nmin, nmax;
};
__host__ __device__ inline Hw1Cam hw1_cam_bounds(const float center[3], const float p00[3], const float pdu[3],
                                                 const float pdv[3], int W, int H) {
    Hw1Cam o;
    const int X0 = -2, X1 = W + 1, Y0 = -2, Y1 = H + 1;  // ix in [x, x+1] (truncation)
    const double cc[3] = {center[0], center[1], center[2]}, p0[3] = {p00[0], p00[1], p00[2]};
    for (int a = 0; a < 3; ++a) {
        o.du[a] = pdu[a];
        o.dv[a] = pdv[a];
    }
    const double xm = fmax(fabs((double)X0), fabs((double)X1)), ym = fmax(fabs((double)Y0), fabs((double)Y1));
    double scale = 0.0;
    for (int a = 0; a < 3; ++a) {
        o.D00[a] = p0[a] - cc[a];
        const double u0 = X0 * o.du[a], u1 = X1 * o.du[a], w0 = Y0 * o.dv[a], w1 = Y1 * o.dv[a];
        o.Dl[a] = o.D00[a] + fmin(u0, u1) + fmin(w0, w1);
        o.Dh[a] = o.D00[a] + fmax(u0, u1) + fmax(w0, w1);
        o.pad[a] = 8.0 * 0x1p-23 * (fabs(cc[a]) + fabs(p0[a]) + xm * fabs(o.du[a]) + ym * fabs(o.dv[a]));
        scale = fmax(scale, fmax(fabs(o.Dl[a]), fabs(o.Dh[a])));
    }
    double nmin2 = 0.0, nmax2 = 0.0;
    for (int a = 0; a < 3; ++a) {
        o.pad[a] += 1e-5 * scale;
        o.Dl[a] -= o.pad[a];
        o.Dh[a] += o.pad[a];
        const double near = o.Dl[a] > 0 ? o.Dl[a] : (o.Dh[a] < 0 ? o.Dh[a] : 0.0);
        const double far = fmax(fabs(o.Dl[a]), fabs(o.Dh[a]));
        nmin2 += near * near;
        nmax2 += far * far;
    }
    o.nmin = sqrt(nmin2) * (1 - 1e-12);
    o.nmax = sqrt(nmax2) * (1 + 1e-12);
    return o;
}

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
    // chunked path (rt_render_hw1_device): work items of at most 2^chunk_log2 list entries
    const uint32_t* __restrict__ chunk_tile;   // per chunk: its tile
    const uint32_t* __restrict__ chunk_first;  // per tile: its first chunk (exclusive prefix; [ntiles] = total)
    uint32_t chunk_cap;                         // chunk_tile's entries
    unsigned long long* __restrict__ keys;      // per (pixel, sample): min over chunks of (t bits << 32 | index)
    uint32_t* zero_counts;  // counts | cursor | done (3 * ntiles): each tile's resolving item zeroes its own
                            // entries for the lane's next frame (after every item of the tile read them)
    int32_t ntiles;
    int32_t chunk_log2;  // work item size (RT_TUNE_HW1_CHUNK)
    Hw1Cam cb;           // the frame's camera bounds for hw1_rect (binned path)
};

// The scan's outputs (hw1_scan_chunks_kernel's arguments, for the scan fused into the count pass).
struct Hw1Scan {
    uint32_t* offsets;       // ntiles + 1
    int32_t n;               // tiles
    uint32_t list_cap;
    uint32_t* chunk_first;   // ntiles + 1
    uint32_t* chunk_tile;    // chunk_cap
    uint32_t chunk_cap;
    unsigned long long* total_out;  // host: tag << 32 | list total
    uint32_t tag;
    uint32_t* arrive;        // blocks done counting (zeroed again by the last)
    int32_t chunk_log2;
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
    // D over the image, per axis, padded as in tile_dirs: the frame's own (hw1_cam_bounds)
    const double* D00 = P.cb.D00;
    const double* Dl = P.cb.Dl;
    const double* Dh = P.cb.Dh;
    const double* pad = P.cb.pad;
    const double* du = P.cb.du;
    const double* dv = P.cb.dv;
    const double nmin = P.cb.nmin, nmax = P.cb.nmax;
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
// 32 entries (the default; RT_TUNE_HW1_CHUNK): c2 0.0399-0.0411 ms per step against 0.0420-0.0422
// with 64, 0.0426 with 16, 0.0465 with 128 (profiles/r06/exp/hw1_chunk/)
constexpr int HW1_CHUNK_LOG2 = 5;

// A tile's work items: one per 2^lg listed entries, or one brute-force item for a list that does
// not fit the capacity; one item with no triangles for an empty tile (no triangle's rectangle
// meets it: every sample misses, and the item resolves the tile).
__device__ __forceinline__ uint32_t hw1_tile_chunks(uint32_t off, uint32_t c, uint32_t list_cap, int lg) {
    return c == 0 ? 1u : (off + c > list_cap ? 1u : (c + (1u << lg) - 1) >> lg);
}

// Inclusive sum of v over a 1024-thread block: a shuffle scan per wave, then the 16 wave totals
// through LDS (two barriers; wsum is free again on return).
__device__ __forceinline__ uint32_t hw1_block_scan(uint32_t v, uint32_t* wsum) {
    const int t = (int)threadIdx.x, lane = t & 63, w = t >> 6;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t u = (uint32_t)__shfl_up((int)v, d);
        if (lane >= d) v += u;
    }
    if (lane == 63) wsum[w] = v;
    __syncthreads();
    uint32_t base = 0;
    for (int i = 0; i < w; ++i) base += wsum[i];
    __syncthreads();
    return v + base;
}

// Inclusive sum of v over the wave's lanes.
__device__ __forceinline__ uint32_t hw1_wave_incl(uint32_t v, uint32_t lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t u = (uint32_t)__shfl_up((int)v, d);
        if ((int)lane >= d) v += u;
    }
    return v;
}

// Exclusive prefix sum of n counts in one workgroup (n is the number of wave tiles); offsets[n] =
// total.  With chunk_first: the same over the tiles' chunk counts, and every chunk's tile in
// chunk_tile (at most chunk_cap; chunks past it are not written, the total in chunk_first[n] says
// how many there were).  total_out (host memory, may be null): the list total, stored from here
// with the frame's tag in the high half for the host's capacity check (a 4-byte copy on the
// frame's stream after the kernels held every frame for its own latency; the tag tells the host
// the total is this frame's without asking the runtime).  Each thread takes PER consecutive tiles, kept in registers (PER 0:
// any number, re-read).
template <int PER>
__global__ __launch_bounds__(1024) void hw1_scan_chunks_kernel(const uint32_t* __restrict__ counts,
                                                               uint32_t* __restrict__ offsets, int n, uint32_t list_cap,
                                                               uint32_t* __restrict__ chunk_first,
                                                               uint32_t* __restrict__ chunk_tile, uint32_t chunk_cap,
                                                               unsigned long long* total_out, uint32_t tag,
                                                               int chunk_log2) {
    __shared__ uint32_t wsum[16];
    const int t = (int)threadIdx.x;
    const int per = PER > 0 ? PER : (n + 1023) / 1024;
    const int lo = min(n, t * per), hi = min(n, lo + per);
    uint32_t c[PER > 0 ? PER : 1];
    uint32_t sum = 0;
    if constexpr (PER > 0) {
#pragma unroll
        for (int j = 0; j < PER; ++j) {  // the loads first, all in flight together
            c[j] = lo + j < hi ? counts[lo + j] : 0u;
            sum += c[j];
        }
    } else {
        for (int i = lo; i < hi; ++i) sum += counts[i];
    }
    auto cnt = [&](int j) {
        if constexpr (PER > 0) return c[j];
        else return counts[lo + j];
    };
    const int m = PER > 0 ? PER : per;
    const uint32_t incl = hw1_block_scan(sum, wsum);
    // the tiles' chunk counts need the tiles' offsets (a list past the capacity: one chunk)
    uint32_t run = incl - sum, csum = 0;
#pragma unroll 32
    for (int j = 0; j < m; ++j) {
        if (lo + j < hi) {
            const uint32_t cj = cnt(j);
            offsets[lo + j] = run;
            csum += hw1_tile_chunks(run, cj, list_cap, chunk_log2);
            run += cj;
        }
    }
    if (t == 1023) {
        offsets[n] = incl;
        if (total_out)
            __hip_atomic_store(total_out, (unsigned long long)tag << 32 | incl, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
    const uint32_t cincl = hw1_block_scan(csum, wsum);
    uint32_t crun = cincl - csum;
    run = incl - sum;
#pragma unroll 32
    for (int j = 0; j < m; ++j) {
        if (lo + j < hi) {
            const uint32_t cj = cnt(j);
            chunk_first[lo + j] = crun;
            const uint32_t nc = hw1_tile_chunks(run, cj, list_cap, chunk_log2);
            for (uint32_t k = 0; k < nc; ++k)
                if (crun + k < chunk_cap) chunk_tile[crun + k] = (uint32_t)(lo + j);
            crun += nc;
            run += cj;
        }
    }
    if (t == 1023) chunk_first[n] = cincl;
}

// The list offsets and work items of n tiles, by one wave (the fused form of
// hw1_scan_chunks_kernel, for n <= 64 * PER): lane l takes PER consecutive tiles, loaded together.
template <int PER>
__device__ __forceinline__ void hw1_wave_scan_tiles(const uint32_t* counts, const Hw1Scan& S, uint32_t lane) {
    const int lo = min(S.n, (int)lane * PER), hi = min(S.n, lo + PER);
    uint32_t c[PER];
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {  // (the other blocks' counts: atomics, read at the coherence point)
        c[j] = lo + j < hi ? __hip_atomic_load(&counts[lo + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        sum += c[j];
    }
    const uint32_t incl = hw1_wave_incl(sum, lane);
    uint32_t run = incl - sum, csum = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        if (lo + j < hi) {
            S.offsets[lo + j] = run;
            csum += hw1_tile_chunks(run, c[j], S.list_cap, S.chunk_log2);
            run += c[j];
        }
    }
    if (lane == 63) {
        S.offsets[S.n] = incl;
        if (S.total_out)
            __hip_atomic_store(S.total_out, (unsigned long long)S.tag << 32 | incl, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
    const uint32_t cincl = hw1_wave_incl(csum, lane);
    uint32_t crun = cincl - csum;
    run = incl - sum;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        if (lo + j < hi) {
            S.chunk_first[lo + j] = crun;
            const uint32_t nc = hw1_tile_chunks(run, c[j], S.list_cap, S.chunk_log2);
            for (uint32_t k = 0; k < nc; ++k)
                if (crun + k < S.chunk_cap) S.chunk_tile[crun + k] = (uint32_t)(lo + j);
            crun += nc;
            run += c[j];
        }
    }
    if (lane == 63) S.chunk_first[S.n] = cincl;
}

// Pass 1: each triangle's rectangle (kept for pass 2) and its count in every tile it meets.
// (Launched with 64-thread blocks: one wave each.)  SCAN_PER > 0: the scan fused in -- the last
// block to finish counting (an arrival counter after a release fence) scans the counts
// (hw1_wave_scan_tiles), so the frame has no kernel boundary and no launch between the passes.
template <int SCAN_PER>
__global__ __launch_bounds__(64) void hw1_rect_count_kernel(Hw1Params P, int4* __restrict__ rects,
                                                            uint32_t* __restrict__ counts, Hw1Scan S) {
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
    if constexpr (SCAN_PER > 0) {
        // the hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, valid forms: 4-byte agent
        // atomics both sides): every block's count atomics have completed (vmcnt) before its
        // arrival add, and the block whose add came last reads the counts with sc1 loads only
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint32_t prev = 0;
        if (lane == 0) prev = atomicAdd(S.arrive, 1u);
        if (uni((uint32_t)__shfl((int)prev, 0)) + 1 != gridDim.x) return;
        if (lane == 0) *S.arrive = 0u;  // for the lane's next frame
        hw1_wave_scan_tiles<SCAN_PER>(counts, S, lane);
    }
}

// One sample of pixel (x, y) from its winner key (~0: no hit): the accepting test's own t, u, v
// (mt_hw1 again), HW1 shade (HW1/include/raytracer.h:21-48), the AOVs.
__device__ __forceinline__ f3 hw1_resolve_sample(const Hw1Params& P, int x, int y, int s, unsigned long long key,
                                                 f3 o, f3 d) {
    const bool hit = key != ~0ull;
    const int32_t besti = hit ? (int32_t)(uint32_t)key : -1;
    f3 p = mk(0.f, 0.f, 0.f), n = p;
    float best = FLT_MAX;
    if (hit) {
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
    if (P.hit_idx) {
        const size_t kk = ((size_t)y * P.W + x) * (size_t)P.spp + (size_t)s;
        P.hit_idx[kk] = besti;
        P.hit_t[kk] = hit ? best : -1.0f;
    }
    return shade_hw1(o, d, hit, p, n, P.lpos, P.lcol);
}

// The camera ray of sample s of pixel (x, y) (HW1/src/render.cpp:95-104: the jittered position
// truncated by get_pixel_position(int, int), the direction normalised as HW1's Ray does, ray.h:25).
__device__ __forceinline__ f3 hw1_dir(const Hw1Params& P, int x, int y, int s) {
    const float pxs = (float)x + P.jitter[2 * s];
    const float pys = (float)y + P.jitter[2 * s + 1];
    const int ix = (int)pxs, iy = (int)pys;
    const f3 pix = add(add(P.p00, scale(P.du, (float)ix)), scale(P.dv, (float)iy));
    return unit(sub(pix, P.center));
}

// One wave per work item, grid-stride over the frame's items: the tile's 64 pixel lanes run mt_hw1
// over the item's chunk of the tile's list and keep each sample's winner as the key
// (t bits << 32 | index).  t >= 0 and never -0 (t + 0.0f), so its bits order like its value; the
// minimum over a tile's chunks is the lexicographic (t, index) minimum of its whole list -- the
// brute-force loop's winner (rec.t < prev.t keeps the first index).  The frame's resolve is fused
// in: a tile of one item (its whole list, an empty list, or the brute-force item of a list past
// the capacity) shades its samples from the keys in registers; a tile of several items folds its
// keys into `keys` with a 64-bit atomicMin and counts its finished items, and the item finishing
// last reads the keys back (agent-scope atomic loads, after every item's atomics completed),
// shades, and resets them.  The tile's counters are left zeroed for the lane's next frame.
// (FUSED false: every item folds its keys with atomicMin and hw1_resolve_kernel resolves.)
template <bool FUSED>
__global__ __launch_bounds__(BLOCK) void render_hw1_chunks_kernel(Hw1Params P) {
    const uint32_t total = uni(P.chunk_first[P.ntiles]);
    const uint32_t nitems = total < P.chunk_cap ? total : P.chunk_cap;
    const int tiles_x = (P.W + HW1_TW - 1) / HW1_TW;
    const uint32_t lane = lane_id();
    const uint32_t waves = gridDim.x * (BLOCK / 64);
    uint32_t* const cursor = P.zero_counts + P.ntiles;
    uint32_t* const done = P.zero_counts + 2 * P.ntiles;
    for (uint32_t j = blockIdx.x * (BLOCK / 64) + threadIdx.x / 64; j < nitems; j += waves) {
        const uint32_t tidx = uni(P.chunk_tile[uni(j)]);
        const uint32_t first = uni(P.chunk_first[tidx]);
        const uint32_t items = uni(P.chunk_first[tidx + 1]) - first;
        const uint32_t c = j - first;
        const uint32_t cnt = uni(P.bin_count[tidx]);
        const uint32_t off = uni(P.bin_offset[tidx]);
        const bool all = cnt > 0 && off + cnt > P.list_cap;  // the list was not written: every triangle, in order
        const uint32_t b = all ? 0u : c << P.chunk_log2;
        const uint32_t e = all ? (uint32_t)P.num_tris : min(cnt, b + (1u << P.chunk_log2));
        const int x = (int)(tidx % tiles_x) * HW1_TW + (int)(lane % HW1_TW);
        const int y = (int)(tidx / tiles_x) * HW1_TH + (int)(lane / HW1_TW);
        const bool valid = x < P.W && y < P.H;
        const bool single = FUSED && items == 1;
        const f3 o = P.center;
        f3 acc = mk(0.f, 0.f, 0.f);
        for (int s = 0; s < P.spp; ++s) {
            const f3 d = hw1_dir(P, x, y, s);
            unsigned long long best = ~0ull;
            // the item's triangle indices, 64 at a time, lane l holding entry ib + l (one
            // coalesced load, then v_readlane: the triangles' scalar loads wait on no second
            // round trip)
            uint32_t idx = 0, ib = b;
            for (uint32_t i = b; i < e; i += 4) {
                if (((i - b) & 63u) == 0) {
                    ib = i;
                    const uint32_t j = i + lane;
                    idx = all ? j : (j < e ? P.bin_list[off + j] : 0u);
                }
                int kk[4];
                float4 tq[12];
#pragma unroll
                for (int q = 0; q < 4; ++q) kk[q] = i + q < e ? (int)rdlane(idx, i + q - ib) : -1;
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
            if (single) {
                if (valid) acc = add(acc, hw1_resolve_sample(P, x, y, s, best, o, d));
            } else if (valid && best != ~0ull) {
                atomicMin(&P.keys[((size_t)y * P.W + x) * (size_t)P.spp + (size_t)s], best);
            }
        }
        bool resolve = single;
        if (FUSED && !single) {
            // the hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, valid forms: 8-byte
            // agent atomics both sides; no fences): this wave's key atomics have completed (vmcnt)
            // before its count, and the wave whose count came last reads the keys with sc1 loads
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            uint32_t prev = 0;
            if (lane == 0) prev = atomicAdd(&done[tidx], 1u);
            resolve = uni((uint32_t)__shfl((int)prev, 0)) + 1 == items;
            if (resolve) {
                for (int s = 0; s < P.spp && valid; ++s) {
                    unsigned long long* kp = &P.keys[((size_t)y * P.W + x) * (size_t)P.spp + (size_t)s];
                    const unsigned long long key = __hip_atomic_load(kp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    *kp = ~0ull;
                    acc = add(acc, hw1_resolve_sample(P, x, y, s, key, o, hw1_dir(P, x, y, s)));
                }
            }
        }
        if (resolve) {
            if (valid) hw1_write_pixel(P, x, y, acc);
            if (lane == 0) {  // (every item of the tile has read its count)
                P.zero_counts[tidx] = 0u;
                cursor[tidx] = 0u;
                done[tidx] = 0u;
            }
        }
    }
}

// The unfused resolve: per pixel, each sample's winner from keys (then reset for the next
// frame), HW1 shade, the average, AOVs; the first threads also zero the tiles' counts and cursors
// for the lane's next frame.
__global__ __launch_bounds__(BLOCK) void hw1_resolve_kernel(Hw1Params P) {
    const int gid = (int)(blockIdx.x * BLOCK + threadIdx.x);
    if (gid < 2 * P.ntiles) P.zero_counts[gid] = 0u;
    if (gid >= P.W * P.H) return;
    const int x = gid % P.W, y = gid / P.W;
    f3 acc = mk(0.f, 0.f, 0.f);
    for (int s = 0; s < P.spp; ++s) {
        const size_t kk = (size_t)gid * (size_t)P.spp + (size_t)s;
        const unsigned long long key = P.keys[kk];
        P.keys[kk] = ~0ull;
        acc = add(acc, hw1_resolve_sample(P, x, y, s, key, P.center, hw1_dir(P, x, y, s)));
    }
    hw1_write_pixel(P, x, y, acc);
}

}  // namespace

using rt::set_error;
using rt::hip_msg;
using rt::DevBuf;
using rt::check_device;
using rt::DeviceGuard;

extern "C" int rt_render_hw1(int device, const rt_vec3* pos, const rt_vec3* nrm, const uint32_t* idx, size_t P,
                             const rt_camera* cam, rt_vec3 lpos, rt_vec3 lcol, int spp, const float* jitter,
                             float* rgb_host, int32_t* hit_idx_host, float* hit_t_host) {
    return rt_render_hw1_ex(device, pos, nrm, idx, P, cam, lpos, lcol, spp, jitter, 0, rgb_host, hit_idx_host,
                            hit_t_host, nullptr);
}

// ---- HW1 resident scene (the C2 configuration's device path) ---------------------------
// The mesh packed once (v0, e1, e2 as ray_intersection computes them, the three normals per
// triangle), the binning buffers kept across frames.  A frame is five launches (rect + count,
// scan, fill, render, resolve) and no host synchronisation: the bin list's capacity is checked
// on the device (a tile whose list would not fit takes the brute-force loop), and the host grows
// it from the latest finished frame's total.
struct rt_hw1_scene {
    int device = 0;
    size_t P = 0;
    DevBuf tri, nrm, jitter;
    // A lane: one frame's binning state.  Direct frames (rt_render_hw1_device) use lane 0 on the
    // caller's stream; delivered frames alternate over the kLanes lanes, each on a stream of its
    // own, so one frame's latency-bound passes (rect + count, the one-workgroup scan and fill:
    // ~60 of the frame's ~97 us with a fraction of the CUs busy) run beside the other frame's
    // render kernel.  Every frame still runs all five passes over its own buffers.
    struct Lane {
        DevBuf rects, bins, list;
        DevBuf chunks;             // chunk_first (ntiles + 1) | chunk_tile (chunk_cap)
        DevBuf keys;               // per (pixel, sample): the chunked pass's winners, kept at ~0 between frames
        int bins_tiles = -1;       // tiles the bins buffer is laid out for
        size_t keys_n = 0;         // samples the keys buffer holds
        uint32_t list_cap = 0, chunk_cap = 0;
        hipStream_t own = nullptr;          // delivered frames' stream (made on first use)
        hipStream_t last_stream = nullptr;  // the stream of the lane's latest frame
        uint64_t last_frame = 0;
        bool used = false;
        int chunk_log2 = -1;       // the item size the chunk table is laid out for
    };
    static constexpr int kLanes = 8;
    Lane lane[kLanes];
    int jitter_spp = -1;
    std::vector<float> jitter_host;
    bool jitter_default = false;  // jitter_host is jittered_samples(jitter_spp, 42)
    static constexpr int kRing = 64;
    hipEvent_t e0[kRing] = {}, e1[kRing] = {};
    hipEvent_t f1[kRing] = {};  // the frame's end, no timestamp
    // the frame's end event: e1 on timed frames, f1 otherwise; set by the frame's last dispatch
    // itself (its stop event), so no marker packet sits between two frames' kernels
    hipEvent_t end_of(int sl) const { return timed[sl] ? e1[sl] : f1[sl]; }
    hipEvent_t frame_end(uint64_t f) const { return end_of(int(f % kRing)); }
    // e0 / e1 (the kernels' start and end timestamps) are recorded for every direct frame but for
    // one delivered frame in RT_TUNE_KERNEL_TIMING_EVERY: a timing event between two kernels holds
    // the next one's dispatch until the previous has completed and the timestamp is written
    // (DESIGN.md §4.13); f1 marks every frame's end without a timestamp
    bool timed[kRing] = {};
    int lane_of[kRing] = {};  // the lane of frame f at [f % kRing]
    bool in_deliver = false;  // rt_render_hw1_deliver is calling render_frame
    unsigned long long* total_host = nullptr;  // pinned: frame f's tag (f mod 2^32) << 32 | its list total, at [f % kRing]
    uint64_t frames = 0;
    const char* last_kernel = "";
    // rt_render_hw1_deliver: frames rendered into a ring of kDeliver device P6 bodies, each body
    // copied to the caller's host buffer on the copy stream while the next frames render
    static constexpr int kDeliver = 8;
    DevBuf dp6[kDeliver];
    // the copies: SDMA (copy_mode 1: a copier thread queues each body on a DMA engine once its
    // frame's end event has fired; dma_done[ticket % kRing] drops to 0 when it has landed), or
    // the HIP runtime's on the copy stream (copy_mode 0: blit kernels on the CUs beside the next
    // frame's; cdone[ticket % kRing] fires when it has landed); -1 until the first delivery
    int copy_mode = -1;
    std::unique_ptr<rt_dma::DmaCopier> dma;
    hsa_signal_t dma_done[kRing] = {};
    bool dma_pending[kRing] = {};
    hipStream_t copy = nullptr;
    hipEvent_t cdone[kRing] = {};  // per ticket: copied
    hipEvent_t caller = nullptr;   // the caller's stream's pending work, for a lane to wait on
    uint64_t tickets = 0;
    // ticket t's body is in host memory
    int wait_copy(uint64_t t) {
        const int r = int(t % kRing);
        if (copy_mode == 1) {
            if (dma_pending[r]) {
                (void)rt_dma::hsa().signal_wait(dma_done[r], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
                dma_pending[r] = false;
            }
            std::string msg;
            const int rc = dma->error(&msg);
            return rc == RT_OK ? RT_OK : set_error(rc, msg);
        }
        if (copy_mode == 0) HIP_TRY(hipEventSynchronize(cdone[r]));
        return RT_OK;
    }
    // every frame of lane L is done (a lane's frames are ordered: one stream, or a wait)
    hipError_t sync_lane(const Lane& L) const { return L.used ? hipEventSynchronize(frame_end(L.last_frame)) : hipSuccess; }
    hipError_t sync_all() const {
        for (const Lane& L : lane) {
            const hipError_t e = sync_lane(L);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    ~rt_hw1_scene() {
        (void)sync_all();
        for (int i = 0; i < kRing; ++i)  // SDMA copies still reading the bodies
            if (dma_pending[i])
                (void)rt_dma::hsa().signal_wait(dma_done[i], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
        dma.reset();  // (the copier thread queries the frames' events)
        for (int i = 0; i < kRing; ++i)
            if (dma_done[i].handle) (void)rt_dma::hsa().signal_destroy(dma_done[i]);
        for (int i = 0; i < kRing; ++i) {
            if (e0[i]) (void)hipEventDestroy(e0[i]);
            if (e1[i]) (void)hipEventDestroy(e1[i]);
            if (f1[i]) (void)hipEventDestroy(f1[i]);
            if (cdone[i]) (void)hipEventSynchronize(cdone[i]);
            if (cdone[i]) (void)hipEventDestroy(cdone[i]);
        }
        if (caller) (void)hipEventDestroy(caller);
        for (Lane& L : lane)
            if (L.own) (void)hipStreamDestroy(L.own);
        if (copy) (void)hipStreamDestroy(copy);
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
    for (rt_hw1_scene::Lane& L : s->lane) {
        if ((rc = L.rects.alloc(P * sizeof(int4))) != RT_OK) return rc;
        // a first capacity: a few tiles per triangle (grown from the frames' totals)
        L.list_cap = uint32_t(std::min<size_t>(std::max<size_t>(4 * P, size_t(1) << 16), 0x7FFFFFFFull));
        if ((rc = L.list.alloc(size_t(L.list_cap) * sizeof(uint32_t))) != RT_OK) return rc;
    }
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&s->total_host), rt_hw1_scene::kRing * sizeof(unsigned long long),
                          hipHostMallocCoherent));
    for (int i = 0; i < rt_hw1_scene::kRing; ++i) {
        s->total_host[i] = ~0ull;  // (no frame's tag)
        HIP_TRY(hipEventCreate(&s->e0[i]));
        HIP_TRY(hipEventCreate(&s->e1[i]));
        HIP_TRY(hipEventCreateWithFlags(&s->f1[i], hipEventDisableTiming));
    }
    *out = s.release();
    return RT_OK;
}

extern "C" void rt_hw1_scene_destroy(rt_hw1_scene* s) {
    if (!s) return;
    DeviceGuard g(s->device);
    delete s;
}

// One frame on lane li, on stream st (rt_render_hw1_device: lane 0, the caller's stream;
// rt_render_hw1_deliver: the lanes in turn, each on its own stream).
static int render_frame(rt_hw1_scene* s, int li, const rt_camera* cam, rt_vec3 lpos, rt_vec3 lcol, int spp,
                        const float* jitter, int flags, float* rgb_dev, uint8_t* p6_dev, int32_t* hit_idx_dev,
                        float* hit_t_dev, hipStream_t st) {
    const int W = cam->pixel_width, H = cam->pixel_height;
    rt_hw1_scene::Lane& L = s->lane[li];
    int rc;
    // jitter_samples(spp, 42u) offsets in [0,1) (HW1/include/antialias.h:12-27), or the caller's
    // (the default table of the scene's current spp is already uploaded: nothing to make)
    const bool have_default = !jitter && s->jitter_default && s->jitter_spp == spp;
    std::vector<float> tab;
    if (!have_default) {
        tab.resize(2 * size_t(spp));
        if (jitter) std::memcpy(tab.data(), jitter, tab.size() * sizeof(float));
        else if ((rc = rt_jittered_samples(spp, 42u, 0, tab.data())) != RT_OK) return rc;
    }
    if (!have_default && (s->jitter_spp != spp || s->jitter_host != tab)) {
        HIP_TRY(s->sync_all());  // every lane's frames read the table
        if ((rc = s->jitter.upload(tab.data(), tab.size() * sizeof(float))) != RT_OK) return rc;
        s->jitter_spp = spp;
        s->jitter_host = tab;
    }
    if (!have_default) s->jitter_default = jitter == nullptr;
    const bool brute = (flags & RT_HW1_BRUTE) != 0;
    const int ntiles = ((W + HW1_TW - 1) / HW1_TW) * ((H + HW1_TH - 1) / HW1_TH);
    // the list total of the latest frame whose scan has run (each total carries its frame's tag:
    // read from pinned memory, no runtime call)
    for (uint64_t b = 1; b <= std::min<uint64_t>(s->frames, uint64_t(rt_hw1_scene::kRing) / 2); ++b) {
        const uint64_t f = s->frames - b;
        const unsigned long long v = __atomic_load_n(&s->total_host[f % rt_hw1_scene::kRing], __ATOMIC_ACQUIRE);
        if (uint32_t(v >> 32) != uint32_t(f)) continue;
        const uint32_t tot = uint32_t(v);
        if (tot > L.list_cap) {  // grow (the old list may still be read by the lane's frames in flight)
            HIP_TRY(s->sync_lane(L));
            L.list_cap = uint32_t(std::min<uint64_t>(uint64_t(tot) + tot / 4 + 1024, 0x7FFFFFFFull));
            if ((rc = L.list.alloc(size_t(L.list_cap) * sizeof(uint32_t))) != RT_OK) return rc;
            L.bins_tiles = -1;  // the chunk table follows the list's capacity
        }
        break;
    }
    const size_t nsamples = size_t(W) * size_t(H) * size_t(spp);
    // work items of 2^lg list entries (RT_TUNE_HW1_CHUNK: 16..256, a power of two)
    int lg = HW1_CHUNK_LOG2;
    {
        const double want = rt::tuning(RT_TUNE_HW1_CHUNK, double(1 << HW1_CHUNK_LOG2));
        while (lg > 4 && double(1 << lg) > want) --lg;
        while (lg < 8 && double(1 << lg) < want) ++lg;
    }
    if (!brute && (L.bins_tiles != ntiles || L.keys_n != nsamples || L.chunk_log2 != lg)) {
        HIP_TRY(s->sync_lane(L));
        // counts | cursor | done (finished items) | arrive | offsets (ntiles + 1): the first four
        // zeroed here, then by every frame's passes (each tile's resolving item, the count pass's
        // last block) for the lane's next
        if ((rc = L.bins.alloc(size_t(4 * ntiles + 2) * sizeof(uint32_t))) != RT_OK) return rc;
        // (on the frame's stream: a null-stream memset is not ordered before a non-blocking
        // stream's kernels)
        HIP_TRY(hipMemsetAsync(L.bins.p, 0, size_t(3 * ntiles + 1) * sizeof(uint32_t), st));
        // items: at most one per 2^lg listed entries plus one per tile
        L.chunk_cap = uint32_t(std::min<uint64_t>((uint64_t(L.list_cap) >> lg) + uint64_t(ntiles) + 1, 0x7FFFFFFFull));
        L.chunk_log2 = lg;
        if ((rc = L.chunks.alloc((size_t(ntiles) + 1 + L.chunk_cap) * sizeof(uint32_t))) != RT_OK) return rc;
        if ((rc = L.keys.alloc(nsamples * sizeof(unsigned long long))) != RT_OK) return rc;
        HIP_TRY(hipMemsetAsync(L.keys.p, 0xFF, nsamples * sizeof(unsigned long long), st));
        L.bins_tiles = ntiles;
        L.keys_n = nsamples;
    }
    Hw1Params hp;
    hp.tri = static_cast<const float4*>(s->tri.p);
    hp.nrm = static_cast<const float4*>(s->nrm.p);
    hp.num_tris = int32_t(s->P);
    hp.center = f3{cam->center.x, cam->center.y, cam->center.z};
    hp.p00 = f3{cam->pixel00_loc.x, cam->pixel00_loc.y, cam->pixel00_loc.z};
    hp.du = f3{cam->pixel_delta_u.x, cam->pixel_delta_u.y, cam->pixel_delta_u.z};
    hp.dv = f3{cam->pixel_delta_v.x, cam->pixel_delta_v.y, cam->pixel_delta_v.z};
    {
        const float c3[3] = {cam->center.x, cam->center.y, cam->center.z};
        const float p3[3] = {cam->pixel00_loc.x, cam->pixel00_loc.y, cam->pixel00_loc.z};
        const float u3[3] = {cam->pixel_delta_u.x, cam->pixel_delta_u.y, cam->pixel_delta_u.z};
        const float v3[3] = {cam->pixel_delta_v.x, cam->pixel_delta_v.y, cam->pixel_delta_v.z};
        hp.cb = hw1_cam_bounds(c3, p3, u3, v3, W, H);
    }
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
    hp.rects = static_cast<const int4*>(L.rects.p);
    hp.bin_count = hp.bin_offset = hp.bin_list = nullptr;
    hp.list_cap = L.list_cap;
    hp.chunk_first = hp.chunk_tile = nullptr;
    hp.chunk_cap = L.chunk_cap;
    hp.keys = static_cast<unsigned long long*>(L.keys.p);
    hp.zero_counts = static_cast<uint32_t*>(L.bins.p);
    hp.ntiles = ntiles;
    hp.chunk_log2 = lg;
    const int sl = int(s->frames % rt_hw1_scene::kRing);
    // the lane's buffers are shared by its frames: a frame on another stream waits for the last
    if (L.used && st != L.last_stream) HIP_TRY(hipStreamWaitEvent(st, s->frame_end(L.last_frame), 0));
    const uint64_t every = uint64_t(std::clamp(rt::tuning(RT_TUNE_KERNEL_TIMING_EVERY, 4.0), 1.0, 256.0));
    s->timed[sl] = !s->in_deliver || s->frames % every == 0;
    s->lane_of[sl] = li;
    // the timestamps are taken by the first and last dispatches themselves (hipExtLaunchKernel
    // start / stop events), not by event packets between them
    hipEvent_t t0 = s->timed[sl] ? s->e0[sl] : nullptr, t1 = s->end_of(sl);
    const int blocks = ((W + 15) / 16) * ((H + 15) / 16);
    if (brute) {
        __atomic_store_n(&s->total_host[sl], (unsigned long long)uint32_t(s->frames) << 32, __ATOMIC_RELEASE);  // (no list)
        hipExtLaunchKernelGGL(render_hw1_kernel, dim3(blocks), dim3(BLOCK), 0, st, t0, t1, 0, hp);
        s->last_kernel = "render_hw1_kernel";
    } else {
        // one wave per 64 triangles (a block each): the per-triangle passes spread over every CU
        // (256-thread blocks kept c2's 19,858 triangles on 78 CUs: 30 + 25 us)
        const dim3 tgrid(unsigned((s->P + 63) / 64));
        uint32_t* counts = static_cast<uint32_t*>(L.bins.p);  // zeroed by the lane's previous frame
        uint32_t* cursor = counts + ntiles;
        Hw1Scan sc;
        sc.arrive = cursor + 2 * ntiles;  // (after done)
        sc.offsets = sc.arrive + 1;       // ntiles + 1 entries
        sc.n = ntiles;
        sc.list_cap = L.list_cap;
        sc.chunk_first = static_cast<uint32_t*>(L.chunks.p);
        sc.chunk_tile = sc.chunk_first + ntiles + 1;
        sc.chunk_cap = L.chunk_cap;
        sc.total_out = s->total_host + sl;
        sc.tag = uint32_t(s->frames);
        sc.chunk_log2 = lg;
        // the scan fused into the count pass up to 64 x 80 tiles (c2: 4800), else its own
        // 1024-thread kernel (PER tiles per thread in registers: 8 up to 8192 tiles, 32 up to
        // 1080p's 32400); the first launch carries the start event only on timed frames
        const int fuse = int(rt::tuning(RT_TUNE_HW1_FUSE, 2.0));
        const bool fused = (fuse & 1) && ntiles <= 64 * 80;
        auto count = fused ? hw1_rect_count_kernel<80> : hw1_rect_count_kernel<0>;
        int4* rects = static_cast<int4*>(L.rects.p);
        if (t0) hipExtLaunchKernelGGL(count, tgrid, dim3(64), 0, st, t0, nullptr, 0, hp, rects, counts, sc);
        else hipLaunchKernelGGL(count, tgrid, dim3(64), 0, st, hp, rects, counts, sc);
        if (!fused) {
            auto scan = ntiles <= 8 * 1024 ? hw1_scan_chunks_kernel<8>
                        : ntiles <= 32 * 1024 ? hw1_scan_chunks_kernel<32> : hw1_scan_chunks_kernel<0>;
            hipLaunchKernelGGL(scan, dim3(1), dim3(1024), 0, st, counts, sc.offsets, ntiles, L.list_cap,
                               sc.chunk_first, sc.chunk_tile, L.chunk_cap, sc.total_out, sc.tag, lg);
        }
        hp.bin_count = counts;
        hp.bin_offset = sc.offsets;
        hp.bin_list = static_cast<const uint32_t*>(L.list.p);
        hp.chunk_first = sc.chunk_first;
        hp.chunk_tile = sc.chunk_tile;
        hipLaunchKernelGGL(hw1_fill_kernel, tgrid, dim3(64), 0, st, hp, cursor, static_cast<uint32_t*>(L.list.p));
        // items grid-stride over a grid of every CU's worth of waves (the count is on the device),
        // 4,096 waves for 64-entry items and as many more as the items are smaller; the resolve
        // fused in, or its own pass
        const int rblocks = 1024 << std::max(0, 6 - lg);
        if (fuse & 2) {
            hipExtLaunchKernelGGL(render_hw1_chunks_kernel<true>, dim3(rblocks), dim3(BLOCK), 0, st, nullptr, t1, 0, hp);
        } else {
            hipLaunchKernelGGL(render_hw1_chunks_kernel<false>, dim3(rblocks), dim3(BLOCK), 0, st, hp);
            const int rgrid = (std::max(W * H, 2 * ntiles) + BLOCK - 1) / BLOCK;
            hipExtLaunchKernelGGL(hw1_resolve_kernel, dim3(rgrid), dim3(BLOCK), 0, st, nullptr, t1, 0, hp);
        }
        s->last_kernel = (fuse & 2) ? "render_hw1_chunks_kernel<true>" : "render_hw1_chunks_kernel<false>";
    }
    HIP_TRY(hipGetLastError());
    L.used = true;
    L.last_stream = st;
    L.last_frame = s->frames;
    s->frames++;
    return RT_OK;
}

extern "C" int rt_render_hw1_device(rt_hw1_scene* s, const rt_camera* cam, rt_vec3 lpos, rt_vec3 lcol, int spp,
                                    const float* jitter, int flags, float* rgb_dev, uint8_t* p6_dev,
                                    int32_t* hit_idx_dev, float* hit_t_dev, void* stream) {
    if (!s || !cam || spp < 1) return set_error(RT_ERR_ARG, "rt_render_hw1_device: bad argument");
    if ((hit_idx_dev == nullptr) != (hit_t_dev == nullptr)) return set_error(RT_ERR_ARG, "hit_idx and hit_t go together");
    if (cam->pixel_width < 1 || cam->pixel_height < 1) return set_error(RT_ERR_ARG, "camera has no pixels");
    DeviceGuard g(s->device);
    return render_frame(s, 0, cam, lpos, lcol, spp, jitter, flags, rgb_dev, p6_dev, hit_idx_dev, hit_t_dev,
                        static_cast<hipStream_t>(stream));
}

// A frame delivered to host memory (C2's bench step, as rt_renderer delivers G/ frames): the
// frame's P6 body is rendered into ring slot k % kDeliver (after that slot's previous copy), and
// copied on the scene's copy stream once the frame's kernels are done, so the copy of frame k
// overlaps the kernels of frame k+1 instead of following them on one stream (VERDICT r05 item 8:
// 0.129 ms per step against 0.096 of kernels when the caller copied on the render stream).
// Frames alternate over the scene's lanes (RT_TUNE_HW1_LANES), each lane's frames in order on its
// own stream after the work already queued on the caller's stream.
extern "C" int rt_render_hw1_deliver(rt_hw1_scene* s, const rt_camera* cam, rt_vec3 lpos, rt_vec3 lcol, int spp,
                                     int flags, uint8_t* host_p6, void* stream, uint64_t* ticket) {
    if (!s || !cam || !host_p6 || !ticket || spp < 1) return set_error(RT_ERR_ARG, "rt_render_hw1_deliver: bad argument");
    const int W = cam->pixel_width, H = cam->pixel_height;
    if (W < 1 || H < 1) return set_error(RT_ERR_ARG, "camera has no pixels");
    DeviceGuard g(s->device);
    hipStream_t st = static_cast<hipStream_t>(stream);
    int rc;
    if (s->copy_mode < 0) {
        // RT_TUNE_COPY_ENGINE: -1 (default) SDMA when the HSA runtime offers it, 0 the runtime's
        // copies, 1 SDMA or fail
        const int want = int(rt::tuning(RT_TUNE_COPY_ENGINE, -1.0));
        hsa_agent_t ga{0}, ca{0};
        if (want != 0 && rt_dma::hsa_agents(s->device, &ga, &ca)) {
            for (hsa_signal_t& d : s->dma_done)
                if (rt_dma::hsa().signal_create(0, 0, nullptr, &d) != HSA_STATUS_SUCCESS)
                    return set_error(RT_ERR_HIP, "hsa_signal_create failed");
            const double cw = rt::tuning(RT_TUNE_COPY_WAIT, -1.0);
            s->dma = std::make_unique<rt_dma::DmaCopier>(ga, ca, cw == 1.0 || cw < 0.0,
                                                         cw >= 2.0 ? int(std::min(cw, 1000.0)) : 0);
            s->copy_mode = 1;
        } else if (want == 1) {
            return set_error(RT_ERR_UNSUPPORTED, "SDMA delivery unavailable: " + rt_dma::hsa().err);
        } else {
            HIP_TRY(hipStreamCreateWithFlags(&s->copy, hipStreamNonBlocking));
            for (int i = 0; i < rt_hw1_scene::kRing; ++i)
                HIP_TRY(hipEventCreateWithFlags(&s->cdone[i], hipEventDisableTiming));
            s->copy_mode = 0;
        }
    }
    const uint64_t k = s->tickets;
    const int slot = int(k % rt_hw1_scene::kDeliver), ring = int(k % rt_hw1_scene::kRing);
    // (a lane's frames overlap the others' only on a hardware queue of its own: HIP gives a process
    // GPU_MAX_HW_QUEUES of them, 4 by default and shared with the caller's streams.  c2: 2 lanes
    // 0.058 ms per frame with 4 queues, 3 lanes 0.073 (two lanes on one queue); with 8 queues
    // 3 lanes 0.046, 4 lanes 0.042)
    const int nl = int(std::clamp(rt::tuning(RT_TUNE_HW1_LANES, 2.0), 1.0, double(rt_hw1_scene::kLanes)));
    const int li = int(k % uint64_t(nl));
    rt_hw1_scene::Lane& L = s->lane[li];
    if (!L.own) HIP_TRY(hipStreamCreateWithFlags(&L.own, hipStreamNonBlocking));
    if (!s->caller) HIP_TRY(hipEventCreateWithFlags(&s->caller, hipEventDisableTiming));
    // work queued on the caller's stream comes first (a wait only while some is pending)
    if (hipStreamQuery(st) != hipSuccess) {
        (void)hipGetLastError();
        HIP_TRY(hipEventRecord(s->caller, st));
        HIP_TRY(hipStreamWaitEvent(L.own, s->caller, 0));
    }
    const size_t bytes = size_t(W) * size_t(H) * 3;
    // ticket k - kRing used this ring entry: its copy must have landed before it is reused
    if (k >= uint64_t(rt_hw1_scene::kRing) && (rc = s->wait_copy(k - rt_hw1_scene::kRing)) != RT_OK) return rc;
    const bool prev = k >= uint64_t(rt_hw1_scene::kDeliver);  // the body's previous frame
    if (s->dp6[slot].n < bytes) {
        if (prev && (rc = s->wait_copy(k - rt_hw1_scene::kDeliver)) != RT_OK) return rc;
        if ((rc = s->dp6[slot].alloc(bytes)) != RT_OK) return rc;
    } else if (prev && s->copy_mode == 1) {
        // the body's previous copy has landed (kDeliver frames back: normally long done)
        if ((rc = s->wait_copy(k - rt_hw1_scene::kDeliver)) != RT_OK) return rc;
    } else if (prev) {
        // the slot's previous copy: a wait on the lane's stream only while it is still running
        // (a cross-stream wait holds the next frame's first kernel even when already satisfied)
        hipEvent_t pe = s->cdone[(k - rt_hw1_scene::kDeliver) % rt_hw1_scene::kRing];
        if (hipEventQuery(pe) != hipSuccess) {
            (void)hipGetLastError();  // not ready is not an error of this call
            HIP_TRY(hipStreamWaitEvent(L.own, pe, 0));
        }
    }
    s->in_deliver = true;
    rc = render_frame(s, li, cam, lpos, lcol, spp, nullptr, flags, nullptr, static_cast<uint8_t*>(s->dp6[slot].p),
                      nullptr, nullptr, L.own);
    s->in_deliver = false;
    if (rc != RT_OK) return rc;
    // the copy waits for the frame's end event, set by its last kernel's dispatch (a marker
    // packet here held the next frame's first kernel: ~16 us between frames)
    hipEvent_t end = s->frame_end(s->frames - 1);
    if (s->copy_mode == 1) {
        rt_dma::hsa().signal_store(s->dma_done[ring], 1);
        s->dma_pending[ring] = true;
        s->dma->push({end, host_p6, s->dp6[slot].p, bytes, s->dma_done[ring]});
    } else {
        HIP_TRY(hipStreamWaitEvent(s->copy, end, 0));
        HIP_TRY(hipMemcpyAsync(host_p6, s->dp6[slot].p, bytes, hipMemcpyDeviceToHost, s->copy));
        HIP_TRY(hipEventRecord(s->cdone[ring], s->copy));
    }
    *ticket = k;
    s->tickets++;
    return RT_OK;
}

// Wait until frame `ticket` of rt_render_hw1_deliver is in its host buffer (one of the last
// 64 delivered frames).
extern "C" int rt_hw1_wait(rt_hw1_scene* s, uint64_t ticket) {
    if (!s) return set_error(RT_ERR_ARG, "rt_hw1_wait: null scene");
    if (ticket >= s->tickets || ticket + rt_hw1_scene::kRing < s->tickets)
        return set_error(RT_ERR_ARG, "rt_hw1_wait: not one of the last 64 delivered frames");
    DeviceGuard g(s->device);
    return s->wait_copy(ticket);
}

extern "C" int rt_hw1_kernel_times(const rt_hw1_scene* s, float* ms_out, int max, int* n_out) {
    if (!s || !ms_out || !n_out || max < 0) return set_error(RT_ERR_ARG, "rt_hw1_kernel_times: bad argument");
    DeviceGuard g(s->device);
    // the latest timed frames (all direct frames; delivered ones are sampled), oldest first
    std::vector<int> slots;
    const uint64_t have = std::min<uint64_t>(s->frames, uint64_t(rt_hw1_scene::kRing));
    for (uint64_t b = 1; b <= have && int(slots.size()) < max; ++b) {
        const int sl = int((s->frames - b) % rt_hw1_scene::kRing);
        if (s->timed[sl]) slots.push_back(sl);
    }
    const int n = int(slots.size());
    for (int i = 0; i < n; ++i) {
        const int sl = slots[size_t(n - 1 - i)];
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
    info[0] = s->lane[0].list_cap;
    info[1] = 0;
    if (s->frames > 0) {
        const int sl = int((s->frames - 1) % rt_hw1_scene::kRing);
        info[0] = s->lane[s->lane_of[sl]].list_cap;
        HIP_TRY(hipEventSynchronize(s->end_of(sl)));
        info[1] = uint32_t(s->total_host[sl]);
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
