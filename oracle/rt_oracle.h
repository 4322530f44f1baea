/* oracle/rt_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference's per-pixel ray path, used as the parity checker
 * by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  It is never linked
 * into or called by the product library (raytracinginonesemester_amd/csrc), whose render
 * path fails loudly when its HIP code object is missing.
 *
 * Pinned against outputs of the reference itself (oracle/_ref/ binaries, built from the sources
 * under /root/reference by `make -C oracle ref`, fixtures in tests/golden (written by
 * tests/golden/gen_golden.py): jitter tables, the 65 ray–triangle KAT answers, camera
 * bases, per-sample primary-hit (triangle index, t), float framebuffers and P6 bytes.
 *
 * Structs mirror the reference's POD layouts byte for byte (sizes checked by tests).
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { float x, y, z; } orc_vec3;                                   /* G/include/vec3.h:302 */
typedef struct { uint32_t parent, left, right, object; } orc_node;            /* G/include/bvh.h:7-13 */
typedef struct { orc_vec3 mn, mx; } orc_aabb;                                 /* G/include/bvh.h:28-52 */
typedef struct { orc_vec3 v0, v1, v2, n0, n1, n2; } orc_tri;                  /* G/include/MeshOBJ.h:42-67 */
typedef struct {                                                              /* G/include/material.h:6-21 */
    orc_vec3 albedo; float kd; orc_vec3 specular; float ks, shininess, kr; orc_vec3 emission;
} orc_material;
typedef struct { orc_vec3 position, color; int32_t intensity; } orc_light;    /* G/include/scene.h:21-25 */

/* Derived pinhole basis of G/include/camera.h:72-94 (and HW1/include/camera.h:55-92). */
typedef struct { orc_vec3 center, pixel00, du, dv; int32_t width, height; } orc_camera;

/* Traversal counters for the algorithmic-bytes model of SURVEY.md §8(d):
 * class 0 = primary, 1 = shadow, 2 = bounce. */
typedef struct {
    uint64_t rays[3], pops[3], internal_entered[3], leaf_entered[3], hits[3];
    uint64_t occluded;
    uint64_t max_pops[3];  /* the most pops of one SearchBVH call */
} orc_stats;

/* std::mt19937(seed) + uniform_real_distribution<float>(0,1), libstdc++ generate_canonical;
 * minus 0.5 when centered != 0 (G/include/antialias.h:12-27), raw [0,1) otherwise
 * (HW1/include/antialias.h:12-27).  out: 2*spp floats (dx, dy) pairs. */
void orc_jitter(int spp, uint32_t seed, int centered, float* out);

/* G/include/camera.h:13-28,72-94 (hw1 != 0: HW1/include/camera.h, which rejects w,h < 1). */
int orc_camera_init(orc_camera* cam, const float pos[3], const float look_at[3], const float up[3],
                    double focal_length_mm, double sensor_height_mm, int width, int height, int hw1);

/* G/include/query.cu:130-166 render() CPU branch, rows [y0, y1) only (out_rgb indexed by
 * full-frame pixel).  jitter: 2*spp floats or NULL (= jittered_samples(spp, 42u)).
 * rebuild_jitter_per_pixel != 0 regenerates the table per pixel like query.cu:142.
 * hit_idx / hit_t (optional, W*H*spp): primary SearchBVH result per (pixel, sample).
 * threads <= 0 uses the OpenMP default. */
int orc_render_g(size_t num_triangles, int W, int H, const orc_camera* cam, orc_vec3 miss_color,
                 int max_depth, int spp, const orc_node* nodes, const orc_aabb* aabbs,
                 const orc_tri* tris, const int32_t* tri_obj_ids, const orc_material* mats,
                 int num_mats, const orc_light* lights, int num_lights, int diffuse_bounce,
                 const float* jitter, int rebuild_jitter_per_pixel, int y0, int y1, int threads,
                 float* out_rgb, int32_t* hit_idx, float* hit_t, orc_stats* stats);

/* One reference SearchBVH (G/include/query.h:224-311) for a given ray; returns triangle
 * index or -1, writes t. */
int orc_search_bvh(size_t num_triangles, const float orig[3], const float dir[3],
                   const orc_node* nodes, const orc_aabb* aabbs, const orc_tri* tris, float* t_out);

/* HW1/src/render.cpp:72-116 brute-force loop with HW1/include/{ray,raytracer}.h semantics.
 * positions/normals indexed by indices (3 per triangle).  jitter: HW1 [0,1) table or NULL. */
int orc_render_hw1(const orc_vec3* positions, const orc_vec3* normals, const uint32_t* indices,
                   size_t num_triangles, const orc_camera* cam, orc_vec3 light_pos,
                   orc_vec3 light_color, int spp, const float* jitter, int y0, int y1, int threads,
                   float* out_rgb, int32_t* hit_idx, float* hit_t);

/* HW1 ray_intersection (HW1/include/ray.h:67-117) for rays from `orig` along dirs[i]
 * (normalised by the HW1 Ray constructor, ray.h:25). */
void orc_kat_hw1(const orc_tri* tri, const float orig[3], const float* dirs, int n,
                 int32_t* hit, float* t);

/* G/ intersectTriangle (G/include/query.h:72-132) with [tmin, tmax]; dir used as given. */
void orc_intersect_g(const orc_tri* tri, const float orig[3], const float* dirs, int n,
                     float tmin, float tmax, int32_t* hit, float* t);

/* ppm_p6 float_to_sample (HW1/ppm_p6_lib/src/ppm_p6.cpp:137-155) over n floats. */
void orc_ppm_quantize(const float* linear, size_t n, int maxval, int clamp, int gamma2, uint16_t* out);

#ifdef __cplusplus
}
#endif
#endif
