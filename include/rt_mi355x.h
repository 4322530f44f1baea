/* include/rt_mi355x.h — C ABI of the MI355X (gfx950) per-pixel ray path.
 *
 * Drop-in boundary for the reference's render entry point
 *     void render(size_t numTriangles, int W, int H, const Camera cam, const Vec3 missColor,
 *                 int max_depth, int spp, const BVHNode* nodes, const AABB* aabbs,
 *                 const Triangle* triangles, const int32_t* triObjectIds,
 *                 const Material* objectMaterials, int numObjectMaterials,
 *                 const Light* lights, int numLights, bool diffuse_bounce, Vec3* output);
 * (HW2/HW2/GPUandCPU/include/query.h:13-29, defined at include/query.cu:79-167) and of the
 * host pieces around it that the reference keeps in C++ (scene JSON + OBJ loading,
 * camera setup, CPU LBVH build, ppm_p6 writer).  Plain C types, plain pointers and sizes;
 * every function returns RT_OK (0) or a negative RT_ERR_* code and never throws;
 * rt_last_error() returns the calling thread's last message.
 *
 * Structs marked "layout = reference" are byte-for-byte the reference's POD types, so a
 * caller holding the reference's arrays passes them unchanged.
 */
#ifndef RT_MI355X_H
#define RT_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 3  /* 2: rt_renderer_opts.host_frame_name, RT_GATHER_HOST_SHARED;
                              3: RT_ERR_INTERNAL, rt_scene_faults, rt_tuning_* (RT_TUNE_*) in place of
                                 environment variables, frame pairs, the resident HW1 scene */

enum {
    RT_OK = 0,
    RT_ERR_ARG = -1,          /* bad argument / malformed arrays */
    RT_ERR_IO = -2,           /* file could not be opened / written */
    RT_ERR_PARSE = -3,        /* OBJ / JSON / PPM syntax */
    RT_ERR_HIP = -4,          /* HIP runtime error (message in rt_last_error) */
    RT_ERR_NOMEM = -5,
    RT_ERR_NODEVICE = -6,     /* no gfx950 device / code object not loadable */
    RT_ERR_UNSUPPORTED = -7,  /* input outside what the kernels handle (see rt_last_error) */
    RT_ERR_COMM = -8,         /* RCCL could not be loaded or a collective failed */
    RT_ERR_INTERNAL = -9      /* a device-side guard fired (rt_scene_faults); the frame is not valid */
};

/* ---- reference POD types ------------------------------------------------------------ */
typedef struct { float x, y, z; } rt_vec3;                       /* layout = reference: Vec3, G/include/vec3.h:299-304 */
typedef struct {                                                  /* layout = reference: BVHNode, G/include/bvh.h:7-13 */
    uint32_t parent_idx, left_idx, right_idx, object_idx;         /* object_idx == 0xFFFFFFFF: internal */
} rt_bvh_node;
typedef struct { rt_vec3 min_corner, max_corner; } rt_aabb;      /* layout = reference: AABB, G/include/bvh.h:28-52 */
typedef struct { rt_vec3 v0, v1, v2, n0, n1, n2; } rt_triangle;  /* layout = reference: Triangle, G/include/MeshOBJ.h:42-67 */
typedef struct {                                                  /* layout = reference: Material, G/include/material.h:6-21 */
    rt_vec3 albedo; float kd;
    rt_vec3 specular_color; float ks; float shininess;
    float kr;
    rt_vec3 emission;
} rt_material;
typedef struct { rt_vec3 position, color; int32_t intensity; } rt_light; /* layout = reference: Light, G/include/scene.h:21-25 */

/* Derived pinhole basis of the reference Camera (G/include/camera.h:208-216): the fields
 * render() reads.  Fill with rt_camera_init (same float/double arithmetic as
 * Camera::initialize, camera.h:72-94). */
typedef struct {
    rt_vec3 center, pixel00_loc, pixel_delta_u, pixel_delta_v;
    int32_t pixel_width, pixel_height;
} rt_camera;

/* Reference Material() defaults (material.h:8-19). */
void rt_material_default(rt_material* m);

/* Camera(pos, lookAt, up, focal_length_mm, sensor_height_mm, width, height)
 * (G/include/camera.h:13-28).  hw1 != 0 follows HW1/include/camera.h (error instead of
 * clamping width/height < 1). */
int rt_camera_init(rt_camera* cam, const float pos[3], const float look_at[3], const float up[3],
                   double focal_length_mm, double sensor_height_mm, int width, int height, int hw1);

/* jittered_samples(spp, seed) (G/include/antialias.h:12-27): std::mt19937 +
 * uniform_real_distribution<float>; centered != 0 subtracts 0.5 (G/), 0 keeps [0,1) (HW1).
 * out: 2*spp floats. */
int rt_jittered_samples(int spp, uint32_t seed, int centered, float* out);

/* ---- host scene: the reference's loaders + CPU LBVH (G/src/main.cu:104-317) -------- */
typedef struct rt_host_scene rt_host_scene;

typedef struct {
    /* settings (G/include/scene.h:15-19), miss colour, camera, counts */
    int32_t max_depth, spp, diffuse_bounce;
    rt_vec3 miss_color;
    rt_vec3 cam_position, cam_look_at, cam_up;
    double focal_length_mm, sensor_height_mm;
    int32_t pixel_width, pixel_height;
    uint64_t num_triangles, num_vertices;
    int32_t num_materials, num_lights, num_objects_loaded;
    int32_t bvh_max_stack;   /* DFS stack depth the traversal of this tree needs */
    int32_t bvh_height;
} rt_scene_info;

typedef struct {  /* views into rt_host_scene storage (valid until rt_host_scene_free) */
    const rt_bvh_node* nodes;        /* 2P-1 */
    const rt_aabb* aabbs;            /* 2P-1 */
    const rt_triangle* triangles;    /* P, packed as G/src/main.cu:388-404 */
    const int32_t* tri_object_ids;   /* P */
    const rt_material* materials;    /* num_materials */
    const rt_light* lights;          /* num_lights (fallback light added as main.cu:328-336) */
    const rt_vec3* positions;        /* num_vertices (transformed) */
    const rt_vec3* normals;          /* num_vertices or NULL */
    const uint32_t* indices;         /* 3P */
} rt_scene_arrays;

/* Scene JSON (G/include/scene.h:242-393) + every mesh object: LoadOBJ_ToMesh
 * (G/include/MeshOBJ.h:260-427), applyObjectTransform (G/src/main.cu:57-96), AppendMesh
 * (MeshOBJ.h:429-466); then calculateAABBs + CPU buildBVH (G/include/bvh.cu:60-89,209-317).
 * Relative mesh paths resolve like G/src/main.cu:119-147 with project_dir (NULL =
 * dirname(dirname(dirname(scene)))). */
int rt_host_scene_load_json(const char* scene_path, const char* project_dir, rt_host_scene** out);
/* OBJ path list without JSON (G/src/main.cu:151-157): default material/camera/settings. */
int rt_host_scene_load_objs(const char* const* obj_paths, int n, rt_host_scene** out);
int rt_host_scene_info(const rt_host_scene* s, rt_scene_info* out);
int rt_host_scene_arrays(const rt_host_scene* s, rt_scene_arrays* out);
void rt_host_scene_free(rt_host_scene* s);

/* CPU LBVH over caller arrays (leaf AABBs from indexed triangles), reference algorithm:
 * nodes/aabbs must hold 2P-1 entries. */
int rt_build_bvh(const rt_vec3* positions, size_t num_vertices, const uint32_t* indices,
                 size_t num_triangles, rt_bvh_node* nodes, rt_aabb* aabbs);
/* The same build on the GPU (the reference's CUDA build bvh.cu:34-206 and
 * its CPU build bvh.cu:209-317): positions_dev (num_vertices Vec3), indices_dev (3*P u32),
 * nodes_dev / aabbs_dev (2P-1 each) are device pointers on `device`.  The arrays are
 * byte-identical to rt_build_bvh's.  Runs on hip_stream and synchronises it before returning
 * (out-of-range vertex indices are reported as RT_ERR_ARG). */
int rt_build_bvh_device(int device, const rt_vec3* positions_dev, size_t num_vertices,
                        const uint32_t* indices_dev, size_t num_triangles, rt_bvh_node* nodes_dev,
                        rt_aabb* aabbs_dev, void* hip_stream);

/* HW1 mesh: LoadOBJ_ToMeshSOA (HW1/src/MeshOBJ.cpp:143-281). */
typedef struct rt_mesh rt_mesh;
typedef struct {
    const rt_vec3* positions; const rt_vec3* normals; const uint32_t* indices;
    uint64_t num_vertices, num_triangles; int32_t has_normals, has_uvs;
} rt_mesh_view;
int rt_mesh_load_obj_hw1(const char* path, rt_mesh** out);
int rt_mesh_view_get(const rt_mesh* m, rt_mesh_view* out);
void rt_mesh_free(rt_mesh* m);

/* ---- ppm_p6 (HW1/ppm_p6_lib/include/ppm_p6.hpp:46-85) ------------------------------- */
typedef struct { int32_t maxval, clamp, gamma2, flip_y; } rt_ppm_options;  /* defaults 255,1,1,0 */
void rt_ppm_options_default(rt_ppm_options* o);
/* rgb: W*H*3 floats, row 0 = top.  Writes "P6\n<W> <H>\n<maxval>\n" + samples. */
int rt_ppm_write(const char* path, const float* rgb, int width, int height, const rt_ppm_options* opt);
/* Same bytes into memory: needs 32 + W*H*3*(maxval<256 ? 1 : 2) bytes; *written = size. */
int rt_ppm_encode(const float* rgb, int width, int height, const rt_ppm_options* opt,
                  uint8_t* buf, size_t cap, size_t* written);
/* read_p6 (ppm_p6.cpp:303-372): rgb_out may be NULL to query W/H first. */
int rt_ppm_read(const char* path, float* rgb_out, size_t cap_floats, int* width, int* height, int* maxval);

/* ---- frame epilogue on the device --------------------------------- */
/* write_p6's header ("P6\n<W> <H>\n<maxval>\n", ppm_p6.cpp:275-277); buf may be NULL to
 * query the size. */
int rt_ppm_header(int width, int height, int maxval, char* buf, size_t cap, size_t* written);
/* write_p6's sample loop (ppm_p6.cpp:284-299 with float_to_sample :137-155) on the device:
 * rgb_dev = rows*W*3 floats (device), out_dev = rows*W*3*(maxval<256 ? 1 : 2) bytes (device),
 * the P6 body without its header; flip_y reverses the given rows.  Asynchronous on
 * hip_stream.  Byte-identical to rt_ppm_encode's body. */
int rt_ppm_quantize_device(const float* rgb_dev, int width, int rows, const rt_ppm_options* opt,
                           uint8_t* out_dev, void* hip_stream);
/* Band un-permute after a gather: strips_dev holds band_count strips back to back, strip r =
 * strip_rows rows of row_bytes bytes in the layout rt_render_device writes for
 * (band_rows, r, band_count) — float rows (W*12 B) or quantised P6 rows.  Writes the
 * height-row frame in image order (flip_y: bottom row first) to frame_dev.  Asynchronous. */
int rt_unpermute_strips_device(const void* strips_dev, int strip_rows, size_t row_bytes, int height,
                               int band_rows, int band_count, int flip_y, void* frame_dev, void* hip_stream);

/* ---- the hot path: device-resident scene + HIP render ---------------------------------- */
typedef struct rt_scene rt_scene;

/* Upload the reference arrays to `device`, validating them (indices in range, a proper
 * binary tree rooted at 0) and repacking them into the gfx950 traversal layout. */
int rt_scene_create(int device, size_t num_triangles, const rt_bvh_node* nodes, const rt_aabb* aabbs,
                    const rt_triangle* triangles, const int32_t* tri_object_ids,
                    const rt_material* materials, int num_materials, const rt_light* lights,
                    int num_lights, rt_scene** out);
void rt_scene_destroy(rt_scene* s);
/* The same scene on another device: device-to-device copies of the packed arrays (no host
 * repacking).  Frames of a scene run in launch order (see rt_render_device). */
int rt_scene_clone(const rt_scene* src, int device, rt_scene** out);
int rt_scene_device(const rt_scene* s);
size_t rt_scene_device_bytes(const rt_scene* s);

enum {
    RT_KERNEL_AUTO = 0,      /* the fastest parity-equivalent kernel */
    RT_KERNEL_WAVE = 1,      /* wave-coherent masked DFS (shared per-wave stack) */
    RT_KERNEL_LANE = 2,      /* one private DFS stack per lane (baseline variant) */
    RT_KERNEL_WAVE_PIXELS = 3 /* WAVE traversal, one pixel per lane looping over its samples */
};

typedef struct {
    int32_t max_depth;        /* TraceRayIterative depth (query.h:156) */
    int32_t spp;
    int32_t diffuse_bounce;
    rt_vec3 miss_color;
    const float* jitter;      /* host, 2*spp floats; NULL = rt_jittered_samples(spp, 42, 1) */
    /* Image sharding: rows are cut into bands of band_rows; this call renders bands b with
     * b % band_count == band_index, written contiguously (band order) into the output
     * ("strip" layout).  band_count <= 1 renders the whole frame in row-major order. */
    int32_t band_rows, band_index, band_count;
    int32_t kernel;           /* RT_KERNEL_* */
    int32_t tile_order;       /* RT_TILES_*: block -> pixel-tile order (speed only) */
    int32_t flags;            /* RT_FLAG_* */
} rt_render_opts;

enum {
    RT_FLAG_NO_CULL = 1,      /* disable tile culling against the root box (A/B; same output) */
    RT_FLAG_BINARY = 4        /* wave traversal over the binary nodes, not the 4-ary records */
};

enum {
    RT_TILES_AUTO = 0,        /* RT_TILES_ROWS */
    RT_TILES_LINEAR = 1,      /* block b renders tile b (dispatch deals blocks round-robin to XCDs) */
    RT_TILES_XCD_CHUNK = 2,   /* each XCD's blocks take one contiguous 1/8 of the tiles */
    RT_TILES_ROWS = 3         /* each XCD's blocks take every 8th row of tiles */
};
void rt_render_opts_default(rt_render_opts* o);

/* Rows covered by (band_rows, band_index, band_count) for an H-row image. */
int rt_shard_rows(int height, int band_rows, int band_index, int band_count);

/* Render into device memory on `hip_stream` (hipStream_t; NULL = the null stream), no
 * host sync.  rgb_dev: rows*W*3 floats.  hit_idx_dev / hit_t_dev (optional, rows*W*spp):
 * primary-ray triangle index (-1 = miss) and t per (pixel, sample).
 * Stream-ordered: the frame's work starts after everything queued on hip_stream before the
 * call and is complete when hip_stream reaches the end of this call's work.  (A frame's tile
 * pre-passes, which write the culled tiles' pixels, run on the scene's own stream after an
 * event wait on hip_stream; rt_renderer, which orders its buffer reuse on the host, lets them
 * overlap the previous frame's render kernel instead.)  Frames of one scene are ordered: a
 * call on another stream than the scene's previous frame makes its stream wait for that frame. */
int rt_render_device(rt_scene* s, const rt_camera* cam, const rt_render_opts* opt,
                     float* rgb_dev, int32_t* hit_idx_dev, float* hit_t_dev, void* hip_stream);

/* rt_render_device that also writes the pixels' P6 samples (write_p6 defaults: maxval 255,
 * clamp, sqrt gamma; ppm_p6.cpp:137-155) to p6_dev (rows*W*3 bytes, same row order as
 * rgb_dev) from the render and cull kernels themselves: the frame epilogue fused into the
 * kernels that produce the pixels (p6_dev may be NULL).  rgb_dev may be NULL when p6_dev is
 * not: the frame is then produced as P6 samples only. */
int rt_render_device_p6(rt_scene* s, const rt_camera* cam, const rt_render_opts* opt,
                        float* rgb_dev, int32_t* hit_idx_dev, float* hit_t_dev, uint8_t* p6_dev,
                        void* hip_stream);

/* Two frames of one scene with the same options (two cameras of the same pixel size, e.g. the
 * next two frames of a sequence), as rt_render_device_p6 twice (frame a, then frame b; the same
 * images), rendered by one launch of the render kernel where it fits them
 * (RT_TUNE_PAIR_FRAMES): the second frame's work fills the first's tail and the launch gap
 * between two frames goes.  This batching is this library's own: the reference renders one
 * frame per render() call (G/src/main.cu:362-378 is a 1x1 warm-up launch, then one timed
 * render).  Outputs of a and b must not overlap. */
int rt_render_device_pair(rt_scene* s, const rt_camera* cam_a, const rt_camera* cam_b,
                          const rt_render_opts* opt, float* rgb_a_dev, uint8_t* p6_a_dev,
                          float* rgb_b_dev, uint8_t* p6_b_dev, void* hip_stream);

/* Synchronous convenience: render into host memory (rows*W*3 floats, + optional AOVs). */
int rt_render(rt_scene* s, const rt_camera* cam, const rt_render_opts* opt,
              float* rgb_host, int32_t* hit_idx_host, float* hit_t_host);

/* Rays one frame of rt_render traces, in the oracle's classes: counts[0] camera rays
 * (W*rows*spp when max_depth > 0), counts[1] shadow rays (IsInShadow calls that cast a ray,
 * shader.h:44-62 behind ShadeDirect's NdotL > 0, shader.h:87-93), counts[2] bounce rays
 * (TraceRayIterative depths > 0, query.h:156-220).  Renders the frame once more with counting
 * kernels (not the timed ones) and discards it; synchronous.  For total rays/s
 * (SURVEY.md §8(d)). */
int rt_count_rays(rt_scene* s, const rt_camera* cam, const rt_render_opts* opt, uint64_t counts[3]);
/* rt_count_rays + counts[3]: the camera rays that are traversed, i.e. those of the pixel tiles
 * the culling pre-passes leave to the render kernel (the others provably miss every box of the
 * tree, their samples are written as misses without a traversal). */
int rt_count_rays_ex(rt_scene* s, const rt_camera* cam, const rt_render_opts* opt, uint64_t counts[4]);

/* The reference signature verbatim (query.h:13-29) over host arrays: uploads to device 0,
 * renders on the GPU, writes W*H Vec3 to `output` (host).  Synchronous. */
int rt_render_reference(size_t num_triangles, int W, int H, const rt_camera* cam, rt_vec3 miss_color,
                        int max_depth, int spp, const rt_bvh_node* nodes, const rt_aabb* aabbs,
                        const rt_triangle* triangles, const int32_t* tri_object_ids,
                        const rt_material* materials, int num_materials, const rt_light* lights,
                        int num_lights, int diffuse_bounce, rt_vec3* output);

/* rt_render_reference over n_gpus devices (0..n_gpus-1) of this process: the image's 8-row
 * bands dealt round-robin over the GPUs, the float strips gathered to device 0 with RCCL and
 * copied into `output` (host).  The frame equals rt_render_reference's bit for bit.
 * (SURVEY.md §8(b) n_gpus / §8(e); G/include/query.h:13-29 has no multi-GPU form.) */
int rt_render_reference_gpus(size_t num_triangles, int W, int H, const rt_camera* cam, rt_vec3 miss_color,
                             int max_depth, int spp, const rt_bvh_node* nodes, const rt_aabb* aabbs,
                             const rt_triangle* triangles, const int32_t* tri_object_ids,
                             const rt_material* materials, int num_materials, const rt_light* lights,
                             int num_lights, int diffuse_bounce, int n_gpus, rt_vec3* output);

/* ---- frame renderer: render(scene, camera) -> frame in host memory on 1..N GPUs ----------
 * The loop around render() in G/src/main.cu:362-378 (render, then the frame copied to host
 * memory), pipelined and sharded.  Per frame, every rank renders the bands b with
 * b % world_size == rank (band_rows-row bands, rt_render_opts sharding) into a device strip on
 * its compute stream; the strips reach rank 0 over RCCL (one grouped ncclSend/ncclRecv per
 * rank on a comm stream, xGMI between GPUs); rank 0 copies them into a pinned host frame on a
 * copy stream, placing every band at its image rows (2-D copies: no un-permute pass).  Frames
 * are double/triple-buffered: frame k+1 renders while frame k is gathered and copied.
 *
 * Ranks: the process drives n_devices GPUs as global ranks rank0 .. rank0+n_devices-1 of
 * world_size.  world_size == n_devices (or 0): one process, the communicator made with
 * ncclCommInitAll.  world_size > n_devices: one rank group of a multi-process job (e.g. one
 * process per GPU under torchrun); every process passes the same 128-byte unique_id, made by
 * rt_comm_unique_id on the process holding rank 0 and shared by the caller.
 * A device id may repeat (several band shards on one GPU, for tests): then gather must be
 * RT_GATHER_DIRECT (one process) or RT_GATHER_HOST_SHARED (several), each rank copying its
 * bands straight into the host frame.
 *
 * RT_GATHER_HOST_SHARED (one process per GPU, e.g. under torchrun): the depth host frames are
 * one POSIX shared-memory segment (host_frame_name, the same on every process; rank 0's
 * process creates it, the others attach, each pins it with hipHostRegister).  Every rank
 * copies its own bands over its own PCIe link into their image rows, then publishes the frame
 * in the segment's per-rank completion word; rank 0's rt_renderer_wait returns once every rank
 * has published.  A rank copies frame t into a slot only after rank 0 has submitted frame t
 * (rank 0's caller then no longer holds frame t-depth).  RCCL is not used on this path. */
typedef struct rt_renderer rt_renderer;

enum {
    RT_DELIVER_P6 = 0,     /* the P6 body (write_p6 defaults), W*H*3 bytes, rows top to bottom */
    RT_DELIVER_F32 = 1,    /* the float framebuffer, W*H*3 floats (the reference's output) */
    RT_DELIVER_DEVICE = 2, /* P6 body assembled in rank 0's device memory; no host copy */
    RT_DELIVER_NONE = 3    /* render only (strips stay on each rank): measurement */
};
enum {
    RT_GATHER_AUTO = 0,    /* one process: DIRECT; several: HOST_SHARED with host_frame_name, else RCCL */
    RT_GATHER_RCCL = 1,    /* strips -> rank 0's GPU over RCCL, then one host copy stream */
    RT_GATHER_DIRECT = 2,  /* each local rank copies its own bands into the host frame (its own
                              PCIe link); single process only */
    RT_GATHER_HOST_SHARED = 3 /* each rank of a multi-process job copies its own bands into one
                                 host frame shared by the processes (host_frame_name); no RCCL */
};
enum { RT_RENDERER_SELF_SEND = 1 /* rank 0's own strip also goes through RCCL (tests at world 1) */ };

typedef struct {
    int32_t n_devices;        /* GPUs this process drives (1..64) */
    const int32_t* devices;   /* their device ids; NULL = 0 .. n_devices-1 */
    int32_t world_size;       /* ranks over all processes; 0 = n_devices */
    int32_t rank0;            /* global rank of devices[0]; the others follow */
    const void* unique_id;    /* 128 bytes (world_size > n_devices) */
    int32_t band_rows;        /* default 8 */
    int32_t deliver;          /* RT_DELIVER_* */
    int32_t gather;           /* RT_GATHER_* */
    int32_t depth;            /* frames in flight, 1..8 (default 3) */
    int32_t flags;            /* RT_RENDERER_* */
    const char* host_frame_name; /* RT_GATHER_HOST_SHARED: shared-memory name ("/..."), same on every
                                    process; RT_GATHER_AUTO picks HOST_SHARED for a multi-process
                                    renderer when it is set (RCCL otherwise) */
} rt_renderer_opts;
void rt_renderer_opts_default(rt_renderer_opts* o);

/* 1 when the renderer delivers its frames with SDMA copies queued through the HSA runtime (one
 * rank, RT_GATHER_DIRECT, a host frame; RT_TUNE_COPY_ENGINE), 0 when with the HIP runtime's
 * copies (blit kernels on the CUs). */
int rt_renderer_copy_engine(const rt_renderer* r);

/* 128-byte RCCL unique id for a multi-process renderer (call on rank 0's process). */
int rt_comm_unique_id(void* id128);

/* Scene upload (rt_scene_create's arguments) to every local device (one upload, then
 * device-to-device clones), stream/event/communicator setup. */
int rt_renderer_create(size_t num_triangles, const rt_bvh_node* nodes, const rt_aabb* aabbs,
                       const rt_triangle* triangles, const int32_t* tri_object_ids,
                       const rt_material* materials, int num_materials, const rt_light* lights,
                       int num_lights, const rt_renderer_opts* opts, rt_renderer** out);
void rt_renderer_destroy(rt_renderer* r);

/* Enqueue one frame (opts: its band fields are the renderer's).  Blocks only to reuse the
 * buffers of frame ticket-depth, which must then be complete.  *ticket numbers the frames. */
int rt_renderer_submit(rt_renderer* r, const rt_camera* cam, const rt_render_opts* opts, uint64_t* ticket);
/* Enqueue two frames (tickets *ticket_a, *ticket_a + 1) with the same options, rendered by one
 * launch per local rank (rt_render_device_pair); delivered as two rt_renderer_submit calls
 * would deliver them.  Needs depth >= 2; blocks to reuse both frames' buffers. */
int rt_renderer_submit_pair(rt_renderer* r, const rt_camera* cam_a, const rt_camera* cam_b,
                            const rt_render_opts* opts, uint64_t* ticket_a);
/* Wait for frame `ticket` (one of the last `depth` submitted, and not from before a change of
 * the frame size, which reallocates the buffers).  On the process holding rank 0,
 * *frame / *bytes give the delivered frame: pinned host memory (RT_DELIVER_P6/F32) or rank 0's
 * device memory (RT_DELIVER_DEVICE), valid until the submit of frame ticket+depth; elsewhere
 * NULL / 0.  Either pointer may be NULL. */
int rt_renderer_wait(rt_renderer* r, uint64_t ticket, const void** frame, size_t* bytes);
/* submit + wait + copy of the frame into out (cap bytes; rank 0 only). */
int rt_renderer_render(rt_renderer* r, const rt_camera* cam, const rt_render_opts* opts, void* out, size_t cap);
/* Local rank i's scene (for rt_frame_times / rt_kernel_times / rt_live_tiles). */
rt_scene* rt_renderer_scene(rt_renderer* r, int i);
int rt_renderer_local_ranks(const rt_renderer* r);
/* Durations (ms) of the gather (RT_TIME_GATHER: rank 0's receives, or its copy wait in DIRECT
 * mode) or of the host copy (RT_TIME_DELIVER) of the last min(max, frames) frames, oldest
 * first, from HIP events on those streams (rank 0's process; n_out = 0 elsewhere). */
enum { RT_TIME_GATHER = 0, RT_TIME_DELIVER = 1, RT_TIME_FRAME = 2 /* first render launch -> frame delivered */ };
int rt_renderer_times(rt_renderer* r, int kind, float* ms_out, int max, int* n_out);

/* HW1 brute-force path on the GPU (HW1/src/render.cpp:72-116 semantics: every triangle,
 * closest t >= 0 with the first index winning ties, HW1 shade).  Synchronous; host I/O. */
int rt_render_hw1(int device, const rt_vec3* positions, const rt_vec3* normals,
                  const uint32_t* indices, size_t num_triangles, const rt_camera* cam,
                  rt_vec3 light_position, rt_vec3 light_color, int spp, const float* jitter,
                  float* rgb_host, int32_t* hit_idx_host, float* hit_t_host);

/* rt_render_hw1 with a kernel selection and the device time of the kernels (HIP events;
 * kernel_ms may be NULL).  flags 0: binned — a conservative per-triangle pixel rectangle
 * (outside it ray_intersection provably rejects every camera ray), then per 16x16 block the
 * brute-force loop over the triangles whose rectangle meets the block, in index order, so
 * the output equals the brute-force loop's bit for bit; RT_HW1_BRUTE: every triangle for
 * every ray (HW1/src/render.cpp:72-116 literally). */
enum { RT_HW1_BRUTE = 1 };
int rt_render_hw1_ex(int device, const rt_vec3* positions, const rt_vec3* normals,
                     const uint32_t* indices, size_t num_triangles, const rt_camera* cam,
                     rt_vec3 light_position, rt_vec3 light_color, int spp, const float* jitter,
                     int flags, float* rgb_host, int32_t* hit_idx_host, float* hit_t_host,
                     float* kernel_ms);

/* Resident HW1 mesh for repeated frames (the C2 configuration on the device): the mesh packed
 * and uploaded once, the binning buffers kept.  rt_render_hw1_device renders one frame on
 * hip_stream (NULL = the default stream) without synchronising: rgb_dev (W*H*3 floats) and/or
 * p6_dev (W*H*3 bytes, write_p6 defaults) and the optional AOVs (W*H*spp each) are device
 * pointers; jitter NULL = jittered_samples(spp, 42) in [0,1).  rt_hw1_kernel_times: ms of the
 * frame's kernels (events around them) for the latest min(max, frames, 64) frames, oldest first;
 * rt_hw1_kernel_name: the render kernel the latest frame launched, as rocprofv3 names it. */
typedef struct rt_hw1_scene rt_hw1_scene;
int rt_hw1_scene_create(int device, const rt_vec3* positions, const rt_vec3* normals, const uint32_t* indices,
                        size_t num_triangles, rt_hw1_scene** out);
void rt_hw1_scene_destroy(rt_hw1_scene* s);
int rt_render_hw1_device(rt_hw1_scene* s, const rt_camera* cam, rt_vec3 light_position, rt_vec3 light_color,
                         int spp, const float* jitter, int flags, float* rgb_dev, uint8_t* p6_dev,
                         int32_t* hit_idx_dev, float* hit_t_dev, void* hip_stream);
/* One frame as rt_render_hw1_device renders it, into one of the scene's 8 device P6 bodies, then
 * that body copied to host_p6 (W*H*3 bytes, pinned) once the frame's kernels are done — by a DMA
 * (SDMA) engine, queued from a copier thread, or with RT_TUNE_COPY_ENGINE 0 by the HIP runtime
 * on the scene's copy stream — so the copy overlaps the next frames' kernels; *ticket numbers the
 * frame.  Frames alternate over the scene's lanes (binning buffers and a stream each,
 * RT_TUNE_HW1_LANES), after the work queued on hip_stream so far.  host_p6 must stay valid until
 * rt_hw1_wait(ticket) returns; a frame reuses the device body of the frame 8 before it (after
 * that frame's copy). */
int rt_render_hw1_deliver(rt_hw1_scene* s, const rt_camera* cam, rt_vec3 light_position, rt_vec3 light_color,
                          int spp, int flags, uint8_t* host_p6, void* hip_stream, uint64_t* ticket);
int rt_hw1_wait(rt_hw1_scene* s, uint64_t ticket);
int rt_hw1_kernel_times(const rt_hw1_scene* s, float* ms_out, int max, int* n_out);
const char* rt_hw1_kernel_name(const rt_hw1_scene* s);
/* info = {entries the bin list holds now, the latest frame's list total (waits for it)}: a
 * total above the capacity its frame ran with means that frame's overflowing tiles took the
 * brute-force loop; the next frame runs with a grown list. */
int rt_hw1_list_info(const rt_hw1_scene* s, int64_t info[2]);

/* Batched ray-triangle queries on the GPU (one triangle, n rays from `origin`), the device
 * Möller–Trumbore used by the kernels:  hw1 != 0 -> HW1 ray_intersection
 * (HW1/include/ray.h:67-117; the HW1 Ray constructor normalises each direction first, ray.h:25),
 * hw1 == 0 -> G/ intersectTriangle (G/include/query.h:72-108) over [tmin, tmax] with the
 * direction used as given.  Host arrays; hit[i] in {0,1}, t[i] = -1 on a miss. */
int rt_intersect_rays(int device, const rt_triangle* tri, const float origin[3], const float* dirs, int n,
                      int hw1, float tmin, float tmax, int32_t* hit, float* t);

/* The Blinn-Phong powf of the kernels (restatement of the reference libm's powf, see
 * csrc/rt_math.hpp): rt_powf_host evaluates the host build, rt_powf_batch the device build
 * over n (x, y) pairs.  Exposed so both can be pinned against the C library's powf. */
float rt_powf_host(float x, float y);
int rt_powf_batch(int device, const float* x, const float* y, int n, float* out);

/* Host build of the kernels' AABB test for n (ray, box, [tmin,tmax]) triples: out_exact =
 * the reference's double slab test (bvh.h:81-129), out_fast = the float-pre-classified test
 * the kernels run (must equal out_exact), out_class = 0 miss / 1 hit / 2 ambiguous (decided
 * in double).  rays: n*6 floats (orig, dir), boxes: n*6 (min, max), tminmax: n*2. */
int rt_box_test_host(const float* rays, const float* boxes, const float* tminmax, int n,
                     int32_t* out_fast, int32_t* out_exact, int32_t* out_class);

/* Host build of the camera rays' frustum records rt_scene_create makes (no device): for a BVH
 * of P triangles (the same arrays as rt_scene_create), the records of arity 2^info[0]
 * (8 x 2^info[0] floats each: per entry the (min, max) pairs of x, y, z, then the entries'
 * refs), info = {log2 arity (2: none fits), DFS stack bound, records}: the largest arity up to
 * 2^max_log2 whose DFS needs at most stack_cap entries (64; 128 for the big-scene kernels).
 * rec is written when rec_cap (floats) suffices; call with a null rec to size it.
 * DESIGN.md §4.12. */
int rt_debug_frustum_records(size_t P, const rt_bvh_node* nodes, const rt_aabb* aabbs, int max_log2, int stack_cap,
                             int64_t* info, float* rec, size_t rec_cap);

/* Durations (ms) of the render kernel of the most recent min(max, launches, 256) timed
 * rt_render_device calls on this scene, oldest first, measured with HIP events recorded
 * on the launch stream around the kernel (direct calls are all timed; an rt_renderer's frames
 * one in RT_TUNE_KERNEL_TIMING_EVERY, *n_out then counts the timed ones).  Waits for those
 * launches to finish. */
int rt_kernel_times(const rt_scene* s, float* ms_out, int max, int* n_out);
/* The same for the whole device frame: the root-box cull pass and the tree-cut cull pass (when
 * it runs), timed on the scene's prep stream, plus the render kernel.  (A frame's pre-passes
 * overlap the previous frame's render kernel, so this is the frame's device work, not the
 * span from its first launch to its end.) */
int rt_frame_times(const rt_scene* s, float* ms_out, int max, int* n_out);
/* The pre-passes alone (root-box cull + tree-cut cull). */
int rt_prepass_times(const rt_scene* s, float* ms_out, int max, int* n_out);
/* Pixel tiles of the most recent rt_render_device call that survived the root-box cull, and
 * all tiles (the tree-cut pass may still cull some of the survivors; those are flagged, not
 * removed from the lists).  Waits for that call to finish. */
int rt_live_tiles(const rt_scene* s, int64_t* live, int64_t* total);
/* Tiles of the most recent rt_render_device call that its render kernel took first (heavy-first
 * dispatch: tiles whose waves took >= 1/4 of the previous finished frame's render kernel in the
 * last frame that rendered them; their order only, never their pixels).  Waits for that call. */
int rt_heavy_tiles(const rt_scene* s, int64_t* heavy);
/* The render kernel instantiation the most recent rt_render_device call launched, as rocprofv3
 * names it ("render_tiles_kernel<49, true, true, 7, 0>"; "" before the first frame): bench.py
 * keys its measured per-launch HBM traffic by it. */
const char* rt_scene_kernel_name(const rt_scene* s);

/* Traversal setup rt_scene_create chose for s: info = {log2 of the camera rays' frustum-record
 * arity (3..5; 2 = the 4-ary records; 0 = no frustum traversal), their DFS stack bound
 * (<= 128 unless RT_TUNE_FRUSTUM_STACK_CAP raised it), 1 if the 4-ary records exist, 1 if the
 * scene takes the deep (512-entry stack) kernels}. */
int rt_scene_traversal_info(const rt_scene* s, int64_t info[4]);
/* Device-side fault flags of s, OR-ed by the kernels since the last clear (waits for the
 * scene's work): bit 0 = a camera-ray frustum traversal needed more than its 128 stack
 * entries (the host bound makes this impossible for records built with the default cap; the
 * wave's answers were poisoned: no hit).  clear != 0 resets the flags.  rt_render
 * returns RT_ERR_INTERNAL when its frame raised one (it clears the flags when the frame starts). */
int rt_scene_faults(rt_scene* s, uint32_t* flags, int clear);

/* ---- Tuning knobs (process-wide; read when a scene is created or a frame is set up) ----
 * The library reads no environment variables: every setting that selects among exact kernel
 * variants or schedules is set here, by tests and A/B scripts.  Frames are identical under
 * every value (order of work only), except RT_TUNE_FRUSTUM_STACK_CAP, a test hook. */
typedef enum {
    RT_TUNE_FRUSTUM_ARITY = 0,   /* log2 of the largest frustum-record arity to build, 2..5 (5) */
    RT_TUNE_HALF_WAVES = 1,      /* -1 auto (default: from 4 band shards, and multi-bounce), 0, 1 */
    RT_TUNE_PAIRED_ONLY = 2,     /* 1 (default): one-light bounce frames take the paired-only kernels */
    RT_TUNE_HEAVY_FRAC = 3,      /* heavy-first class threshold, fraction of a frame (0.10; 0 = off) */
    RT_TUNE_HEAVY_CAP = 4,       /* heavy-list entries per (class, list) (512) */
    RT_TUNE_CULL_COVERAGE = 5,   /* the cut pass runs when the root box covers <= this (0.3; >= 1: always) */
    RT_TUNE_CULL_BOXES = 6,      /* boxes of the tile-culling cut (64; at scene creation) */
    RT_TUNE_BIG_SCENE_BYTES = 7, /* scenes above this take the 8-wave depth-1 kernel (64 MiB) */
    RT_TUNE_FRUSTUM_STACK_CAP = 8, /* TEST HOOK: stack bound the frustum records may need (128) */
    RT_TUNE_PEER_TIMEOUT_S = 9,  /* rt_renderer: seconds to wait for a peer rank (120) */
    RT_TUNE_RENDERER_THREADS = 10, /* rt_renderer: -1 auto (default: a thread per further distinct
                                      GPU), 0 submit every rank from the caller, 1 threads always */
    RT_TUNE_COPY_ENGINE = 11,    /* rt_renderer's host delivery: -1 auto (SDMA where it applies: one rank,
                                    DIRECT, a host frame), 0 the HIP runtime's copies, 1 SDMA or fail */
    RT_TUNE_QUANT_RECORDS = 12,  /* quantised frustum records for the big-scene kernels, at scene creation:
                                    0 never (default; measured slower on c5), -1 scenes whose float
                                    records exceed 1/8 of RT_TUNE_BIG_SCENE_BYTES, 1 always */
    RT_TUNE_PREPASS_GATE = 13,   /* f in (0, 1]: a frame's render kernel opens the next frame's cull/cut
                                    pre-passes when its first work queue has handed out the fraction
                                    f of its items (0.5 default; 1: drained, they then fill its
                                    tail); 0: they start when the frame before it has finished.
                                    Off while RT_TUNE_OVERLAP_FRAMES is on */
    RT_TUNE_OVERLAP_FRAMES = 14, /* rt_renderer frames: 1 lets a frame's render kernel start while the previous
                                    one's tail still runs (two render streams per scene); 0 (default) */
    RT_TUNE_KERNEL_TIMING_EVERY = 15, /* rt_renderer frames: the render kernel's start event (kernel times) in one
                                    frame of this many (4); an event before every kernel held each
                                    dispatch ~5 us */
    RT_TUNE_RECORD_GREEDY = 16,  /* frustum records grown by expanding the entry of largest weight: 2
                                    (default) surface area x sqrt(leaves below), 1 surface area;
                                    0: every path to the same depth; at scene creation */
    RT_TUNE_WIDE4_GREEDY = 17,   /* the 4-ary records (shadow and bounce rays) grown by expanding the
                                    largest-area entry (1, default; 2: x sqrt(leaves below)) instead
                                    of the grandchildren (0); at scene creation */
    RT_TUNE_PAIR_FRAMES = 18,    /* rt_render_device_pair / rt_renderer_submit_pair: 1 (default) renders the
                                    two frames in one launch of the render kernel where it is
                                    instantiated for them (depth-1 sample kernels of the wave
                                    traversal and the paired-only bounce kernels, scene within
                                    RT_TUNE_BIG_SCENE_BYTES); 0 two launches */
    RT_TUNE_PAIR_RESERVE = 19,   /* pair kernels: block slots per CU left free for the next pair's pre-passes
                                    (default 1 for depth-1 frames, 0 for the bounce kernels'
                                    pairs; fractions: that many per CU on average) */
    RT_TUNE_CUT_SUB = 20,        /* sub-boxes per box of the tile-culling cut, tested for the tiles whose rays
                                    may reach that box (16; a power of two <= 64; < 2: one level);
                                    at scene creation */
    RT_TUNE_HW1_LANES = 21,      /* rt_render_hw1_deliver: frames alternate over this many lanes (binning
                                    buffers + a stream each, 1..8; default 2): a lane
                                    overlaps the others only on a hardware queue of its own (HIP:
                                    GPU_MAX_HW_QUEUES per process, 4 by default) */
    RT_TUNE_COPY_WAIT = 22,      /* the SDMA copier threads (rt_renderer's and rt_hw1_scene's deliveries): 1 waits
                                    for a frame with hipEventSynchronize, 0 polls hipEventQuery spinning,
                                    2..1000 polls every that many microseconds; default -1: the renderer
                                    spins, the HW1 scene waits; at the copier's creation */
    RT_TUNE_HW1_FUSE = 23,       /* the HW1 scene's frames: bit 0 the scan fused into the count pass (its last
                                    block, up to 5,120 tiles), bit 1 the resolve fused into the render pass
                                    (each tile's last item); default 2 */
    RT_TUNE_HW1_CHUNK = 24,      /* the HW1 scene's render work items: list entries per item, 16..256, a power of two
                                    (32) */
    RT_TUNE_COUNT = 25
} rt_tune_id;
/* Set knob id (NaN restores the default).  RT_ERR_ARG for an unknown id. */
int rt_tuning_set(int id, double value);
/* The value set for id, or NaN when it has its default. */
int rt_tuning_get(int id, double* value);
void rt_tuning_reset(void);

int rt_device_count(int* n);
const char* rt_last_error(void);
int rt_abi_version(void);
/* sha256 (hex) of the csrc/ and include/ sources and compile flags this library was built from
 * (raytracinginonesemester_amd/build.py: source_build_id), so a caller can prove which sources
 * the loaded binary came from. */
const char* rt_build_id(void);

#ifdef __cplusplus
}
#endif
#endif /* RT_MI355X_H */
