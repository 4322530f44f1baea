// oracle/ref/ref_g.cpp — TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// Driver around the reference's own HW2 "GPUandCPU" CPU build
// (/root/reference/HW2/HW2/GPUandCPU, abbreviated G/ below), compiled from the
// sources where they lie by oracle/Makefile into oracle/_ref/ref_g.  It calls the
// reference functions directly and dumps their outputs so that tests/golden can be
// generated from the reference itself (tests/golden/gen_golden.py).
//
// The reference's app keeps its pipeline inline in main() (G/src/main.cu:98-436),
// so this driver pulls that translation unit in with its main renamed and replays
// the same call sequence:
//   SceneIO::LoadSceneFromFile            G/include/scene.h:382
//   LoadOBJ_ToMesh / applyObjectTransform / AppendMesh   G/src/main.cu:168-190
//   BVH::calculateAABBs, std::accumulate(AABB::merge), BVH::buildBVH (CPU)
//                                         G/src/main.cu:256-317
//   triangle packing                      G/src/main.cu:388-404
//   render() CPU branch                   G/include/query.cu:130-166
//   SearchBVH on the primary rays         G/include/query.h:224-311
// Nothing here changes reference arithmetic; it only chooses inputs and writes outputs.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cfloat>
#include <cmath>
#include <string>
#include <vector>
#include <random>
#include <numeric>
#include <chrono>
#include <fstream>
#include <iostream>
#include <sstream>
#include <algorithm>
#include <functional>
#include <unordered_map>
#include <utility>
#include <limits>
#include <stdexcept>

// Camera keeps its derived basis private (G/include/camera.h:208-216); the dump needs it.
#define private public
#define main ref_g_shipped_main
#include "main.cu"
#undef main
#undef private

namespace {

bool write_bin(const std::string& path, const void* p, size_t n) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    size_t w = n ? std::fwrite(p, 1, n, f) : 0;
    std::fclose(f);
    return w == n;
}

void hexf(FILE* f, const char* name, float v) { std::fprintf(f, "  \"%s\": \"%a\",\n", name, (double)v); }
void hexv(FILE* f, const char* name, const Vec3& v) {
    std::fprintf(f, "  \"%s\": [\"%a\", \"%a\", \"%a\"],\n", name, (double)v.x, (double)v.y, (double)v.z);
}

int usage() {
    std::fprintf(stderr,
        "usage: ref_g jitter <spp> <seed>\n"
        "       ref_g scene <scene.json> <project_dir> <outdir> [W H spp max_depth diffuse(0/1|-1) hits(0/1)]\n"
        "       ref_g arrays <indir> <outdir> W H spp max_depth diffuse(0/1)\n");
    return 2;
}

int cmd_jitter(int argc, char** argv) {
    if (argc < 4) return usage();
    const int spp = std::atoi(argv[2]);
    const unsigned seed = (unsigned)std::strtoul(argv[3], nullptr, 10);
    auto offs = jittered_samples(spp, seed);  // G/include/antialias.h:12-27
    for (auto& o : offs) std::printf("%a %a\n", (double)o.first, (double)o.second);
    return 0;
}

// Path resolution as in G/src/main.cu:119-147 (scene-relative, cwd, project-relative),
// except that the "project" directory is passed explicitly so the scene JSON can live
// outside the reference tree.
std::string resolve(const std::string& scene_dir, const std::string& project_dir, std::string path) {
    if (SceneIO::is_abs_path(path)) return path;
    auto exists = [](const std::string& p) { std::ifstream f(p); return static_cast<bool>(f); };
    const std::string scene_rel = SceneIO::join_path(scene_dir, path);
    std::string proj_rel = path;
    if (proj_rel.rfind("./", 0) == 0) proj_rel = proj_rel.substr(2);
    proj_rel = SceneIO::join_path(project_dir, proj_rel);
    if (exists(scene_rel)) return scene_rel;
    if (exists(proj_rel)) return proj_rel;
    return scene_rel;
}

int cmd_scene(int argc, char** argv) {
    if (argc < 5) return usage();
    const std::string scene_path = argv[2];
    const std::string project_dir = argv[3];
    const std::string outdir = argv[4];
    int W = argc > 5 ? std::atoi(argv[5]) : 0;
    int H = argc > 6 ? std::atoi(argv[6]) : 0;
    int spp_o = argc > 7 ? std::atoi(argv[7]) : 0;
    int depth_o = argc > 8 ? std::atoi(argv[8]) : 0;
    int diffuse_o = argc > 9 ? std::atoi(argv[9]) : -1;
    int want_hits = argc > 10 ? std::atoi(argv[10]) : 1;

    Scene scene;
    std::string err;
    if (!SceneIO::LoadSceneFromFile(scene_path, scene, &err)) {
        std::fprintf(stderr, "scene load failed: %s\n", err.c_str());
        return 1;
    }
    const std::string scene_dir = SceneIO::dirname(scene_path);

    // G/src/main.cu:164-190
    Mesh globalMesh;
    std::vector<Material> objectMaterials;
    int nextObjectId = 0;
    for (const auto& o : scene.objects) {
        if (!o.type.empty() && o.type != "mesh") continue;
        SceneObject obj = o;
        obj.path = resolve(scene_dir, project_dir, obj.path);
        Mesh tempMesh;
        const int objIdBegin = nextObjectId;
        if (!LoadOBJ_ToMesh(obj.path, tempMesh, nextObjectId)) {
            std::fprintf(stderr, "failed to load OBJ %s\n", obj.path.c_str());
            continue;
        }
        applyObjectTransform(tempMesh, obj);
        if (objectMaterials.size() < static_cast<size_t>(nextObjectId))
            objectMaterials.resize(nextObjectId, Material());
        for (int oid = objIdBegin; oid < nextObjectId; ++oid) objectMaterials[oid] = obj.material;
        AppendMesh(globalMesh, tempMesh);
    }
    if (globalMesh.positions.empty()) { std::fprintf(stderr, "no geometry\n"); return 1; }

    // G/src/main.cu:197-317 (CPU branch)
    const size_t P = globalMesh.indices.size() / 3;
    size_t chunk_size = required<RayTracer::BVHState>(P);
    char* chunk = new char[chunk_size];
    char* chunk_base = chunk;
    RayTracer::BVHState bvhState = RayTracer::BVHState::fromChunk(chunk, P);
    AccStruct::BVH bvh;
    MeshView h_mesh = globalMesh.getView();
    bvh.calculateAABBs(h_mesh, bvhState.AABBs);
    AABB SceneBoundingBox = std::accumulate(
        bvhState.AABBs + (P - 1), bvhState.AABBs + (2 * P - 1), AABB(),
        [](const AABB& l, const AABB& r) { return AABB::merge(l, r); });
    std::vector<unsigned int> TriangleIndices(P);
    std::iota(TriangleIndices.begin(), TriangleIndices.end(), 0);
    bvh.buildBVH(bvhState.Nodes, bvhState.AABBs, SceneBoundingBox, TriangleIndices, static_cast<int>(P));

    // G/src/main.cu:321-338 with the config's overrides.
    int max_depth = scene.settings.max_depth;
    int spp = scene.settings.spp;
    bool diffuse_bounce = scene.settings.diffuse_bounce;
    if (spp_o > 0) spp = spp_o;
    if (depth_o > 0) max_depth = depth_o;
    if (diffuse_o >= 0) diffuse_bounce = diffuse_o != 0;
    Vec3 miss_color = scene.miss_color;
    Camera cam = scene.camera;
    if (W > 0 && H > 0) {
        cam = Camera(cam.get_center(), cam.get_look_at(), cam.get_up_vector(),
                     cam.get_focal_length_mm(), cam.get_sensor_height_mm(), W, H);
    }
    std::vector<Light> lights = scene.lights;
    if (lights.empty()) {
        Light fb;
        fb.position = make_vec3(-3.0f, 0.0f, 1.0f);
        fb.color = make_vec3(1.0f, 1.0f, 1.0f);
        fb.intensity = 1;
        lights.push_back(fb);
    }
    const int img_w = cam.pixel_width, img_h = cam.pixel_height;

    // G/src/main.cu:388-404
    std::vector<Triangle> h_tris(P);
    for (size_t i = 0; i < P; ++i) {
        const uint32_t i0 = globalMesh.indices[i * 3 + 0];
        const uint32_t i1 = globalMesh.indices[i * 3 + 1];
        const uint32_t i2 = globalMesh.indices[i * 3 + 2];
        Vec3 n0 = make_vec3(0, 0, 0), n1 = make_vec3(0, 0, 0), n2 = make_vec3(0, 0, 0);
        if (!globalMesh.normals.empty()) {
            n0 = globalMesh.normals[i0]; n1 = globalMesh.normals[i1]; n2 = globalMesh.normals[i2];
        }
        h_tris[i] = Triangle(globalMesh.positions[i0], globalMesh.positions[i1], globalMesh.positions[i2], n0, n1, n2);
    }

    std::vector<Vec3> image((size_t)img_w * img_h, make_vec3(0, 0, 0));
    auto t0 = std::chrono::high_resolution_clock::now();
    render(P, img_w, img_h, cam, miss_color, max_depth, spp, bvhState.Nodes, bvhState.AABBs, h_tris.data(),
           globalMesh.triangleObjIds.data(), objectMaterials.data(), (int)objectMaterials.size(),
           lights.data(), (int)lights.size(), diffuse_bounce, image.data());
    auto t1 = std::chrono::high_resolution_clock::now();
    const double render_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();

    const size_t nn = 2 * P - 1;
    bool ok = true;
    ok &= write_bin(outdir + "/nodes.bin", bvhState.Nodes, nn * sizeof(BVHNode));
    ok &= write_bin(outdir + "/aabbs.bin", bvhState.AABBs, nn * sizeof(AABB));
    ok &= write_bin(outdir + "/tris.bin", h_tris.data(), P * sizeof(Triangle));
    ok &= write_bin(outdir + "/triobj.bin", globalMesh.triangleObjIds.data(), P * sizeof(int32_t));
    ok &= write_bin(outdir + "/mats.bin", objectMaterials.data(), objectMaterials.size() * sizeof(Material));
    ok &= write_bin(outdir + "/lights.bin", lights.data(), lights.size() * sizeof(Light));
    ok &= write_bin(outdir + "/fb.f32", image.data(), image.size() * sizeof(Vec3));

    if (want_hits) {
        // Primary-hit AOV: the exact rays render() shoots (G/include/query.cu:146-158), each
        // through the reference SearchBVH; triangleIdx and t per (pixel, sample).
        const size_t ns = (size_t)img_w * img_h * spp;
        std::vector<int32_t> hit_idx(ns);
        std::vector<float> hit_t(ns);
        auto offsets = jittered_samples(spp, 42u);
        for (int y = 0; y < img_h; ++y)
            for (int x = 0; x < img_w; ++x)
                for (int si = 0; si < spp; ++si) {
                    float px = float(x) + offsets[si].first;
                    float py = float(y) + offsets[si].second;
                    const Ray ray = cam.get_ray(px, py);
                    HitRecord rec;
                    SearchBVH((int)P, ray, bvhState.Nodes, bvhState.AABBs, h_tris.data(), rec);
                    const size_t k = ((size_t)y * img_w + x) * spp + si;
                    hit_idx[k] = rec.hit ? rec.triangleIdx : -1;
                    hit_t[k] = rec.hit ? (float)rec.t : -1.0f;
                }
        ok &= write_bin(outdir + "/hits.i32", hit_idx.data(), ns * sizeof(int32_t));
        ok &= write_bin(outdir + "/hitt.f32", hit_t.data(), ns * sizeof(float));
    }

    FILE* m = std::fopen((outdir + "/meta.json").c_str(), "w");
    if (!m) return 1;
    std::fprintf(m, "{\n");
    std::fprintf(m, "  \"num_triangles\": %zu,\n  \"width\": %d,\n  \"height\": %d,\n", P, img_w, img_h);
    std::fprintf(m, "  \"spp\": %d,\n  \"max_depth\": %d,\n  \"diffuse_bounce\": %d,\n", spp, max_depth, (int)diffuse_bounce);
    std::fprintf(m, "  \"num_materials\": %zu,\n  \"num_lights\": %zu,\n", objectMaterials.size(), lights.size());
    std::fprintf(m, "  \"sizeof_camera\": %zu,\n  \"sizeof_material\": %zu,\n  \"sizeof_light\": %zu,\n",
                 sizeof(Camera), sizeof(Material), sizeof(Light));
    hexv(m, "miss_color", miss_color);
    hexv(m, "center", cam.center);
    hexv(m, "pixel00_loc", cam.pixel00_loc);
    hexv(m, "pixel_delta_u", cam.pixel_delta_u);
    hexv(m, "pixel_delta_v", cam.pixel_delta_v);
    hexf(m, "focal_length_mm", (float)cam.focal_length_mm);
    std::fprintf(m, "  \"render_ms\": %.3f\n}\n", render_ms);
    std::fclose(m);
    delete[] chunk_base;
    return ok ? 0 : 1;
}

template <class T>
bool read_bin(const std::string& path, std::vector<T>& out) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    out.resize(size_t(n) / sizeof(T));
    const size_t r = out.empty() ? 0 : std::fread(out.data(), sizeof(T), out.size(), f);
    std::fclose(f);
    return r == out.size() && size_t(n) % sizeof(T) == 0;
}

// Caller-supplied scene arrays (any tree, e.g. one deeper than SearchBVH's 512-entry stack)
// straight into the reference render() and SearchBVH (G/include/query.cu:79-167,
// G/include/query.h:224-311): <indir>/{nodes,aabbs,tris,triobj,mats,lights}.bin in the
// reference layouts and <indir>/camera.txt = "pos(3) look_at(3) up(3) focal_mm sensor_mm" (%a).
int cmd_arrays(int argc, char** argv) {
    if (argc < 9) return usage();
    const std::string indir = argv[2], outdir = argv[3];
    const int W = std::atoi(argv[4]), H = std::atoi(argv[5]), spp = std::atoi(argv[6]);
    const int max_depth = std::atoi(argv[7]);
    const bool diffuse_bounce = std::atoi(argv[8]) != 0;
    std::vector<BVHNode> nodes;
    std::vector<AABB> aabbs;
    std::vector<Triangle> tris;
    std::vector<int32_t> triobj;
    std::vector<Material> mats;
    std::vector<Light> lights;
    if (!read_bin(indir + "/nodes.bin", nodes) || !read_bin(indir + "/aabbs.bin", aabbs) ||
        !read_bin(indir + "/tris.bin", tris) || !read_bin(indir + "/triobj.bin", triobj) ||
        !read_bin(indir + "/mats.bin", mats) || !read_bin(indir + "/lights.bin", lights)) {
        std::fprintf(stderr, "cannot read the arrays in %s\n", indir.c_str());
        return 1;
    }
    double c[11];
    FILE* cf = std::fopen((indir + "/camera.txt").c_str(), "r");
    if (!cf) return 1;
    for (double& v : c)
        if (std::fscanf(cf, "%la", &v) != 1) { std::fclose(cf); return 1; }
    std::fclose(cf);
    const Camera cam(make_vec3(float(c[0]), float(c[1]), float(c[2])), make_vec3(float(c[3]), float(c[4]), float(c[5])),
                     make_vec3(float(c[6]), float(c[7]), float(c[8])), c[9], c[10], W, H);
    const size_t P = tris.size();
    const Vec3 miss_color = make_vec3(0.0f, 0.0f, 0.0f);
    std::vector<Vec3> image((size_t)W * H, make_vec3(0, 0, 0));
    render(P, W, H, cam, miss_color, max_depth, spp, nodes.data(), aabbs.data(), tris.data(), triobj.data(),
           mats.data(), (int)mats.size(), lights.data(), (int)lights.size(), diffuse_bounce, image.data());
    const size_t ns = (size_t)W * H * spp;
    std::vector<int32_t> hit_idx(ns);
    std::vector<float> hit_t(ns);
    auto offsets = jittered_samples(spp, 42u);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            for (int si = 0; si < spp; ++si) {
                const Ray ray = cam.get_ray(float(x) + offsets[si].first, float(y) + offsets[si].second);
                HitRecord rec;
                SearchBVH((int)P, ray, nodes.data(), aabbs.data(), tris.data(), rec);
                const size_t k = ((size_t)y * W + x) * spp + si;
                hit_idx[k] = rec.hit ? rec.triangleIdx : -1;
                hit_t[k] = rec.hit ? (float)rec.t : -1.0f;
            }
    bool ok = write_bin(outdir + "/fb.f32", image.data(), image.size() * sizeof(Vec3));
    ok &= write_bin(outdir + "/hits.i32", hit_idx.data(), ns * sizeof(int32_t));
    ok &= write_bin(outdir + "/hitt.f32", hit_t.data(), ns * sizeof(float));
    FILE* m = std::fopen((outdir + "/meta.json").c_str(), "w");
    if (!m) return 1;
    std::fprintf(m, "{\n");
    std::fprintf(m, "  \"num_triangles\": %zu,\n  \"width\": %d,\n  \"height\": %d,\n", P, W, H);
    std::fprintf(m, "  \"spp\": %d,\n  \"max_depth\": %d,\n  \"diffuse_bounce\": %d,\n", spp, max_depth, (int)diffuse_bounce);
    hexv(m, "center", cam.center);
    hexv(m, "pixel00_loc", cam.pixel00_loc);
    hexv(m, "pixel_delta_u", cam.pixel_delta_u);
    hexv(m, "pixel_delta_v", cam.pixel_delta_v);
    std::fprintf(m, "  \"num_lights\": %zu\n}\n", lights.size());
    std::fclose(m);
    return ok ? 0 : 1;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) return usage();
    if (!std::strcmp(argv[1], "jitter")) return cmd_jitter(argc, argv);
    if (!std::strcmp(argv[1], "scene")) return cmd_scene(argc, argv);
    if (!std::strcmp(argv[1], "arrays")) return cmd_arrays(argc, argv);
    return usage();
}
