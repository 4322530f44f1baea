// oracle/ref/ref_hw1.cpp — TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// Driver around the reference's HW1 brute-force CPU path (/root/reference/HW1),
// built from the sources where they lie by oracle/Makefile into oracle/_ref/ref_hw1.
//
//   kat     — the ray–triangle known-answer rays of
//             HW1/test_ray_tri_inter_STANDALONE/test_ray_triangle_inter.cpp:17-126
//             (8 fixed rays + the 0.1-step barycentric sweep), each run through the
//             reference ray_intersection (HW1/include/ray.h:67-117); prints the outcome.
//             Catch2 is absent from the image, so the TEST_CASE bodies are not compiled;
//             this driver shoots the same rays and records the reference's answers.
//   render  — the per-pixel loop of HW1/src/render.cpp:72-116 with the camera,
//             resolution, light and spp as arguments (render.cpp hard-codes them at :43-58),
//             dumping the float framebuffer and the winning triangle index per sample.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cfloat>
#include <cmath>
#include <string>
#include <vector>
#include <limits>
#include "MeshOBJ.h"
#include "camera.h"
#include "ray.h"
#include "raytracer.h"
#include "vec3.h"
#include "antialias.h"

namespace {

bool write_bin(const std::string& path, const void* p, size_t n) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    size_t w = n ? std::fwrite(p, 1, n, f) : 0;
    std::fclose(f);
    return w == n;
}

void kat_one(const Triangle& T, const Vec3& d) {
    Ray r(Vec3{0.0f, 0.0f, 0.0f}, d);
    HitRecord rec = ray_intersection(r, T);
    std::printf("%a %a %a %d %a\n", (double)d.x, (double)d.y, (double)d.z, rec.hit ? 1 : 0,
                rec.hit ? (double)(float)rec.t : -1.0);
}

int cmd_kat() {
    // test_ray_triangle_inter.cpp:21-29
    Vec3 v0{-5.0f, -5.0f, -10.0f};
    Vec3 v1{0.0f, 5.0f, -10.0f};
    Vec3 v2{5.0f, -5.0f, -10.0f};
    Vec3 n{0.0f, 0.0f, 1.0f};
    Triangle T{v0, v1, v2, n, n, n};
    // :32-89 — vertex, inside, outside, edge midpoint, parallel, behind, near-edge in/out
    kat_one(T, Vec3{0.0f, 5.0f, -10.0f});
    kat_one(T, Vec3{0.0f, 0.0f, -10.0f});
    kat_one(T, Vec3{0.0f, 20.0f, -10.0f});
    Vec3 pointOnEdge = (v2 + v1) * 0.5;
    kat_one(T, pointOnEdge);
    kat_one(T, Vec3{5.0f, 0.0f, 0.0f});
    kat_one(T, Vec3{0.0f, 0.0f, 10.0f});
    kat_one(T, Vec3{0.0f, -4.999f, -10.0f});
    kat_one(T, Vec3{0.0f, -5.001f, -10.0f});
    // :116-125 — the sweep, same float loop variables
    for (float alpha = 0.0f; alpha <= 1.0f; alpha += 0.1f) {
        for (float beta = 0.0f; beta <= 1 - alpha; beta += 0.1f) {
            float gamma = 1 - alpha - beta;
            Vec3 ray = alpha * v0 + beta * v1 + gamma * v2;
            kat_one(T, ray);
        }
    }
    return 0;
}

Vec3 v3(char** a) { return make_vec3(std::strtof(a[0], nullptr), std::strtof(a[1], nullptr), std::strtof(a[2], nullptr)); }

int cmd_render(int argc, char** argv) {
    // render <obj> <outdir> W H cx cy cz lx ly lz ux uy uz focal sensor Lx Ly Lz Cr Cg Cb spp
    if (argc < 24) { std::fprintf(stderr, "render: bad args\n"); return 2; }
    const std::string path = argv[2], outdir = argv[3];
    const int W = std::atoi(argv[4]), H = std::atoi(argv[5]);
    const Vec3 pos = v3(argv + 6), look = v3(argv + 9), up = v3(argv + 12);
    const double focal = std::strtod(argv[15], nullptr), sensor = std::strtod(argv[16], nullptr);
    Light light;
    light.position = v3(argv + 17);
    light.color = v3(argv + 20);
    const int spp = std::atoi(argv[23]);

    MeshSOA mesh;
    if (!LoadOBJ_ToMeshSOA(path, mesh)) { std::fprintf(stderr, "load failed\n"); return 1; }
    const size_t indexCount = mesh.indices.size();
    camera cam(pos, look, up, focal, sensor, W, H);

    std::vector<Vec3> image((size_t)W * H);
    std::vector<int32_t> hit_idx((size_t)W * H * spp);
    std::vector<float> hit_t((size_t)W * H * spp);
    auto offsets = jittered_samples(spp, 42u);
    auto center = cam.get_center();
#pragma omp parallel for schedule(dynamic, 1)
    for (int j = 0; j < H; j++) {
        for (int i = 0; i < W; i++) {
            Vec3 accum_color = make_vec3(0.0f, 0.0f, 0.0f);
            int si = 0;
            for (const auto& o : offsets) {
                float px = float(i) + o.first;
                float py = float(j) + o.second;
                // render.cpp:86 — get_pixel_position takes int, so px/py truncate.
                Ray r = Ray(center, cam.get_pixel_position(px, py) - center);
                HitRecord prev;
                prev.hit = false;
                prev.t = std::numeric_limits<float>::max();
                auto color = shade(r, prev, light);
                int best = -1;
                for (int k = 0; k < (int)indexCount; k += 3) {
                    Triangle tri;
                    tri.v0 = mesh.positions[mesh.indices[k]];
                    tri.v1 = mesh.positions[mesh.indices[k + 1]];
                    tri.v2 = mesh.positions[mesh.indices[k + 2]];
                    tri.n0 = mesh.normals[mesh.indices[k]];
                    tri.n1 = mesh.normals[mesh.indices[k + 1]];
                    tri.n2 = mesh.normals[mesh.indices[k + 2]];
                    HitRecord rec = ray_intersection(r, tri);
                    if (rec.hit && rec.t < prev.t) {
                        color = shade(r, rec, light);
                        prev = rec;
                        best = k / 3;
                    }
                }
                accum_color = accum_color + color;
                const size_t kk = ((size_t)j * W + i) * spp + si;
                hit_idx[kk] = best;
                hit_t[kk] = best >= 0 ? (float)prev.t : -1.0f;
                ++si;
            }
            image[(size_t)j * W + i] = accum_color / float(offsets.size());
        }
    }
    bool ok = write_bin(outdir + "/fb.f32", image.data(), image.size() * sizeof(Vec3));
    ok &= write_bin(outdir + "/hits.i32", hit_idx.data(), hit_idx.size() * sizeof(int32_t));
    ok &= write_bin(outdir + "/hitt.f32", hit_t.data(), hit_t.size() * sizeof(float));
    std::printf("triangles %zu\n", indexCount / 3);
    return ok ? 0 : 1;
}

int cmd_jitter(int argc, char** argv) {
    if (argc < 4) return 2;
    auto offs = jittered_samples(std::atoi(argv[2]), (unsigned)std::strtoul(argv[3], nullptr, 10));
    for (auto& o : offs) std::printf("%a %a\n", (double)o.first, (double)o.second);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc >= 2 && !std::strcmp(argv[1], "kat")) return cmd_kat();
    if (argc >= 2 && !std::strcmp(argv[1], "render")) return cmd_render(argc, argv);
    if (argc >= 2 && !std::strcmp(argv[1], "jitter")) return cmd_jitter(argc, argv);
    std::fprintf(stderr, "usage: ref_hw1 kat | render ... | jitter spp seed\n");
    return 2;
}
