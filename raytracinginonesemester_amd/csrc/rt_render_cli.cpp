// rt_render_cli.cpp — command-line renderer over the C++ host API (the role of the
// reference app G/src/main.cu:98-436): scene JSON (or OBJ list) in, ppm_p6 P6 out.
//
//   rt_render_cli scene.json [-o out.ppm] [--width W --height H] [--spp S] [--depth D]
//                 [--project DIR] [--kernel wave|lane]
//   rt_render_cli a.obj b.obj ... [-o out.ppm]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rt_mi355x.hpp"

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s scene.json|mesh.obj... [-o out.ppm] [--width W] [--height H] "
                             "[--spp S] [--depth D] [--project DIR] [--kernel wave|lane]\n", argv[0]);
        return 2;
    }
    std::vector<std::string> inputs;
    std::string out = "render.ppm";
    const char* project = nullptr;
    int W = 0, H = 0, spp = 0, depth = 0, kernel = RT_KERNEL_AUTO;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> const char* {
            if (i + 1 >= argc) { std::fprintf(stderr, "missing value for %s\n", a.c_str()); std::exit(2); }
            return argv[++i];
        };
        if (a == "-o") out = next();
        else if (a == "--width") W = std::atoi(next());
        else if (a == "--height") H = std::atoi(next());
        else if (a == "--spp") spp = std::atoi(next());
        else if (a == "--depth") depth = std::atoi(next());
        else if (a == "--project") project = next();
        else if (a == "--kernel") kernel = std::strcmp(next(), "lane") == 0 ? RT_KERNEL_LANE : RT_KERNEL_WAVE;
        else inputs.push_back(a);
    }
    try {
        const bool is_scene = inputs.size() == 1 &&
                              (inputs[0].size() >= 5 && (inputs[0].rfind(".json") == inputs[0].size() - 5 ||
                                                         inputs[0].rfind(".scene") == inputs[0].size() - 6));
        rt::HostScene hs = is_scene ? rt::HostScene::load_json(inputs[0], project) : rt::HostScene::load_objs(inputs);
        std::printf("Loaded %llu triangles (%d objects), BVH height %d\n",
                    (unsigned long long)hs.info().num_triangles, hs.info().num_objects_loaded, hs.info().bvh_height);
        rt::Camera cam = hs.camera(W, H);
        rt_render_opts o = hs.options();
        if (spp > 0) o.spp = spp;
        if (depth > 0) o.max_depth = depth;
        o.kernel = kernel;
        rt::DeviceScene ds(hs);
        (void)rt::render(ds, rt::Camera(hs.info().cam_position, hs.info().cam_look_at, hs.info().cam_up,
                                        hs.info().focal_length_mm, hs.info().sensor_height_mm, 1, 1), o);  // warm-up
        const auto t0 = std::chrono::high_resolution_clock::now();
        rt::Framebuffer fb = rt::render(ds, cam, o);
        const auto t1 = std::chrono::high_resolution_clock::now();
        const double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        const double samples = double(fb.width) * fb.height * o.spp;
        std::printf("GPU Render Time: %.3f ms (%dx%d, %d spp, depth %d): %.1f Msamples/s\n", ms, fb.width,
                    fb.height, o.spp, o.max_depth, samples / ms * 1e-3);
        rt::write_p6(out, fb);
        std::printf("Image saved to %s\n", out.c_str());
    } catch (const rt::Error& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
