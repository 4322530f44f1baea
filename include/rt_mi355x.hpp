// include/rt_mi355x.hpp — C++ host API over the C ABI (header-only).
//
// The north-star drop-in shape `render(scene, camera) -> framebuffer`: the reference's app
// (G/src/main.cu:98-436) loads a scene, builds the LBVH, calls render() and writes an
// image; the same flow here is
//     rt::HostScene hs = rt::HostScene::load_json("frog.json");
//     rt::DeviceScene ds(hs);                       // arrays resident on the MI355X
//     rt::Camera cam = hs.camera();                 // Camera(pos, lookAt, up, mm, mm, W, H)
//     rt::Framebuffer fb = rt::render(ds, cam, hs.options());
//     rt::write_p6("out.ppm", fb);                  // ppm_p6 defaults
// Errors from the C ABI become rt::Error exceptions on this (C++) side only.
#pragma once

#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "rt_mi355x.h"

namespace rt {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

inline void check(int rc) {
    if (rc != RT_OK) throw Error(rc, rt_last_error());
}

struct Camera {
    rt_camera c{};
    Camera() = default;
    Camera(rt_vec3 pos, rt_vec3 look_at, rt_vec3 up, double focal_mm, double sensor_mm, int w, int h,
           bool hw1 = false) {
        const float p[3] = {pos.x, pos.y, pos.z}, l[3] = {look_at.x, look_at.y, look_at.z},
                    u[3] = {up.x, up.y, up.z};
        check(rt_camera_init(&c, p, l, u, focal_mm, sensor_mm, w, h, hw1 ? 1 : 0));
    }
    int width() const { return c.pixel_width; }
    int height() const { return c.pixel_height; }
};

struct Framebuffer {
    int width = 0, height = 0;
    std::vector<float> rgb;  // height*width*3, row 0 = top (G/include/query.cu:148)
};

class HostScene {
public:
    static HostScene load_json(const std::string& path, const char* project_dir = nullptr) {
        HostScene s;
        check(rt_host_scene_load_json(path.c_str(), project_dir, &s.h_));
        s.refresh();
        return s;
    }
    static HostScene load_objs(const std::vector<std::string>& paths) {
        std::vector<const char*> p;
        for (auto& s : paths) p.push_back(s.c_str());
        HostScene s;
        check(rt_host_scene_load_objs(p.data(), int(p.size()), &s.h_));
        s.refresh();
        return s;
    }
    HostScene() = default;
    HostScene(HostScene&& o) noexcept : h_(o.h_), info_(o.info_), arr_(o.arr_) { o.h_ = nullptr; }
    HostScene& operator=(HostScene&& o) noexcept {
        std::swap(h_, o.h_);
        info_ = o.info_;
        arr_ = o.arr_;
        return *this;
    }
    HostScene(const HostScene&) = delete;
    HostScene& operator=(const HostScene&) = delete;
    ~HostScene() { if (h_) rt_host_scene_free(h_); }

    const rt_scene_info& info() const { return info_; }
    const rt_scene_arrays& arrays() const { return arr_; }
    Camera camera(int w = 0, int h = 0) const {
        return Camera(info_.cam_position, info_.cam_look_at, info_.cam_up, info_.focal_length_mm,
                      info_.sensor_height_mm, w > 0 ? w : info_.pixel_width, h > 0 ? h : info_.pixel_height);
    }
    rt_render_opts options() const {
        rt_render_opts o;
        rt_render_opts_default(&o);
        o.max_depth = info_.max_depth;
        o.spp = info_.spp;
        o.diffuse_bounce = info_.diffuse_bounce;
        o.miss_color = info_.miss_color;
        return o;
    }

private:
    void refresh() {
        check(rt_host_scene_info(h_, &info_));
        check(rt_host_scene_arrays(h_, &arr_));
    }
    rt_host_scene* h_ = nullptr;
    rt_scene_info info_{};
    rt_scene_arrays arr_{};
};

class DeviceScene {
public:
    explicit DeviceScene(const HostScene& hs, int device = 0) {
        const auto& a = hs.arrays();
        const auto& i = hs.info();
        check(rt_scene_create(device, size_t(i.num_triangles), a.nodes, a.aabbs, a.triangles, a.tri_object_ids,
                              a.materials, i.num_materials, a.lights, i.num_lights, &s_));
    }
    DeviceScene(const DeviceScene&) = delete;
    DeviceScene& operator=(const DeviceScene&) = delete;
    ~DeviceScene() { if (s_) rt_scene_destroy(s_); }
    rt_scene* get() const { return s_; }

private:
    rt_scene* s_ = nullptr;
};

inline Framebuffer render(const DeviceScene& ds, const Camera& cam, const rt_render_opts& opt) {
    Framebuffer fb;
    fb.width = cam.width();
    fb.height = rt_shard_rows(cam.height(), opt.band_rows, opt.band_index, opt.band_count);
    if (fb.height < 0) throw Error(RT_ERR_ARG, "bad band parameters");
    fb.rgb.resize(size_t(fb.width) * size_t(fb.height) * 3);
    check(rt_render(ds.get(), &cam.c, &opt, fb.rgb.data(), nullptr, nullptr));
    return fb;
}

inline void write_p6(const std::string& path, const Framebuffer& fb, const rt_ppm_options* opt = nullptr) {
    check(rt_ppm_write(path.c_str(), fb.rgb.data(), fb.width, fb.height, opt));
}

}  // namespace rt
