// rt_hip_host.hpp — host-side HIP helpers shared by the device translation units
// (error mapping into the C ABI's RT_ERR_HIP, owned device buffers, gfx950 check).
#pragma once

#include <hip/hip_runtime.h>

#include <cstring>
#include <string>

#include "rt_common.hpp"

namespace rt {

inline std::string hip_msg(hipError_t e, const char* what) {
    return std::string(what) + ": " + hipGetErrorString(e);
}
#define HIP_TRY(expr)                                                          \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess) return set_error(RT_ERR_HIP, hip_msg(e_, #expr)); \
    } while (0)

struct DevBuf {
    void* p = nullptr;
    size_t n = 0;
    ~DevBuf() { if (p) (void)hipFree(p); }
    int alloc(size_t bytes) {
        if (p) { (void)hipFree(p); p = nullptr; }
        n = bytes;
        if (bytes == 0) return RT_OK;
        hipError_t e = hipMalloc(&p, bytes);
        if (e != hipSuccess) { p = nullptr; return set_error(RT_ERR_HIP, hip_msg(e, "hipMalloc")); }
        return RT_OK;
    }
    int upload(const void* src, size_t bytes) {
        int rc = alloc(bytes);
        if (rc != RT_OK || bytes == 0) return rc;
        hipError_t e = hipMemcpy(p, src, bytes, hipMemcpyHostToDevice);
        if (e != hipSuccess) return set_error(RT_ERR_HIP, hip_msg(e, "hipMemcpy H2D"));
        return RT_OK;
    }
};

inline int check_device(int device) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) return set_error(RT_ERR_NODEVICE, "no HIP device visible");
    if (device < 0 || device >= n) return set_error(RT_ERR_ARG, "device index out of range");
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) return set_error(RT_ERR_HIP, hip_msg(e, "hipGetDeviceProperties"));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return set_error(RT_ERR_NODEVICE, std::string("kernels are built for gfx950, device is ") + prop.gcnArchName);
    return RT_OK;
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        (void)hipSetDevice(d);
    }
    ~DeviceGuard() { if (prev >= 0) (void)hipSetDevice(prev); }
};

// The HIP events around the most recent frame of a scene (rt_render_device*, rt_device.hip):
// before its first launch and after its render kernel, both on the frame's stream and owned
// by the scene (valid for the scene's next 255 frames); nullptr before the first frame.
// rt_renderer synchronises on these instead of recording events of its own on that stream.
// back: the frame that many frames before the most recent (1: frame A of a pair just rendered).
void scene_frame_events(const rt_scene* s, hipEvent_t* first, hipEvent_t* last, int back = 0);
// A caller that orders the reuse of its output buffers itself (rt_renderer: host waits per
// frame slot) lets a scene's frame pre-passes skip the wait for the work queued before the
// frame on its stream, so they overlap the previous frame's render kernel (rt_device.hip).
void scene_set_caller_ordered(rt_scene* s, bool on);

}  // namespace rt
