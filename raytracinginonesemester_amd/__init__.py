"""MI355X-native per-pixel ray path of nirajbabar/raytracinginonesemester.

The compute lives in librt_mi355x.so (HIP kernels for gfx950 + the C ABI of
include/rt_mi355x.h); this package is the host-side mirror of the reference interface.
"""
from ._lib import (RTError, RT_DELIVER_DEVICE, RT_DELIVER_F32, RT_DELIVER_NONE, RT_DELIVER_P6,  # noqa: F401
                   RT_GATHER_AUTO, RT_GATHER_DIRECT, RT_GATHER_HOST_SHARED, RT_GATHER_RCCL, RT_KERNEL_AUTO, RT_KERNEL_LANE,
                   RT_KERNEL_WAVE, RT_RENDERER_SELF_SEND, RT_TILES_AUTO, RT_TILES_LINEAR, RT_TILES_ROWS,
                   RT_TILES_XCD_CHUNK, RT_TIME_DELIVER, RT_TIME_FRAME, RT_TIME_GATHER)
from .api import (  # noqa: F401
    LIGHT_DTYPE, Camera, DeviceScene, HostScene, HW1Scene, MeshHW1, Renderer, build_bvh, comm_unique_id, build_bvh_device, default_material, device_count,
    encode_p6, encode_p6_device, intersect_rays, jittered_samples, p6_header, quantize_p6_device, read_p6,
    render, render_hw1, unpermute_strips_device, write_p6, set_tuning, get_tuning, reset_tuning, tuning,
)
