"""ctypes binding of include/rt_mi355x.h (librt_mi355x.so, built in-tree by build.py).

The library is loaded lazily on first use and never replaced by a Python/CPU fallback:
if the shared object is missing or a render call finds no gfx950 device, the call raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("RT_MI355X_LIB", PKG / "lib" / "librt_mi355x.so"))

RT_OK = 0
RT_ERR = {
    -1: "RT_ERR_ARG", -2: "RT_ERR_IO", -3: "RT_ERR_PARSE", -4: "RT_ERR_HIP",
    -5: "RT_ERR_NOMEM", -6: "RT_ERR_NODEVICE", -7: "RT_ERR_UNSUPPORTED", -8: "RT_ERR_COMM",
    -9: "RT_ERR_INTERNAL",
}
RT_KERNEL_AUTO, RT_KERNEL_WAVE, RT_KERNEL_LANE, RT_KERNEL_WAVE_PIXELS = 0, 1, 2, 3
RT_TILES_AUTO, RT_TILES_LINEAR, RT_TILES_XCD_CHUNK, RT_TILES_ROWS = 0, 1, 2, 3
RT_FLAG_NO_CULL = 1
RT_FLAG_BINARY = 4
RT_DELIVER_P6, RT_DELIVER_F32, RT_DELIVER_DEVICE, RT_DELIVER_NONE = 0, 1, 2, 3
RT_GATHER_AUTO, RT_GATHER_RCCL, RT_GATHER_DIRECT, RT_GATHER_HOST_SHARED = 0, 1, 2, 3
RT_RENDERER_SELF_SEND = 1
RT_TIME_GATHER, RT_TIME_DELIVER, RT_TIME_FRAME = 0, 1, 2
RT_FAULT_FRUSTUM_STACK = 1
# rt_tune_id (include/rt_mi355x.h): knob name -> id
TUNE = {"frustum_arity": 0, "half_waves": 1, "paired_only": 2, "heavy_frac": 3, "heavy_cap": 4,
        "cull_coverage": 5, "cull_boxes": 6, "big_scene_bytes": 7, "frustum_stack_cap": 8,
        "peer_timeout_s": 9, "renderer_threads": 10, "copy_engine": 11,
        "quant_records": 12, "prepass_gate": 13,
        "overlap_frames": 14, "kernel_timing_every": 15,
        "record_greedy": 16, "wide4_greedy": 17, "pair_frames": 18, "pair_reserve": 19,
        "cut_sub": 20, "hw1_lanes": 21, "copy_wait": 22, "hw1_fuse": 23, "hw1_chunk": 24}


class RTError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{RT_ERR.get(code, code)}: {msg}")
        self.code = code


class Vec3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]

    def __iter__(self):
        return iter((self.x, self.y, self.z))


class BVHNode(C.Structure):
    _fields_ = [("parent_idx", C.c_uint32), ("left_idx", C.c_uint32),
                ("right_idx", C.c_uint32), ("object_idx", C.c_uint32)]


class AABB(C.Structure):
    _fields_ = [("min_corner", Vec3), ("max_corner", Vec3)]


class Triangle(C.Structure):
    _fields_ = [("v0", Vec3), ("v1", Vec3), ("v2", Vec3), ("n0", Vec3), ("n1", Vec3), ("n2", Vec3)]


class Material(C.Structure):
    _fields_ = [("albedo", Vec3), ("kd", C.c_float), ("specular_color", Vec3), ("ks", C.c_float),
                ("shininess", C.c_float), ("kr", C.c_float), ("emission", Vec3)]


class Light(C.Structure):
    _fields_ = [("position", Vec3), ("color", Vec3), ("intensity", C.c_int32)]


class CameraT(C.Structure):
    _fields_ = [("center", Vec3), ("pixel00_loc", Vec3), ("pixel_delta_u", Vec3),
                ("pixel_delta_v", Vec3), ("pixel_width", C.c_int32), ("pixel_height", C.c_int32)]


class SceneInfo(C.Structure):
    _fields_ = [("max_depth", C.c_int32), ("spp", C.c_int32), ("diffuse_bounce", C.c_int32),
                ("miss_color", Vec3), ("cam_position", Vec3), ("cam_look_at", Vec3), ("cam_up", Vec3),
                ("focal_length_mm", C.c_double), ("sensor_height_mm", C.c_double),
                ("pixel_width", C.c_int32), ("pixel_height", C.c_int32),
                ("num_triangles", C.c_uint64), ("num_vertices", C.c_uint64),
                ("num_materials", C.c_int32), ("num_lights", C.c_int32),
                ("num_objects_loaded", C.c_int32), ("bvh_max_stack", C.c_int32),
                ("bvh_height", C.c_int32)]


class SceneArrays(C.Structure):
    _fields_ = [("nodes", C.c_void_p), ("aabbs", C.c_void_p), ("triangles", C.c_void_p),
                ("tri_object_ids", C.c_void_p), ("materials", C.c_void_p), ("lights", C.c_void_p),
                ("positions", C.c_void_p), ("normals", C.c_void_p), ("indices", C.c_void_p)]


class MeshView(C.Structure):
    _fields_ = [("positions", C.c_void_p), ("normals", C.c_void_p), ("indices", C.c_void_p),
                ("num_vertices", C.c_uint64), ("num_triangles", C.c_uint64),
                ("has_normals", C.c_int32), ("has_uvs", C.c_int32)]


class PPMOptions(C.Structure):
    _fields_ = [("maxval", C.c_int32), ("clamp", C.c_int32), ("gamma2", C.c_int32), ("flip_y", C.c_int32)]


class RenderOpts(C.Structure):
    _fields_ = [("max_depth", C.c_int32), ("spp", C.c_int32), ("diffuse_bounce", C.c_int32),
                ("miss_color", Vec3), ("jitter", C.c_void_p), ("band_rows", C.c_int32),
                ("band_index", C.c_int32), ("band_count", C.c_int32), ("kernel", C.c_int32),
                ("tile_order", C.c_int32), ("flags", C.c_int32)]


class RendererOpts(C.Structure):
    _fields_ = [("n_devices", C.c_int32), ("devices", C.c_void_p), ("world_size", C.c_int32),
                ("rank0", C.c_int32), ("unique_id", C.c_void_p), ("band_rows", C.c_int32),
                ("deliver", C.c_int32), ("gather", C.c_int32), ("depth", C.c_int32), ("flags", C.c_int32),
                ("host_frame_name", C.c_void_p)]


P = C.c_void_p
I = C.c_int
SZ = C.c_size_t

# name -> (restype, argtypes); every symbol declared in include/rt_mi355x.h
SIGNATURES = {
    "rt_material_default": (None, [P]),
    "rt_camera_init": (I, [P, P, P, P, C.c_double, C.c_double, I, I, I]),
    "rt_jittered_samples": (I, [I, C.c_uint32, I, P]),
    "rt_host_scene_load_json": (I, [C.c_char_p, C.c_char_p, P]),
    "rt_host_scene_load_objs": (I, [P, I, P]),
    "rt_host_scene_info": (I, [P, P]),
    "rt_host_scene_arrays": (I, [P, P]),
    "rt_host_scene_free": (None, [P]),
    "rt_build_bvh": (I, [P, SZ, P, SZ, P, P]),
    "rt_build_bvh_device": (I, [I, P, SZ, P, SZ, P, P, P]),
    "rt_mesh_load_obj_hw1": (I, [C.c_char_p, P]),
    "rt_mesh_view_get": (I, [P, P]),
    "rt_mesh_free": (None, [P]),
    "rt_ppm_options_default": (None, [P]),
    "rt_ppm_write": (I, [C.c_char_p, P, I, I, P]),
    "rt_ppm_encode": (I, [P, I, I, P, P, SZ, P]),
    "rt_ppm_read": (I, [C.c_char_p, P, SZ, P, P, P]),
    "rt_ppm_header": (I, [I, I, I, P, SZ, P]),
    "rt_ppm_quantize_device": (I, [P, I, I, P, P, P]),
    "rt_unpermute_strips_device": (I, [P, I, SZ, I, I, I, I, P, P]),
    "rt_scene_create": (I, [I, SZ, P, P, P, P, P, I, P, I, P]),
    "rt_scene_destroy": (None, [P]),
    "rt_scene_clone": (I, [P, I, P]),
    "rt_scene_device": (I, [P]),
    "rt_scene_device_bytes": (SZ, [P]),
    "rt_render_opts_default": (None, [P]),
    "rt_shard_rows": (I, [I, I, I, I]),
    "rt_render_device": (I, [P, P, P, P, P, P, P]),
    "rt_render_device_p6": (I, [P, P, P, P, P, P, P, P]),
    "rt_render_device_pair": (I, [P, P, P, P, P, P, P, P, P]),
    "rt_render": (I, [P, P, P, P, P, P]),
    "rt_count_rays": (I, [P, P, P, P]),
    "rt_count_rays_ex": (I, [P, P, P, P]),
    "rt_render_reference": (I, [SZ, I, I, P, Vec3, I, I, P, P, P, P, P, I, P, I, I, P]),
    "rt_render_reference_gpus": (I, [SZ, I, I, P, Vec3, I, I, P, P, P, P, P, I, P, I, I, I, P]),
    "rt_renderer_opts_default": (None, [P]),
    "rt_comm_unique_id": (I, [P]),
    "rt_renderer_create": (I, [SZ, P, P, P, P, P, I, P, I, P, P]),
    "rt_renderer_destroy": (None, [P]),
    "rt_renderer_submit": (I, [P, P, P, P]),
    "rt_renderer_submit_pair": (I, [P, P, P, P, P]),
    "rt_renderer_wait": (I, [P, C.c_uint64, P, P]),
    "rt_renderer_render": (I, [P, P, P, P, SZ]),
    "rt_renderer_scene": (P, [P, I]),
    "rt_renderer_local_ranks": (I, [P]),
    "rt_renderer_copy_engine": (I, [P]),
    "rt_renderer_times": (I, [P, I, P, I, P]),
    "rt_render_hw1": (I, [I, P, P, P, SZ, P, Vec3, Vec3, I, P, P, P, P]),
    "rt_render_hw1_ex": (I, [I, P, P, P, SZ, P, Vec3, Vec3, I, P, I, P, P, P, P]),
    "rt_hw1_scene_create": (I, [I, P, P, P, SZ, P]),
    "rt_hw1_scene_destroy": (None, [P]),
    "rt_render_hw1_device": (I, [P, P, Vec3, Vec3, I, P, I, P, P, P, P, P]),
    "rt_render_hw1_deliver": (I, [P, P, Vec3, Vec3, I, I, P, P, P]),
    "rt_hw1_wait": (I, [P, C.c_uint64]),
    "rt_hw1_kernel_times": (I, [P, P, I, P]),
    "rt_hw1_kernel_name": (C.c_char_p, [P]),
    "rt_hw1_list_info": (I, [P, P]),
    "rt_intersect_rays": (I, [I, P, P, P, I, I, C.c_float, C.c_float, P, P]),
    "rt_powf_host": (C.c_float, [C.c_float, C.c_float]),
    "rt_debug_frustum_records": (C.c_int, [C.c_size_t, P, P, C.c_int, C.c_int, P, P, C.c_size_t]),
    "rt_powf_batch": (I, [I, P, P, I, P]),
    "rt_box_test_host": (I, [P, P, P, I, P, P, P]),
    "rt_kernel_times": (I, [P, P, I, P]),
    "rt_frame_times": (I, [P, P, I, P]),
    "rt_prepass_times": (I, [P, P, I, P]),
    "rt_live_tiles": (I, [P, P, P]),
    "rt_heavy_tiles": (I, [P, P]),
    "rt_scene_kernel_name": (C.c_char_p, [P]),
    "rt_scene_traversal_info": (I, [P, P]),
    "rt_scene_faults": (I, [P, P, I]),
    "rt_tuning_set": (I, [I, C.c_double]),
    "rt_tuning_get": (I, [I, P]),
    "rt_tuning_reset": (None, []),
    "rt_device_count": (I, [P]),
    "rt_last_error": (C.c_char_p, []),
    "rt_abi_version": (I, []),
    "rt_build_id": (C.c_char_p, []),
}

_lib = None


def lib() -> C.CDLL:
    """Load librt_mi355x.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RTError(-6, f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        # One HIP runtime per process: when torch is installed, its bundled HIP runtime must be
        # the one this library binds to (device pointers and streams are shared with torch), so
        # torch is loaded first.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            # experiment builds of older sources (scripts/ab_libs.py) may lack newer entry points:
            # those raise AttributeError when called; the in-tree library exports them all
            # (tests/test_host.py checks every symbol of include/rt_mi355x.h)
            if LIB_PATH != PKG / "lib" / "librt_mi355x.so" and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != RT_OK:
        msg = lib().rt_last_error()
        raise RTError(rc, msg.decode() if msg else "")


def ptr(a) -> int | None:
    """Address of a numpy array / ctypes object (None passes NULL)."""
    if a is None:
        return None
    if hasattr(a, "ctypes"):
        return a.ctypes.data
    return C.addressof(a)
