"""Python mirror of the reference's host interface for the per-pixel ray path.

Names and argument meaning follow the reference (citations relative to the reference repo,
G/ = HW2/HW2/GPUandCPU):

* :class:`Camera`       — ``Camera(pos, lookAt, up, focal_length_mm, sensor_height_mm, w, h)``
                          (G/include/camera.h:13-28).
* :class:`HostScene`    — ``SceneIO::LoadSceneFromFile`` + the mesh/BVH pipeline of
                          G/src/main.cu:104-317 (loaders, transforms, CPU LBVH).
* :class:`DeviceScene`  — the scene arrays resident on one MI355X.
* :func:`render`        — ``render(numTriangles, W, H, cam, missColor, max_depth, spp, nodes,
                          aabbs, triangles, triObjectIds, objectMaterials, numObjectMaterials,
                          lights, numLights, diffuse_bounce, output)`` (G/include/query.h:13-29).
* :func:`render_hw1`    — the HW1 brute-force loop (HW1/src/render.cpp:72-116) on the GPU.
* :func:`write_p6` / :func:`read_p6` — ppm_p6 (HW1/ppm_p6_lib/include/ppm_p6.hpp:46-85).

All compute goes through librt_mi355x.so; there is no CPU render path here.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path
from typing import Optional, Sequence

import numpy as np

from . import _lib as L
from ._lib import check, lib, ptr

LIGHT_DTYPE = np.dtype([("position", "<f4", 3), ("color", "<f4", 3), ("intensity", "<i4")])
assert LIGHT_DTYPE.itemsize == C.sizeof(L.Light) == 28
assert C.sizeof(L.Material) == 52 and C.sizeof(L.Triangle) == 72 and C.sizeof(L.AABB) == 24


def _v3(v) -> L.Vec3:
    x, y, z = (float(c) for c in v)
    return L.Vec3(x, y, z)


def _f3(v) -> "C.Array":
    return (C.c_float * 3)(*[float(c) for c in v])


class Camera:
    """Pinhole camera; ``hw1=True`` follows HW1/include/camera.h (rejects w, h < 1)."""

    def __init__(self, pos=(0.0, 0.0, 0.0), look_at=(0.0, 1.0, 0.0), up=(0.0, 0.0, 1.0),
                 focal_length_mm: float = 50.0, sensor_height_mm: float = 24.0,
                 width: int = 100, height: int = 100, hw1: bool = False):
        self.pos, self.look_at, self.up = tuple(pos), tuple(look_at), tuple(up)
        self.focal_length_mm, self.sensor_height_mm = float(focal_length_mm), float(sensor_height_mm)
        self.c = L.CameraT()
        check(lib().rt_camera_init(C.byref(self.c), _f3(pos), _f3(look_at), _f3(up),
                                   self.focal_length_mm, self.sensor_height_mm, int(width), int(height),
                                   1 if hw1 else 0))

    @property
    def pixel_width(self) -> int:
        return self.c.pixel_width

    @property
    def pixel_height(self) -> int:
        return self.c.pixel_height

    def basis(self) -> dict:
        """center, pixel00_loc, pixel_delta_u, pixel_delta_v as float32 arrays."""
        return {k: np.array(tuple(getattr(self.c, k)), np.float32)
                for k in ("center", "pixel00_loc", "pixel_delta_u", "pixel_delta_v")}

    def resized(self, width: int, height: int) -> "Camera":
        return Camera(self.pos, self.look_at, self.up, self.focal_length_mm, self.sensor_height_mm,
                      width, height)


def jittered_samples(spp: int, seed: int = 42, centered: bool = True) -> np.ndarray:
    """(spp, 2) float32 sub-pixel offsets (G/include/antialias.h:12-27; HW1 when not centered)."""
    out = np.zeros((spp, 2), np.float32)
    check(lib().rt_jittered_samples(int(spp), int(seed), 1 if centered else 0, ptr(out)))
    return out


def default_material() -> np.ndarray:
    m = L.Material()
    lib().rt_material_default(C.byref(m))
    return np.frombuffer(bytes(m), np.float32).copy()


class HostScene:
    """A G/-dialect scene loaded and BVH-built on the host (arrays in the reference layouts)."""

    def __init__(self, handle: int):
        self._h = C.c_void_p(handle)
        info = L.SceneInfo()
        check(lib().rt_host_scene_info(self._h, C.byref(info)))
        self.info = info
        arr = L.SceneArrays()
        check(lib().rt_host_scene_arrays(self._h, C.byref(arr)))
        P = int(info.num_triangles)
        NN = 2 * P - 1
        nv = int(info.num_vertices)

        def view(addr, dtype, shape):
            if not addr:
                return None
            n = int(np.prod(shape)) * np.dtype(dtype).itemsize
            buf = (C.c_char * n).from_address(addr)
            return np.frombuffer(buf, dtype).reshape(shape).copy()  # own the data

        self.num_triangles = P
        self.nodes = view(arr.nodes, np.uint32, (NN, 4))
        self.aabbs = view(arr.aabbs, np.float32, (NN, 6))
        self.triangles = view(arr.triangles, np.float32, (P, 18))
        self.tri_object_ids = view(arr.tri_object_ids, np.int32, (P,))
        self.materials = view(arr.materials, np.float32, (info.num_materials, 13))
        self.lights = view(arr.lights, LIGHT_DTYPE, (info.num_lights,))
        self.positions = view(arr.positions, np.float32, (nv, 3))
        self.normals = view(arr.normals, np.float32, (nv, 3))
        self.indices = view(arr.indices, np.uint32, (P, 3))

    @classmethod
    def load_json(cls, path, project_dir=None) -> "HostScene":
        h = C.c_void_p()
        check(lib().rt_host_scene_load_json(str(path).encode(),
                                            None if project_dir is None else str(project_dir).encode(),
                                            C.byref(h)))
        return cls(h.value)

    @classmethod
    def load_objs(cls, paths: Sequence) -> "HostScene":
        enc = [str(p).encode() for p in paths]
        arr = (C.c_char_p * len(enc))(*enc)
        h = C.c_void_p()
        check(lib().rt_host_scene_load_objs(C.cast(arr, C.c_void_p), len(enc), C.byref(h)))
        return cls(h.value)

    def camera(self, width: Optional[int] = None, height: Optional[int] = None) -> Camera:
        i = self.info
        return Camera(tuple(i.cam_position), tuple(i.cam_look_at), tuple(i.cam_up), i.focal_length_mm,
                      i.sensor_height_mm, width or i.pixel_width, height or i.pixel_height)

    @property
    def settings(self) -> dict:
        i = self.info
        return {"max_depth": i.max_depth, "spp": i.spp, "diffuse_bounce": bool(i.diffuse_bounce),
                "miss_color": tuple(i.miss_color)}

    def close(self) -> None:
        if self._h:
            lib().rt_host_scene_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MeshHW1:
    """LoadOBJ_ToMeshSOA (HW1/src/MeshOBJ.cpp:143-281)."""

    def __init__(self, path):
        h = C.c_void_p()
        check(lib().rt_mesh_load_obj_hw1(str(path).encode(), C.byref(h)))
        self._h = h
        v = L.MeshView()
        check(lib().rt_mesh_view_get(self._h, C.byref(v)))
        nv, nt = int(v.num_vertices), int(v.num_triangles)
        self.positions = np.frombuffer((C.c_char * (nv * 12)).from_address(v.positions), np.float32).reshape(nv, 3).copy()
        self.normals = (np.frombuffer((C.c_char * (nv * 12)).from_address(v.normals), np.float32).reshape(nv, 3).copy()
                        if v.normals else None)
        self.indices = np.frombuffer((C.c_char * (nt * 12)).from_address(v.indices), np.uint32).reshape(nt, 3).copy()
        self.num_triangles = nt

    def __del__(self):
        try:
            if self._h:
                lib().rt_mesh_free(self._h)
        except Exception:
            pass


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


class DeviceScene:
    """Reference arrays uploaded to one device (rt_scene_create)."""

    def __init__(self, num_triangles: int, nodes, aabbs, triangles, tri_object_ids=None,
                 materials=None, lights=None, device: int = 0):
        P = int(num_triangles)
        self._keep = [_c(nodes, np.uint32), _c(aabbs, np.float32), _c(triangles, np.float32)]
        objs = None if tri_object_ids is None else _c(tri_object_ids, np.int32)
        mats = None if materials is None else _c(materials, np.float32).reshape(-1, 13)
        lts = None if lights is None else np.ascontiguousarray(lights, dtype=LIGHT_DTYPE)
        nmat = 0 if mats is None else mats.shape[0]
        nl = 0 if lts is None else lts.shape[0]
        h = C.c_void_p()
        check(lib().rt_scene_create(int(device), P, ptr(self._keep[0]), ptr(self._keep[1]), ptr(self._keep[2]),
                                    ptr(objs), ptr(mats), nmat, ptr(lts), nl, C.byref(h)))
        self._h = h
        self._owned = True
        self.num_triangles = P
        self.device = device

    @classmethod
    def _borrow(cls, handle, num_triangles: int, owner) -> "DeviceScene":
        """A scene owned by a Renderer (its timing queries; destroyed with the renderer, which
        then invalidates this view: later calls raise instead of touching freed memory)."""
        self = cls.__new__(cls)
        self._h = C.c_void_p(handle)
        self._owned = False
        self._owner = owner
        self._keep = []
        self.num_triangles = num_triangles
        self.device = int(lib().rt_scene_device(self._h))
        return self

    def _handle(self) -> C.c_void_p:
        if not self._h:
            raise L.RTError(-1, "scene is closed (or its Renderer was closed)")
        return self._h

    @classmethod
    def from_host(cls, hs: HostScene, device: int = 0) -> "DeviceScene":
        return cls(hs.num_triangles, hs.nodes, hs.aabbs, hs.triangles, hs.tri_object_ids, hs.materials,
                   hs.lights, device)

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    @property
    def device_bytes(self) -> int:
        return int(lib().rt_scene_device_bytes(self._handle()))

    @staticmethod
    def make_opts(spp: int = 1, max_depth: int = 1, diffuse_bounce: bool = True, miss_color=(0, 0, 0),
                  jitter=None, band_rows: int = 8, band_index: int = 0, band_count: int = 1,
                  kernel: int = L.RT_KERNEL_AUTO, tile_order: int = L.RT_TILES_AUTO, flags: int = 0):
        o = L.RenderOpts()
        lib().rt_render_opts_default(C.byref(o))
        o.spp, o.max_depth, o.diffuse_bounce = int(spp), int(max_depth), 1 if diffuse_bounce else 0
        o.miss_color = _v3(miss_color)
        jit = None
        if jitter is not None:
            jit = _c(jitter, np.float32).reshape(-1)
            o.jitter = jit.ctypes.data
        o.band_rows, o.band_index, o.band_count, o.kernel = int(band_rows), int(band_index), int(band_count), int(kernel)
        o.tile_order = int(tile_order)
        o.flags = int(flags)
        return o, jit

    def render(self, camera: Camera, spp: int = 1, max_depth: int = 1, diffuse_bounce: bool = True,
               miss_color=(0, 0, 0), jitter=None, aov: bool = False, band_rows: int = 8,
               band_index: int = 0, band_count: int = 1, kernel: int = L.RT_KERNEL_AUTO,
               tile_order: int = L.RT_TILES_AUTO, flags: int = 0):
        """Synchronous render to host: (rows, W, 3) float32 [+ (rows, W, spp) hit idx / t]."""
        o, _jit = self.make_opts(spp, max_depth, diffuse_bounce, miss_color, jitter, band_rows, band_index,
                                 band_count, kernel, tile_order, flags)
        W = camera.pixel_width
        rows = lib().rt_shard_rows(camera.pixel_height, o.band_rows, o.band_index, o.band_count)
        if rows < 0:
            raise L.RTError(-1, "bad band parameters")
        rgb = np.zeros((rows, W, 3), np.float32)
        hi = ht = None
        if aov:
            hi = np.zeros((rows, W, spp), np.int32)
            ht = np.zeros((rows, W, spp), np.float32)
        check(lib().rt_render(self._handle(), C.byref(camera.c), C.byref(o), ptr(rgb), ptr(hi), ptr(ht)))
        return (rgb, hi, ht) if aov else rgb

    def count_rays(self, camera: Camera, spp: int = 1, max_depth: int = 1, diffuse_bounce: bool = True,
                   miss_color=(0, 0, 0), band_rows: int = 8, band_index: int = 0, band_count: int = 1) -> dict:
        """Rays one frame traces (rt_count_rays_ex): camera, shadow and bounce counts, the classes
        of the oracle's stats["rays"], and camera_traced, the camera rays of the tiles the culling
        passes leave to the render kernel (the rest provably miss and are not traversed)."""
        o, _jit = self.make_opts(spp, max_depth, diffuse_bounce, miss_color, None, band_rows, band_index,
                                 band_count)
        out = (C.c_uint64 * 4)()
        check(lib().rt_count_rays_ex(self._handle(), C.byref(camera.c), C.byref(o), out))
        return {"camera": int(out[0]), "shadow": int(out[1]), "bounce": int(out[2]), "camera_traced": int(out[3])}

    def render_device(self, camera: Camera, opts, rgb_dev_ptr: int, hit_idx_ptr=None, hit_t_ptr=None,
                      stream: Optional[int] = None, p6_dev_ptr=None) -> None:
        """Render into device memory (rt_render_device); with ``p6_dev_ptr`` the render and cull
        kernels also write the pixels' P6 samples (write_p6 defaults), rt_render_device_p6."""
        check(lib().rt_render_device_p6(self._handle(), C.byref(camera.c), C.byref(opts), rgb_dev_ptr, hit_idx_ptr,
                                        hit_t_ptr, p6_dev_ptr, stream))

    def render_device_pair(self, camera_a: Camera, camera_b: Camera, opts, rgb_a=None, p6_a=None, rgb_b=None,
                           p6_b=None, stream: Optional[int] = None) -> None:
        """Two frames with one launch of the render kernel where it fits them
        (rt_render_device_pair): the images of two render_device calls."""
        check(lib().rt_render_device_pair(self._handle(), C.byref(camera_a.c), C.byref(camera_b.c), C.byref(opts),
                                          rgb_a, p6_a, rgb_b, p6_b, stream))

    def kernel_times(self, max_launches: int = 256) -> np.ndarray:
        """ms of the render kernel for the most recent launches (HIP events on its stream)."""
        out = np.zeros(max_launches, np.float32)
        n = C.c_int()
        check(lib().rt_kernel_times(self._handle(), ptr(out), max_launches, C.byref(n)))
        return out[:n.value]

    def live_tiles(self) -> tuple:
        """(traced tiles, all tiles) of the most recent render."""
        live, total = C.c_int64(), C.c_int64()
        check(lib().rt_live_tiles(self._handle(), C.byref(live), C.byref(total)))
        return live.value, total.value

    def kernel_name(self) -> str:
        """The render kernel instantiation of the most recent frame, as rocprofv3 names it."""
        return lib().rt_scene_kernel_name(self._handle()).decode()

    def heavy_tiles(self) -> int:
        """Tiles the most recent render dispatched first (heavy-first order, speed only)."""
        n = C.c_int64()
        check(lib().rt_heavy_tiles(self._handle(), C.byref(n)))
        return n.value

    def frame_times(self, max_launches: int = 256) -> np.ndarray:
        """ms of the frame's device work (cull pre-passes + render kernel)."""
        out = np.zeros(max_launches, np.float32)
        n = C.c_int()
        check(lib().rt_frame_times(self._handle(), ptr(out), max_launches, C.byref(n)))
        return out[:n.value]

    def prepass_times(self, max_launches: int = 256) -> np.ndarray:
        """ms of the cull pre-passes (root-box cull + tree-cut cull) alone."""
        out = np.zeros(max_launches, np.float32)
        n = C.c_int()
        check(lib().rt_prepass_times(self._handle(), ptr(out), max_launches, C.byref(n)))
        return out[:n.value]

    def traversal_info(self) -> dict:
        """The traversal rt_scene_create chose (rt_scene_traversal_info)."""
        info = (C.c_int64 * 4)()
        check(lib().rt_scene_traversal_info(self._handle(), info))
        return {"frustum_log2": int(info[0]), "frustum_bound": int(info[1]), "wide": bool(info[2]),
                "deep": bool(info[3])}

    def faults(self, clear: bool = True) -> int:
        """RT_FAULT_* bits the device guards raised since the last clear (rt_scene_faults)."""
        f = C.c_uint32()
        check(lib().rt_scene_faults(self._handle(), C.byref(f), 1 if clear else 0))
        return f.value

    def close(self) -> None:
        if self._h and self._owned:
            lib().rt_scene_destroy(self._h)
        self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Renderer:
    """render(scene, camera) -> frame in host memory on 1..N GPUs (rt_renderer, include/rt_mi355x.h).

    Every rank renders its 8-row bands (band b -> rank b % world) into a device strip with the
    fused P6 epilogue; the strips reach the host frame band by band, pipelined `depth` frames
    deep: each GPU over its own PCIe link (RT_GATHER_DIRECT in one process; RT_GATHER_HOST_SHARED
    across processes, into the shared-memory frame ``host_frame_name``), or over RCCL to rank 0
    first (RT_GATHER_RCCL).  ``devices``: the GPUs this process drives;
    ``world_size``/``rank0``/``unique_id`` join a multi-process job (one process per GPU): rank
    0's process makes the RCCL id with :func:`comm_unique_id` and shares it.
    """

    def __init__(self, num_triangles: int, nodes, aabbs, triangles, tri_object_ids=None, materials=None,
                 lights=None, devices=(0,), world_size: int = 0, rank0: int = 0, unique_id: bytes = None,
                 band_rows: int = 8, deliver: int = L.RT_DELIVER_P6, gather: int = L.RT_GATHER_AUTO,
                 depth: int = 3, flags: int = 0, host_frame_name: Optional[str] = None):
        P = int(num_triangles)
        keep = [_c(nodes, np.uint32), _c(aabbs, np.float32), _c(triangles, np.float32)]
        objs = None if tri_object_ids is None else _c(tri_object_ids, np.int32)
        mats = None if materials is None else _c(materials, np.float32).reshape(-1, 13)
        lts = None if lights is None else np.ascontiguousarray(lights, dtype=LIGHT_DTYPE)
        devs = np.ascontiguousarray(list(devices), np.int32)
        o = L.RendererOpts()
        lib().rt_renderer_opts_default(C.byref(o))
        o.n_devices, o.devices = len(devs), devs.ctypes.data
        o.world_size, o.rank0 = int(world_size), int(rank0)
        uid = None
        if unique_id is not None:
            uid = C.create_string_buffer(bytes(unique_id), 128)
            o.unique_id = C.addressof(uid)
        o.band_rows, o.deliver, o.gather, o.depth, o.flags = int(band_rows), int(deliver), int(gather), int(depth), int(flags)
        name = None
        if host_frame_name:
            name = C.create_string_buffer(str(host_frame_name).encode())
            o.host_frame_name = C.addressof(name)
        h = C.c_void_p()
        check(lib().rt_renderer_create(P, ptr(keep[0]), ptr(keep[1]), ptr(keep[2]), ptr(objs), ptr(mats),
                                       0 if mats is None else mats.shape[0], ptr(lts),
                                       0 if lts is None else lts.shape[0], C.byref(o), C.byref(h)))
        self._h = h
        self._name = name
        self._borrowed = []  # DeviceScene views of this renderer's scenes (invalidated by close)
        self.num_triangles = P
        self.deliver = int(deliver)
        self.world = int(world_size) or len(devs)
        self.rank0 = int(rank0)

    @classmethod
    def from_host(cls, hs: HostScene, **kw) -> "Renderer":
        return cls(hs.num_triangles, hs.nodes, hs.aabbs, hs.triangles, hs.tri_object_ids, hs.materials,
                   hs.lights, **kw)

    @property
    def copy_engine(self) -> str:
        """"sdma" (copies queued through the HSA runtime on a DMA engine) or "runtime" (HIP's)."""
        return "sdma" if lib().rt_renderer_copy_engine(self._h) else "runtime"

    @property
    def local_ranks(self) -> int:
        return int(lib().rt_renderer_local_ranks(self._h))

    def scene(self, i: int = 0) -> DeviceScene:
        """Local rank i's device scene (frame/kernel timing queries)."""
        h = lib().rt_renderer_scene(self._h, int(i))
        if not h:
            raise L.RTError(-1, f"no local rank {i}")
        v = DeviceScene._borrow(h, self.num_triangles, self)
        self._borrowed.append(v)
        return v

    def submit(self, camera: Camera, opts) -> int:
        t = C.c_uint64()
        check(lib().rt_renderer_submit(self._h, C.byref(camera.c), C.byref(opts), C.byref(t)))
        return t.value

    def submit_pair(self, camera_a: Camera, camera_b: Camera, opts) -> tuple:
        """Two frames, one render launch per local rank (rt_renderer_submit_pair): their tickets."""
        t = C.c_uint64()
        check(lib().rt_renderer_submit_pair(self._h, C.byref(camera_a.c), C.byref(camera_b.c), C.byref(opts),
                                            C.byref(t)))
        return t.value, t.value + 1

    def wait(self, ticket: int):
        """(address, bytes) of the delivered frame on rank 0's process, else (None, 0)."""
        f, n = C.c_void_p(), C.c_size_t()
        check(lib().rt_renderer_wait(self._h, int(ticket), C.byref(f), C.byref(n)))
        return f.value, n.value

    def render(self, camera: Camera, spp: int = 1, max_depth: int = 1, diffuse_bounce: bool = True,
               miss_color=(0, 0, 0), jitter=None, kernel: int = L.RT_KERNEL_AUTO, flags: int = 0):
        """One synchronous frame: (H, W, 3) uint8 P6 samples or float32 (rank 0; None elsewhere)."""
        o, _jit = DeviceScene.make_opts(spp, max_depth, diffuse_bounce, miss_color, jitter, kernel=kernel, flags=flags)
        W, H = camera.pixel_width, camera.pixel_height
        f32 = self.deliver == L.RT_DELIVER_F32
        out = np.zeros((H, W, 3), np.float32 if f32 else np.uint8)
        check(lib().rt_renderer_render(self._h, C.byref(camera.c), C.byref(o), ptr(out), out.nbytes))
        return out if self.rank0 == 0 and self.deliver != L.RT_DELIVER_NONE else None

    def times(self, kind: int, max_frames: int = 256) -> np.ndarray:
        out = np.zeros(max_frames, np.float32)
        n = C.c_int()
        check(lib().rt_renderer_times(self._h, int(kind), ptr(out), int(max_frames), C.byref(n)))
        return out[:n.value]

    def close(self) -> None:
        for v in getattr(self, "_borrowed", []):
            v._h = C.c_void_p()
        self._borrowed = []
        if self._h:
            lib().rt_renderer_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def comm_unique_id() -> bytes:
    """128-byte RCCL unique id for a multi-process Renderer (made on rank 0's process)."""
    b = C.create_string_buffer(128)
    check(lib().rt_comm_unique_id(b))
    return b.raw


def render(numTriangles, W, H, cam: Camera, missColor, max_depth, spp, nodes, aabbs, triangles,
           triObjectIds, objectMaterials, numObjectMaterials, lights, numLights, diffuse_bounce, output,
           n_gpus: int = 1):
    """The reference entry point (G/include/query.h:13-29) with host arrays; fills ``output``
    (H*W*3 float32, row-major, row 0 = top) like the CPU branch of query.cu:130-166.
    n_gpus > 1 shards the bands over GPUs 0..n_gpus-1 (rt_render_reference_gpus)."""
    out = np.asarray(output)
    if out.dtype != np.float32 or not out.flags.c_contiguous or out.size != W * H * 3:
        raise ValueError("output must be a contiguous float32 array of W*H*3")
    mats = _c(objectMaterials, np.float32).reshape(-1, 13)[:numObjectMaterials]
    lts = np.ascontiguousarray(lights, dtype=LIGHT_DTYPE)[:numLights]
    nd, ab, tr = _c(nodes, np.uint32), _c(aabbs, np.float32), _c(triangles, np.float32)
    ob = None if triObjectIds is None else _c(triObjectIds, np.int32)
    args = (int(numTriangles), int(W), int(H), C.byref(cam.c), _v3(missColor), int(max_depth), int(spp), ptr(nd),
            ptr(ab), ptr(tr), ptr(ob), ptr(mats), int(numObjectMaterials), ptr(lts), int(numLights),
            1 if diffuse_bounce else 0)
    if n_gpus == 1:
        check(lib().rt_render_reference(*args, ptr(out)))
    else:
        check(lib().rt_render_reference_gpus(*args, int(n_gpus), ptr(out)))
    return out


RT_HW1_BRUTE = 1


def render_hw1(positions, normals, indices, camera: Camera, light_position, light_color, spp: int = 1,
               jitter=None, aov: bool = False, device: int = 0, brute: bool = False, timing: bool = False):
    """HW1 path on the GPU (HW1/src/render.cpp:72-116 semantics): (H, W, 3) float32 [+ per-sample
    winning triangle / t] [+ device ms of the kernels when ``timing``].  ``brute`` runs every
    triangle for every ray; the default skips triangles outside their conservative pixel
    rectangle (same output bit for bit, see rt_render_hw1_ex)."""
    pos, nrm, idx = _c(positions, np.float32), _c(normals, np.float32), _c(indices, np.uint32)
    W, H = camera.pixel_width, camera.pixel_height
    rgb = np.zeros((H, W, 3), np.float32)
    hi = ht = None
    if aov:
        hi = np.zeros((H, W, spp), np.int32)
        ht = np.zeros((H, W, spp), np.float32)
    jit = None if jitter is None else _c(jitter, np.float32).reshape(-1)
    ms = C.c_float(0.0)
    check(lib().rt_render_hw1_ex(int(device), ptr(pos), ptr(nrm), ptr(idx), idx.size // 3, C.byref(camera.c),
                                 _v3(light_position), _v3(light_color), int(spp), ptr(jit),
                                 RT_HW1_BRUTE if brute else 0, ptr(rgb), ptr(hi), ptr(ht),
                                 C.byref(ms) if timing else None))
    out = (rgb, hi, ht) if aov else (rgb,)
    if timing:
        out = out + (ms.value,)
    return out if len(out) > 1 else out[0]


class HW1Scene:
    """A HW1 mesh resident on one MI355X (rt_hw1_scene): repeated frames of the HW1 path
    (HW1/src/render.cpp:72-116) without re-uploading it."""

    def __init__(self, positions, normals, indices, device: int = 0):
        pos, nrm, idx = _c(positions, np.float32), _c(normals, np.float32), _c(indices, np.uint32)
        h = C.c_void_p()
        check(lib().rt_hw1_scene_create(int(device), ptr(pos), ptr(nrm), ptr(idx), idx.size // 3, C.byref(h)))
        self._h = h
        self.device = device

    def render_device(self, camera: Camera, light_position, light_color, spp: int = 1, rgb_ptr=None, p6_ptr=None,
                      hit_idx_ptr=None, hit_t_ptr=None, stream=None, jitter=None, brute: bool = False) -> None:
        """One frame into device buffers (raw pointers) on a HIP stream (handle), asynchronously."""
        jit = None if jitter is None else _c(jitter, np.float32).reshape(-1)
        check(lib().rt_render_hw1_device(self._h, C.byref(camera.c), _v3(light_position), _v3(light_color), int(spp),
                                         ptr(jit), RT_HW1_BRUTE if brute else 0, rgb_ptr, p6_ptr, hit_idx_ptr,
                                         hit_t_ptr, stream))

    def render_deliver(self, camera: Camera, light_position, light_color, spp: int, host_p6_ptr: int, stream=None,
                       brute: bool = False) -> int:
        """One frame's P6 body (write_p6 defaults) delivered to host memory at host_p6_ptr
        (W*H*3 bytes, pinned) by the scene's own copy stream, overlapping the next frames'
        kernels (rt_render_hw1_deliver); returns the frame's ticket for wait()."""
        t = C.c_uint64()
        check(lib().rt_render_hw1_deliver(self._h, C.byref(camera.c), _v3(light_position), _v3(light_color), int(spp),
                                          RT_HW1_BRUTE if brute else 0, host_p6_ptr, stream, C.byref(t)))
        return int(t.value)

    def wait(self, ticket: int) -> None:
        check(lib().rt_hw1_wait(self._h, int(ticket)))

    def kernel_times(self, max_frames: int = 64) -> np.ndarray:
        out = np.zeros(max_frames, np.float32)
        n = C.c_int()
        check(lib().rt_hw1_kernel_times(self._h, ptr(out), max_frames, C.byref(n)))
        return out[:n.value]

    def kernel_name(self) -> str:
        return lib().rt_hw1_kernel_name(self._h).decode()

    def list_info(self) -> tuple:
        """(bin-list capacity now, the latest frame's list total)."""
        info = (C.c_int64 * 2)()
        check(lib().rt_hw1_list_info(self._h, info))
        return int(info[0]), int(info[1])

    def close(self) -> None:
        if self._h:
            lib().rt_hw1_scene_destroy(self._h)
        self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def intersect_rays(triangle18, dirs, origin=(0.0, 0.0, 0.0), hw1: bool = True, tmin: float = 0.0,
                   tmax: float = 3.4028234663852886e38, device: int = 0):
    """Device Möller–Trumbore over a batch of rays against one triangle (v0,v1,v2,n0,n1,n2 as 18
    floats): HW1 ray_intersection semantics when hw1, else G/ intersectTriangle with [tmin, tmax]."""
    tri = L.Triangle.from_buffer_copy(_c(triangle18, np.float32).tobytes())
    d = _c(dirs, np.float32).reshape(-1, 3)
    n = d.shape[0]
    hit = np.zeros(n, np.int32)
    t = np.zeros(n, np.float32)
    check(lib().rt_intersect_rays(int(device), C.byref(tri), _f3(origin), ptr(d), n, 1 if hw1 else 0,
                                  float(tmin), float(tmax), ptr(hit), ptr(t)))
    return hit, t


def build_bvh(positions, indices):
    """CPU LBVH (G/include/bvh.cu:209-317) over an indexed mesh: (nodes (2P-1,4), aabbs (2P-1,6))."""
    pos, idx = _c(positions, np.float32), _c(indices, np.uint32)
    P = idx.size // 3
    if P == 0:  # what rt_build_bvh answers for an empty mesh (no arrays to size)
        check(lib().rt_build_bvh(ptr(pos), pos.size // 3, None, 0, None, None))
    nodes = np.zeros((2 * P - 1, 4), np.uint32)
    aabbs = np.zeros((2 * P - 1, 6), np.float32)
    check(lib().rt_build_bvh(ptr(pos), pos.size // 3, ptr(idx), P, ptr(nodes), ptr(aabbs)))
    return nodes, aabbs


def build_bvh_device(positions, indices, device: int = 0, stream=None, tensors: bool = False):
    """The LBVH build on the GPU (rt_build_bvh_device): the same (nodes (2P-1,4), aabbs (2P-1,6))
    as build_bvh.  positions (nv,3) float32 / indices (P,3) uint32 may be numpy arrays or device
    tensors; tensors=True returns device tensors (nodes as int32 bit patterns) instead of numpy."""
    import torch

    dev = torch.device("cuda", device)

    def on_dev(a, dt_np):
        if isinstance(a, torch.Tensor):
            return a.to(dev).contiguous()
        return torch.from_numpy(np.ascontiguousarray(a, dt_np).view(np.int32 if dt_np == np.uint32 else dt_np)
                                .copy()).to(dev)

    pos = on_dev(positions, np.float32).reshape(-1, 3)
    idx = on_dev(indices, np.uint32).reshape(-1, 3)
    P = idx.shape[0]
    nodes = torch.empty((max(2 * P - 1, 1), 4), dtype=torch.int32, device=dev)
    aabbs = torch.empty((max(2 * P - 1, 1), 6), dtype=torch.float32, device=dev)
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    check(lib().rt_build_bvh_device(device, pos.data_ptr(), pos.shape[0], idx.data_ptr(), P, nodes.data_ptr(),
                                    aabbs.data_ptr(), stream))
    if tensors:
        return nodes, aabbs
    return nodes.cpu().numpy().view(np.uint32), aabbs.cpu().numpy()


def _ppm_opts(maxval=255, clamp=True, gamma2=True, flip_y=False) -> L.PPMOptions:
    return L.PPMOptions(int(maxval), 1 if clamp else 0, 1 if gamma2 else 0, 1 if flip_y else 0)


def encode_p6(rgb, maxval=255, clamp=True, gamma2=True, flip_y=False) -> bytes:
    a = _c(rgb, np.float32)
    H, W = a.shape[0], a.shape[1]
    o = _ppm_opts(maxval, clamp, gamma2, flip_y)
    n = C.c_size_t()
    check(lib().rt_ppm_encode(ptr(a), W, H, C.byref(o), None, 0, C.byref(n)))
    buf = (C.c_uint8 * n.value)()
    check(lib().rt_ppm_encode(ptr(a), W, H, C.byref(o), C.cast(buf, C.c_void_p), n.value, C.byref(n)))
    return bytes(buf)


def write_p6(path, rgb, maxval=255, clamp=True, gamma2=True, flip_y=False) -> None:
    a = _c(rgb, np.float32)
    o = _ppm_opts(maxval, clamp, gamma2, flip_y)
    check(lib().rt_ppm_write(str(path).encode(), ptr(a), a.shape[1], a.shape[0], C.byref(o)))


def read_p6(path) -> np.ndarray:
    w, h, mv = C.c_int(), C.c_int(), C.c_int()
    check(lib().rt_ppm_read(str(path).encode(), None, 0, C.byref(w), C.byref(h), C.byref(mv)))
    out = np.zeros((h.value, w.value, 3), np.float32)
    check(lib().rt_ppm_read(str(path).encode(), ptr(out), out.size, C.byref(w), C.byref(h), C.byref(mv)))
    return out


def p6_header(width: int, height: int, maxval: int = 255) -> bytes:
    """write_p6's header bytes (ppm_p6.cpp:275-277)."""
    n = C.c_size_t()
    check(lib().rt_ppm_header(width, height, maxval, None, 0, C.byref(n)))
    buf = C.create_string_buffer(n.value)
    check(lib().rt_ppm_header(width, height, maxval, buf, n.value, C.byref(n)))
    return buf.raw[:n.value]


def quantize_p6_device(rgb_dev, width: int, rows: int, out_dev, maxval=255, clamp=True, gamma2=True,
                       flip_y=False, stream=None) -> None:
    """P6 body of a device framebuffer on the device (rt_ppm_quantize_device).  rgb_dev / out_dev
    are device addresses (ints, e.g. tensor.data_ptr()); asynchronous on `stream`."""
    o = _ppm_opts(maxval, clamp, gamma2, flip_y)
    check(lib().rt_ppm_quantize_device(rgb_dev, width, rows, C.byref(o), out_dev, stream))


def unpermute_strips_device(strips_dev, strip_rows: int, row_bytes: int, height: int, band_rows: int,
                            band_count: int, frame_dev, flip_y=False, stream=None) -> None:
    """Band un-permute of back-to-back gathered strips into an image-order frame on the device."""
    check(lib().rt_unpermute_strips_device(strips_dev, strip_rows, row_bytes, height, band_rows, band_count,
                                           1 if flip_y else 0, frame_dev, stream))


def encode_p6_device(rgb, maxval=255, clamp=True, gamma2=True, flip_y=False):
    """P6 file bytes of an (H, W, 3) float32 CUDA tensor, quantised on the device (only the
    quantised body crosses PCIe).  Same bytes as encode_p6 on the host copy."""
    import torch

    if not (isinstance(rgb, torch.Tensor) and rgb.is_cuda and rgb.dtype == torch.float32 and rgb.dim() == 3
            and rgb.shape[2] == 3):
        raise ValueError("encode_p6_device: expects an (H, W, 3) float32 device tensor")
    rgb = rgb.contiguous()
    H, W = rgb.shape[0], rgb.shape[1]
    bps = 1 if maxval < 256 else 2
    body = torch.empty(H * W * 3 * bps, dtype=torch.uint8, device=rgb.device)
    stream = torch.cuda.current_stream(rgb.device).cuda_stream
    quantize_p6_device(rgb.data_ptr(), W, H, body.data_ptr(), maxval, clamp, gamma2, flip_y, stream)
    return p6_header(W, H, maxval) + body.cpu().numpy().tobytes()


def set_tuning(name: str, value) -> None:
    """Process-wide tuning knob (rt_tuning_set; include/rt_mi355x.h rt_tune_id): None restores
    its default.  Read when a scene is created or a frame is set up."""
    check(lib().rt_tuning_set(L.TUNE[name], float("nan") if value is None else float(value)))


def get_tuning(name: str):
    """The value set for a knob, or None when it has its default."""
    v = C.c_double()
    check(lib().rt_tuning_get(L.TUNE[name], C.byref(v)))
    return None if v.value != v.value else v.value


def reset_tuning() -> None:
    lib().rt_tuning_reset()


class tuning:
    """Context manager: ``with rt.tuning(half_waves=1): ...`` sets knobs, restores them after."""

    def __init__(self, **knobs):
        self.knobs = knobs
        self.saved = {}

    def __enter__(self):
        for k, v in self.knobs.items():
            self.saved[k] = get_tuning(k)
            set_tuning(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.saved.items():
            set_tuning(k, v)
        return False


def device_count() -> int:
    n = C.c_int()
    rc = lib().rt_device_count(C.byref(n))
    return n.value if rc == 0 else 0
