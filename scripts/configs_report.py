"""Measure every BASELINE.json config that fits one GPU and print one JSON line each (the rows of
BASELINE.md §4; C4 = C3 on N GPUs comes from bench.py under torch.distributed.run).

    python scripts/configs_report.py [--out gpurun_out/configs.jsonl] [--cpu-threads 16]

* c1 — HW1 brute force, sphere 256x256x1: GPU (rt_render_hw1, synchronous call incl. mesh
  upload and read-back) and the oracle's CPU restatement (1 thread and all threads).
* c2 — HW1 brute force, frog 640x480x1 primary rays: GPU as c1; CPU on a 48-row band.
* c3 — frog 1920x1080x16, max_bounces 1: rt_render_device, scene resident, HIP-event kernel time.
* c5 — 1M-triangle heightfield 3840x2160x64 on ONE GPU (the config names 8): as c3.
Parity: hit indices / framebuffer / P6 against the reference's fixtures (tests/golden) for
c1-c3; for c5 a band of rows against the oracle (the full frame is too long for the CPU).
"""
from __future__ import annotations

import argparse
import gzip
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import raytracinginonesemester_amd as rt  # noqa: E402
from raytracinginonesemester_amd import configs  # noqa: E402
from oracle import pyoracle as orc  # noqa: E402

GOLD = REPO / "tests" / "golden" / "scenes"
# shadow rays per camera sample (oracle counter replay, configs.BYTES_PER_SAMPLE comment)
SHADOW_PER_SAMPLE = {"c3": 0.02072, "c5": 0.2105}


def gold(name, f, dt):
    return np.frombuffer(gzip.open(GOLD / name / f).read(), dt)


def ppm_maxabs(rgb, name):
    ref = gzip.open(GOLD / name / "image.ppm.gz").read()
    mine = rt.encode_p6(rgb)
    n = len(rt.p6_header(rgb.shape[1], rgb.shape[0]))
    return int(np.abs(np.frombuffer(mine[n:], np.uint8).astype(int)
                      - np.frombuffer(ref[n:], np.uint8).astype(int)).max())


def median_time(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def hw1(cfg, threads, reps, cpu_rows):
    c = configs.HW1_CONFIGS[cfg]
    W, H, spp = c["width"], c["height"], c["spp"]
    mesh = rt.MeshHW1(configs.MESHES / c["mesh"])
    cam = rt.Camera(c["position"], c["look_at"], c["up"], c["focal_mm"], c["sensor_mm"], W, H, hw1=True)
    args = (mesh.positions, mesh.normals, mesh.indices, cam, c["light_pos"], c["light_color"])
    rgb, hi, _ = rt.render_hw1(*args, spp=spp, aov=True)
    t_gpu = median_time(lambda: rt.render_hw1(*args, spp=spp), reps)
    k_ms = float(np.median([rt.render_hw1(*args, spp=spp, timing=True)[1] for _ in range(reps)]))
    kb_ms = float(np.median([rt.render_hw1(*args, spp=spp, timing=True, brute=True)[1] for _ in range(reps)]))
    oc = orc.camera_from_basis(*(cam.basis()[k] for k in ("center", "pixel00_loc", "pixel_delta_u",
                                                          "pixel_delta_v")), W, H)
    rows = (0, H) if cpu_rows is None else (H // 2 - cpu_rows // 2, H // 2 + cpu_rows // 2)
    n_cpu = (rows[1] - rows[0]) * W * spp
    cpu = {}
    for th in sorted({1, threads}):
        t0 = time.perf_counter()
        orc.render_hw1(mesh.positions, mesh.normals, mesh.indices, oc, c["light_pos"], c["light_color"], spp=spp,
                       rows=rows, threads=th)
        cpu[th] = n_cpu / (time.perf_counter() - t0) / 1e6
    name = f"{cfg}_full"
    samples = W * H * spp
    return {"config": cfg, "gpus": 1, "Mrays_s": samples / t_gpu / 1e6, "total_rays_s": samples / t_gpu,
            "timing": "synchronous rt_render_hw1 call (mesh upload + kernel + read-back), median",
            "ms": t_gpu * 1e3, "cpu_Mrays_s": {str(k): v for k, v in cpu.items()},
            "device_Mrays_s": samples / k_ms / 1e3, "device_ms": k_ms,
            "device_timing": "HIP events around the binned pipeline (rect, bin, scan, fill, render kernels)",
            "brute_device_Mrays_s": samples / kb_ms / 1e3, "brute_device_ms": kb_ms,
            "cpu_sample": f"oracle HW1 restatement rows {rows[0]}..{rows[1]}",
            "hit_idx_mismatches": int((hi.reshape(-1) != gold(name, "hits.i32.gz", np.int32)).sum()),
            "rgb_maxabs": float(np.abs(rgb.reshape(-1) - gold(name, "fb.f32.gz", np.float32)).max()),
            "ppm_maxabs": ppm_maxabs(rgb, name)}


def gpath(cfg, threads, reps, cpu_rows):
    g = configs.G_CONFIGS[cfg]
    sp = configs.scene_path(g["scene"])
    hs = rt.HostScene.load_json(sp, REPO if sp.parent == configs.SCENES else sp.parent)
    cam = hs.camera(g["width"], g["height"])
    W, H, spp = cam.pixel_width, cam.pixel_height, g["spp"]
    ds = rt.DeviceScene.from_host(hs, device=0)
    opts, _j = ds.make_opts(spp=spp, max_depth=g["max_depth"], miss_color=hs.settings["miss_color"])
    dev = torch.device("cuda", 0)
    rgb = torch.zeros((H, W, 3), dtype=torch.float32, device=dev)
    hit = torch.zeros((H, W, spp), dtype=torch.int32, device=dev)
    ht = torch.zeros((H, W, spp), dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    ds.render_device(cam, opts, rgb.data_ptr(), hit.data_ptr(), ht.data_ptr(), stream=st)
    torch.cuda.synchronize()
    for _ in range(2):
        ds.render_device(cam, opts, rgb.data_ptr(), stream=st)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        ds.render_device(cam, opts, rgb.data_ptr(), stream=st)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / reps
    kt = ds.kernel_times(reps)
    samples = W * H * spp
    B = configs.BYTES_PER_SAMPLE[cfg]
    out = {"config": cfg, "gpus": 1, "Mrays_s": samples / t / 1e6,
           "total_rays_s": samples * (1 + SHADOW_PER_SAMPLE[cfg]) / t,
           "timing": "rt_render_device per frame (scene resident, stream-ordered), mean of reps",
           "ms": t * 1e3, "kernel_ms": float(kt.mean()),
           # SURVEY §8(d) reference-layout byte model: what the reference's per-ray traversal
           # would fetch, NOT this kernel's traffic (that is profiles/traffic.json / bench.py)
           "reference_equivalent_frac": samples * B / (float(kt.mean()) / 1e3) / 8.0e12}
    tr = {}
    try:
        tr = json.loads((REPO / "profiles" / "traffic.json").read_text()).get(cfg, {})
    except Exception:
        pass
    if tr.get("bytes_per_launch"):
        out["hbm_frac_measured"] = tr["bytes_per_launch"] / (float(kt.mean()) / 1e3) / 8.0e12
        out["hbm_bytes_per_launch"] = tr["bytes_per_launch"]
    rgb_h = rgb.cpu().numpy()
    hit_h = hit.cpu().numpy()
    oc = orc.camera_from_basis(*(cam.basis()[k] for k in ("center", "pixel00_loc", "pixel_delta_u",
                                                          "pixel_delta_v")), W, H)
    rows = (0, H) if cpu_rows is None else (H // 2 - cpu_rows // 2, H // 2 + cpu_rows // 2)
    t0 = time.perf_counter()
    ref, rhi, _ = orc.render_g(hs.num_triangles, oc, hs.nodes, hs.aabbs, hs.triangles, hs.tri_object_ids,
                               hs.materials, hs.lights, spp=spp, max_depth=g["max_depth"],
                               miss=hs.settings["miss_color"], rows=rows, threads=threads, aov=True)
    out["cpu_Mrays_s"] = {str(threads): (rows[1] - rows[0]) * W * spp / (time.perf_counter() - t0) / 1e6}
    out["cpu_sample"] = f"oracle restatement rows {rows[0]}..{rows[1]}"
    y0, y1 = rows
    out["hit_idx_mismatches"] = int((hit_h[y0:y1] != rhi[y0:y1]).sum())
    out["rgb_maxabs"] = float(np.abs(rgb_h[y0:y1] - ref[y0:y1]).max())
    if cfg == "c3":
        import hashlib

        meta = json.loads((GOLD / "c3_full" / "meta.json").read_text())["sha256"]
        out["hit_idx_sha256_equals_reference"] = hashlib.sha256(hit_h.tobytes()).hexdigest() == meta["hits.i32"]
        out["hit_t_sha256_equals_reference"] = hashlib.sha256(ht.cpu().numpy().tobytes()).hexdigest() == meta["hitt.f32"]
        out["rgb_maxabs_vs_reference"] = float(np.abs(rgb_h.reshape(-1) - gold("c3_full", "fb.f32.gz", np.float32)).max())
        out["ppm_maxabs"] = ppm_maxabs(rgb_h, "c3_full")
    out["parity_rows"] = [y0, y1]
    ds.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=str(REPO / "gpurun_out" / "configs.jsonl"))
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "0") or 16))
    ap.add_argument("--only", default="c1,c2,c3,c5")
    a = ap.parse_args()
    lines = []
    for cfg in a.only.split(","):
        if cfg == "c1":
            r = hw1("c1", a.cpu_threads, 5, None)
        elif cfg == "c2":
            r = hw1("c2", a.cpu_threads, 5, 48)
        elif cfg == "c3":
            r = gpath("c3", a.cpu_threads, 20, None)
        else:
            r = gpath("c5", a.cpu_threads, 3, 16)
        r = {k: (round(v, 6) if isinstance(v, float) else v) for k, v in r.items()}
        print(json.dumps(r), flush=True)
        lines.append(json.dumps(r))
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
