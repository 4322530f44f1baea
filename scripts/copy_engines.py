"""Frame delivery (rt_renderer, P6 frames to pinned host memory) under different HIP copy-engine
settings, each in its own child process (the runtime reads them at start-up).

    python scripts/copy_engines.py [--steps 200]

Per setting: ms per delivered frame (3-deep pipeline), render-kernel ms, device-frame ms and
host-copy ms (HIP events), for deliver none (render only) and deliver p6.
"""
import json
import os
import subprocess
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
SETTINGS = {
    "default": {},
    "blit_engine_2": {"GPU_BLIT_ENGINE_TYPE": "2"},
    "blit_engine_1": {"GPU_BLIT_ENGINE_TYPE": "1"},
    "force_blit_0": {"GPU_FORCE_BLIT_COPY_SIZE": "0"},
    "no_large_bar": {"ROC_ENABLE_LARGE_BAR": "0"},
    "host_coherent": {"HIP_HOST_COHERENT": "1"},
}


def child(steps: int):
    sys.path.insert(0, str(REPO))
    import numpy as np
    import torch  # noqa: F401

    import raytracinginonesemester_amd as rt
    from raytracinginonesemester_amd import configs

    cfg = configs.G_CONFIGS["c3"]
    hs = rt.HostScene.load_json(configs.scene_path(cfg["scene"]), REPO)
    cam = hs.camera(cfg["width"], cfg["height"])
    opts, _j = rt.DeviceScene.make_opts(spp=cfg["spp"], max_depth=1, miss_color=hs.settings["miss_color"])
    out = {}
    ds = rt.DeviceScene.from_host(hs)
    p6 = torch.zeros((cam.pixel_height * cam.pixel_width * 3,), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for n in (10, steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            ds.render_device(cam, opts, 0, stream=st, p6_dev_ptr=p6.data_ptr())
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    out["device_loop"] = {"ms_per_frame": round(dt / steps * 1e3, 4)}
    if os.environ.get("RT_EXP_EVENTS", "7") == "7":
        out["device_loop"]["frame_ms"] = round(float(np.median(ds.frame_times(steps))), 4)
        out["device_loop"]["kernel_ms"] = round(float(np.median(ds.kernel_times(steps))), 4)
    ds.close()
    if os.environ.get("RT_EXP_EVENTS", "7") != "7":
        print("RESULT " + json.dumps(out), flush=True)
        return
    for name, d in (("none", rt.RT_DELIVER_NONE), ("p6", rt.RT_DELIVER_P6), ("f32", rt.RT_DELIVER_F32)):
        r = rt.Renderer.from_host(hs, deliver=d)
        for n, timed in ((10, False), (steps, True)):
            t0 = time.perf_counter()
            ts = []
            for _ in range(n):
                ts.append(r.submit(cam, opts))
                if len(ts) >= 3:
                    r.wait(ts.pop(0))
            for t in ts:
                r.wait(t)
            dt = time.perf_counter() - t0
        sc = r.scene(0)
        out[name] = {"ms_per_frame": round(dt / steps * 1e3, 4),
                     "kernel_ms": round(float(np.median(sc.kernel_times(steps))), 4),
                     "frame_ms": round(float(np.median(sc.frame_times(steps))), 4),
                     "deliver_ms": round(float(np.median(r.times(rt.RT_TIME_DELIVER, steps))), 4)}
        r.close()
    print("RESULT " + json.dumps(out), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(int(sys.argv[2]))
        return
    steps = 200
    arg = sys.argv[1] if len(sys.argv) > 1 else None
    if arg and arg.startswith("@"):
        arg = Path(arg[1:]).read_text()
    settings = json.loads(arg) if arg else SETTINGS
    for name, env in settings.items():
        e = dict(os.environ, **env)
        p = subprocess.run([sys.executable, __file__, "--child", str(steps)], env=e, capture_output=True, text=True,
                           timeout=180)
        res = [ln[7:] for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
        print(json.dumps({"setting": name, "env": env, "rc": p.returncode,
                          "result": json.loads(res[0]) if res else p.stderr[-400:]}), flush=True)


if __name__ == "__main__":
    main()
