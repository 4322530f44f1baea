"""Quick GPU sanity check: render small golden scenes on cuda:0 and compare with the oracle."""
import gzip, json, sys, time
from pathlib import Path
import numpy as np
REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import raytracinginonesemester_amd as rt
from raytracinginonesemester_amd import configs
G = REPO / "tests" / "golden" / "scenes"
print("devices", rt.device_count(), flush=True)
for name, scene in [("c3_small", "frog.json"), ("cornell", "cornell.json"), ("sphere_single", "sphere_single.json"), ("frog_bounce", "frog.json")]:
    meta = json.loads((G / name / "meta.json").read_text())
    sp = configs.scene_path(scene)
    hs = rt.HostScene.load_json(sp, REPO)
    cam = hs.camera(meta["width"], meta["height"])
    ds = rt.DeviceScene.from_host(hs)
    ref = np.frombuffer(gzip.open(G / name / "fb.f32.gz").read(), np.float32).reshape(meta["height"], meta["width"], 3)
    rh = np.frombuffer(gzip.open(G / name / "hits.i32.gz").read(), np.int32).reshape(meta["height"], meta["width"], -1)
    for kern in (rt.RT_KERNEL_WAVE, rt.RT_KERNEL_LANE):
        t = time.time()
        rgb, hi, ht = ds.render(cam, spp=meta["spp"], max_depth=meta["max_depth"], diffuse_bounce=bool(meta["diffuse_bounce"]),
                                miss_color=hs.settings["miss_color"], aov=True, kernel=kern)
        dt = time.time() - t
        d = np.abs(rgb - ref)
        print(f"{name} kernel={kern} {dt*1e3:.1f}ms hits_equal={np.array_equal(hi, rh)} hit_mism={(hi != rh).sum()} "
              f"fb_exact={(rgb.view(np.uint32) == ref.view(np.uint32)).mean():.6f} maxabs={d.max():.3g}", flush=True)
