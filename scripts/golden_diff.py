"""Debug helper: render a golden scene with the current library (RT_MI355X_LIB) and report the
pixels whose float framebuffer differs from the golden one.
    python scripts/golden_diff.py sphere_single [kernel] [flags]"""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))
import torch  # noqa: E402,F401

from conftest import G_SCENES, golden_array, golden_meta, hexv, host_scene  # noqa: E402
import raytracinginonesemester_amd as rt  # noqa: E402

name = sys.argv[1]
kernel = int(sys.argv[2]) if len(sys.argv) > 2 else 1
flags = int(sys.argv[3]) if len(sys.argv) > 3 else 0
meta = golden_meta(name)
hs = host_scene(G_SCENES[name])
cam = hs.camera(meta["width"], meta["height"])
ds = rt.DeviceScene.from_host(hs, device=0)
rgb, hi, ht = ds.render(cam, spp=meta["spp"], max_depth=meta["max_depth"], diffuse_bounce=bool(meta["diffuse_bounce"]),
                        miss_color=hexv(meta["miss_color"]), aov=True, kernel=kernel, flags=flags)
ref = golden_array(name, "fb.f32.gz", np.float32).reshape(meta["height"], meta["width"], 3)
rgb = np.asarray(rgb, np.float32).reshape(ref.shape)
bad = np.nonzero((rgb.view(np.uint32) != ref.view(np.uint32)).any(axis=2))
print(name, "kernel", kernel, "flags", flags, "differing pixels", len(bad[0]), "of", ref.shape[0] * ref.shape[1],
      "max-abs", float(np.abs(rgb - ref).max()))
for y, x in list(zip(*bad))[:12]:
    print(" ", (int(x), int(y)), rgb[y, x].tolist(), ref[y, x].tolist())
