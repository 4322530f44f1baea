"""Algorithmic bytes per camera sample (SURVEY.md §8(d) traffic model), from the oracle's
replay of the reference SearchBVH order:
    B_ray = 24*(pops + 2*internal_entered) + 16*(internal_entered + leaf_entered) + 72*leaf_entered
    B_sample = (sum over all rays of B_ray) / camera samples  (+ 12 B/pixel framebuffer / spp)
c3: whole 1920x1080x16 frame.  c5: every 27th row of the 3840x2160x64 frame (80 rows).
Prints a JSON line; the numbers are frozen into raytracinginonesemester_amd/configs.py."""
import json, sys, time
from pathlib import Path
import numpy as np
REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import raytracinginonesemester_amd as rt
from raytracinginonesemester_amd import configs
from oracle import pyoracle as orc

def run(name, rows_step):
    c = configs.G_CONFIGS[name]
    sp = configs.scene_path(c["scene"])
    hs = rt.HostScene.load_json(sp, REPO if sp.parent == configs.SCENES else sp.parent)
    cam = hs.camera(c["width"], c["height"])
    b = cam.basis()
    oc = orc.camera_from_basis(b["center"], b["pixel00_loc"], b["pixel_delta_u"], b["pixel_delta_v"], c["width"], c["height"])
    tot = None
    t = time.time()
    for y in range(0, c["height"], rows_step):
        _, st = orc.render_g(hs.num_triangles, oc, hs.nodes, hs.aabbs, hs.triangles, hs.tri_object_ids, hs.materials,
                             hs.lights, spp=c["spp"], max_depth=c["max_depth"], miss=hs.settings["miss_color"],
                             rows=(y, y + 1), stats=True)
        if tot is None:
            tot = st
        else:
            for k in st:
                tot[k] = [a + b for a, b in zip(tot[k], st[k])] if isinstance(st[k], list) else tot[k] + st[k]
    samples = tot["rays"][0]
    byts = sum(orc.bytes_per_ray(tot, k) * tot["rays"][k] for k in range(3))
    return {"config": name, "rows_step": rows_step, "samples": samples, "B_sample": byts / samples,
            "B_primary": orc.bytes_per_ray(tot, 0), "B_shadow": orc.bytes_per_ray(tot, 1),
            "shadow_per_sample": tot["rays"][1] / samples, "primary_hit_rate": tot["hits"][0] / samples,
            "fb_B_sample": 12.0 / c["spp"], "secs": time.time() - t, "stats": tot}

for name, step in (("c3", 1), ("c5", 27)):
    print(json.dumps(run(name, step)), flush=True)
