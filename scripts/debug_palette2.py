import numpy as np
import voxelhex_amd as vhx
from voxelhex_amd import _native as N
from tests._oracle import Oracle
from tests.test_gpu_parity import rand_rays
orc = Oracle()
rt = vhx.Raytracer(0)
t = vhx.BoxTree(64, 4)
rng = np.random.default_rng(3)
for i in range(3000):
    p = rng.integers(0, 64, 3)
    k = i % 4
    e = (vhx.Albedo(int(p[0] * 4), int(p[1] * 4), int(p[2] * 4), 255) if k == 0 else
         int(1 + i % 7) if k == 1 else (vhx.Albedo(10, 20, 30, 255), 3) if k == 2 else vhx.Albedo.from_u32(0x11223344))
    t.insert(p, e)
flat = t.flatten()
rt.upload(flat)
o, d = rand_rays(np.random.default_rng(9), 64, 5000)
for fields in (("value",), ("value", "cell", "voxel", "impact", "normal", "depth", "rgba")):
    g = rt.trace_rays(o, d, fields=fields, count_bytes=True)
    r = orc.trace_rays(flat, o, d, fields=fields, count_bytes=True)
    bad = np.flatnonzero(g["value"] != r["value"])
    print(fields, "bad", bad.size, "bytes bad", np.count_nonzero(g["bytes"] != r["bytes"]))
    for i in bad[:4]:
        print(i, {k: (g[k][i].tolist(), r[k][i].tolist()) for k in g})
# per-ray single traces for the first bad ray
if bad.size:
    i = bad[0]
    g1 = rt.trace_rays(o[i:i+1], d[i:i+1], count_bytes=True)
    print("single", {k: g1[k][0].tolist() for k in g1})
