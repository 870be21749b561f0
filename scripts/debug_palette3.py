import numpy as np
import voxelhex_amd as vhx
from voxelhex_amd import _native as N
from tests._oracle import Oracle
from tests.test_gpu_parity import rand_rays
orc = Oracle()
rt = vhx.Raytracer(0)


def tree(kind):
    t = vhx.BoxTree(64, 4)
    rng = np.random.default_rng(3)
    for i in range(3000):
        p = rng.integers(0, 64, 3)
        k = i % 4 if kind == 4 else kind
        e = (vhx.Albedo(int(p[0] * 4), int(p[1] * 4), int(p[2] * 4), 255) if k == 0 else
             int(1 + i % 7) if k == 1 else (vhx.Albedo(10, 20, 30, 255), 3) if k == 2 else vhx.Albedo.from_u32(0x11223344))
        t.insert(p, e)
    return t


trees = {k: tree(k) for k in range(5)}
flats = {k: trees[k].flatten() for k in range(5)}
o, d = rand_rays(np.random.default_rng(9), 64, 5000)
ref = {k: orc.trace_rays(flats[k], o, d) for k in range(5)}
for seq in ([4, 4], [3, 4, 4], [0, 1, 2, 3, 4, 4], [1, 4], [0, 4], [2, 4]):
    res = []
    for k in seq:
        rt._tree = None
        rt.upload(flats[k])
        g = rt.trace_rays(o, d)
        res.append(int(np.count_nonzero(g["value"] != ref[k]["value"])))
    print(seq, res, flush=True)
# fresh context per upload
for k in range(5):
    r2 = vhx.Raytracer(0); r2.upload(flats[k]); g = r2.trace_rays(o, d); r2.close()
    print("fresh", k, int(np.count_nonzero(g["value"] != ref[k]["value"])), flush=True)
