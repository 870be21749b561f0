"""Bisects the palette-tree GPU/oracle mismatch (diagnostic)."""
import numpy as np
import voxelhex_amd as vhx
from voxelhex_amd import _native as N
from tests._oracle import Oracle
from tests.test_gpu_parity import rand_rays

orc = Oracle()
rt = vhx.Raytracer(0)


def host_occ(flat):
    bd = flat.brick_dim
    n3 = bd ** 3
    v = flat.voxels.reshape(-1, n3)
    col = flat.color_palette
    dat = flat.data_palette
    ci = v & 0xFFFF
    di = v >> 16
    cn = (ci == 0xFFFF) | (ci >= col.size) | (((col[np.minimum(ci, max(col.size - 1, 0))] >> 24) & 0xFF) == 0 if col.size else True)
    dn = (di == 0xFFFF) | (di >= dat.size) | ((dat[np.minimum(di, max(dat.size - 1, 0))] == 0) if dat.size else True)
    full = ~(cn & dn)
    words = np.zeros(v.shape[0], np.uint64)
    for b in range(64):
        words |= full[:, b].astype(np.uint64) << np.uint64(b)
    return words


def check(tag, t):
    flat = t.flatten()
    rt.upload(flat)
    rng = np.random.default_rng(9)
    o, d = rand_rays(rng, 64, 5000)
    g = rt.trace_rays(o, d)
    r = orc.trace_rays(flat, o, d)
    bad = np.count_nonzero(g["value"] != r["value"])
    hdr = rt.read_derived(N.VHX_DERIVED_NODE_HDR, 0, flat.desc.node_count)
    occ = rt.read_derived(N.VHX_DERIVED_BRICK_OCC, 0, flat.desc.brick_count)
    hocc = host_occ(flat)
    hdr_ok = np.array_equal(hdr[:, 2], flat.node_type) and np.array_equal(
        (hdr[:, 0].astype(np.uint64) | (hdr[:, 1].astype(np.uint64) << np.uint64(32))), flat.node_ocbits)
    print(f"{tag}: nodes {flat.desc.node_count} bricks {flat.desc.brick_count} colors {flat.desc.color_count} "
          f"data {flat.desc.data_count}: mismatching rays {bad}, hdr ok {hdr_ok}, occ ok {np.array_equal(occ, hocc)} "
          f"(occ diff words {np.count_nonzero(occ != hocc)})", flush=True)


for kind in range(5):
    t = vhx.BoxTree(64, 4)
    rng = np.random.default_rng(3)
    for i in range(3000):
        p = rng.integers(0, 64, 3)
        k = i % 4 if kind == 4 else kind
        e = (vhx.Albedo(int(p[0] * 4), int(p[1] * 4), int(p[2] * 4), 255) if k == 0 else
             int(1 + i % 7) if k == 1 else (vhx.Albedo(10, 20, 30, 255), 3) if k == 2 else vhx.Albedo.from_u32(0x11223344))
        t.insert(p, e)
    check(f"kind {kind}", t)
