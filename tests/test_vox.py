"""MagicaVoxel .vox import (vhx_boxtree_load_vox <- BoxTree::load_vox_file, src/convert/magicavoxel.rs:234-374).

Pinning: parse_rotation_matrix against the reference's KATs (magicavoxel.rs:377-404); the rest against an
independent Python restatement of magicavoxel.rs (below) over .vox files written by this test, and the reference's
own models when the checkout is present. The .vox reader itself is restated from the file format; dot_vox 5.1.1 is
not vendored, so byte-level parity with it is unpinned.
"""
import ctypes
import os
import struct

import numpy as np
import pytest

import voxelhex_amd as vhx
from voxelhex_amd import _native as N

REF_MODELS = ["/root/reference/assets/models/navigate.vox",
              "/root/reference/whisp/assets/models/gingerbread_house_by_kirra_luan.vox"]


# ----------------------------------------------------------------------------------------------- .vox writer
def _chunk(cid, content=b"", children=b""):
    return cid.encode() + struct.pack("<ii", len(content), len(children)) + content + children


def _str(s):
    b = s.encode()
    return struct.pack("<i", len(b)) + b


def _dict(d):
    return struct.pack("<i", len(d)) + b"".join(_str(k) + _str(v) for k, v in d.items())


def write_vox(models, palette, scene):
    """models: [(size (x,y,z), [(x,y,z,file_colour_index), ...])]; palette: 256 (r,g,b,a);
    scene: list of ("T", attrs, child, frames) | ("G", attrs, children) | ("S", attrs, [(model_id, attrs)])."""
    body = b""
    for size, voxels in models:
        body += _chunk("SIZE", struct.pack("<iii", *size))
        body += _chunk("XYZI", struct.pack("<i", len(voxels)) + b"".join(struct.pack("<BBBB", *v) for v in voxels))
    for i, node in enumerate(scene):
        if node[0] == "T":
            _, attrs, child, frames = node
            c = struct.pack("<i", i) + _dict(attrs) + struct.pack("<iiii", child, -1, 0, len(frames))
            c += b"".join(_dict(f) for f in frames)
            body += _chunk("nTRN", c)
        elif node[0] == "G":
            _, attrs, children = node
            body += _chunk("nGRP", struct.pack("<i", i) + _dict(attrs) + struct.pack("<i", len(children)) +
                           b"".join(struct.pack("<i", ch) for ch in children))
        else:
            _, attrs, models_ = node
            body += _chunk("nSHP", struct.pack("<i", i) + _dict(attrs) + struct.pack("<i", len(models_)) +
                           b"".join(struct.pack("<i", mid) + _dict(a) for mid, a in models_))
    body += _chunk("MATL", struct.pack("<i", 1) + _dict({"_type": "_diffuse"}))  # skipped chunk
    if palette is not None:
        body += _chunk("RGBA", b"".join(struct.pack("<BBBB", *c) for c in palette))
    return b"VOX " + struct.pack("<i", 200) + _chunk("MAIN", b"", body)


# ----------------------------------------------- independent restatement of src/convert/magicavoxel.rs (Python)
def _rot(b):
    m = [[0] * 3 for _ in range(3)]
    r0, r1 = b & 3, (b >> 2) & 3
    r2 = (~(r0 ^ r1)) & 3
    m[0][r0] = -1 if b & 0x10 else 1
    m[1][r1] = -1 if b & 0x20 else 1
    m[2][r2] = -1 if b & 0x40 else 1
    return m


def _mm(a, b):
    return [[sum(a[i][k] * b[k][j] for k in range(3)) for j in range(3)] for i in range(3)]


def _tr(v, m):
    return tuple(v[0] * m[r][0] + v[1] * m[r][1] + v[2] * m[r][2] for r in range(3))


def _div2(v):  # Rust i32 division truncates toward zero
    return tuple(int(x / 2) for x in v)


def _walk(scene, models, fun):
    ident = [[1, 0, 0], [0, 1, 0], [0, 0, 1]]
    stack = [[scene[0][2], (0, 0, 0), ident, 0]]
    while stack:
        node, t, rot, idx = stack[-1]
        n = scene[node]
        if n[0] == "T":
            fr = n[3][0]
            if "_t" in fr:
                t = tuple(a + int(b) for a, b in zip(t, fr["_t"].split(" ")))
            orient = _mm(rot, _rot(int(fr["_r"]))) if "_r" in fr else ident
            if idx == 0:
                stack[-1][3] += 1
                stack.append([n[2], t, orient, 0])
            else:
                stack.pop()
        elif n[0] == "G":
            if idx < len(n[2]):
                stack[-1][3] += 1
                stack.append([n[2][idx], t, rot, 0])
            else:
                stack.pop()
        else:
            for mid, a in n[2]:
                if int(a.get("_f", "0")) == 0:
                    fun(models[mid], t, rot)
            stack.pop()
            if stack:
                stack[-1][3] += 1


def py_load(models, palette, scene, bd):
    mn, mx = [2 ** 31 - 1] * 3, [-2 ** 31] * 3

    def bounds(m, t, rot):
        h = _div2(_tr(m[0], rot))
        for k in range(3):
            mn[k] = min(mn[k], t[k] - h[k], t[k] + h[k])
            mx[k] = max(mx[k], t[k] + h[k], t[k] - h[k])

    _walk(scene, models, bounds)
    min_ly = (mn[0], mn[2], mn[1])
    max_ly = (mx[0], mx[2], mx[1])
    ext = max(b - a for a, b in zip(min_ly, max_ly))
    libm = ctypes.CDLL("libm.so.6")
    libm.logf.restype = ctypes.c_float
    libm.logf.argtypes = [ctypes.c_float]
    q = np.float32(libm.logf(np.float32(ext) / np.float32(bd))) / np.float32(libm.logf(np.float32(4.0)))
    size = 4 ** max(0, int(np.ceil(q))) * bd
    min_rz = (min_ly[0], min_ly[2], min_ly[1])
    out = {}

    def place(m, t, rot):
        h = _div2(_tr(m[0], rot))
        bl = tuple(t[k] - h[k] - min_rz[k] + (-1 if h[k] < 0 else 0) for k in range(3))
        for v in m[1]:
            tv = _tr(v[:3], rot)
            p = (bl[0] + tv[0], bl[2] + tv[2], bl[1] + tv[1])
            c = palette[max(0, v[3] - 1)]
            out[p] = c[0] | c[1] << 8 | c[2] << 16 | c[3] << 24

    _walk(scene, models, place)
    return size, out


PALETTE = [((k * 37) % 256, (k * 91) % 256, (k * 13) % 256, 255) for k in range(256)]


def _scene_cases():
    cube = ((4, 4, 4), [(x, y, z, 1 + (x + 2 * y + 3 * z) % 200) for x in range(4) for y in range(4) for z in range(4)
                        if (x + y + z) % 2 == 0])
    slab = ((6, 2, 3), [(x, y, z, 7) for x in range(6) for y in range(2) for z in range(3) if x != y])
    lone = ((1, 1, 1), [(0, 0, 0, 255)])
    return {
        "single": ([cube], [("T", {}, 1, [{}]), ("G", {}, [2]), ("T", {}, 3, [{"_t": "10 -3 7"}]),
                            ("S", {}, [(0, {})])]),
        "rotated_pair": ([cube, slab],
                         [("T", {}, 1, [{}]), ("G", {}, [2, 4]),
                          ("T", {}, 3, [{"_t": "0 0 0", "_r": str((1 << 0) | (2 << 2) | (1 << 5) | (1 << 6))}]),
                          ("S", {}, [(0, {})]),
                          ("T", {}, 5, [{"_t": "9 4 -2", "_r": "20"}]), ("S", {}, [(1, {})])]),
        "frames_and_nested": ([cube, lone],
                              [("T", {}, 1, [{}]), ("G", {}, [2, 6]),
                               ("T", {}, 3, [{"_t": "3 3 3", "_r": "4"}]), ("G", {}, [4]),
                               ("T", {}, 5, [{"_t": "-4 8 1"}, {"_t": "100 100 100"}]),
                               ("S", {}, [(0, {}), (1, {"_f": "1"})]),
                               ("T", {}, 7, [{"_t": "12 0 5"}]), ("S", {}, [(1, {"_f": "0"})])]),
        "spread": ([cube, slab, lone],
                   [("T", {}, 1, [{}]), ("G", {}, [2, 4, 6]),
                    ("T", {}, 3, [{"_t": "-30 5 2", "_r": "17"}]), ("S", {}, [(0, {})]),
                    ("T", {}, 5, [{"_t": "40 -20 9", "_r": str(2 | (0 << 2) | (1 << 4))}]), ("S", {}, [(1, {})]),
                    ("T", {}, 7, [{"_t": "5 60 -33"}]), ("S", {}, [(2, {})])]),
    }


# ----------------------------------------------------------------------------------------------------- tests
def test_rotation_matrix_kats():
    """parse_rotation_matrix test (magicavoxel.rs:377-404)."""
    m = (ctypes.c_int32 * 9)()
    assert N.lib().vhx_vox_rotation(4, ctypes.byref(m)) == 0
    assert list(m) == [1, 0, 0, 0, 1, 0, 0, 0, 1]
    assert N.lib().vhx_vox_rotation((1 << 0) | (2 << 2) | (0 << 4) | (1 << 5) | (1 << 6), ctypes.byref(m)) == 0
    assert list(m) == [0, 1, 0, 0, 0, -1, -1, 0, 0]
    valid = 0
    for b in range(128):
        rc = N.lib().vhx_vox_rotation(b, ctypes.byref(m))
        r0, r1 = b & 3, (b >> 2) & 3
        ok = r0 < 3 and r1 < 3 and r0 != r1
        assert (rc == 0) == ok, b
        if ok:
            valid += 1
            a = np.array(list(m)).reshape(3, 3)
            assert (np.abs(a).sum(0) == 1).all() and (np.abs(a).sum(1) == 1).all()
            assert a.tolist() == _rot(b)
    assert valid == 48  # 6 permutations x 8 sign patterns


def test_model_size_to_tree_size():
    for (sx, sy, sz), bd in [((1, 1, 1), 8), ((8, 2, 3), 8), ((9, 1, 1), 8), ((32, 31, 5), 8), ((33, 1, 1), 8),
                             ((64, 64, 64), 4), ((65, 2, 2), 4), ((126, 40, 80), 2), ((300, 1, 1), 16)]:
        got = N.lib().vhx_vox_tree_size(sx, sy, sz, bd)
        m = max(sx, sy, sz)
        assert got % bd == 0 and got >= min(m, got)
        k = round(np.log(got // bd) / np.log(4))
        assert 4 ** k * bd == got


@pytest.mark.parametrize("name", list(_scene_cases()))
@pytest.mark.parametrize("bd", [1, 2, 4, 8])
def test_synthetic_scene_matches_restatement(name, bd):
    models, scene = _scene_cases()[name]
    data = write_vox(models, PALETTE, scene)
    size, want = py_load(models, PALETTE, scene, bd)
    if size < 4 * bd:  # BoxTree::new rejects it; the reference panics in load_vox_file
        with pytest.raises(vhx.OctreeError):
            vhx.BoxTree.load_vox_bytes(data, bd)
        return
    t = vhx.BoxTree.load_vox_bytes(data, bd)
    assert t.info()["size"] == size
    for p, albedo in want.items():
        e = t.get(p)
        assert e.kind == "Visual" and e.albedo().packed() == albedo, (name, p, e)
    assert t.flatten().desc.boxtree_size == size
    rng = np.random.default_rng(bd)
    for p in rng.integers(0, size, (2000, 3)):
        p = tuple(int(v) for v in p)
        assert (t.get(p).kind != "Empty") == (p in want), p


def test_file_roundtrip_and_errors(tmp_path):
    models, scene = _scene_cases()["single"]
    p = tmp_path / "m.vox"
    p.write_bytes(write_vox(models, PALETTE, scene))
    t = vhx.BoxTree.load_vox_file(p, 2)
    assert t.get((0, 0, 0)).kind == "Visual"
    with pytest.raises(N.VhxError):
        vhx.BoxTree.load_vox_file(tmp_path / "missing.vox", 4)
    bad = [b"VOX!" + b"\0" * 40, write_vox(models, PALETTE, scene)[:-20], write_vox(models, None, scene),
           write_vox(models, PALETTE, [("S", {}, [(0, {})])]),
           write_vox(models, PALETTE, [("T", {}, 1, [{}]), ("S", {}, [(5, {})])]),
           write_vox(models, PALETTE, [("T", {}, 1, [{}]), ("T", {}, 2, [{"_r": "3"}]), ("S", {}, [(0, {})])])]
    for b in bad:
        with pytest.raises(N.VhxError):
            vhx.BoxTree.load_vox_bytes(b, 2)
    # odd-sized model mirrored in x lands at -1 (the reference panics on the insert)
    odd = ((3, 1, 1), [(0, 0, 0, 1), (2, 0, 0, 1)])
    with pytest.raises(vhx.InvalidPosition):
        vhx.BoxTree.load_vox_bytes(write_vox([odd], PALETTE, [("T", {}, 1, [{}]), ("T", {}, 2, [{"_r": "20"}]),
                                                              ("S", {}, [(0, {})])]), 1)


def _corrupt_cases():
    """Malformed inputs a parser of untrusted bytes must refuse without reading out of bounds (VERDICT r02 next 6;
    reference entry: magicavoxel.rs:236-253 hands the bytes to dot_vox): chunk lengths past the end, negative chunk,
    string, dictionary, voxel, child and frame counts, negative model sizes."""
    models, scene = _scene_cases()["single"]
    good = write_vox(models, PALETTE, scene)
    cases = {}
    main_at = 8  # "MAIN" chunk header: id, content length, children length
    b = bytearray(good)
    struct.pack_into("<i", b, main_at + 8, 1 << 30)  # MAIN's children length far past the end
    cases["main_children_past_end"] = bytes(b)
    b = bytearray(good)
    struct.pack_into("<i", b, main_at + 8, -64)
    cases["main_children_negative"] = bytes(b)
    b = bytearray(good)
    struct.pack_into("<i", b, main_at + 4, -1)
    cases["main_content_negative"] = bytes(b)
    first = 20  # the first child chunk (SIZE)
    b = bytearray(good)
    struct.pack_into("<i", b, first + 4, 0x7FFFFFF0)  # SIZE content length past the end
    cases["chunk_content_past_end"] = bytes(b)
    b = bytearray(good)
    struct.pack_into("<i", b, first + 4, -12)
    cases["chunk_content_negative"] = bytes(b)
    b = bytearray(good)
    struct.pack_into("<i", b, first + 8, -5)
    cases["chunk_children_negative"] = bytes(b)
    b = bytearray(good)
    struct.pack_into("<iii", b, first + 12, -4, 2, 2)  # negative model size
    cases["size_negative"] = bytes(b)
    xyzi = good.index(b"XYZI")
    b = bytearray(good)
    struct.pack_into("<i", b, xyzi + 12, -3)  # negative voxel count
    cases["xyzi_count_negative"] = bytes(b)
    b = bytearray(good)
    struct.pack_into("<i", b, xyzi + 12, 1 << 29)  # voxel count past the chunk
    cases["xyzi_count_past_chunk"] = bytes(b)
    trn = write_vox(models, PALETTE, [("T", {"_name": "x"}, 1, [{"_t": "1 2 3"}]), ("S", {}, [(0, {})])])
    at = trn.index(b"nTRN") + 12 + 4  # node id, then the attribute dictionary
    b = bytearray(trn)
    struct.pack_into("<i", b, at, -2)  # negative dictionary count
    cases["dict_count_negative"] = bytes(b)
    b = bytearray(trn)
    struct.pack_into("<i", b, at + 4, -7)  # negative key length
    cases["string_length_negative"] = bytes(b)
    b = bytearray(trn)
    struct.pack_into("<i", b, at + 4, 1 << 28)  # key length past the chunk
    cases["string_length_past_chunk"] = bytes(b)
    frames_at = trn.index(b"nTRN") + 12 + 4 + len(_dict({"_name": "x"})) + 12
    b = bytearray(trn)
    struct.pack_into("<i", b, frames_at, -1)  # negative frame count
    cases["frame_count_negative"] = bytes(b)
    grp = write_vox(models, PALETTE, [("T", {}, 1, [{}]), ("G", {}, [2]), ("T", {}, 3, [{}]), ("S", {}, [(0, {})])])
    at = grp.index(b"nGRP") + 12 + 4 + len(_dict({}))
    b = bytearray(grp)
    struct.pack_into("<i", b, at, -9)  # negative child count
    cases["group_children_negative"] = bytes(b)
    b = bytearray(grp)
    struct.pack_into("<i", b, at, 1 << 27)
    cases["group_children_past_chunk"] = bytes(b)
    shp = grp.index(b"nSHP") + 12 + 4 + len(_dict({}))
    b = bytearray(grp)
    struct.pack_into("<i", b, shp, -1)  # negative model count
    cases["shape_models_negative"] = bytes(b)
    cases["truncated_header"] = good[:10]
    cases["empty"] = b""
    return good, cases


@pytest.mark.parametrize("name", sorted(_corrupt_cases()[1]))
def test_corrupt_files_are_refused(name):
    good, cases = _corrupt_cases()
    assert vhx.BoxTree.load_vox_bytes(good, 2) is not None  # the unmodified file loads
    with pytest.raises(N.VhxError):
        vhx.BoxTree.load_vox_bytes(cases[name], 2)


def _read_vox(path):
    """Independent minimal reader: models, palette and scene of a real .vox file (for the restatement)."""
    b = open(path, "rb").read()
    n, m = struct.unpack("<ii", b[12:20])
    off, end = 20 + n, 20 + n + m
    models, scene, palette, pending = [], [], None, None

    def rd_dict(c, o):
        k = struct.unpack("<i", c[o:o + 4])[0]
        o += 4
        d = {}
        for _ in range(k):
            ln = struct.unpack("<i", c[o:o + 4])[0]
            key = c[o + 4:o + 4 + ln].decode()
            o += 4 + ln
            ln = struct.unpack("<i", c[o:o + 4])[0]
            d[key] = c[o + 4:o + 4 + ln].decode()
            o += 4 + ln
        return d, o

    while off < end:
        cid = b[off:off + 4].decode("latin1")
        cn, cm = struct.unpack("<ii", b[off + 4:off + 12])
        c = b[off + 12:off + 12 + cn]
        if cid == "SIZE":
            pending = struct.unpack("<iii", c[:12])
        elif cid == "XYZI":
            k = struct.unpack("<i", c[:4])[0]
            v = np.frombuffer(c[4:4 + 4 * k], np.uint8).reshape(-1, 4)
            models.append((pending, [tuple(int(x) for x in r) for r in v]))
        elif cid == "RGBA":
            palette = [tuple(c[4 * i:4 * i + 4]) for i in range(256)]
        elif cid == "nTRN":
            _, o = rd_dict(c, 4)
            child = struct.unpack("<i", c[o:o + 4])[0]
            nf = struct.unpack("<i", c[o + 12:o + 16])[0]
            o += 16
            frames = []
            for _ in range(nf):
                f, o = rd_dict(c, o)
                frames.append(f)
            scene.append(("T", {}, child, frames))
        elif cid == "nGRP":
            _, o = rd_dict(c, 4)
            k = struct.unpack("<i", c[o:o + 4])[0]
            scene.append(("G", {}, list(struct.unpack(f"<{k}i", c[o + 4:o + 4 + 4 * k]))))
        elif cid == "nSHP":
            _, o = rd_dict(c, 4)
            k = struct.unpack("<i", c[o:o + 4])[0]
            o += 4
            ms = []
            for _ in range(k):
                mid = struct.unpack("<i", c[o:o + 4])[0]
                a, o = rd_dict(c, o + 4)
                ms.append((mid, a))
            scene.append(("S", {}, ms))
        off += 12 + cn + cm
    return models, palette, scene


@pytest.mark.parametrize("path", REF_MODELS, ids=lambda p: os.path.basename(p))
def test_reference_models(path):
    """The reference's own .vox assets (CPU-only; skipped where the checkout is absent)."""
    if not os.path.exists(path):
        pytest.skip("reference checkout not present")
    models, palette, scene = _read_vox(path)
    size, want = py_load(models, palette, scene, 8)
    t = vhx.BoxTree.load_vox_file(path, 8)
    assert t.info()["size"] == size
    keys = list(want)
    rng = np.random.default_rng(0)
    for i in rng.choice(len(keys), size=min(len(keys), 3000), replace=False):
        p = keys[i]
        e = t.get(p)
        assert e.kind == "Visual" and e.albedo().packed() == want[p], (p, e)


def test_gingerbread_fixture_is_the_imported_asset():
    """tests/golden/gingerbread_bd8.npz (the GPU tests' copy of the reference's gingerbread model) equals what
    vhx_boxtree_load_vox builds from the asset, where the reference checkout exists."""
    import hashlib
    import os
    from tests._arraytree import ArrayTree, FIELDS
    from tests.golden.make_vox_fixture import SRC, build
    fx = ArrayTree(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "gingerbread_bd8.npz"))
    assert fx.brick_dim == 8 and fx.boxtree_size == 2048 and fx.desc.node_count > 0
    if not os.path.exists(SRC):
        pytest.skip("reference checkout not present (the GPU box): fixture checked for shape only")
    assert hashlib.sha256(open(SRC, "rb").read()).hexdigest() == fx.source_sha256
    arrays = build()
    for k in FIELDS:
        assert np.array_equal(arrays[k], fx.arrays[k]), k
