"""A compiled C consumer of the C ABI (tests/abi_c/consumer.c, gcc -std=c99 against include/*.h, linked to the in-tree
libvhx.so): the call shape of the reference-side Rust `extern "C"` block. The CPU test builds and
links it and runs its no-device path; the GPU test feeds it the BASELINE config-2 tree and camera through a file and
checks what it wrote: the first frame against the committed golden digests (tests/golden/frames.json), five frames of
two back-to-back vhx_trace_primary_batch calls on one context against the same digests and a two-frame
vhx_trace_shadows_batch against the oracle's shadow pass, the frame after its ranged write against the oracle, and the
one-rank vhx_mgpu frame against the golden RGBA / depth."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

import voxelhex_amd as vhx
from voxelhex_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "abi_c", "_build", "consumer")
CASE = "c2_256_bd4_1920x1080"


def build_consumer():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "abi_c")], check=True)
    return EXE


def _write_tree(path, flat, cam):
    d = flat.desc
    counts = np.array([d.boxtree_size, d.brick_dim, d.node_count, d.brick_count, d.solid_count, d.color_count,
                       d.data_count, 0], np.uint32)
    with open(path, "wb") as f:
        f.write(b"VHXT")
        f.write(np.array([1, __import__("ctypes").sizeof(cam)], np.uint32).tobytes())
        f.write(counts.tobytes())
        f.write(bytes(cam))
        for a in (flat.node_type, flat.node_ocbits, flat.node_children, flat.voxels, flat.solid_values,
                  flat.color_palette, flat.data_palette):
            f.write(np.ascontiguousarray(a).tobytes())


def test_c_consumer_builds_links_and_reports_no_device(tmp_path):
    exe = build_consumer()
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, 32, 8)
    tree = str(tmp_path / "tree.bin")
    _write_tree(tree, flat, vhx.glass_camera(32, 16, 16))
    n = __import__("ctypes").c_int()
    N.lib().vhx_device_count(__import__("ctypes").byref(n))
    r = subprocess.run([exe, tree, str(tmp_path)], capture_output=True, text=True, timeout=120)
    if n.value == 0:
        assert r.returncode == 3 and "no_device 1" in r.stdout, (r.returncode, r.stdout, r.stderr)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "usage" in r.stderr


@pytest.mark.gpu
def test_c_consumer_frames(tmp_path, oracle):
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "frames.json")))[CASE]
    size, bd, W, H = meta["size"], meta["brick_dim"], meta["width"], meta["height"]
    flat = vhx.FlatTree.build_scene(meta["scene"], size, bd)
    cam = vhx.glass_camera(size, W, H, target=(size / 2,) * 3)
    tree = str(tmp_path / "tree.bin")
    _write_tree(tree, flat, cam)
    exe = EXE if os.path.exists(EXE) else build_consumer()
    r = subprocess.run([exe, tree, str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    out = r.stdout
    assert "shared_equal 1" in out and "past_end -3" in out and "through_shared -5" in out and \
           "empty_frame -1" in out and out.strip().endswith("ok"), out
    n = W * H
    raw = np.fromfile(str(tmp_path / "frame0.bin"), np.uint32)
    widths = {"value": 1, "cell": 1, "voxel": 3, "impact": 3, "normal": 3, "depth": 1, "rgba": 1}
    off = 0
    for k in ("value", "cell", "voxel", "impact", "normal", "depth", "rgba"):
        part = raw[off:off + n * widths[k]]
        off += n * widths[k]
        assert hashlib.sha256(part.tobytes()).hexdigest() == meta["sha256"][k], f"frame0 {k} differs from golden"
    # the batches: five frames of two back-to-back vhx_trace_primary_batch calls on one context, then the shadow batch
    assert "batch_overlap -1" in out and "batch frames 5 shadow_frames 2" in out, out
    bt = np.fromfile(str(tmp_path / "batch.bin"), np.uint32).reshape(17, n)
    for k in range(5):
        for i, f in enumerate(("value", "depth", "rgba")):
            assert hashlib.sha256(bt[3 * k + i].tobytes()).hexdigest() == meta["sha256"][f], f"batch frame {k} {f}"
    hits = oracle.trace_primary(flat, cam, 0, 0, W, H, fields=("value", "impact", "normal", "rgba"))
    sh = oracle.trace_shadows(flat, (float(size),) * 3, hits)["shadowed"]
    assert sh.sum() > 0
    for k in range(2):
        assert np.array_equal(bt[15 + k], sh), f"shadow batch frame {k}"
    # frame 1: the C program cleared the first brick_count // 3 bricks' voxels through vhx_update_range
    clear = int(out.split("cleared_voxels ")[1].split()[0])
    flat.voxels[:clear] = N.VHX_EMPTY
    ref = oracle.trace_primary(flat, cam, 0, 0, W, H, fields=("value", "depth", "rgba"))
    f1 = np.fromfile(str(tmp_path / "frame1.bin"), np.uint32).reshape(3, n)
    for i, k in enumerate(("value", "depth", "rgba")):
        assert np.array_equal(f1[i], ref[k].view(np.uint32)), f"frame1 {k} differs from the oracle"
    assert not np.array_equal(f1[0], raw[:n])
    if "mgpu skipped" not in out:
        mg = np.fromfile(str(tmp_path / "mgpu.bin"), np.uint32).reshape(2, n)
        assert hashlib.sha256(mg[0].tobytes()).hexdigest() == meta["sha256"]["rgba"]
        assert hashlib.sha256(mg[1].tobytes()).hexdigest() == meta["sha256"]["depth"]
