"""The multi-rank code of vhx_mgpu on one GPU (VERDICT r02 "the N>1 branches of vhx_mgpu have never
executed"). tests/abi_c/mgpu_ranks.c runs N rank threads, each with its own vhx_ctx on device 0, against libvhx with
VHX_RCCL_LIB pointing at the loopback communicator of tests/loopback/loopback_rccl.cpp (test infrastructure: RCCL's C
ABI, stream-ordered device-to-device copies instead of xGMI links). So the tree broadcast's receive side on ranks >= 1,
the deal of the tiles over R + N - 1 slots, the point-to-point group into rank 0's slot-major buffer, the untile, frames
in flight and vhx_mgpu_balance with peers all run for real; only the transport differs from the 8-GPU node.

Rank 0's frames are checked bit for bit: camera A against the committed golden digests of c2_256_bd4_1920x1080
(tests/golden/frames.json, the oracle's frame), camera B (a second view, frames alternate A / B and are all submitted
without waiting) against the oracle."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

import voxelhex_amd as vhx
from voxelhex_amd.multigpu import tile_plan

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "tests", "abi_c", "_build")
EXE = os.path.join(BUILD, "mgpu_ranks")
LOOPBACK = os.path.join(BUILD, "libvhx_loopback_rccl.so")
CASE = "c2_256_bd4_1920x1080"
SYMBOLS = ("ncclGetUniqueId", "ncclCommInitRank", "ncclCommDestroy", "ncclCommCount", "ncclCommUserRank",
           "ncclBroadcast", "ncclSend", "ncclRecv", "ncclGroupStart", "ncclGroupEnd", "ncclGetErrorString")


def _build():
    if not (os.path.exists(EXE) and os.path.exists(LOOPBACK)):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "abi_c")], check=True)


def test_loopback_communicator_builds_and_exports_rccl_abi():
    """CPU: the driver and the loopback library build, and the library exports every RCCL symbol libvhx binds
    (voxelhex_amd/csrc/vhx_mgpu.hip, rccl())."""
    import ctypes
    _build()
    lib = ctypes.CDLL(LOOPBACK)
    for s in SYMBOLS:
        assert hasattr(lib, s), s
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "usage" in r.stderr


@pytest.fixture(scope="module")
def scene(tmp_path_factory, oracle):
    from tests.test_abi_c import _write_tree
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "frames.json")))[CASE]
    size, bd, W, H = meta["size"], meta["brick_dim"], meta["width"], meta["height"]
    flat = vhx.FlatTree.build_scene(meta["scene"], size, bd)
    cam_a = vhx.glass_camera(size, W, H, target=(size / 2,) * 3)
    cam_b = vhx.glass_camera(size, W, H, angle=40.7, target=(size / 2,) * 3)
    d = tmp_path_factory.mktemp("mgpu_ranks")
    tree = str(d / "tree.bin")
    _write_tree(tree, flat, cam_a)
    camb = str(d / "camb.bin")
    with open(camb, "wb") as f:
        f.write(bytes(cam_b))
    ref_b = oracle.trace_primary(flat, cam_b, 0, 0, W, H, fields=("depth", "rgba"))
    return dict(meta=meta, tree=tree, camb=camb, ref_b=ref_b, W=W, H=H, dir=d)


@pytest.mark.gpu
@pytest.mark.parametrize("nranks,root_slots,inflight,overlap,frames,mode", [
    (2, 1, 1, 1, 4, "plain"),
    (3, 2, 3, 1, 7, "plain"),
    (4, 1, 2, 0, 5, "plain"),
    (8, 3, 1, 1, 4, "plain"),
    (2, 1, 2, 1, 4, "balance"),
    (3, 1, 1, 1, 4, "balance"),
    (2, 1, 1, 1, 4, "rgba"),
    (8, 3, 2, 1, 5, "rgba"),
    (2, 1, 1, 1, 5, "batch"),
    (4, 2, 2, 1, 7, "batch"),
    (8, 1, 3, 0, 6, "batchrgba"),
    (3, 3, 2, 1, 4, "batchrgba"),
])
def test_ranks_frames_equal_golden_and_oracle(scene, nranks, root_slots, inflight, overlap, frames, mode):
    _build()
    W, H = scene["W"], scene["H"]
    out = str(scene["dir"] / f"fb_{nranks}_{root_slots}_{inflight}_{overlap}_{mode}.bin")
    env = dict(os.environ, VHX_RCCL_LIB=LOOPBACK, VHX_LOOPBACK_TIMEOUT_S="60")
    r = subprocess.run([EXE, scene["tree"], scene["camb"], out, str(nranks), str(root_slots), str(inflight),
                        str(overlap), str(frames), mode], capture_output=True, text=True, timeout=240, env=env)
    print(r.stdout)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (r.returncode, r.stdout, r.stderr[-3000:])
    # every ray traced exactly once over the ranks (vhx_mgpu_info)
    assert f"rays {W * H}" in r.stdout.split("root_slots")[1]
    R = int(r.stdout.split("root_slots ")[1].split()[0])
    assert 1 <= R <= 4 and (mode == "balance" or R == root_slots)
    n = W * H
    fb = np.fromfile(out, np.uint32).reshape(4, n)
    sha = scene["meta"]["sha256"]
    assert hashlib.sha256(fb[0].tobytes()).hexdigest() == sha["rgba"], "camera A rgba differs from golden"
    ref = scene["ref_b"]
    assert np.array_equal(fb[2], ref["rgba"].view(np.uint32)), "camera B rgba differs from the oracle"
    # bytes into rank 0 per frame (vhx_mgpu_frame_bytes, every rank reports the same): the other N - 1 slots' parts,
    # one plane of 32-bit words per tile entry in RGBA-only mode, two otherwise
    root_bytes = {int(line.split("root_bytes ")[1].split()[0]) for line in r.stdout.splitlines() if "root_bytes" in line}
    plan = tile_plan(nranks, R, 64, W, H, 0)
    planes = 1 if mode in ("rgba", "batchrgba") else 2
    assert root_bytes == {(nranks - 1) * plan["tiles_per_slot"] * 64 * 64 * 4 * planes}, root_bytes
    if mode in ("rgba", "batchrgba"):  # no depth plane crossed: rank 0's depth framebuffers keep their fill
        assert (fb[1] == 0xABABABAB).all() and (fb[3] == 0xABABABAB).all()
        return
    assert hashlib.sha256(fb[1].tobytes()).hexdigest() == sha["depth"], "camera A depth differs from golden"
    assert np.array_equal(fb[3], ref["depth"].view(np.uint32)), "camera B depth differs from the oracle"
