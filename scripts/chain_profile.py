"""The lone frame's dependent chain, per node iteration.

Traces rays of the bench frame (3840x2160, scene S 1024^3 bd 4, glass camera) one per wave through the VHX_CHAIN build
(libvhx_chain.so, vhx_chain_profile: s_memtime stamps around every block of a node iteration) and writes the cycle
breakdown -- node-load waits, leaf probes (brick walks), POP/PUSH bookkeeping, ADVANCE walks, loop overhead -- and the
histogram of the node-load waits, for three sets of pixels: the 256 longest rays of the frame (the lone frame's
critical path), 256 rays around the median of the rays that leave pass 0 (24..72 steps), and 256 random rays that
enter the tree. Step counts per pixel come from the oracle (CPU, test infrastructure: only the pixel choice).
usage: VHX_LIB=voxelhex_amd/_lib/libvhx_chain.so chain_profile.py OUT_DIR"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("VHX_LIB", os.path.join(ROOT, "voxelhex_amd", "_lib", "libvhx_chain.so"))
import numpy as np  # noqa: E402

import voxelhex_amd as vhx  # noqa: E402
from voxelhex_amd import _native as N  # noqa: E402
from tests._oracle import ORACLE_LIB  # noqa: E402

CLASSES = ("load", "probe", "move", "advance", "other")
BUCKET = 64  # cycles per histogram bucket (trace.hpp, VHX_CHAIN_HIST)


def profile(rt, cam, pix):
    out = np.zeros((len(pix), 64), np.uint64)
    p = np.ascontiguousarray(pix, np.uint32)
    rc = N.lib().vhx_chain_profile(rt._h, ctypes.byref(cam), p.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                   len(p), out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    if rc != N.VHX_OK:
        raise RuntimeError(f"vhx_chain_profile = {rc}: {N.lib().vhx_last_error(rt._h)}")
    return out


def summarise(out, name):
    tot = out[:, 0].astype(np.float64)
    cls = {c: out[:, 1 + k].astype(np.float64) for k, c in enumerate(CLASSES)}
    nload, nprobe, nadv, steps = (out[:, k].astype(np.float64) for k in (6, 7, 8, 9))
    hist = out[:, 16:64].sum(0).astype(np.int64)
    acc = sum(cls.values())
    cum = np.cumsum(hist) / max(1, hist.sum())
    pct = {q: int(np.searchsorted(cum, q / 100.0) + 1) * BUCKET for q in (10, 50, 90, 99)}
    s = {
        "rays": int(len(out)),
        "cycles_per_ray_mean": float(tot.mean()), "cycles_per_ray_max": float(tot.max()),
        "steps_per_ray_mean": float(steps.mean()), "node_iterations_per_ray_mean": float(nload.mean()),
        "probes_per_ray_mean": float(nprobe.mean()), "advance_walks_per_ray_mean": float(nadv.mean()),
        "share": {c: float(cls[c].sum() / max(1.0, tot.sum())) for c in CLASSES},
        "stamped_fraction": float(acc.sum() / max(1.0, tot.sum())),
        "cycles_per_node_iteration": float(tot.sum() / max(1.0, nload.sum())),
        "node_load_wait_mean": float(cls["load"].sum() / max(1.0, nload.sum())),
        "node_load_wait_percentiles_le": pct,
        "node_load_wait_histogram_64cyc": hist.tolist(),
        "probe_cycles_mean": float(cls["probe"].sum() / max(1.0, nprobe.sum())),
        "advance_cycles_mean": float(cls["advance"].sum() / max(1.0, nadv.sum())),
        "cycles_per_step": float(tot.sum() / max(1.0, steps.sum())),
    }
    lines = [f"[{name}] {s['rays']} rays, one per wave: {s['cycles_per_ray_mean']:.0f} cycles per ray (max "
             f"{s['cycles_per_ray_max']:.0f}), {s['steps_per_ray_mean']:.1f} steps, {s['node_iterations_per_ray_mean']:.1f} "
             f"node iterations, {s['cycles_per_node_iteration']:.0f} cycles per node iteration, {s['cycles_per_step']:.0f} per step",
             "  share of the traversal: " + ", ".join(f"{c} {100 * v:.1f}%" for c, v in s["share"].items())
             + f" (stamped {100 * s['stamped_fraction']:.1f}%)",
             f"  node-load wait: mean {s['node_load_wait_mean']:.0f} cycles, p10/p50/p90/p99 <= "
             + "/".join(str(pct[q]) for q in (10, 50, 90, 99)) + " cycles",
             f"  per probe {s['probe_cycles_mean']:.0f} cycles, per ADVANCE walk {s['advance_cycles_mean']:.0f} cycles"]
    return s, "\n".join(lines)


def main():
    od = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "chain")
    os.makedirs(od, exist_ok=True)
    W, H, S = 3840, 2160, 1024
    flat = vhx.FlatTree.build_scene(N.VHX_SCENE_LATTICE_CUBE, S, 4, threads=16)
    cam = vhx.glass_camera(S, W, H, target=(S / 2.0,) * 3)
    lib = ctypes.CDLL(ORACLE_LIB)
    steps = np.zeros(W * H, np.uint32)
    assert lib.vhx_oracle_ray_steps(ctypes.byref(flat.desc), ctypes.byref(cam), 0, 0, W, H,
                                    steps.ctypes.data_as(ctypes.c_void_p), 0) == 0
    order = np.argsort(-steps.astype(np.int64), kind="stable")
    rng = np.random.default_rng(0)
    mid = np.nonzero((steps > 24) & (steps <= 72))[0]
    ent = np.nonzero(steps > 0)[0]
    sets = {"longest256": order[:256], "pass1_256": rng.choice(mid, 256, replace=False),
            "random256": rng.choice(ent, 256, replace=False)}
    rt = vhx.Raytracer(0)
    rt.upload(flat)
    res, text = {}, []
    for name, pix in sets.items():
        profile(rt, cam, pix[:8])  # warm-up launch (code and tables)
        out = profile(rt, cam, pix)
        s, t = summarise(out, name)
        s["steps_equal_oracle"] = bool(np.array_equal(out[:, 9].astype(np.uint32), steps[pix]))
        s["oracle_steps_mean"] = float(steps[pix].mean())
        res[name] = s
        text.append(t)
        np.save(os.path.join(od, f"{name}.npy"), out)
    res["clock"] = "s_memtime ticks = shader cycles (MI355X_MICROARCH.md); 2.4 GHz peak"
    json.dump(res, open(os.path.join(od, "chain.json"), "w"), indent=1)
    open(os.path.join(od, "chain.txt"), "w").write("\n".join(text) + "\n")
    print("\n".join(text))
    rt.close()


if __name__ == "__main__":
    main()
