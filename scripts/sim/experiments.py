"""The wave-simulator experiments of docs/DESIGN_LOG.md §14.6 (diagnostics): the current design's block counts (compare with
profiles/r03/blocks_default.log), capped brick walks, vote-aligned phases, budget schedules and the critical path of
tail splits. Output: profiles/r03/sim_r03.txt.    python scripts/sim/experiments.py > profiles/r03/sim_r03.txt"""
import contextlib
import ctypes
import io
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import scripts.sim.wavesim as S  # noqa: E402


def main():
    import voxelhex_amd as vhx
    lib = S.build()
    lib.wavesim_build.restype = ctypes.c_int64
    flat = vhx.FlatTree.build_scene(1, 1024, 4, threads=8)
    cam = vhx.glass_camera(1024, 3840, 2160, target=(512.0,) * 3)
    print("iteration records", lib.wavesim_build(ctypes.byref(flat.desc), ctypes.byref(cam), 3840, 2160))

    def go(budgets, design=0, cap=0, rpw=(), show=False):
        s = S.run(lib, budgets, design, cap, 12, rpw)
        f = io.StringIO()
        with contextlib.redirect_stdout(f):
            tot = S.report(s, f"budgets {budgets} design {design} cap {cap} rpw {rpw}")
        if show:
            print(f.getvalue(), end="")
        n = len(budgets) + 1
        return tot / 1e6, [s.rays_in[p] for p in range(n)], [round(s.max_wave[p] / 1e3) for p in range(n)]

    print("\n# current design, default schedule (block counts = the VHX_PROF GPU build)")
    base = go((24, 96, 768), show=True)[0]
    print("\n# capped brick walks (design 1): VALU estimate vs current")
    for cap in (6, 4, 3, 2):
        v = go((24, 96, 768), 1, cap)[0]
        print(f"  cap {cap}: {v:.1f}M ({v / base - 1:+.1%})")
    print("\n# vote-aligned phases (design 2): node blocks run when >= kn lanes need them, brick walks when >= kw")
    for kn in (1, 16, 32, 48):
        for kw in (1, 16, 32, 48):
            v = go((24, 96, 768), 2, kn | (kw << 8))[0]
            print(f"  kn {kn:2d} kw {kw:2d}: {v:.1f}M ({v / base - 1:+.1%})")
    print("\n# budget schedules: VALU estimate, rays per pass, costliest wave per pass (k instructions)")
    for b, rpw in [((24, 96, 768), ()), ((64,), ()), ((24, 64, 256, 1024), ()), ((16, 48, 192, 768), ()),
                   ((24, 72, 216, 648), ()), ((32, 96, 288, 864), ()), ((24, 96, 768, 1536), ()),
                   ((24, 96, 768, 1536), (0, 0, 0, 0, 1)), ((24, 96, 768), (0, 0, 0, 16)),
                   ((24, 96, 768, 1280), (0, 0, 0, 0, 4))]:
        v, rays, mw = go(b, 0, 0, rpw)
        print(f"  {str(b):22s} rpw {str(rpw):18s} VALU {v:6.1f}M ({v / base - 1:+.1%}) rays {rays} max-wave {mw} "
              f"(sum {sum(mw)}k)")


if __name__ == "__main__":
    main()
