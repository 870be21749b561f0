"""Prices the workgroup-level regroup of the walks in the wave simulator before any kernel is
written: designs 6 (brick walks of a workgroup's 4 waves compacted into full waves through LDS) and 7 (brick and
ADVANCE walks) against the current design 0, on the bench frame with the default frames-in-flight schedule ({24, 72,
216, 648}, sparse 12, 64z queue order), for exchange costs of 0, 30 and 60 VALU-equivalent instructions per wave and
walk phase. The measure is the VALU-weighted wave trips of the simulator (block executions x block cost).
    python scripts/sim/regroup.py > profiles/r06/sim_regroup.txt"""
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
    budgets = (24, 72, 216, 648)
    for order in (1, 0):
        print(f"\n# queue order {order} ({'64z tiles, the busy default' if order == 1 else 'frame rows'})")
        base = None
        for design in (0, 6, 7):
            for cost in ((0, 30, 60) if design else (30,)):
                S.COSTS[16] = cost
                s = S.run(lib, budgets, design, 0, 12, (), order=order)
                f = io.StringIO()
                with contextlib.redirect_stdout(f):
                    tot = S.report(s, f"design {design} exchange cost {cost}")
                print(f.getvalue(), end="")
                walk = sum(s.waves[p][b] * S.COSTS[b] for p in range(S.NP) for b in (2, 6))
                lanes2 = sum(s.lanes[p][2] for p in range(S.NP)) / max(1, sum(s.waves[p][2] for p in range(S.NP)))
                lanes6 = sum(s.lanes[p][6] for p in range(S.NP)) / max(1, sum(s.waves[p][6] for p in range(S.NP)))
                if base is None:
                    base = tot
                print(f"  -> total {tot / 1e6:.1f}M ({tot / base - 1:+.1%} vs design 0), walk trips {walk / 1e6:.1f}M VALU, "
                      f"lanes per brick trip {lanes2:.1f}, per advance trip {lanes6:.1f}")


if __name__ == "__main__":
    main()
