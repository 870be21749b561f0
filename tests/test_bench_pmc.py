"""bench.py's in-run PMC reduction (parse_pmc_dir): FETCH_SIZE and the SQ counters of the frame kernels summed and
divided by the pass-0 dispatches, with the x1024 B x2 gfx950 correction; other kernels are ignored."""
import csv
import os

import bench


def _write(d, rows):
    os.makedirs(os.path.join(d, "box"), exist_ok=True)
    with open(os.path.join(d, "box", "pmc_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for r in rows:
            w.writerow(dict(zip(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"], r)))


def test_parse_pmc_dir(tmp_path):
    p0 = "void k_trace_primary<false, 4, false, false>(vhx::DevTree, CamD)"
    q = "void k_trace_queue<false, 4, false>(vhx::DevTree)"
    rows = []
    for disp in (1, 5):  # two frames
        rows += [(disp, p0, "FETCH_SIZE", 100), (disp, p0, "SQ_INSTS_VALU", 1000),
                 (disp, p0, "SQ_THREAD_CYCLES_VALU", 3200), (disp, p0, "SQ_ACTIVE_INST_VALU", 100),
                 (disp + 1, q, "FETCH_SIZE", 50), (disp + 1, q, "SQ_INSTS_VALU", 2000),
                 (disp + 1, q, "SQ_THREAD_CYCLES_VALU", 1600), (disp + 1, q, "SQ_ACTIVE_INST_VALU", 100),
                 (disp + 2, "void k_trace_primary<true, 4, false, false>(x)", "FETCH_SIZE", 10 ** 9),  # instrumented
                 (disp + 3, "void k_brick_occ_ballot(x)", "FETCH_SIZE", 10 ** 9)]
    _write(str(tmp_path), rows)
    r = bench.parse_pmc_dir(str(tmp_path))
    assert r["frames"] == 2
    assert r["bytes"] == (2 * 150) * 1024 * 2 / 2
    assert r["valu"] == (2 * 3000) / 2
    assert r["lanes"] == {"k_trace_primary": 32.0, "k_trace_queue": 16.0}
    assert abs(r["useful"] - (2 * 4800) / (64 * 2 * 200)) < 1e-12


def test_parse_pmc_dir_empty(tmp_path):
    assert bench.parse_pmc_dir(str(tmp_path)) is None
