"""Per-frame PMC figures of the bench frame from a gpu_profile.sh directory (rocprofv3 --pmc passes of bench.py).

A frame = one vhx_trace_primary launch: pass 0 (k_trace_primary<false,..>), the queue passes (k_trace_queue<false,..>)
and the compaction kernels between them. With frames in flight the dispatches of different frames interleave, so the
figures are totals over every frame kernel divided by the number of pass-0 dispatches (every traced frame is the same
view). Recipe (/opt/skills/guides/MI355X_MICROARCH.md, HBM section): FETCH_SIZE (KB) derives from TCC_EA0_RDREQ and
reads half the bytes on gfx950, so bytes = FETCH_SIZE x 1024 x 2 (Infinity-Cache hits counted: an upper bound of HBM
bytes). Issue side: CDNA4 SIMDs are 32 lanes wide, a wave64 VALU instruction takes 2 issue cycles (MI355X_MICROARCH.md,
per-instruction cycle constants), so the chip issues at most 1024 SIMDs x 2.4 GHz / 2 = 1228.8 G wave-instructions per
second; SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU is the
mean number of active lanes per VALU instruction.

usage: pmc_frame.py PROFILE_DIR WORKLOAD_KEY OUT_JSON
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

FRAME_KERNELS = ("k_trace_primary<false", "k_trace_queue<false", "k_count_flags", "k_scan_counts", "k_emit_flags",
                 "k_gather_chunks", "k_put_queue_args")
PEAK_VALU_WAVE_INSTR_PER_S = 1024 * 2.4e9 / 2


def kname(row):
    return row["Kernel_Name"].replace("void ", "")


def totals(d):
    tot = defaultdict(float)
    per_kernel = defaultdict(lambda: defaultdict(float))
    frames = defaultdict(set)
    for f in glob.glob(os.path.join(d, "pmc*_counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            n = kname(row)
            if not n.startswith(FRAME_KERNELS):
                continue
            c = row["Counter_Name"]
            v = float(row["Counter_Value"])
            tot[c] += v
            per_kernel[n.split("(")[0]][c] += v
            if n.startswith("k_trace_primary<false"):
                frames[os.path.basename(f)].add(row["Dispatch_Id"])
    nfr = {k: len(v) for k, v in frames.items()}
    return tot, per_kernel, nfr


def main():
    d, key, out = sys.argv[1], sys.argv[2], sys.argv[3]
    tot, per_kernel, nfr = totals(d)
    nf = max(nfr.values())
    if any(v != nf for v in nfr.values()):
        sys.exit(f"passes traced different frame counts: {nfr}")
    per = {c: v / nf for c, v in tot.items()}
    fetch_kb = per["FETCH_SIZE"]
    lanes = {k.split("<")[0]: per_kernel[k]["SQ_THREAD_CYCLES_VALU"] / max(1.0, per_kernel[k]["SQ_ACTIVE_INST_VALU"])
             for k in per_kernel if "trace" in k and "SQ_ACTIVE_INST_VALU" in per_kernel[k]}
    useful = per["SQ_THREAD_CYCLES_VALU"] / (64.0 * per["SQ_ACTIVE_INST_VALU"])
    entry = {
        "read_bytes_per_launch": fetch_kb * 1024.0 * 2.0, "fetch_size_kb": fetch_kb, "gfx950_correction": 2.0,
        "source": f"rocprofv3 --pmc FETCH_SIZE (x1024 B, x2 gfx950), frame kernels / frames ({nf}); "
                  f"{os.path.basename(d.rstrip('/'))}",
        "issue": {
            "valu_wave_instructions_per_frame": per["SQ_INSTS_VALU"],
            "salu_instructions_per_frame": per["SQ_INSTS_SALU"],
            "peak_valu_wave_instructions_per_s": PEAK_VALU_WAVE_INSTR_PER_S,
            "active_lanes_per_valu": {k: round(v, 2) for k, v in lanes.items()},
            "useful_lane_frac": round(useful, 4),
            "source": f"rocprofv3 --pmc SQ_INSTS_VALU, SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU; frame kernels / "
                      f"frames ({nf}); {os.path.basename(d.rstrip('/'))}"},
    }
    try:
        allv = json.load(open(out))
    except (OSError, ValueError):
        allv = {}
    allv[key] = entry
    json.dump(allv, open(out, "w"), indent=1, sort_keys=True)
    print(key, json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
