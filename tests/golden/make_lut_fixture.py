"""Extracts the three lookup tables of VoxelHex's src/spatial/lut.rs (lines 4-161) as data into luts.json.

Run in the build container (where /root/reference exists):  python tests/golden/make_lut_fixture.py
The JSON holds only the table values (expected outputs of the reference's LUT generators
src/bin/sectant_region_offset_lut.rs and src/bin/sectant_step_result_lut.rs, and the generator-less
RAY_TO_NODE_OCCUPANCY_BITMASK_LUT); tests pin the oracle's regenerated tables against it.
"""
import json
import os
import re
import sys

SRC = os.environ.get("VHX_REFERENCE", "/root/reference") + "/src/spatial/lut.rs"


def block(text, name):
    start = text.index(name)
    start = text.index("= [", start) + 2
    depth, i = 0, start
    while True:
        if text[i] == "[":
            depth += 1
        elif text[i] == "]":
            depth -= 1
            if depth == 0:
                return text[start:i + 1]
        i += 1


def main():
    text = open(SRC).read()
    off = block(text, "SECTANT_OFFSET_LUT")
    offsets = [[float(a), float(b), float(c)] for a, b, c in
               re.findall(r"x:\s*([0-9.]+),\s*y:\s*([0-9.]+),\s*z:\s*([0-9.]+)", off)]
    step = block(text, "SECTANT_STEP_RESULT_LUT")
    step_vals = [int(v) for v in re.findall(r"\d+", step)]
    occ = block(text, "RAY_TO_NODE_OCCUPANCY_BITMASK_LUT")
    occ_vals = [int(v) for v in re.findall(r"\d+", occ)]
    assert len(offsets) == 64 and len(step_vals) == 64 * 27 and len(occ_vals) == 64 * 8
    out = {
        "source": "VoxelHex src/spatial/lut.rs:4-161",
        "sectant_offset": offsets,
        "sectant_step_result": step_vals,
        "ray_to_node_occupancy_bitmask": [str(v) for v in occ_vals],
    }
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "luts.json")
    json.dump(out, open(dst, "w"), separators=(",", ":"))
    print("wrote", dst)


if __name__ == "__main__":
    sys.exit(main())
