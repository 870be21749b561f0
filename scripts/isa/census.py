"""ISA census of one kernel in a hipcc --save-temps .s file: per basic block the instruction
count by class (VALU, SALU, VMEM, SMEM, LDS, branch, wait), its successors, and the loops (back edges), so that the
traversal blocks can be matched to the source (trace.hpp) and weighted by block-execution counts.

Usage: census.py FILE.s 'k_trace_queue<false, 4, false>' [--asm LABEL...]   (--asm prints those blocks' code)
       census.py FILE.s KERNEL --lines [FILE_SUBSTR]   (a -gline-tables-only build: instructions per source line of
                                                        FILE_SUBSTR, default trace.hpp, with the blocks they fall in)
"""
import re
import subprocess
import sys


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
    return dict(zip(names, out))


def extract(path, want):
    lines = open(path).read().split("\n")
    labels = [(i, m.group(1)) for i, l in enumerate(lines) for m in [re.match(r"^(_Z\w+):", l)] if m]
    dm = demangle([n for _, n in labels])
    for i, n in labels:
        d = dm[n]
        if d.startswith("void " + want + "(") or d.startswith(want + "("):
            body = []
            for l in lines[i + 1:]:
                if l.startswith(".Lfunc_end"):
                    break
                body.append(l)
            return d, body
    raise SystemExit("kernel not found: " + want)


def klass(op):
    if op.startswith("s_waitcnt") or op.startswith("s_wait_"):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc")) or op == "s_endpgm":
        return "branch"
    if op.startswith(("s_load", "s_buffer_load", "s_store", "s_atomic", "s_dcache", "s_buffer_store")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("v_"):
        return "valu"
    return "other"


def blocks_of(body):
    blocks, cur = [], None
    for l in body:
        m = re.match(r"^(\.LBB[0-9_]+):", l)
        if m:
            cur = {"label": m.group(1), "ins": [], "text": []}
            blocks.append(cur)
            continue
        s = l.strip()
        if not s or s.startswith((";", ".", "//")):
            continue
        if cur is None:
            cur = {"label": "entry", "ins": [], "text": []}
            blocks.append(cur)
        op = s.split()[0]
        cur["ins"].append(op)
        cur["text"].append(s)
    return blocks


def lines_census(body, want):
    files, cur, per = {}, None, {}
    block = "entry"
    for l in body:
        t = l.strip()
        m = re.match(r"^\.file\s+(\d+)\s+\"([^\"]*)\"\s+\"([^\"]*)\"", t)
        if m:
            files[m.group(1)] = m.group(3)
            continue
        m = re.match(r"^\.loc\s+(\d+)\s+(\d+)", t)
        if m:
            cur = (m.group(1), int(m.group(2)))
            continue
        m = re.match(r"^(\.LBB[0-9_]+):", l)
        if m:
            block = m.group(1)
            continue
        if not t or t.startswith((";", ".", "//")):
            continue
        k = klass(t.split()[0])
        e = per.setdefault(cur, {"valu": 0, "salu": 0, "other": 0, "blocks": set()})
        e["valu" if k == "valu" else ("salu" if k == "salu" else "other")] += 1
        e["blocks"].add(block)
    return files, per


def main():
    if "--lines" in sys.argv:
        i = sys.argv.index("--lines")
        want = sys.argv[i + 1] if len(sys.argv) > i + 1 else "trace.hpp"
        text = open(sys.argv[1]).read().split("\n")
        name, body = extract(sys.argv[1], sys.argv[2])
        files, per = lines_census([l for l in text if l.strip().startswith(".file")] + body, want)
        print(name)
        rows = sorted(((files.get(f, f), ln, e) for (f, ln), e in ((k, v) for k, v in per.items() if k)),
                      key=lambda r: (r[0], r[1]))
        tot = {}
        for fn, ln, e in rows:
            tot[fn] = tot.get(fn, 0) + e["valu"]
            if want in fn:
                print(f"{fn}:{ln:<5d} valu {e['valu']:4d} salu {e['salu']:3d} other {e['other']:3d}  "
                      + " ".join(sorted(e["blocks"]))[:90])
        print("VALU per file:", tot)
        return
    name, body = extract(sys.argv[1], sys.argv[2])
    show = sys.argv[sys.argv.index("--asm") + 1:] if "--asm" in sys.argv else []
    blocks = blocks_of(body)
    pos = {b["label"]: k for k, b in enumerate(blocks)}
    tot = {}
    print(name)
    for k, b in enumerate(blocks):
        c = {}
        for op in b["ins"]:
            c[klass(op)] = c.get(klass(op), 0) + 1
        for kk, v in c.items():
            tot[kk] = tot.get(kk, 0) + v
        succ = []
        for t in b["text"]:
            m = re.match(r"^s_c?branch\w*\s+(\.LBB[0-9_]+)", t)
            if m:
                tgt = m.group(1)
                succ.append(("^" if pos.get(tgt, 1 << 30) <= k else "") + tgt)
        print(f"{b['label']:>14} n={len(b['ins']):4d} " + " ".join(f"{kk}={v}" for kk, v in sorted(c.items()))
              + (("  -> " + " ".join(succ)) if succ else ""))
        if b["label"] in show:
            for t in b["text"]:
                print("        " + t)
    print("total", sum(tot.values()), dict(sorted(tot.items())))


if __name__ == "__main__":
    main()
