"""Instruction histogram of a kernel's basic blocks from the gfx950 ISA (development tool).

Compiles one translation unit of libmpt with --save-temps (the same flags as mpt/_build.py),
finds the kernel's symbol in the assembly and prints, per basic block with at least MIN_VALU
vector-ALU instructions, the instruction count and the most frequent opcodes -- e.g. the BVH8
node test of k_trace<TM_PATH> (profiles/r04_k_trace_node_isa.txt) -- plus the kernel's
resource usage (VGPRs, scratch, LDS, occupancy).
usage: python tools/isa_hist.py <source under csrc> <kernel symbol prefix> [-DDEFINE ...]
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hiprt-path-tracer_amd"))
from mpt import _build  # noqa: E402

MIN_VALU = 24


def main():
    src, prefix, defs = sys.argv[1], sys.argv[2], sys.argv[3:]
    with tempfile.TemporaryDirectory() as d:
        cmd = [_build.HIPCC, *_build.CXXFLAGS, *defs, "-c", str(_build.CSRC / src), "-o", os.path.join(d, "x.o"),
               "--save-temps", "-Rpass-analysis=kernel-resource-usage"]
        r = subprocess.run(cmd, cwd=d, capture_output=True, text=True)
        if r.returncode != 0:
            sys.exit(r.stdout + r.stderr)
        asm = [f for f in os.listdir(d) if f.endswith("gfx950.s")][0]
        lines = open(os.path.join(d, asm)).read().split("\n")
        usage = [l for l in r.stderr.split("\n") if "remark" in l]
    start = next(i for i, l in enumerate(lines) if l.startswith(prefix) and re.match(r"^[\w.$]+:", l))
    name = lines[start].split(":")[0]
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    print(f"kernel {name}")
    grab = False
    for l in usage:
        if "Function Name:" in l:
            grab = name in l
        elif grab:
            m = re.search(r"remark: [^ ]+ +(.*) \[-Rpass-analysis", l)
            if m:
                print("  " + m.group(1).strip())
    blocks, cur, label = [], [], "entry"
    for l in lines[start + 1:end]:
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            blocks.append((label, cur))
            label, cur = m.group(1), []
            continue
        t = l.strip()
        if t and not t.startswith((".", ";")):
            cur.append(t.split()[0])
    blocks.append((label, cur))
    total = sum(len(b) for _, b in blocks)
    print(f"  {total} instructions in {len(blocks)} basic blocks")
    for label, ins in blocks:
        valu = sum(1 for i in ins if i.startswith("v_"))
        if valu >= MIN_VALU:
            c = collections.Counter(ins)
            print(f"  {label}: {len(ins)} instructions ({valu} VALU): " + ", ".join(f"{k} {v}" for k, v in c.most_common(14)))


if __name__ == "__main__":
    main()
