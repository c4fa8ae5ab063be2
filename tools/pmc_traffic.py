"""Per-kernel HBM traffic per launch from tools/profile_round.sh's PMC passes.

Corrections (MI355X_MICROARCH.md, HBM / rocprofv3): on gfx950 FETCH_SIZE tallies a
128-B memory-side read request as 64 B, so read bytes are rebuilt from the request-size
counters, 128 * TCC_EA0_RDREQ_128B + 64 * TCC_EA0_RDREQ_64B + 32 * TCC_EA0_RDREQ_32B
(cross-checked against 2 x FETCH_SIZE); write bytes are WRITE_SIZE (KiB, exact for
streaming stores).  Calibration in the same run: k_accumulate moves a known byte count
(reads 100 B / pixel, writes 36 B / pixel).  Pass 5: SQ_INSTS_VALU (wave-level VALU
instructions, the traversal's issue roofline), SQ_WAVES, GRBM_GUI_ACTIVE (summed over the
8 XCDs: effective clock = GRBM_GUI_ACTIVE / 8 / kernel time).
usage: python tools/pmc_traffic.py gpurun_out/prof_<tag> profiles/<name>.json
"""
import collections
import csv
import json
import os
import sys


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    p = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(p):
        return agg
    for r in csv.DictReader(open(p)):
        agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def mean(x):
    return sum(x) / len(x) if x else None


def main(src, dst):
    passes = [load(os.path.join(src, f"pmc{i}")) for i in (1, 2, 3, 4, 5)]
    names = set().union(*[set(p) for p in passes])
    out = {}
    for k in sorted(names):
        f = passes[0].get(k, {}).get("FETCH_SIZE", [])
        w = passes[1].get(k, {}).get("WRITE_SIZE", [])
        q = passes[2].get(k, {})
        n128, n64, n32 = (mean(q.get(c, [])) for c in ("TCC_EA0_RDREQ_128B_sum", "TCC_EA0_RDREQ_64B_sum",
                                                         "TCC_EA0_RDREQ_32B_sum"))
        rd = 128 * n128 + 64 * n64 + 32 * (n32 or 0.0) if n128 is not None else (2 * 1024 * mean(f) if f else None)
        wr = 1024 * mean(w) if w else None
        hm = passes[3].get(k, {})
        hit, miss = mean(hm.get("TCC_HIT_sum", [])), mean(hm.get("TCC_MISS_sum", []))
        sq = passes[4].get(k, {})
        valu = mean(sq.get("SQ_INSTS_VALU", []))
        grbm = mean(sq.get("GRBM_GUI_ACTIVE", []))
        out[k] = {"launches": len(f) or len(w), "read_bytes": rd, "write_bytes": wr,
                  "valu_insts": valu, "waves": mean(sq.get("SQ_WAVES", [])),
                  "grbm_gui_active": grbm,
                  "traffic_bytes": (rd or 0.0) + (wr or 0.0) if rd is not None and wr is not None else None,
                  "fetch_size_x2_bytes": 2 * 1024 * mean(f) if f else None,
                  "l2_hit_rate": hit / (hit + miss) if hit is not None and hit + miss > 0 else None}
    json.dump({"source": src, "note": __doc__.strip().splitlines()[0], "kernels": out}, open(dst, "w"), indent=1)
    for k, v in sorted(out.items(), key=lambda kv: -(kv[1]["traffic_bytes"] or 0)):
        if v["traffic_bytes"]:
            print(f"{k[:60]:60s} {v['launches']:4d}  rd {v['read_bytes'] / 1e6:9.2f} MB  wr {v['write_bytes'] / 1e6:9.2f} MB"
                  f"  (2xFETCH {v['fetch_size_x2_bytes'] / 1e6:9.2f} MB)  L2 hit {v['l2_hit_rate'] or 0:.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
