"""Per-kernel HBM traffic per launch from tools/profile_round.sh's PMC passes.

Corrections (MI355X_MICROARCH.md, HBM / rocprofv3): on gfx950 FETCH_SIZE tallies a
128-B memory-side read request as 64 B, so read bytes are rebuilt from the request-size
counters, 128 * TCC_EA0_RDREQ_128B + 64 * TCC_EA0_RDREQ_64B + 32 * TCC_EA0_RDREQ_32B
(cross-checked against 2 x FETCH_SIZE); write bytes are WRITE_SIZE (KiB, exact for
streaming stores).  Pass 5: SQ_INSTS_VALU (wave-level VALU instructions, the issue
roofline), SQ_WAVES, GRBM_GUI_ACTIVE (summed over the 8 XCDs).

Normalisation.  Every pass runs the same bench command, whose JSON line lists its timed kernel
lines ("kernel_lines": symbol prefix, launches, units per launch).  For each line the LAST
`launches` dispatches of the kernels matching the prefix are the timed region's launches (the
profiled command runs with --no-parity --no-cpu-baseline, so nothing follows them); their
counters, their kernel-trace durations (trace pass) and the line's units per launch all describe
the same launches, and the "timed" entry of the kernel holds bytes per unit, bytes per launch,
the average launch time and the resulting HBM / VALU fractions.  bench.py reads that entry, so
its counter fields are reproducible from profiles/ for any --steps.
usage: python tools/pmc_traffic.py gpurun_out/prof_<tag> profiles/<name>.json
"""
import collections
import csv
import json
import os
import sys

HBM_PEAK = 8.0e12
VALU_PEAK = 256 * 4 * 2.4e9 / 2


def load(d):
    """kernel name -> {dispatch id -> {counter: value}}"""
    agg = collections.defaultdict(lambda: collections.defaultdict(dict))
    p = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(p):
        return agg
    for r in csv.DictReader(open(p)):
        agg[r["Kernel_Name"]][int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    return agg


def load_trace(d):
    """kernel name -> {dispatch id -> duration ns}"""
    out = collections.defaultdict(dict)
    p = os.path.join(d, "run_kernel_trace.csv")
    if not os.path.exists(p):
        return out
    for r in csv.DictReader(open(p)):
        out[r["Kernel_Name"]][int(r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return out


def bench_line(log):
    if not os.path.exists(log):
        return None
    for ln in reversed(open(log, errors="replace").read().splitlines()):
        if ln.startswith('{"metric"'):
            return json.loads(ln)
    return None


def mean(x):
    x = list(x)
    return sum(x) / len(x) if x else None


def per_dispatch(passes, name, did):
    """read / write bytes, VALU instructions of one dispatch (None where a pass lacks it)"""
    q = passes[2].get(name, {}).get(did, {})
    f = passes[0].get(name, {}).get(did, {}).get("FETCH_SIZE")
    if "TCC_EA0_RDREQ_128B_sum" in q:
        rd = 128 * q["TCC_EA0_RDREQ_128B_sum"] + 64 * q.get("TCC_EA0_RDREQ_64B_sum", 0.0) + 32 * q.get("TCC_EA0_RDREQ_32B_sum", 0.0)
    else:
        rd = 2 * 1024 * f if f is not None else None
    w = passes[1].get(name, {}).get(did, {}).get("WRITE_SIZE")
    wr = 1024 * w if w is not None else None
    valu = passes[4].get(name, {}).get(did, {}).get("SQ_INSTS_VALU")
    return rd, wr, valu


def timed_entry(passes, trace, names, launches, units):
    """counters of the last `launches` dispatches of the kernels `names`.  Each pass is its own
    process, so dispatch ids are selected per pass (the order of the launches is the same)."""
    def last(dmap):
        ids = sorted((did, n) for n in names for did in dmap.get(n, {}))
        return ids[-launches:] if launches else []
    if any(n in passes[2] for n in names):
        rds = [per_dispatch(passes, n, did)[0] for did, n in last(passes[2])]
    else:   # no request-size pass: 2 x FETCH_SIZE
        rds = [2 * 1024 * passes[0][n][did]["FETCH_SIZE"] for did, n in last(passes[0])]
    wrs = [1024 * passes[1][n][did]["WRITE_SIZE"] for did, n in last(passes[1]) if "WRITE_SIZE" in passes[1][n][did]]
    valus = [passes[4][n][did]["SQ_INSTS_VALU"] for did, n in last(passes[4]) if "SQ_INSTS_VALU" in passes[4][n][did]]
    durs = [trace[n][did] for did, n in last(trace)]
    rd, wr, valu, avg_ns = mean(x for x in rds if x is not None), mean(wrs), mean(valus), mean(durs)
    if rd is None or wr is None or not avg_ns or not units:
        return None
    tb = rd + wr
    e = {"launches": launches, "units_per_launch": units, "avg_ns": avg_ns, "read_bytes": rd, "write_bytes": wr,
         "traffic_bytes": tb, "read_per_unit": rd / units, "write_per_unit": wr / units, "traffic_per_unit": tb / units,
         "hbm_frac": tb / (avg_ns * 1e-9) / HBM_PEAK, "kernels": sorted(names)}
    if valu is not None:
        e.update(valu_insts=valu, valu_rate=valu / (avg_ns * 1e-9), valu_frac=valu / (avg_ns * 1e-9) / VALU_PEAK)
    return e


def main(src, dst):
    passes = [load(os.path.join(src, f"pmc{i}")) for i in (1, 2, 3, 4, 5)]
    trace = load_trace(os.path.join(src, "trace"))
    line = bench_line(os.path.join(src, "trace.log"))
    names = set().union(*[set(p) for p in passes])
    out = {}
    for k in sorted(names):
        f = [v.get("FETCH_SIZE") for v in passes[0].get(k, {}).values()]
        f = [x for x in f if x is not None]
        w = [v.get("WRITE_SIZE") for v in passes[1].get(k, {}).values()]
        w = [x for x in w if x is not None]
        rds = [per_dispatch(passes, k, did)[0] for did in passes[2].get(k, {})]
        rds = [x for x in rds if x is not None] or [2 * 1024 * x for x in f]
        hm = passes[3].get(k, {})
        hit = mean(v.get("TCC_HIT_sum", 0.0) for v in hm.values()) if hm else None
        miss = mean(v.get("TCC_MISS_sum", 0.0) for v in hm.values()) if hm else None
        sq = passes[4].get(k, {})
        rd, wr = mean(rds), (1024 * mean(w) if w else None)
        out[k] = {"launches": len(f) or len(w), "read_bytes": rd, "write_bytes": wr,
                  "valu_insts": mean(v.get("SQ_INSTS_VALU", 0.0) for v in sq.values()) if sq else None,
                  "waves": mean(v.get("SQ_WAVES", 0.0) for v in sq.values()) if sq else None,
                  "grbm_gui_active": mean(v.get("GRBM_GUI_ACTIVE", 0.0) for v in sq.values()) if sq else None,
                  "traffic_bytes": rd + wr if rd is not None and wr is not None else None,
                  "fetch_size_x2_bytes": 2 * 1024 * mean(f) if f else None,
                  "l2_hit_rate": hit / (hit + miss) if hit is not None and miss is not None and hit + miss > 0 else None,
                  "avg_ns_all_launches": mean(trace.get(k, {}).values()) if trace.get(k) else None}
    lines = (line or {}).get("kernel_lines") or []
    for ln in lines:
        match = sorted(k for k in names if k.startswith(ln["symbol"]))
        if not match:
            continue
        e = timed_entry(passes, trace, match, int(ln["launches"]), float(ln["units_per_launch"]))
        if e:
            for k in match:
                out[k]["timed"] = e
    meta = {"source": src, "note": __doc__.strip().splitlines()[0],
            "bench_command_line": {kk: line.get(kk) for kk in ("steps", "warmup", "config", "ms_per_step", "value")} if line else None,
            # the library the profiled command ran (bench.py compares it with the one it runs)
            "libmpt_sha256_16": ((line or {}).get("device") or {}).get("libmpt_sha256_16"),
            "kernels": out}
    json.dump(meta, open(dst, "w"), indent=1)
    for k, v in sorted(out.items(), key=lambda kv: -(kv[1]["traffic_bytes"] or 0)):
        if v["traffic_bytes"]:
            t = v.get("timed")
            extra = (f"  timed: {t['traffic_per_unit']:.1f} B/unit over {t['launches']} launches of {t['units_per_launch']:.0f} units,"
                     f" {t['avg_ns'] / 1e6:.3f} ms, HBM frac {t['hbm_frac']:.3f}" if t else "")
            print(f"{k[:60]:60s} {v['launches']:4d}  rd {v['read_bytes'] / 1e6:9.2f} MB  wr {v['write_bytes'] / 1e6:9.2f} MB"
                  f"  L2 hit {v['l2_hit_rate'] or 0:.2f}{extra}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
