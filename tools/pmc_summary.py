"""Per-kernel summary of rocprofv3 --pmc passes (tools/gpu_probe.sh): the mean per dispatch
of every counter, plus derived ratios (issue / wait split, VALU and f64 mix per wave,
texture-address busy fraction).
usage: python tools/pmc_summary.py gpurun_out/<tag> [kernel substrings...]"""
import collections
import csv
import glob
import os
import sys


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in sorted(glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(p)):
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main(d, *names):
    agg = load(d)
    for k in sorted(agg):
        if names and not any(n in k for n in names):
            continue
        c = {n: sum(v) / len(v) for n, v in agg[k].items()}
        print(k[:90])
        for n in sorted(c):
            print(f"    {n:40s} {c[n]:16.4g}")
        w = c.get("SQ_WAVES")
        if c.get("SQ_WAVE_CYCLES"):
            wc = c["SQ_WAVE_CYCLES"]
            print(f"    -> issue/wait: active {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f} wait {c.get('SQ_WAIT_ANY', 0) / wc:.3f} "
                  f"wait_inst {c.get('SQ_WAIT_INST_ANY', 0) / wc:.3f} valu {c.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f} "
                  f"vmem {c.get('SQ_ACTIVE_INST_VMEM', 0) / wc:.3f}")
        if w:
            f64 = sum(c.get(n, 0) for n in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                             "SQ_INSTS_VALU_TRANS_F64"))
            f32 = sum(c.get(n, 0) for n in ("SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_FMA_F32"))
            print(f"    -> per wave: valu {c.get('SQ_INSTS_VALU', 0) / w:.0f} f64 {f64 / w:.0f} f32 add/mul/fma {f32 / w:.0f} "
                  f"vmem {c.get('SQ_INSTS_VMEM', 0) / w:.0f} lds {c.get('SQ_INSTS_LDS', 0) / w:.0f} salu {c.get('SQ_INSTS_SALU', 0) / w:.0f}")
        if c.get("GRBM_GUI_ACTIVE") and c.get("TA_BUSY_avr") is not None:
            print(f"    -> TA busy {c['TA_BUSY_avr'] / c['GRBM_GUI_ACTIVE']:.3f} of GUI-active cycles; "
                  f"TCP tag accesses / L2 read req {c.get('TCP_TOTAL_CACHE_ACCESSES_sum', 0) / max(1, c.get('TCP_TCC_READ_REQ_sum', 1)):.2f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
