"""GPU idle time between kernels in a rocprofv3 --kernel-trace run (development tool).

Reads the run's kernel_trace.csv, takes the dispatches of the last `window_ms` of the trace
(the bench's timed region sits at its end), and prints the busy fraction of the GPU over that
window (union of kernel intervals), the number of dispatches, their mean duration and the
mean gap between consecutive dispatches -- the cost of a launch chain of small kernels.
With a third argument, also the window's dispatches per kernel (count, total and mean
duration; the busy time they overlap with other kernels is counted in each).
usage: python tools/trace_gaps.py <rocprofv3 output dir> [window_ms] [per-kernel: 1]
"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    window = float(sys.argv[2]) if len(sys.argv) > 2 else 50.0
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = list(csv.DictReader(open(f)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    t_end = max(e for _, e, _ in iv)
    t0 = t_end - window * 1e6
    iv = [x for x in iv if x[0] >= t0]
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = iv[-1][1] - iv[0][0]
    gaps = [max(0, iv[i + 1][0] - iv[i][1]) for i in range(len(iv) - 1)]
    # the largest gap is usually a host synchronisation (the timed region's boundary): reported
    # apart, and the busy fraction also given without it
    top = max(gaps) if gaps else 0
    rest = sorted(gaps)[:-1] if gaps else []
    print(f"window {span / 1e6:.3f} ms, {len(iv)} dispatches, busy {busy / span:.3f} "
          f"({busy / max(1, span - top):.3f} without the largest gap, {top / 1e3:.1f} us), "
          f"mean kernel {sum(e - s for s, e, _ in iv) / len(iv) / 1e3:.1f} us, "
          f"mean gap {sum(rest) / max(1, len(rest)) / 1e3:.1f} us without it, gaps > 20 us: {sum(1 for g in rest if g > 20000)}")
    if len(sys.argv) > 3:
        per = {}
        for s, e, n in iv:
            k = n.split("(")[0][:90]
            c, t = per.get(k, (0, 0))
            per[k] = (c + 1, t + e - s)
        for k, (c, t) in sorted(per.items(), key=lambda x: -x[1][1]):
            print(f"{c:6d} {t / 1e3:10.1f} us {t / c / 1e3:8.2f} us/call  {k}")


if __name__ == "__main__":
    main()
