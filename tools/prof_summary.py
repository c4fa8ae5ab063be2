"""Summarises a rocprofv3 --kernel-trace --stats run (rocpd SQLite db or the
kernel_stats.csv of --output-format csv) into a plain-text table for profiles/."""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute(
        "select name, count(*), sum(duration)/1000.0, avg(duration)/1000.0, min(duration)/1000.0, max(duration)/1000.0,"
        " max(vgpr_count), max(sgpr_count), max(scratch_size), max(lds_size), max(grid_x), max(workgroup_x)"
        " from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1.0
    out = ["%-70s %6s %12s %10s %10s %10s %5s %5s %7s %6s %9s" % (
        "kernel", "calls", "total_us", "avg_us", "min_us", "max_us", "vgpr", "sgpr", "scratch", "lds", "grid")]
    for r in rows:
        out.append("%-70s %6d %12.1f %10.2f %10.2f %10.2f %5d %5d %7d %6d %9d  (%.1f%%)" % (
            r[0][:70], r[1], r[2], r[3], r[4], r[5], r[6], r[7], r[8], r[9], r[10], 100.0 * r[2] / total))
    return "\n".join(out)


def from_csv(path):
    with open(path) as f:
        rows = list(csv.DictReader(f))
    out = ["%-70s %6s %12s %10s %8s" % ("kernel", "calls", "total_us", "avg_us", "pct")]
    for r in rows:
        out.append("%-70s %6s %12.1f %10.2f %8.2f" % (r["Name"][:70], r["Calls"], float(r["TotalDurationNs"]) / 1e3,
                                                   float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
    return "\n".join(out)


def main(src, dst=None):
    if os.path.isdir(src):
        dbs = glob.glob(os.path.join(src, "**", "*.db"), recursive=True)
        csvs = glob.glob(os.path.join(src, "**", "*kernel_stats.csv"), recursive=True)
        text = from_csv(csvs[0]) if csvs else from_db(dbs[0])
    elif src.endswith(".db"):
        text = from_db(src)
    else:
        text = from_csv(src)
    if dst:
        with open(dst, "w") as f:
            f.write(text + "\n")
    print(text)


if __name__ == "__main__":
    main(*sys.argv[1:])
