import sys, time
first = sys.argv[1]
if first == "torch":
    import torch
sys.path.insert(0, "hiprt-path-tracer_amd"); sys.path.insert(0, ".")
import __graft_entry__ as g
t = time.time(); g.smoke(); print(first, "smoke", time.time() - t)
import os
maps = open("/proc/self/maps").read()
print(sorted(set(l.split()[-1] for l in maps.splitlines() if "amdhip64" in l or "hsa-runtime" in l)))
