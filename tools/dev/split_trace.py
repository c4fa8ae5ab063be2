"""Dev helper: print the GPU per-bounce trace and the oracle's last (cumulative) block of a debug log."""
import sys
lines = open(sys.argv[1]).read().splitlines()
print("\n".join(l for l in lines if l.startswith("GPU b") or (l.startswith("=== frame") and "GPU" in l)))
blocks, cur = [], None
for l in lines:
    if l.startswith("=== frame") and "CPU" in l:
        cur = []
        blocks.append(cur)
    elif cur is not None and l.startswith("CPU"):
        cur.append(l)
print("----")
print("\n".join(blocks[-1] if blocks else []))
print([l for l in lines if l.startswith("GPU [")])
