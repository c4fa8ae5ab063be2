"""Runs bench.py once per libmpt variant (MPT_LIB_PATH) and prints the per-kernel times.
Development tool for A/B experiments on the GPU box:
    python tools/bench_variants.py path/to/a/libmpt.so path/to/b/libmpt.so [-- bench args]
A variant may carry environment settings: path/to/libmpt.so@MPT_SHADE_SPLIT=1,MPT_X=2
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    args = sys.argv[1:]
    extra = []
    if "--" in args:
        i = args.index("--")
        args, extra = args[:i], args[i + 1:]
    for spec in args:
        lib, _, sets = spec.partition("@")
        env = dict(os.environ, MPT_LIB_PATH=os.path.abspath(lib))
        env.update(kv.split("=", 1) for kv in sets.split(",") if kv)
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "16", "--warmup", "2", "--no-cpu-baseline",
               "--no-parity", "--configs", "none", "--batch1-steps", "0", *extra]
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            print(spec, "FAILED", r.returncode, r.stderr[-2000:], flush=True)
            sys.exit(r.returncode)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
        j = json.loads(line)
        print(json.dumps({"lib": spec, "ms_per_step": j["ms_per_step"], "value": j["value"],
                          "kernels": j["kernel_ms_per_step"], "trav": j.get("traversal_stages")}), flush=True)


if __name__ == "__main__":
    main()
