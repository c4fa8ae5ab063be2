#!/bin/bash
# Round-end style GPU pass: parity tests, smoke, profile (kernel trace + PMC passes), bench.
# usage: tools/gpu_round.sh <tag> [bench args...]
set -o pipefail
tag=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/round_$tag; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -n 30 $o/pytest_gpu.log; exit 1; }
tail -n 1 $o/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { cat $o/smoke.log; exit 1; }
tail -n 1 $o/smoke.log
bash tools/profile_round.sh $tag --steps 16 --warmup 16 "$@" || exit 1
timeout -k 10 400 python bench.py "$@" > $o/bench.json 2> $o/bench.err || { tail -n 20 $o/bench.err; exit 1; }
cat $o/bench.json
echo done
