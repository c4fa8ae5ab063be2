#!/bin/bash
# Round-end refresh after a ReSTIR DI change (gpurun): the whole GPU suite, smoke, and the C4
# bench line with its CPU baseline and parity leg.
# usage: tools/gpu_c4_final.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/final_$1
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -n 30 $o/pytest_gpu.log; exit 1; }
tail -n 1 $o/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { cat $o/smoke.log; exit 1; }
tail -n 1 $o/smoke.log
timeout -k 10 600 python bench.py --workload c4 --steps 64 --cpu-seconds 10 --parity-seconds 60 > $o/c4.json 2> $o/c4.err || { tail -n 20 $o/c4.err; exit 1; }
echo c4 && tail -c 400 $o/c4.json
