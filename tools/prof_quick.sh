#!/bin/bash
# rocprofv3 kernel-trace stats of one bench command (gpurun); summary printed.
# usage: tools/prof_quick.sh <tag> [bench args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
o=gpurun_out/pq_$tag; mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/trace -o run --output-format csv -- python3 bench.py "$@" --no-cpu-baseline --no-parity > $o/trace.log 2>&1 || { tail -20 $o/trace.log; exit 1; }
python3 tools/prof_summary.py $o/trace | head -40
