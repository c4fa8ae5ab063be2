#!/bin/bash
# One rocprofv3 --pmc pass (counters given) over a short bench command (gpurun); per-kernel
# counter sums printed for the kernels whose name matches a pattern.
# usage: tools/pmc_quick.sh <tag> "<counters>" "<kernel regex>" [bench args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; ctrs=$2; pat=$3; shift 3
o=gpurun_out/pmcq_$tag; mkdir -p $o
timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-trace -d $o/pmc -o run --output-format csv -- python3 bench.py "$@" --no-cpu-baseline --no-parity > $o/pmc.log 2>&1 || { tail -20 $o/pmc.log; exit 1; }
python3 tools/pmc_summary.py $o $pat
