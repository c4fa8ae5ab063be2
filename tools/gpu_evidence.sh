#!/bin/bash
# Evidence for one workload on the GPU box (gpurun): rocprofv3 kernel table + separate PMC passes
# of the bench command (tools/profile_round.sh), the per-kernel traffic summary normalised by
# the profiled run's own launches (tools/pmc_traffic.py, copied into profiles/ so the bench line
# below reads it), then the bench line itself.
# usage: tools/gpu_evidence.sh <tag> <workload> "<profile args>" "<bench args>"
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; w=$2; pargs=$3; bargs=$4
o=gpurun_out/ev_$tag; mkdir -p $o
bash tools/profile_round.sh ${tag}_$w --workload $w $pargs || exit $?
python tools/pmc_traffic.py gpurun_out/prof_${tag}_$w $o/${tag}_${w}_pmc_traffic.json > $o/${tag}_${w}_pmc.txt || exit 1
cp $o/${tag}_${w}_pmc_traffic.json profiles/
python tools/prof_summary.py gpurun_out/prof_${tag}_$w/trace > $o/${tag}_${w}_kernel_stats.txt 2>/dev/null || true
timeout -k 10 600 python bench.py --workload $w --configs none $bargs > $o/${tag}_${w}_bench.json 2> $o/${tag}_${w}_bench.err || { tail -n 20 $o/${tag}_${w}_bench.err; exit 1; }
tail -c 400 $o/${tag}_${w}_bench.json
echo
