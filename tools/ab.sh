#!/bin/bash
# A/B timing on the GPU box: alternates bench runs of two libmpt builds (default: ab/base vs
# the in-tree library), printing ms/step and the per-kernel breakdown of each run.
# usage: tools/ab.sh <tag> <rounds> [bench args...]
set -o pipefail
tag=$1; rounds=$2; shift 2
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/ab_$tag
mkdir -p $out
for r in $(seq 1 $rounds); do
  for v in base new; do
    lib=$([ $v = base ] && echo ab/base/libmpt.so || echo hiprt-path-tracer_amd/mpt/libmpt.so)
    MPT_LIB_PATH=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity "$@" > $out/$v$r.json 2> $out/$v$r.err || { tail -5 $out/$v$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$out/$v$r.json')); k=d['kernel_ms_per_step']; print('$v$r', d['ms_per_step'], d['value'], {x: k[x] for x in ('trace_path','trace_nee_any','trace_nee_closest','shade','shade_generic','resolve','restir')})"
  done
done
