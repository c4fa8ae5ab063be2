#!/bin/bash
# Focused GPU-box pass (gpurun): the named test files, then optional bench lines.
# usage: tools/gpu_focus.sh <tag> "<pytest files / -k expr>" [bench args; ...]  (bench runs separated by ';')
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; tests=$2; benches=$3
o=gpurun_out/focus_$tag; mkdir -p $o
if [ -n "$tests" ]; then
  timeout -k 10 900 python -u -m pytest $tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 || { tail -n 40 $o/pytest.log; exit 1; }
  tail -n 3 $o/pytest.log
fi
i=0
IFS=';' read -ra B <<< "$benches"
for b in "${B[@]}"; do
  [ -z "${b// }" ] && continue
  i=$((i+1))
  timeout -k 10 400 python bench.py $b > $o/bench$i.json 2> $o/bench$i.err || { tail -n 20 $o/bench$i.err; exit 1; }
  python -c "import json;d=json.load(open('$o/bench$i.json'));print('$b', d['value'], d['ms_per_step'], json.dumps(d['kernel_ms_per_step']), d['roofline']['kernel'], d['roofline']['frac'])"
done
echo done
