#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/batch3; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -k batched > $o/pytest.log 2>&1 || { tail -n 20 $o/pytest.log; exit 1; }
tail -n 1 $o/pytest.log
true
timeout -k 10 300 python bench.py --steps 128 --emulate-rank-of 8 > $o/e8.json 2>> $o/err.log || exit 1
timeout -k 10 300 python bench.py --steps 128 --emulate-rank-of 4 > $o/e2.json 2>> $o/err.log || exit 1
for f in e2 e8; do python -c "import json;d=json.load(open('$o/$f.json'));print('$f', d['value'], d['ms_per_step'], d['samples_per_launch'])"; done
