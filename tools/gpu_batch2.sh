#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/batch2; mkdir -p $o
for b in 8 16; do
  timeout -k 10 200 python bench.py --steps 64 --batch $b --no-cpu-baseline --no-parity > $o/b1_$b.json 2>> $o/err.log || exit 1
  python -c "import json;d=json.load(open('$o/b1_$b.json'));print('1gpu batch', $b, d['ms_per_step'], d['samples_per_launch'], d['value'])"
done
timeout -k 10 200 python bench.py --steps 64 --emulate-rank-of 8 > $o/e8_auto.json 2>> $o/err.log || exit 1
python -c "import json;d=json.load(open('$o/e8_auto.json'));print('rank of 8 auto', d['ms_per_step'], d['samples_per_launch'])"
timeout -k 10 400 python bench.py > $o/bench_c3.json 2>> $o/err.log || exit 1
cat $o/bench_c3.json
echo done
