#!/bin/bash
# batched-sample parity tests + bench sweeps over the batch size (1 GPU and the 8-way rehearsal)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/batch; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "batched or partition or city" > $o/pytest.log 2>&1 || { tail -n 30 $o/pytest.log; exit 1; }
tail -n 2 $o/pytest.log
for b in 1 2 4; do
  timeout -k 10 200 python bench.py --steps 64 --batch $b --no-cpu-baseline --no-parity > $o/b1_$b.json 2>> $o/err.log || exit 1
  python -c "import json;d=json.load(open('$o/b1_$b.json'));print('1gpu batch', $b, d['ms_per_step'], d['samples_per_launch'], d['value'])"
done
for b in 1 4 8 16; do
  timeout -k 10 200 python bench.py --steps 64 --batch $b --emulate-rank-of 8 > $o/e8_$b.json 2>> $o/err.log || exit 1
  python -c "import json;d=json.load(open('$o/e8_$b.json'));print('rank of 8, batch', $b, d['ms_per_step'], d['samples_per_launch'])"
done
for b in 2 4; do
  timeout -k 10 200 python bench.py --steps 64 --batch $b --emulate-rank-of $b > $o/e${b}_$b.json 2>> $o/err.log || exit 1
  python -c "import json;d=json.load(open('$o/e${b}_$b.json'));print('rank of', $b, 'batch', $b, d['ms_per_step'], d['samples_per_launch'])"
done
echo done
