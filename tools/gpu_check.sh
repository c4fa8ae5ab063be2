#!/bin/bash
# One GPU-box pass (gpurun): GPU parity tests, smoke, default bench, scaling rehearsal
# (rank 0's share of an N-way split on one GPU), kernel-trace stats of the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/check; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -n 30 $o/pytest_gpu.log; exit 1; }
tail -n 2 $o/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { cat $o/smoke.log; exit 1; }
cat $o/smoke.log
timeout -k 10 400 python bench.py > $o/bench_c3.json 2> $o/bench_c3.err || { tail -n 20 $o/bench_c3.err; exit 1; }
cat $o/bench_c3.json
for n in 2 4 8; do
  timeout -k 10 200 python bench.py --steps 64 --emulate-rank-of $n > $o/emu_$n.json 2>> $o/emu.err || exit 1
  python -c "import json;d=json.load(open('$o/emu_$n.json'));print($n, d['ms_per_step'], d['kernel_ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/trace -o run --output-format csv -- python3 bench.py --steps 16 --warmup 2 --no-cpu-baseline --no-parity > $o/trace.log 2>&1 || exit 1
echo done
