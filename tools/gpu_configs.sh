#!/bin/bash
# bench lines of the other BASELINE configs + 8-way scaling rehearsals (one GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/configs; mkdir -p $o
timeout -k 10 300 python bench.py --workload c5 --steps 64 --warmup 2 > $o/c5.json 2>> $o/err.log || exit 1
timeout -k 10 200 python bench.py --workload c2 > $o/c2.json 2>> $o/err.log || exit 1
timeout -k 10 300 python bench.py --workload c4 --steps 64 > $o/c4.json 2>> $o/err.log || exit 1
true
timeout -k 10 300 python bench.py --workload c5 --steps 64 --warmup 2 --emulate-rank-of 8 > $o/c5_e8.json 2>> $o/err.log || exit 1
for f in c5 c2 c4 c5_e8; do python -c "import json;d=json.load(open('$o/$f.json'));print('$f', d['value'], d['ms_per_step'], d.get('samples_per_launch'), d['kernel_ms_per_step']['frame_gpu'], (d.get('parity_vs_oracle') or {}).get('bit_exact'))"; done
