# the final build: GPU suite, smoke, default bench, C4 rank-of-8; then one rank of a 2 / 4 / 8-way
# C3 split at the driver's 20 steps (the library's defaults)
bash tools/gpu_suite.sh r05u || exit 1
o=gpurun_out/r05u
for r in 2 4 8; do
  timeout -k 10 300 python -u bench.py --emulate-rank-of $r --steps 20 --no-parity --no-cpu-baseline --configs none --batch1-steps 0 > $o/c3_rank${r}_s20.json 2> $o/c3_rank${r}_s20.err || { tail -20 $o/c3_rank${r}_s20.err; exit 1; }
  python -c "import json; print('c3 rank of $r at 20 steps', json.load(open('$o/c3_rank${r}_s20.json'))['ms_per_step'])"
done
