# the final build: GPU suite, smoke, the driver's default bench, the C4 rank-of-8 rehearsal, then one
# C3 rank of 8 at the driver's 20 steps (overlapped halves by default on a rank's wavefront)
bash tools/gpu_suite.sh r05n || exit 1
o=gpurun_out/r05n
timeout -k 10 300 python -u bench.py --emulate-rank-of 8 --steps 20 --no-parity --no-cpu-baseline --configs none > $o/c3_rank8_s20.json 2> $o/c3_rank8_s20.err || { tail -20 $o/c3_rank8_s20.err; exit 1; }
python -c "import json; print('c3 rank8 s20', json.load(open('$o/c3_rank8_s20.json'))['ms_per_step'])"
