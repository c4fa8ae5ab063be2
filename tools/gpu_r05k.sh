# round-5 evidence at the final build: rocprofv3 kernel tables + PMC passes + bench lines (C3, C4),
# then the C3 rank-of-8 rehearsal
bash tools/gpu_evidence.sh r05k c3 "--steps 32" "--steps 64" && bash tools/gpu_evidence.sh r05k c4 "--steps 32" "--steps 32" || exit 1
o=gpurun_out/ev_r05k
timeout -k 10 300 python -u bench.py --emulate-rank-of 8 --steps 64 > $o/c3_rank8.json 2> $o/c3_rank8.err || { tail -20 $o/c3_rank8.err; exit 1; }
tail -c 300 $o/c3_rank8.json
