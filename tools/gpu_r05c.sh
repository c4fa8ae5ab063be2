# kernel trace of one C4 rank of 8 (band 3, the slowest) and of the whole C4 frame
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r05c; mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/rank3 -o run --output-format csv -- python3 bench.py --workload c4 --emulate-rank-of 8 --emulate-band 3 --steps 32 > $o/rank3.log 2>&1 || { tail -20 $o/rank3.log; exit 1; }
python tools/prof_summary.py $o/rank3 > $o/rank3_kernel_stats.txt 2>&1; head -40 $o/rank3_kernel_stats.txt
python tools/trace_gaps.py $o/rank3 40
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/whole -o run --output-format csv -- python3 bench.py --workload c4 --steps 16 --configs none --batch1-steps 0 --no-parity --no-cpu-baseline > $o/whole.log 2>&1 || { tail -20 $o/whole.log; exit 1; }
python tools/prof_summary.py $o/whole > $o/whole_kernel_stats.txt 2>&1; head -30 $o/whole_kernel_stats.txt
python tools/trace_gaps.py $o/whole 100
