# C5 alone, twice, with a rocprofv3 kernel table: the r05q config line's path traversal ran at 6.44
# instead of ~3.85 ms/spp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r05r; mkdir -p $o
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --workload c5 --steps 8 --configs none --no-parity --no-cpu-baseline > $o/c5_$k.json 2> $o/c5_$k.err || { tail -20 $o/c5_$k.err; exit 1; }
  python -c "import json; d=json.load(open('$o/c5_$k.json')); print('c5 run $k', d['ms_per_step'], d['kernel_ms_per_step']['trace_path'])"
done
timeout -k 10 300 python -u bench.py --steps 8 --configs c5 --no-parity --no-cpu-baseline --batch1-steps 0 > $o/c3_then_c5.json 2> $o/c3_then_c5.err || { tail -20 $o/c3_then_c5.err; exit 1; }
python -c "
import json; d=json.load(open('$o/c3_then_c5.json')); c=d['configs'][0]
print('c5 after c3 in one process', c['ms_per_step'], c['kernel_ms_per_step']['trace_path'])"
