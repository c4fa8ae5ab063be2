# The GPU suite and smoke, then the driver's default bench command and the C4 rank-of-8 rehearsal
# (gpurun: bash tools/gpu_suite.sh [tag]; outputs under gpurun_out/<tag>)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/${1:-suite}; mkdir -p $o
timeout -k 10 900 python -u -m pytest -q -x --durations=25 --timeout 300 --timeout-method thread -m gpu tests > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -5 $o/smoke.log; exit 1; }
cat $o/smoke.log
timeout -k 10 400 python -u bench.py > $o/bench_default.json 2> $o/bench_default.err || { tail -20 $o/bench_default.err; exit 1; }
python -c "
import json; d = json.load(open('$o/bench_default.json'))
print('c3', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('batch1'))
for c in d.get('configs', []): print(c['workload'][:3], c.get('value'), c.get('ms_per_step'), c.get('parity_vs_oracle', {}).get('bit_exact'))"
timeout -k 10 300 python -u bench.py --workload c4 --emulate-rank-of 8 --steps 20 > $o/c4_rank8.json 2> $o/c4_rank8.err || { tail -20 $o/c4_rank8.err; exit 1; }
python -c "import json; d=json.load(open('$o/c4_rank8.json')); print('c4 rank8 slowest', d['ms_per_spp_slowest_rank'], 'mean', d['ms_per_spp_mean_rank'])"
