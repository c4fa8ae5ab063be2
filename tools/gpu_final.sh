# The round's closing measurements on the GPU box (gpurun: bash tools/gpu_final.sh <tag>): the
# driver's default bench command, the C3 rank-of-2 / 4 / 8 rehearsals and the C4 rank-of-8
# rehearsal at the driver's 20 steps; outputs under gpurun_out/<tag>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/${1:-final}; mkdir -p $o
timeout -k 10 400 python -u bench.py > $o/bench_default.json 2> $o/bench_default.err || { tail -20 $o/bench_default.err; exit 1; }
python -c "
import json; d = json.load(open('$o/bench_default.json'))
print('c3', d['value'], d['ms_per_step'], d['roofline']['frac'], (d['roofline'].get('solo') or {}).get('frac'), d['roofline'].get('traffic_same_library'), d.get('batch1', {}).get('ms_per_step'))
for c in d.get('configs', []): print(c['workload'][:3], c.get('value'), c.get('ms_per_step'), c.get('parity_vs_oracle', {}).get('bit_exact'))"
for n in 2 4 8; do
  timeout -k 10 300 python -u bench.py --emulate-rank-of $n --steps 20 > $o/c3_rank$n.json 2> $o/c3_rank$n.err || { tail -20 $o/c3_rank$n.err; exit 1; }
  python -c "import json; d=json.load(open('$o/c3_rank$n.json')); print('c3 rank of $n', d['ms_per_step'], d['value'])"
done
timeout -k 10 300 python -u bench.py --workload c4 --emulate-rank-of 8 --steps 20 > $o/c4_rank8.json 2> $o/c4_rank8.err || { tail -20 $o/c4_rank8.err; exit 1; }
python -c "import json; d=json.load(open('$o/c4_rank8.json')); print('c4 rank8 slowest', d['ms_per_spp_slowest_rank'], 'mean', d['ms_per_spp_mean_rank'])"
