# traversal occupancy A/B: any-hit / list traversals at 6 waves/SIMD (path rays at 5), and all at 6
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r05m; mkdir -p $o
B=hiprt-path-tracer_amd/mpt/libmpt.so; A=ab/w6any/libmpt.so; W=ab/w6/libmpt.so
timeout -k 10 400 python tools/bench_variants.py $B $A $W $B $A $W > $o/c3.jsonl 2> $o/c3.err || { tail -20 $o/c3.err; exit 1; }
timeout -k 10 300 python tools/bench_variants.py $B $A $W -- --workload c5 --steps 32 > $o/c5.jsonl 2> $o/c5.err || { tail -20 $o/c5.err; exit 1; }
for w in c3 c5; do python -c "
import json
for l in open('$o/$w.jsonl'):
    j = json.loads(l); k = j['kernels']
    print('$w', j['lib'].split('/')[-2], j['ms_per_step'], 'trace', k['trace_path'], k['trace_nee_any'], k['trace_nee_closest'])"; done
# the driver's 20 steps on one rank of 8: overlapped sample-batch halves (MPT_OVERLAP) or not
for v in 0 1; do
  MPT_OVERLAP=$v timeout -k 10 300 python -u bench.py --emulate-rank-of 8 --steps 20 --no-parity --no-cpu-baseline --configs none > $o/c3_rank8_s20_ov$v.json 2> $o/c3_rank8_s20_ov$v.err || { tail -20 $o/c3_rank8_s20_ov$v.err; exit 1; }
  MPT_OVERLAP=$v timeout -k 10 300 python -u bench.py --emulate-rank-of 8 --steps 20 --no-parity --no-cpu-baseline --configs none > $o/c3_rank8_s20_ov${v}b.json 2> $o/c3_rank8_s20_ov${v}b.err || { tail -20 $o/c3_rank8_s20_ov${v}b.err; exit 1; }
  python -c "import json; print('overlap=$v', json.load(open('$o/c3_rank8_s20_ov$v.json'))['ms_per_step'], json.load(open('$o/c3_rank8_s20_ov${v}b.json'))['ms_per_step'])"
done
