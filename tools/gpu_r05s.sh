# the ReSTIR DI list traversals at 6 waves / SIMD (ab/wl6: MPT_TRACE_WAVES_LIST=6, their grid at 6
# blocks per CU) against 5 (ab/wl5, the same code): parity, then C4 whole frame and rank of 8
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r05s; mkdir -p $o
W6=$PWD/ab/wl6/libmpt.so; W5=$PWD/ab/wl5/libmpt.so
MPT_LIB_PATH=$W6 timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_restir.py tests/test_configs.py -k "restir or c4" > $o/pytest_wl6.log 2>&1 || { tail -30 $o/pytest_wl6.log; exit 1; }
tail -1 $o/pytest_wl6.log
timeout -k 10 400 python tools/bench_variants.py $W5 $W6 $W5 $W6 -- --workload c4 --steps 32 > $o/c4_ab.jsonl 2> $o/c4_ab.err || { tail -20 $o/c4_ab.err; exit 1; }
python -c "
import json
for l in open('$o/c4_ab.jsonl'):
    j = json.loads(l); k = j['kernels']; print(j['lib'].split('/')[-2], j['ms_per_step'], 'restir', k.get('restir'))"
for v in wl5 wl6; do
  MPT_LIB_PATH=$PWD/ab/$v/libmpt.so timeout -k 10 300 python -u bench.py --workload c4 --emulate-rank-of 8 --steps 128 > $o/c4_rank8_$v.json 2> $o/c4_rank8_$v.err || { tail -20 $o/c4_rank8_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$o/c4_rank8_$v.json')); print('$v rank8 slowest', d['ms_per_spp_slowest_rank'], 'mean', d['ms_per_spp_mean_rank'])"
done
