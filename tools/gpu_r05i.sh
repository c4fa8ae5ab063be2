# chunked ReSTIR DI initial candidates (ab/ci): the ReSTIR / C4 parity tests with the variant,
# then C4 whole frame base vs ci and the rank-of-8 rehearsal with ci
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r05i; mkdir -p $o
CI=$PWD/ab/ci/libmpt.so
MPT_LIB_PATH=$CI timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_restir.py tests/test_configs.py -k "restir or c4" > $o/pytest_ci.log 2>&1 || { tail -30 $o/pytest_ci.log; exit 1; }
tail -2 $o/pytest_ci.log
timeout -k 10 400 python tools/bench_variants.py hiprt-path-tracer_amd/mpt/libmpt.so $CI hiprt-path-tracer_amd/mpt/libmpt.so $CI -- --workload c4 --steps 32 > $o/c4_ab.jsonl 2> $o/c4_ab.err || { tail -20 $o/c4_ab.err; exit 1; }
python -c "
import json
for l in open('$o/c4_ab.jsonl'):
    j = json.loads(l); k = j['kernels']; print('c4', j['lib'].split('/')[-2], j['ms_per_step'], 'restir', k.get('restir'), k.get('restir_kernels'))"
MPT_LIB_PATH=$CI timeout -k 10 300 python -u bench.py --workload c4 --emulate-rank-of 8 --steps 128 > $o/c4_rank8_ci.json 2> $o/c4_rank8_ci.err || { tail -20 $o/c4_rank8_ci.err; exit 1; }
python -c "import json; d=json.load(open('$o/c4_rank8_ci.json')); print('c4 rank8 ci slowest', d['ms_per_spp_slowest_rank'], 'mean', d['ms_per_spp_mean_rank'], [b['restir_ms_per_spp'] for b in d['bands']])"
