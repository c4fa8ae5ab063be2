# Packed-FMA / v_bfm node test (ab/pk, -DMPT_TRAV_PK): parity with the variant, the graph test
# with its replay counters, then base vs pk on C3, C5 and C3T (alternating, two runs each)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r05f; mkdir -p $o
MPT_LIB_PATH=$PWD/ab/pk/libmpt.so timeout -k 10 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_restir.py tests/test_alpha.py -k "not c4 and not c5" > $o/pytest_pk.log 2>&1 || { tail -30 $o/pytest_pk.log; exit 1; }
tail -2 $o/pytest_pk.log
timeout -k 10 200 python -u -m pytest -q -x --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py -k graph > $o/pytest_graph.log 2>&1 || { tail -30 $o/pytest_graph.log; exit 1; }
tail -1 $o/pytest_graph.log
B=hiprt-path-tracer_amd/mpt/libmpt.so; P=ab/pk/libmpt.so
timeout -k 10 300 python tools/bench_variants.py $B $P $B $P > $o/c3.jsonl 2> $o/c3.err || { tail -20 $o/c3.err; exit 1; }
timeout -k 10 300 python tools/bench_variants.py $B $P $B $P -- --workload c5 --steps 64 > $o/c5.jsonl 2> $o/c5.err || { tail -20 $o/c5.err; exit 1; }
timeout -k 10 300 python tools/bench_variants.py $B $P $B $P -- --workload c3t > $o/c3t.jsonl 2> $o/c3t.err || { tail -20 $o/c3t.err; exit 1; }
timeout -k 10 200 python -u bench.py --steps 16 --warmup 2 --configs none --no-parity --no-cpu-baseline --batch1-steps 16 > $o/c3_batch1.json 2> $o/c3_batch1.err || { tail -20 $o/c3_batch1.err; exit 1; }
for w in c3 c5 c3t; do python -c "
import json
for l in open('$o/$w.jsonl'):
    j = json.loads(l); k = j['kernels']
    print('$w', j['lib'].split('/')[-2], j['ms_per_step'], 'trace', k['trace_path'], k['trace_nee_any'], k['trace_nee_closest'])"; done
python -c "import json; print(json.load(open('$o/c3_batch1.json'))['batch1'])"
bash tools/gpu_r05g.sh
