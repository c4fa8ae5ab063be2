cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r05a; mkdir -p $o
timeout -k 10 480 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_low_res.py tests/test_adaptive.py tests/test_gpu_parity.py tests/test_restir.py tests/test_host_cpp.py tests/test_configs.py -k "low_res or partition or halo or aux or cpp or display_nans or adaptive or c3t" > $o/pytest.log 2>&1; rc=$?
tail -3 $o/pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
L=hiprt-path-tracer_amd/mpt/libmpt.so
timeout -k 10 200 python -u tools/bench_variants.py $L@MPT_MAT_PRIVATE=1 $L@MPT_MAT_PRIVATE=0 -- --workload c3t > $o/ab_c3t.jsonl 2>&1 || { tail -20 $o/ab_c3t.jsonl; exit 1; }
cut -c1-220 $o/ab_c3t.jsonl
timeout -k 10 300 python -u bench.py --workload c4 --emulate-rank-of 8 --steps 128 > $o/c4_rank8.json 2> $o/c4_rank8.err || { tail -20 $o/c4_rank8.err; exit 1; }
python -c "import json; d=json.load(open('$o/c4_rank8.json')); print('c4 rank8 slowest', d['ms_per_spp_slowest_rank'], 'mean', d['ms_per_spp_mean_rank'])"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $o/bench_default.json 2> $o/bench_default.err || { tail -20 $o/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('$o/bench_default.json')); print(d['value'], d['ms_per_step'], d.get('batch1')); [print(c.get('workload','')[:40], c.get('value'), c.get('ms_per_step'), c.get('error')) for c in d.get('configs', [])]"
