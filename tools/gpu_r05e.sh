# HIP-graph replay of one-sample launch sets: parity tests, then batch-1 C3 and 1-spp-per-launch C1
# with graphs on / off
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r05e; mkdir -p $o
timeout -k 10 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_low_res.py tests/test_adaptive.py tests/test_alpha.py tests/test_configs.py -k "not c4 and not c5" > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
for g in 1 0; do
  MPT_GRAPHS=$g timeout -k 10 200 python -u bench.py --steps 16 --warmup 2 --configs none --no-parity --no-cpu-baseline --batch1-steps 16 > $o/c3_graphs$g.json 2> $o/c3_graphs$g.err || { tail -20 $o/c3_graphs$g.err; exit 1; }
  MPT_GRAPHS=$g timeout -k 10 200 python -u bench.py --workload c1 --steps 32 --batch 1 --configs none --no-parity --no-cpu-baseline > $o/c1_graphs$g.json 2> $o/c1_graphs$g.err || { tail -20 $o/c1_graphs$g.err; exit 1; }
  python -c "import json; a=json.load(open('$o/c3_graphs$g.json')); b=json.load(open('$o/c1_graphs$g.json')); print('graphs=$g', 'c3 batch1', a['batch1'], 'c1 1spp/launch ms', b['ms_per_step'])"
done
