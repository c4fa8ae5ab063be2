cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05a
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_low_res.py tests/test_adaptive.py tests/test_gpu_parity.py tests/test_restir.py tests/test_host_cpp.py tests/test_configs.py -k "low_res or partition or halo or aux or cpp or display_nans or adaptive" > gpurun_out/r05a/pytest.log 2>&1 || { tail -40 gpurun_out/r05a/pytest.log; exit 1; }
tail -3 gpurun_out/r05a/pytest.log
timeout -k 10 600 python -u bench.py --workload c4 --emulate-rank-of 8 --steps 32 > gpurun_out/r05a/c4_rank8.json 2> gpurun_out/r05a/c4_rank8.err || { tail -20 gpurun_out/r05a/c4_rank8.err; exit 1; }
tail -c 600 gpurun_out/r05a/c4_rank8.json
