set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/g6
timeout -k 10 900 python -u -m pytest tests/test_restir.py tests/test_configs.py tests/test_host_cpp.py tests/test_gather.py -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/g6/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -n 3 gpurun_out/g6/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 900 python tools/bench_variants.py abv/vs_split.so abv/aos.so abv/vs_split.so abv/aos.so -- --workload c4 --steps 16 --no-parity > gpurun_out/g6/ab_c4.log 2>&1
echo "ab rc $?"; cut -c1-600 gpurun_out/g6/ab_c4.log
