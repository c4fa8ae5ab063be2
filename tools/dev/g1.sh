set -o pipefail
mkdir -p gpurun_out/g1
timeout -k 10 300 python -u -m pytest tests/test_gather.py tests/test_host_cpp.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/g1/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -n 25 gpurun_out/g1/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 500 python tools/bench_variants.py abv/base.so abv/ub.so abv/base.so abv/ub.so -- --no-parity > gpurun_out/g1/ab.log 2>&1
rc=$?; echo "ab rc $rc"; cut -c1-900 gpurun_out/g1/ab.log
