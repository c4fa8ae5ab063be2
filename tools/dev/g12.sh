set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/g12
L=hiprt-path-tracer_amd/mpt/libmpt.so
timeout -k 10 600 python tools/bench_variants.py abv/base/libmpt.so $L abv/base/libmpt.so $L -- --no-parity --workload c4 > gpurun_out/g12/ab_c4.log 2>&1
echo "ab c4 rc $?"
timeout -k 10 500 python -u -m pytest tests/test_restir.py tests/test_configs.py -k "restir or c4 or C4" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g12/pytest.log 2>&1
echo "pytest rc $?"; tail -n 2 gpurun_out/g12/pytest.log
