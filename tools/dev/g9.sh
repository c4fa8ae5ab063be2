# full GPU suite after the texture-decided plain class + stages; A/B of the routing on C3T
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/g9
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g9/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -n 5 gpurun_out/g9/pytest.log; [ $rc -eq 0 ] || exit $rc
L=hiprt-path-tracer_amd/mpt/libmpt.so
timeout -k 10 500 python tools/bench_variants.py $L@MPT_SHADE_TEXMETAL=0 $L@MPT_SHADE_TEXMETAL=1 -- --no-parity --workload c3t > gpurun_out/g9/ab.log 2>&1
rc=$?; echo "ab rc $rc"; cut -c1-700 gpurun_out/g9/ab.log
