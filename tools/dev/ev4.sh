set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/g5
timeout -k 10 600 python -u -m pytest tests/test_configs.py -k c3t -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/g5/pytest.log 2>&1
rc=$?; echo "pytest c3t rc $rc"; tail -n 3 gpurun_out/g5/pytest.log
[ $rc -le 1 ] || exit $rc
bash tools/gpu_evidence.sh r04b c3t "--steps 16 --warmup 4" "--steps 64 --cpu-seconds 10" || exit $?
