# stage tests + C3T parity + C3T evidence
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/g8
timeout -k 10 400 python -u -m pytest tests/test_shade_classes.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/g8/stages.log 2>&1
rc=$?; echo "stages rc $rc"; tail -n 3 gpurun_out/g8/stages.log; [ $rc -eq 0 ] || exit $rc
bash tools/dev/ev4.sh
