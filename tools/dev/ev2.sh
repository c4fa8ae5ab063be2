set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_evidence.sh r04b c2 "--steps 16 --warmup 4" "--steps 64 --cpu-seconds 10" || exit $?
bash tools/gpu_evidence.sh r04b c5 "--steps 8 --warmup 2" "--steps 64 --cpu-seconds 10" || exit $?
