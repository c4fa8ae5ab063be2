# round-4 final evidence, part 2: C2, C5, C1
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_evidence.sh r04c c2 "--steps 16 --warmup 4" "--steps 64 --cpu-seconds 10" || exit $?
bash tools/gpu_evidence.sh r04c c5 "--steps 8 --warmup 2" "--steps 64 --cpu-seconds 10" || exit $?
bash tools/gpu_evidence.sh r04c c1 "" "" || exit $?
