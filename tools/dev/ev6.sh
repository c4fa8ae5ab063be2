# round-4 final evidence, part 1: C4 and C3T (profiles + PMC + bench line)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_evidence.sh r04c c4 "--steps 16 --warmup 4" "--steps 64 --cpu-seconds 10 --parity-seconds 60" || exit $?
bash tools/gpu_evidence.sh r04c c3t "--steps 16 --warmup 4" "--steps 64 --cpu-seconds 10" || exit $?
