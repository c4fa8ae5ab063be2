set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/g10
timeout -k 10 500 python tools/bench_variants.py abv/base/libmpt.so abv/noslot/libmpt.so abv/base/libmpt.so abv/noslot/libmpt.so -- --no-parity --workload c3t > gpurun_out/g10/ab.log 2>&1
echo "ab rc $?"
