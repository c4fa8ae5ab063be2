# A/B of libmpt variants (tools/bench_variants.py): bench.py per variant, alternating
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python tools/bench_variants.py "$@" -- --no-parity > gpurun_out/ab/ab.log 2>&1
rc=$?; echo "ab rc $rc"; cut -c1-1200 gpurun_out/ab/ab.log
