set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c4probe
timeout -k 10 300 python tools/bench_variants.py hiprt-path-tracer_amd/mpt/libmpt.so ab/notrace/libmpt.so -- --workload c4 --no-parity > gpurun_out/c4probe/variants.txt 2>&1 || exit 1
cat gpurun_out/c4probe/variants.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c4probe/trace -o run --output-format csv -- python3 bench.py --workload c4 --steps 8 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/c4probe/trace.log 2>&1 || exit 1
echo done
