set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/g11
L=hiprt-path-tracer_amd/mpt/libmpt.so
timeout -k 10 400 python tools/bench_variants.py abv/base/libmpt.so $L abv/base/libmpt.so $L -- --no-parity --workload c3t > gpurun_out/g11/ab_c3t.log 2>&1
echo "ab c3t rc $?"
timeout -k 10 400 python tools/bench_variants.py abv/base/libmpt.so $L abv/base/libmpt.so $L -- --no-parity > gpurun_out/g11/ab_c3.log 2>&1
echo "ab c3 rc $?"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_lobes.py tests/test_shade_classes.py tests/test_gltf_textures.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g11/pytest.log 2>&1
echo "pytest rc $?"; tail -n 2 gpurun_out/g11/pytest.log
