# plain-class shading stages: parity under each split, then A/B against the one-kernel shading
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/g7
T="tests/test_gpu_parity.py tests/test_configs.py tests/test_lobes.py tests/test_gltf_textures.py tests/test_restir.py tests/test_light_samples.py tests/test_adaptive.py"
MPT_SHADE_SPLIT=1 timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g7/split1.log 2>&1
rc=$?; echo "split1 rc $rc"; tail -n 3 gpurun_out/g7/split1.log; [ $rc -eq 0 ] || exit $rc
MPT_SHADE_SPLIT=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py tests/test_gltf_textures.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g7/split2.log 2>&1
rc=$?; echo "split2 rc $rc"; tail -n 3 gpurun_out/g7/split2.log; [ $rc -eq 0 ] || exit $rc
MPT_SHADE_SPLIT=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py tests/test_gltf_textures.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g7/split3.log 2>&1
rc=$?; echo "split3 rc $rc"; tail -n 3 gpurun_out/g7/split3.log; [ $rc -eq 0 ] || exit $rc
L=hiprt-path-tracer_amd/mpt/libmpt.so
timeout -k 10 500 python tools/bench_variants.py $L $L@MPT_SHADE_SPLIT=1 $L@MPT_SHADE_SPLIT=2 $L@MPT_SHADE_SPLIT=3 abv/late2/libmpt.so@MPT_SHADE_SPLIT=1 $L -- --no-parity > gpurun_out/g7/ab.log 2>&1
rc=$?; echo "ab rc $rc"; cut -c1-900 gpurun_out/g7/ab.log
