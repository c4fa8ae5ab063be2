set -o pipefail
mkdir -p gpurun_out/g3
export MPT_LIB_PATH=$PWD/abv/ntA.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_light_samples.py tests/test_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g3/pytest.log 2>&1
rc=$?; echo "pytest(ntA) rc $rc"; tail -n 3 gpurun_out/g3/pytest.log
[ $rc -le 1 ] || exit $rc
unset MPT_LIB_PATH
bash tools/dev/ab.sh abv/base.so abv/ntA.so abv/ntB.so abv/rich.so abv/base.so abv/ntA.so abv/ntB.so abv/rich.so
