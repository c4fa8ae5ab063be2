set -o pipefail
mkdir -p gpurun_out/g4
export MPT_LIB_PATH=$PWD/abv/ntC.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_light_samples.py tests/test_configs.py tests/test_restir.py tests/test_lobes.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g4/pytest.log 2>&1
rc=$?; echo "pytest(ntC) rc $rc"; tail -n 3 gpurun_out/g4/pytest.log
[ $rc -le 1 ] || exit $rc
unset MPT_LIB_PATH
bash tools/dev/ab.sh abv/base.so abv/ntA.so abv/ntC.so abv/base.so abv/ntA.so abv/ntC.so
