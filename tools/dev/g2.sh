set -o pipefail
mkdir -p gpurun_out/g2
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_light_samples.py tests/test_configs.py tests/test_shade_classes.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g2/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -n 15 gpurun_out/g2/pytest.log
[ $rc -le 1 ] || exit $rc
bash tools/dev/ab.sh abv/base.so abv/pf.so abv/base.so abv/pf.so
