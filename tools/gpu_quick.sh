# New / changed GPU tests, then the driver's default bench (gpurun: bash tools/gpu_quick.sh <tag> [pytest -k expr])
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/${1:-quick}; mkdir -p $o
k=${2:-halo_native or overlapped_batch_then or graph_captured_once}
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests -k "$k" > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
[ -n "$3" ] && exit 0
timeout -k 10 400 python -u bench.py > $o/bench_default.json 2> $o/bench_default.err || { tail -20 $o/bench_default.err; exit 1; }
python -c "
import json; d = json.load(open('$o/bench_default.json'))
print('c3', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('batch1', {}).get('ms_per_spp'))
print(json.dumps(d['kernel_ms_per_step']))
for c in d.get('configs', []): print(c['workload'][:3], c.get('value'), c.get('ms_per_step'), c.get('parity_vs_oracle', {}).get('bit_exact'))"
