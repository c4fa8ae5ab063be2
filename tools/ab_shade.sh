# GPU parity of the shading paths at the current library, then an alternating A/B of libmpt variants
# (gpurun: bash tools/ab_shade.sh <tag> "<pytest -k expr>" <variant>... [-- bench args])
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/$1; mkdir -p $o; k=$2; shift 2
if [ -n "$k" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests -k "$k" > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
  tail -2 $o/pytest.log
fi
timeout -k 10 900 python -u tools/bench_variants.py "$@" > $o/ab.jsonl 2> $o/ab.err || { tail -20 $o/ab.err; exit 1; }
python -c "
import json
for l in open('$o/ab.jsonl'):
    d = json.loads(l); k = d['kernels']
    print(d['lib'][-40:], d['ms_per_step'], 'shade', k['shade'], 'path', k['trace_path'], 'any', k['trace_nee_any'], 'restir', k['restir'])"
