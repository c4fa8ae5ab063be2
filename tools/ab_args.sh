# Alternating A/B of bench argument sets (gpurun: bash tools/ab_args.sh <tag> "<args 1>" "<args 2>" ...)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/$1; shift; mkdir -p $o
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-parity --configs none --batch1-steps 0 $args > $o/run_$i.json 2> $o/run_$i.err || { tail -20 $o/run_$i.err; exit 1; }
  python -c "
import json; d=json.load(open('$o/run_$i.json'))
print('[$args]', d['ms_per_step'], d['value'], d.get('samples_per_launch'))"
done
