# Alternating A/B of one environment switch on a bench command (gpurun: bash tools/ab_env.sh <tag> <VAR> "<values>" <bench args...>)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/$1; var=$2; vals=$3; shift 3; mkdir -p $o
i=0
for v in $vals; do
  i=$((i+1))
  env $var=$v timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-parity --configs none --batch1-steps 0 "$@" > $o/ab_${i}_$v.json 2> $o/ab_${i}_$v.err || { tail -20 $o/ab_${i}_$v.err; exit 1; }
  python -c "
import json; d=json.load(open('$o/ab_${i}_$v.json'))
if 'ms_per_spp_slowest_rank' in d: print('$var=$v', 'slowest', d['ms_per_spp_slowest_rank'], 'mean', d['ms_per_spp_mean_rank'], [b['ms_per_spp'] for b in d['bands']], 'restir', [b['restir_ms_per_spp'] for b in d['bands']])
else: print('$var=$v', d['ms_per_step'], 'restir', d['kernel_ms_per_step']['restir'], d['kernel_ms_per_step']['restir_kernels'])"
done
