# C4 rank-of-8 band timings at the driver's 20 steps against the samples per batch (gpurun:
# bash tools/ab_c4_band_batch.sh <tag> <band> "<batches>"); outputs under gpurun_out/<tag>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/$1; band=$2; mkdir -p $o
for b in $3; do
  timeout -k 10 300 python -u bench.py --workload c4 --emulate-rank-of 8 --emulate-band $band --steps 20 --batch $b > $o/b$b.json 2> $o/b$b.err || { tail -20 $o/b$b.err; exit 1; }
  python -c "import json; d=json.load(open('$o/b$b.json')); x=d['bands'][0]; print('batch $b', x['ms_per_spp'], 'restir', x['restir_ms_per_spp'])"
done
