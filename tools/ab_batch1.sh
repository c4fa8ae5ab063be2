# batch-1 (one sample per wavefront) C3 timing with and without the row halves (gpurun: bash tools/ab_batch1.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/$1; mkdir -p $o
for v in ${PARTS:-0 2 3 4 0 2 3 4}; do
  MPT_PIX_PARTS=$v timeout -k 10 300 python -u bench.py --steps 16 --warmup 2 --no-cpu-baseline --no-parity --configs none --batch1-steps 16 > $o/b1_$v.json 2> $o/b1_$v.err || { tail -20 $o/b1_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$o/b1_$v.json')); print('pix_parts', $v, 'batched', d['ms_per_step'], 'batch1', d['batch1'])"
done
