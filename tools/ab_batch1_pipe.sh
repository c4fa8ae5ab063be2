# Batch-1 C3 (bench.py batch1) for row-part settings (gpurun: bash tools/ab_batch1_pipe.sh <tag> "<parts:pipe> ...")
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/$1; mkdir -p $o
i=0
for v in $2; do
  i=$((i+1)); parts=${v%:*}; pipe=${v#*:}
  MPT_PIX_PARTS=$parts MPT_PIX_PIPE=$pipe timeout -k 10 300 python -u bench.py --steps 16 --no-cpu-baseline --no-parity --no-solo --configs none --batch1-steps 16 > $o/r$i.json 2> $o/r$i.err || { tail -20 $o/r$i.err; exit 1; }
  python -c "import json; d=json.load(open('$o/r$i.json')); print('parts $parts pipe $pipe', d['batch1']['ms_per_step'], d['ms_per_step'])"
done
