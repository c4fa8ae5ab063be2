# Batch-1 and batched C3 against the HIP runtime's hardware queues per process and the row-part
# settings (gpurun: bash tools/ab_hwq.sh <tag> "<queues>:<parts>:<pix_pipe> ...")
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/$1; mkdir -p $o
i=0
for v in $2; do
  i=$((i+1)); q=${v%%:*}; rest=${v#*:}; parts=${rest%:*}; pipe=${rest#*:}
  GPU_MAX_HW_QUEUES=$q MPT_PIX_PARTS=$parts MPT_PIX_PIPE=$pipe timeout -k 10 300 python -u bench.py --steps 32 --no-cpu-baseline --no-parity --no-solo --configs none --batch1-steps 16 > $o/r$i.json 2> $o/r$i.err || { tail -20 $o/r$i.err; exit 1; }
  python -c "import json; d=json.load(open('$o/r$i.json')); print('queues $q parts $parts pipe $pipe', d['batch1']['ms_per_step'], d['ms_per_step'])"
done
