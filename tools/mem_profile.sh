#!/bin/bash
# Memory-pipeline counter passes (TA / vL1D / UTCL1 / L2) of the bench command; runs on the GPU box.
# usage: tools/mem_profile.sh <tag> [bench args...]
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/mem_$tag
mkdir -p $out
args="$* --no-cpu-baseline"
i=0
for pmc in "GRBM_GUI_ACTIVE TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum" \
           "TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum" \
           "TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_UTCL1_REQUEST_sum TCP_PENDING_STALL_CYCLES_sum" \
           "TA_FLAT_READ_WAVEFRONTS_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCC_TAG_STALL_sum"; do
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --pmc $pmc --kernel-trace -d $out/p$i -o run --output-format csv -- python3 bench.py $args > $out/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i failed rc=$rc"; tail -5 $out/p$i.log; exit $rc; fi
done
echo done
