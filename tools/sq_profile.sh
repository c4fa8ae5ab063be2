#!/bin/bash
# SQ counter pass (issue / wait breakdown per kernel) of the bench command; runs on the GPU box.
# usage: tools/sq_profile.sh <tag> [bench args...]
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/sq_$tag
mkdir -p $out
args="$* --no-cpu-baseline"
i=0
for pmc in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_VMEM" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc --kernel-trace -d $out/p$i -o run --output-format csv -- python3 bench.py $args > $out/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i failed rc=$rc"; tail -5 $out/p$i.log; case $rc in 124|137|134|139) exit $rc;; esac; fi
done
echo done
