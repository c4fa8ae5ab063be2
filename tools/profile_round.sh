#!/bin/bash
# Runs on the GPU box (gpurun): kernel-trace stats of the bench command, then separate
# PMC passes (counters never combined with other trace domains), for tools/pmc_traffic.py.
# usage: tools/profile_round.sh <tag> [bench args...]
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/prof_$tag
mkdir -p $out
args="$* --no-cpu-baseline --no-parity --no-solo --configs none --batch1-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 bench.py $args > $out/trace.log 2>&1 || exit $?
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc --kernel-trace -d $out/pmc$i -o run --output-format csv -- python3 bench.py $args > $out/pmc$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "pmc pass $i ($pmc) failed rc=$rc"; tail -5 $out/pmc$i.log
    case $rc in 124|137|134|139) exit $rc;; esac
  fi
done
echo done
