#!/bin/bash
# Measurement batch on the GPU box (gpurun): optional GPU tests, the C3 bench for the in-tree
# libmpt and every build_variants/<name>/libmpt.so (A/B), then separate rocprofv3 --pmc passes
# (SQ issue / wait, f64 VALU mix, texture-address / L1 counters) of the in-tree build.
# usage: tools/gpu_probe.sh <tag> [tests] [pmc] [-- bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
tests=0; pmc=0
while [ $# -gt 0 ] && [ "$1" != "--" ]; do
  case $1 in tests) tests=1;; pmc) pmc=1;; esac; shift
done
[ "$1" == "--" ] && shift
bargs="--steps 32 --warmup 2 --no-cpu-baseline --no-parity $*"
out=gpurun_out/$tag
mkdir -p $out
fail() { echo "$1 failed rc=$2"; tail -20 "$3"; exit $2; }
if [ $tests == 1 ]; then
  echo "== pytest -m gpu"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || fail pytest $? $out/pytest.log
  tail -3 $out/pytest.log
fi
echo "== bench (in-tree)"
timeout -k 10 300 python3 bench.py $bargs > $out/bench.json 2> $out/bench.err || fail bench $? $out/bench.err
for v in build_variants/*/libmpt.so; do
  [ -f "$v" ] || continue
  n=$(basename $(dirname $v))
  echo "== bench $n"
  timeout -k 10 300 env MPT_LIB_PATH=$PWD/$v python3 bench.py $bargs > $out/bench_$n.json 2> $out/bench_$n.err || fail "bench $n" $? $out/bench_$n.err
done
if [ $pmc == 1 ]; then
  i=0
  for c in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VMEM" \
           "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_FLAT SQ_LDS_BANK_CONFLICT"; do
    i=$((i+1))
    echo "== pmc $i"
    timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace -d $out/pmc$i -o run --output-format csv -- python3 bench.py $bargs > $out/pmc$i.log 2>&1 || fail "pmc $i" $? $out/pmc$i.log
  done
fi
echo done
