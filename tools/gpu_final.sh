#!/bin/bash
# Round-end measurement batch on the GPU box (gpurun): GPU tests, smoke, kernel trace + PMC
# passes of the C3 bench, the default C3 bench line, and the other configs' bench lines.
# usage: tools/gpu_final.sh <tag> [a|b]   (a: tests, smoke, profiles, C3; b: the other configs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1
part=${2:-ab}
o=gpurun_out/final_$tag
mkdir -p $o
if [[ $part == *a* ]]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -n 30 $o/pytest_gpu.log; exit 1; }
tail -n 1 $o/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { cat $o/smoke.log; exit 1; }
tail -n 1 $o/smoke.log
bash tools/profile_round.sh $tag --steps 16 --warmup 16 || exit 1
timeout -k 10 400 python bench.py > $o/c3.json 2> $o/c3.err || { tail -n 20 $o/c3.err; exit 1; }
echo c3 && tail -c 300 $o/c3.json
fi
[[ $part == *b* ]] || { echo done; exit 0; }
timeout -k 10 400 python bench.py --workload c2 --cpu-seconds 10 > $o/c2.json 2> $o/c2.err || { tail -n 20 $o/c2.err; exit 1; }
echo c2
timeout -k 10 600 python bench.py --workload c4 --steps 64 --cpu-seconds 10 --parity-seconds 60 > $o/c4.json 2> $o/c4.err || { tail -n 20 $o/c4.err; exit 1; }
echo c4
timeout -k 10 400 python bench.py --workload c5 --steps 64 --cpu-seconds 10 > $o/c5.json 2> $o/c5.err || { tail -n 20 $o/c5.err; exit 1; }
echo c5
timeout -k 10 300 python bench.py --workload c1 > $o/c1.json 2> $o/c1.err || { tail -n 20 $o/c1.err; exit 1; }
echo c1
timeout -k 10 300 python bench.py --emulate-rank-of 8 > $o/c3_rank_of_8.json 2> $o/c3_rank_of_8.err || { tail -n 20 $o/c3_rank_of_8.err; exit 1; }
echo done
