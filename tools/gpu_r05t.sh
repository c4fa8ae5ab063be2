# overlapped halves on one rank of a 2- / 4-way C3 split at the driver's 20 steps (10-21 M paths per
# wavefront), each A/B pair twice
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r05t; mkdir -p $o
for r in 2 4; do
  for v in 0 1 0 1; do
    MPT_OVERLAP=$v timeout -k 10 300 python -u bench.py --emulate-rank-of $r --steps 20 --no-parity --no-cpu-baseline --configs none --batch1-steps 0 > $o/r${r}_ov$v.json 2> $o/r${r}_ov$v.err || { tail -20 $o/r${r}_ov$v.err; exit 1; }
    python -c "import json; print('rank of $r overlap=$v', json.load(open('$o/r${r}_ov$v.json'))['ms_per_step'])"
  done
done
