# C3 rank-of-8 rehearsals (64 steps, and the driver's 20 against the whole frame at 20), then the
# C4 small-band A/B of monolithic reuse passes
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r05l; mkdir -p $o
timeout -k 10 300 python -u bench.py --emulate-rank-of 8 --steps 64 > $o/c3_rank8.json 2> $o/c3_rank8.err || { tail -20 $o/c3_rank8.err; exit 1; }
tail -c 300 $o/c3_rank8.json
timeout -k 10 300 python -u bench.py --emulate-rank-of 8 --steps 20 > $o/c3_rank8_s20.json 2> $o/c3_rank8_s20.err || { tail -20 $o/c3_rank8_s20.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --configs none --no-parity --no-cpu-baseline > $o/c3_s20.json 2> $o/c3_s20.err || { tail -20 $o/c3_s20.err; exit 1; }
python -c "
import json
a = json.load(open('$o/c3_rank8_s20.json')); b = json.load(open('$o/c3_s20.json'))
print('c3 steps 20: whole', b['ms_per_step'], 'rank-of-8', a['ms_per_step'], 'ratio', b['ms_per_step'] / a['ms_per_step'])"
# the reuse passes monolithic on a small band (the initial pass staged and chunked)
for m in 0 1; do
  MPT_RESTIR_MONO_REUSE=$m timeout -k 10 300 python -u bench.py --workload c4 --emulate-rank-of 8 --steps 128 > $o/c4_rank8_mono$m.json 2> $o/c4_rank8_mono$m.err || { tail -20 $o/c4_rank8_mono$m.err; exit 1; }
  python -c "import json; d=json.load(open('$o/c4_rank8_mono$m.json')); print('c4 rank8 mono_reuse=$m slowest', d['ms_per_spp_slowest_rank'], 'mean', d['ms_per_spp_mean_rank'])"
done
bash tools/gpu_r05m.sh
