# the whole GPU suite and smoke; then (only if both are clean) the C4 overlap A/B and the C4
# rank-of-8 rehearsal at 128 and 32 samples per batch
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r05d; mkdir -p $o
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -5 $o/smoke.log; exit 1; }
cat $o/smoke.log
L=hiprt-path-tracer_amd/mpt/libmpt.so
timeout -k 10 300 python -u tools/bench_variants.py $L@MPT_RESTIR_OVERLAP=1 $L@MPT_RESTIR_OVERLAP=0 -- --workload c4 --steps 32 > $o/ab_c4_overlap.jsonl 2>&1 || { tail -20 $o/ab_c4_overlap.jsonl; exit 1; }
cut -c1-200 $o/ab_c4_overlap.jsonl
timeout -k 10 300 python -u bench.py --workload c4 --emulate-rank-of 8 --steps 128 > $o/c4_rank8.json 2> $o/c4_rank8.err || { tail -20 $o/c4_rank8.err; exit 1; }
python -c "import json; d=json.load(open('$o/c4_rank8.json')); print('c4 rank8 b128 slowest', d['ms_per_spp_slowest_rank'], 'mean', d['ms_per_spp_mean_rank'])"
timeout -k 10 300 python -u bench.py --workload c4 --emulate-rank-of 8 --steps 128 --batch 32 > $o/c4_rank8_b32.json 2> $o/c4_rank8_b32.err || { tail -20 $o/c4_rank8_b32.err; exit 1; }
python -c "import json; d=json.load(open('$o/c4_rank8_b32.json')); print('c4 rank8 b32 slowest', d['ms_per_spp_slowest_rank'], 'mean', d['ms_per_spp_mean_rank'])"
