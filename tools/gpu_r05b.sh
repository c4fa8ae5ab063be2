# A/B on the GPU box: private-memory resolved materials (default build) vs the per-slot global
# copy (ab/matslot), C3 and C3T; the C4 rank-of-8 rehearsal at 128 / 32 samples per batch; the
# default bench line (C3 headline + the other configs)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r05b; mkdir -p $o
L=hiprt-path-tracer_amd/mpt/libmpt.so
timeout -k 10 400 python -u tools/bench_variants.py $L ab/matslot/libmpt.so $L ab/matslot/libmpt.so -- --workload c3 > $o/ab_c3.jsonl 2>&1 || { tail -20 $o/ab_c3.jsonl; exit 1; }
timeout -k 10 400 python -u tools/bench_variants.py $L ab/matslot/libmpt.so $L ab/matslot/libmpt.so -- --workload c3t > $o/ab_c3t.jsonl 2>&1 || { tail -20 $o/ab_c3t.jsonl; exit 1; }
cut -c1-200 $o/ab_c3.jsonl $o/ab_c3t.jsonl
timeout -k 10 600 python -u bench.py --workload c4 --emulate-rank-of 8 --steps 32 > $o/c4_rank8_b128.json 2> $o/c4_rank8_b128.err || { tail -20 $o/c4_rank8_b128.err; exit 1; }
MPT_RESTIR_MAX_BATCH=32 timeout -k 10 600 python -u bench.py --workload c4 --emulate-rank-of 8 --steps 32 > $o/c4_rank8_b32.json 2> $o/c4_rank8_b32.err || { tail -20 $o/c4_rank8_b32.err; exit 1; }
python -c "import json; [print(f, json.load(open('$o/'+f))['ms_per_spp_slowest_rank']) for f in ('c4_rank8_b128.json','c4_rank8_b32.json')]"
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $o/bench_default.json 2> $o/bench_default.err || { tail -20 $o/bench_default.err; exit 1; }
tail -c 300 $o/bench_default.json
