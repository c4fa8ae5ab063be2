# k_chunk_join (frame_begin + G-buffer merge + reservoir merge of a chunk's sample in one pass,
# ab/join): the ReSTIR / C4 parity tests with it, then the C4 rank-of-8 rehearsal base vs join
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r05o; mkdir -p $o
J=$PWD/ab/join/libmpt.so
MPT_LIB_PATH=$J timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_restir.py tests/test_configs.py -k "restir or c4" > $o/pytest_join.log 2>&1 || { tail -30 $o/pytest_join.log; exit 1; }
tail -2 $o/pytest_join.log
for v in base join base join; do
  L=hiprt-path-tracer_amd/mpt/libmpt.so; [ $v = join ] && L=$J
  MPT_LIB_PATH=$(realpath $L) timeout -k 10 300 python -u bench.py --workload c4 --emulate-rank-of 8 --steps 128 > $o/c4_rank8_$v.json 2> $o/c4_rank8_$v.err || { tail -20 $o/c4_rank8_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$o/c4_rank8_$v.json')); print('$v slowest', d['ms_per_spp_slowest_rank'], 'mean', d['ms_per_spp_mean_rank'])"
done
