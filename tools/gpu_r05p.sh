# the final build again (k_chunk_join): GPU suite, smoke, default bench, C4 rank-of-8; then the
# whole 1080p C4 frame with chunks of 2 / 4 against one sample at a time
bash tools/gpu_suite.sh r05p || exit 1
o=gpurun_out/r05p
L=hiprt-path-tracer_amd/mpt/libmpt.so
timeout -k 10 400 python tools/bench_variants.py $L@MPT_RESTIR_CHUNK=1 $L@MPT_RESTIR_CHUNK=2 $L@MPT_RESTIR_CHUNK=4 $L@MPT_RESTIR_CHUNK=1 $L@MPT_RESTIR_CHUNK=2 $L@MPT_RESTIR_CHUNK=4 -- --workload c4 --steps 32 > $o/c4_chunk_ab.jsonl 2> $o/c4_chunk_ab.err || { tail -20 $o/c4_chunk_ab.err; exit 1; }
python -c "
import json
for l in open('$o/c4_chunk_ab.jsonl'):
    j = json.loads(l); k = j['kernels']; print(j['lib'].split('@')[-1], j['ms_per_step'], 'restir', k.get('restir'), k.get('restir_kernels'))"
