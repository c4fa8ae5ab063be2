# whole-frame C4 in chunks of 4 (default) vs 8 vs 12; C5 with overlapped halves forced on
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r05v; mkdir -p $o
L=hiprt-path-tracer_amd/mpt/libmpt.so
timeout -k 10 500 python tools/bench_variants.py $L $L@MPT_RESTIR_CHUNK=8 $L@MPT_RESTIR_CHUNK=12 $L $L@MPT_RESTIR_CHUNK=8 $L@MPT_RESTIR_CHUNK=12 -- --workload c4 --steps 48 > $o/c4_chunk.jsonl 2> $o/c4_chunk.err || { tail -20 $o/c4_chunk.err; exit 1; }
python -c "
import json
for l in open('$o/c4_chunk.jsonl'):
    j = json.loads(l); print(j['lib'].split('@')[-1], j['ms_per_step'])"
timeout -k 10 300 python tools/bench_variants.py $L $L@MPT_OVERLAP=1 $L $L@MPT_OVERLAP=1 -- --workload c5 --steps 16 > $o/c5_ov.jsonl 2> $o/c5_ov.err || { tail -20 $o/c5_ov.err; exit 1; }
python -c "
import json
for l in open('$o/c5_ov.jsonl'):
    j = json.loads(l); print(j['lib'].split('@')[-1], j['ms_per_step'])"
