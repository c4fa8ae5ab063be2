# f32 transcendentals (ab/f32, -DMPT_TMATH_F32) and packed node test + f32 (ab/pkf32): the
# device functions against libm-derived expectations are checked on the CPU; here C3 / C3T / C5
# per-kernel times, base vs variants, alternating
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r05g; mkdir -p $o
B=hiprt-path-tracer_amd/mpt/libmpt.so; F=ab/f32/libmpt.so; PF=ab/pkf32/libmpt.so
timeout -k 10 300 python tools/bench_variants.py $B $F $PF $B $F $PF > $o/c3.jsonl 2> $o/c3.err || { tail -20 $o/c3.err; exit 1; }
timeout -k 10 300 python tools/bench_variants.py $B $F $PF -- --workload c3t > $o/c3t.jsonl 2> $o/c3t.err || { tail -20 $o/c3t.err; exit 1; }
for w in c3 c3t; do python -c "
import json
for l in open('$o/$w.jsonl'):
    j = json.loads(l); k = j['kernels']
    print('$w', j['lib'].split('/')[-2], j['ms_per_step'], 'shade', k['shade'], k['shade_generic'], 'trace', k['trace_path'], k['trace_nee_any'], k['trace_nee_closest'])"; done
