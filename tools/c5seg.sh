cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for c in c5 c5d; do for s in ${SEGS:-1024 2048 4096 8192}; do
  timeout -k 10 120 python3 bench.py --config $c --no-cpu-baseline --segments $s > gpurun_out/seg_${c}_$s.json 2>gpurun_out/seg.err || { tail -5 gpurun_out/seg.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/seg_${c}_$s.json').read().strip().splitlines()[-1]); print('$c', $s, round(d['ms_per_step'],4), {k:(v['launches'],round(v['avg_ms'],4)) for k,v in d['kernels'].items()})"
done; done
