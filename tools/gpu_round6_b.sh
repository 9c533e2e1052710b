#!/bin/bash
# Round-6 evidence, call B: the detector's per-layer profile of this build (tools/gpu_det_profile.sh,
# TAG=r06, no C4 trace), then -- with this call's PMC tables placed where bench.py looks for them
# (profiles/r06/, in the box's copy of the tree) -- the bench lines of every config and the serving
# latencies, each carrying this build's figures.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
DET=1 C4=0 TAG=r06 timeout -k 10 600 tools/gpu_det_profile.sh > gpurun_out/r06_det.log 2>&1 || { tail -20 gpurun_out/r06_det.log; exit 3; }
tail -12 gpurun_out/det_r06/det_layers_pmc.txt
mkdir -p profiles/r06
[ -f gpurun_out/prof_r06/layers_pmc.json ] && cp gpurun_out/prof_r06/layers_pmc.json profiles/r06/layers_pmc.json
cp gpurun_out/det_r06/det_layers_pmc.json profiles/r06/c4_layers_pmc.json
for c in c3 c4 c2 c5; do
  timeout -k 10 400 python3 bench.py --config $c > gpurun_out/r06_bench_$c.json 2> gpurun_out/r06_bench_$c.err || exit 3
  python3 -c "import json;d=json.load(open('gpurun_out/r06_bench_$c.json'));r=d['roofline'];print('$c', d['value'], d['ms_per_step'], r['frac'], r.get('traffic'), (r.get('detector') or {}).get('frac'), (r.get('detector') or {}).get('traffic'))"
done
timeout -k 10 400 python3 -u tools/serve_latency.py --json gpurun_out/r06_serve_latency.json > gpurun_out/r06_serve_latency.txt 2>&1 || exit 3
tail -6 gpurun_out/r06_serve_latency.txt
