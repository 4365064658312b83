#!/bin/bash
# Round 4, box y: the C3/C4/C5 bench lines again (CPU baselines included) now that per-class PMC traffic
# summaries exist at those shapes (tools/r04_gpu_x.sh), so each line carries traffic beside its roofline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/r04y; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
for c in c3 c4 c5; do
  timeout -k 10 600 python bench.py --config $c > $O/bench_$c.log 2>&1 && echo "$c ok" || exit 1
done
for f in $O/bench_*.log; do
  echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], d["value"], r["kernel"], r["frac"], r.get("traffic_over_algorithmic"), {k: v.get("traffic_over_algorithmic") for k, v in d["roofline_classes"].items()})')"
done
