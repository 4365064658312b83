#!/bin/bash
# Round 4 final artifacts from one box: smoke, the default bench line (C2 bf16, CPU baseline, Vocos), C2 fp16,
# C1/C3/C4/C5 lines (CPU baselines, extrapolated where BASELINE.md §3 says so), and the rocprofv3 kernel
# trace + stats of the default bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${R04_OUT:-r04final}; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 240 python __graft_entry__.py smoke > $O/smoke.log 2>&1 && echo "smoke ok" || exit 1
timeout -k 10 500 python bench.py > $O/bench_c2.log 2>&1 && echo "c2 ok" || exit 1
timeout -k 10 500 python bench.py --compute fp16 > $O/bench_c2_fp16.log 2>&1 && echo "c2 fp16 ok" || exit 1
for c in c1 c3 c4 c5; do
  timeout -k 10 600 python bench.py --config $c > $O/bench_$c.log 2>&1 && echo "$c ok" || exit 1
done
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py \
  --no-cpu-baseline > $O/trace.log 2>&1 && echo "trace ok" || exit 1
for f in $O/bench_*.log; do
  echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], d["value"], r["kernel"], r["frac"], r.get("rocprof_frac"), (d.get("cpu_baseline") or {}).get("value"))')"
done
