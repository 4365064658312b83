#!/bin/bash
# Round-end bench lines on one box: C1..C5 (bf16) and C2 fp16, each with its CPU baseline and the Vocos timing,
# as `python bench.py --config cN` prints them (the driver's default run is C2). Output: gpurun_out/$OUT.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-bench_all}; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
for c in ${CONFIGS:-c1 c2 c3 c4 c5}; do
  case $c in c1|c2) ST="";; *) ST="--steps 3 --warmup 1";; esac
  timeout -k 10 900 python bench.py --config $c $ST > $O/bench_$c.log 2>&1 || { echo "bench $c failed"; exit 1; }
  echo "$c $(tail -1 $O/bench_$c.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], d["value"], r["kernel"], r["frac"], d["cpu_baseline"]["value"] if d.get("cpu_baseline") else None)')"
done
if [ "${FP16:-1}" = 1 ]; then
  timeout -k 10 900 python bench.py --config c2 --compute fp16 > $O/bench_c2_fp16.log 2>&1 || { echo "bench c2 fp16 failed"; exit 1; }
  echo "c2 fp16 $(tail -1 $O/bench_c2_fp16.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
fi
