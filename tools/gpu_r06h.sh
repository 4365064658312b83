#!/bin/bash
# LayerNorm fold after the MFMA u/v kernel and the division-free statistics: diagnostic, envelopes, one-box A/B,
# kernel-trace stats of the fold-on bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; O=$PWD/gpurun_out/${OUT:-r06h}; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python tools/diag_fold.py 2>&1 | grep -v amdgpu.ids | tee $O/diag_fold.log || exit 1
F5H_ENVELOPE_LOG=$O/envelopes.jsonl timeout -k 10 400 python -u -m pytest tests/test_gpu_envelope.py -q -rf -s --timeout 200 \
  --timeout-method thread > $O/envelope.log 2>&1; rc=$?
grep -E "envelope|passed|failed|Error" $O/envelope.log | head -30
timeout -k 10 400 python -u tools/ab_c2.py --config c2 --rounds 4 --calls 4 --arms fold0,fold1 > $O/ab_fold_bf16.log 2>&1 || exit 1
grep -v amdgpu $O/ab_fold_bf16.log
cd /tmp && F5H_LNFOLD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fold1 -o run -- python3 $R/bench.py --config c2 --steps 4 --warmup 2 --no-cpu-baseline --no-vocos --probe none > $O/prof_fold1.log 2>&1 || exit 1
f=$(find $O/prof_fold1 -name '*kernel_stats.csv' | head -1); python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print("total kernel ms", sum(float(r["TotalDurationNs"]) for r in rows) / 1e6)
for r in rows[:12]:
    print(f'{r["Name"][:90]:90s} {r["Calls"]:>7s} {float(r["AverageNs"])/1e3:9.2f} us {float(r["TotalDurationNs"])/1e6:9.2f} ms')
for r in rows:
    if "lnfold" in r["Name"]: print("LNFOLD", r["Calls"], float(r["AverageNs"]) / 1e3, "us")
PY
rm -f $O/prof_fold1/*kernel_trace.csv
exit $rc
