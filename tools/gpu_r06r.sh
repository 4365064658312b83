#!/bin/bash
# kernel-trace stats of a config's bench with the fold off and on (CONFIG, default c5)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; O=$PWD/gpurun_out/${OUT:-r06r}; mkdir -p $O; export TMPDIR=/tmp
C=${CONFIG:-c5}
for f in 0 1; do
  cd /tmp && F5H_LNFOLD=$f timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fold$f -o run -- python3 $R/bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --no-vocos --probe none > $O/prof_fold$f.log 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' $O/prof_fold$f.log
  f=$(find $O/prof_fold$f -name '*kernel_stats.csv' | head -1); python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print("total kernel ms", sum(float(r["TotalDurationNs"]) for r in rows) / 1e6)
for r in rows[:12]:
    print(f'{r["Name"][:90]:90s} {r["Calls"]:>7s} {float(r["AverageNs"])/1e3:9.2f} us {float(r["TotalDurationNs"])/1e6:9.2f} ms')
PY
  find $O/prof_fold$f -name '*kernel_trace.csv' -delete
done
