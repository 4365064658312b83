#!/bin/bash
# kernel-trace stats of the C2 bench with the LayerNorm fold off and on
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; O=$PWD/gpurun_out/${OUT:-r06g}; mkdir -p $O; export TMPDIR=/tmp
for f in 0 1; do
  cd /tmp && F5H_LNFOLD=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fold$f -o run -- python3 $R/bench.py --config c2 --steps 4 --warmup 2 --no-cpu-baseline --no-vocos --probe none > $O/prof_fold$f.log 2>&1 || exit 1
  tail -1 $O/prof_fold$f.log
  f=$(find $O/prof_fold$f -name '*kernel_stats.csv' | head -1); python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total kernel ms", tot / 1e6)
for r in rows[:16]:
    print(f'{r["Name"][:90]:90s} {r["Calls"]:>7s} {float(r["AverageNs"])/1e3:9.2f} us {float(r["TotalDurationNs"])/1e6:9.2f} ms')
PY
done
