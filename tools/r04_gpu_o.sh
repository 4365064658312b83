#!/bin/bash
# Round 4, box o: rocprofv3 kernel traces of C3 and C4 calls at the scalar-DMA HEAD (per-class launch averages that
# bench.py attaches beside its in-kernel stamps), within the profiler's graph-dispatch limit (1 warm + 1-2 calls).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/r04o; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
export F5H_TRACE_WARM=1
for cfg in c3 c4; do
  if [ $cfg = c3 ]; then export F5H_TRACE_CALLS=1; else export F5H_TRACE_CALLS=2; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$cfg -o run -- \
    python tools/trace_c2.py run $cfg > $O/trace_$cfg.log 2>&1 || { echo "trace $cfg failed"; exit 1; }
  python tools/class_profile.py trace $O/trace_$cfg/run_kernel_trace.csv $cfg $O/r04_rocprof_classes_$cfg.json > /dev/null \
    && echo "trace $cfg ok"
done
python - <<'PY'
import json
for c in ("c3", "c4"):
    d = json.load(open(f"gpurun_out/r04o/r04_rocprof_classes_{c}.json"))
    print(c, {k: (v["avg_launch_us"], v["dispatches"]) for k, v in d["classes"].items()})
PY
