#!/bin/bash
# Which HIP call of the graph-eviction test waits behind the other stream's spin: the test under
# rocprofv3 --hip-runtime-trace --stats; keeps the stats and the calls over 20 ms, drops the full trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-diag_evict}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-runtime-trace --stats --output-format csv -d $O/rp -o evict -- \
  python -u -m pytest tests/test_gpu_contract.py -q -rf -k "${TESTS:-eviction_never_waits}" --timeout 200 --timeout-method thread \
  > $O/evict.log 2>&1
rc=$?; echo "diag rc=$rc"; tail -3 $O/evict.log
python - "$O" <<'PY'
import csv, glob, os, sys
o = sys.argv[1]
rows = []
for f in glob.glob(f"{o}/rp/**/*hip_api_trace.csv", recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            try:
                d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            except (KeyError, ValueError):
                continue
            if d > 20:
                rows.append((int(r["Start_Timestamp"]), d, r.get("Function", "?"), r.get("Thread_Id", "?")))
    os.remove(f)
rows.sort()
with open(f"{o}/slow_calls.txt", "w") as fh:
    for t, d, fn, tid in rows:
        fh.write(f"{t} {d:9.2f} ms {fn} thread {tid}\n")
print(open(f"{o}/slow_calls.txt").read()[-3000:])
PY
exit $rc
