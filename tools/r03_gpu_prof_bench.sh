#!/bin/bash
# rocprofv3 kernel trace + stats of the bench command itself (C2 defaults minus the CPU baseline and the
# Vocos timing), so the bench line's live attention average can be checked against rocprof's.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/r03pb; mkdir -p $O; export TMPDIR=/tmp
# (rocprofv3 of this build exits 1 after a complete run whose outputs are written: judge by the files)
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof -o run -- \
  python bench.py --no-cpu-baseline --no-vocos > $O/bench.log 2>&1; rc=$?
[ $rc -le 1 ] && ls $O/prof/run_kernel_stats.csv > /dev/null || { echo "prof failed rc=$rc"; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
python - "$O" <<'PY'
import csv, json, sys, glob
o = sys.argv[1]
line = json.loads([l for l in open(f"{o}/bench.log") if l.startswith('{"metric"')][-1])
r = line["roofline"]
st = glob.glob(f"{o}/prof/**/run_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(st)))
att = [x for x in rows if "attn16_kernel" in x["Name"]]
out = [f"bench line: {line['ms_per_step']} ms/call, {r['kernel']} avg {r['avg_launch_us']} us (in-kernel stamps, timed region)"]
for x in att:
    out.append(f"rocprofv3 --stats: {x['Name'][:60]} calls {x['Calls']} avg {float(x['AverageNs'])/1e3:.2f} us "
               f"min {float(x['MinNs'])/1e3:.2f} max {float(x['MaxNs'])/1e3:.2f}")
print("\n".join(out)); open(f"{o}/compare.txt", "w").write("\n".join(out) + "\n")
PY
