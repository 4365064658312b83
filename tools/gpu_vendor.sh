#!/bin/bash
# Same-box yardstick: hipBLASLt (torch.mm) and torch SDPA at the C2 and C4 shapes of every
# kernel class under rocprofv3 --kernel-trace --stats, then this build's kernel trace at C2 and C4 per rank
# (graph mode, 1 warm + 2 marked calls, phase chain off: every class its own launch) summarised per class by
# tools/class_profile.py. Output: $O.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-vendor}; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/vendor -o run -- \
  python tools/vendor_ref.py $O/vendor_ops.json > $O/vendor.log 2>&1 || { echo "vendor failed"; exit 1; }
echo "vendor ok"
for c in c2 c4; do
  F5H_CHAIN=0 F5H_TRACE_WARM=1 F5H_TRACE_CALLS=2 timeout -s KILL 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$c -o run -- \
    python tools/trace_c2.py run $c > $O/tr_$c.log 2>&1 || { echo "trace $c failed"; exit 1; }
  (cd tools && python class_profile.py trace $O/tr_$c/run_kernel_trace.csv $c $O/classes_$c.json > /dev/null) \
    && echo "trace $c ok"
done
# the vendor trace is summarised into the JSON by hand (profiles/r05_vendor_c2_c4.json); keep it, drop ours
find $O -path "*tr_c*" -name "*_kernel_trace.csv" -delete
