#!/bin/bash
# Round 4, box c: GPU suite (pool allocations, pad skip, attention TU without SLP), engine-drop diagnostic,
# attention row-max / row-sum variants (F5H_ATTN_VAR) interleaved at C2, the 8-phase 256x256 GEMM (cfg 12):
# bitwise tile-config tests, op-level timing against the ping-pong kernel (cfg 11) at the large-batch shapes,
# interleaved C4 / C5 benches (F5H_LARGE_CFG).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/r04c; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo "tests rc=$?"; grep -E "passed|failed" $O/gputest.log | tail -3; grep -E "^drop" $O/gputest.log
timeout -k 10 120 python tools/diag_drop.py > $O/diag_drop.log 2>&1; echo "diag rc=$?"; tail -1 $O/diag_drop.log
for i in 1 2; do
  for v in 0 1 2 3; do
    F5H_ATTN_VAR=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-vocos --probe attention > $O/attn_v${v}_$i.log 2>&1 || exit 1
  done
done
for f in $O/attn_v*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_launch_us"])')"; done
F5H_ATTN_VAR=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "attention or c2_sample or base_batch" -q -rf --timeout 300 --timeout-method thread > $O/attn_v3_tests.log 2>&1
echo "attn var3 tests rc=$?"; tail -2 $O/attn_v3_tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "tile_config" -q -rf --timeout 300 --timeout-method thread > $O/tiles.log 2>&1
rc=$?; echo "tile tests rc=$rc"; tail -3 $O/tiles.log
[ $rc -eq 0 ] || exit 1
GT_CFGS=11,12 GT_SHAPES=c3_qkv,c3_ffn1,c3_ffn2,c3_out,c5_qkv timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/gt -o run -- \
  python tools/gemm_tune.py > $O/gt.log 2>&1 || { echo "gemm_tune failed"; exit 1; }
GT_CFGS=11,12 GT_SHAPES=c3_qkv,c3_ffn1,c3_ffn2,c3_out,c5_qkv python tools/gemm_tune.py --report $O/gt/run_kernel_trace.csv > $O/gt_report.txt; cat $O/gt_report.txt
for i in 1 2; do
  for c in 11 12; do
    F5H_LARGE_CFG=$c timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-vocos --probe none > $O/c4_${c}_$i.log 2>&1 || exit 1
    F5H_LARGE_CFG=$c timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-vocos --probe none > $O/c5_${c}_$i.log 2>&1 || exit 1
  done
done
for f in $O/c4_*.log $O/c5_*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"; done
