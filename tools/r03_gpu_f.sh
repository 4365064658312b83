#!/bin/bash
# Round 3 GPU pass F: (1) the pipelined attention kernel (F5H_ATTN_PIPE=1) against the attention
# tests; (2) GEMM tile tests with two-blocks-per-CU launch bounds; (3) interleaved C2 benches:
# old launch bounds (libf5h_lb1.so) / new / new + pipelined attention; (4) C2 timeline, new build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03f; export TMPDIR=/tmp
F5H_ATTN_PIPE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rf --timeout 120 --timeout-method thread -k "attention or c2 or sample_fp32 or masked" > gpurun_out/r03f/pipe_tests.log 2>&1; echo "pipe tests rc=$?"; tail -3 gpurun_out/r03f/pipe_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_envelope.py -m gpu -q -rf --timeout 120 --timeout-method thread -k "linear or tile or envelope" > gpurun_out/r03f/gemm_tests.log 2>&1; echo "gemm tests rc=$?"; tail -3 gpurun_out/r03f/gemm_tests.log
LIB=$PWD/f5-tts_amd/f5_tts_amd/lib
for i in 1 2; do
  F5H_LIB=$LIB/libf5h_lb1.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe qkv > gpurun_out/r03f/lb1_$i.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe qkv > gpurun_out/r03f/lb2_$i.log 2>&1 || exit 1
  F5H_ATTN_PIPE=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe attention > gpurun_out/r03f/pipe_$i.log 2>&1 || exit 1
done
for f in gpurun_out/r03f/lb1_*.log gpurun_out/r03f/lb2_*.log gpurun_out/r03f/pipe_*.log; do echo "$f $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r.get("kernel"), r.get("avg_launch_us"), r.get("frac"))')"; done
timeout -k 10 300 python tools/timeline_c2.py > gpurun_out/r03f/timeline_c2.log 2>&1; echo "timeline rc=$?"; tail -7 gpurun_out/r03f/timeline_c2.log
F5H_ATTN_PIPE=1 timeout -k 10 300 python tools/timeline_c2.py > gpurun_out/r03f/timeline_c2_pipe.log 2>&1; echo "timeline pipe rc=$?"; tail -6 gpurun_out/r03f/timeline_c2_pipe.log
