#!/bin/bash
# Round 3 GPU pass H: operand-intake probe (LDS-DMA vs register staging), the fused LayerNorm tail's
# bitwise test, the register-staged GEMM configurations (40-42) against every tile config, their op-level
# timing at the C2 shapes (kernel trace), C2 benches interleaved: tails on / off (F5H_LN_FUSE=0) /
# LayerNorm skipped (timing-only bound), then a kernel trace of C2 calls.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/r03h; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 60 ./tools/probes/intake 8 > $O/intake_8mb.log 2>&1 && timeout -k 10 60 ./tools/probes/intake 64 > $O/intake_64mb.log 2>&1 || exit 1
cat $O/intake_8mb.log $O/intake_64mb.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_contract.py tests/test_gpu_parity.py -m gpu -q -rf -x --timeout 120 --timeout-method thread -k "ln_fuse or tile_config" > $O/targeted_tests.log 2>&1; rc=$?
echo "targeted tests rc=$rc"; tail -3 $O/targeted_tests.log
[ $rc -eq 0 ] || exit $rc
GT_CFGS=0,1,5,40,41,42,43,44,45 GT_SHAPES=c2_qkv,c2_ffn1,c2_out,c2_ffn2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $PWD/$O/gt -o run -- python tools/gemm_tune.py > $O/gt.log 2>&1 || { echo "tune failed"; exit 1; }
GT_CFGS=0,1,5,40,41,42,43,44,45 GT_SHAPES=c2_qkv,c2_ffn1,c2_out,c2_ffn2 python tools/gemm_tune.py --report $O/gt/run_kernel_trace.csv | tee $O/gemm_tune_rs.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > $O/fuse_$i.log 2>&1 || exit 1
  F5H_LN_FUSE=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > $O/sep_$i.log 2>&1 || exit 1
  F5H_LN_FUSE=0 F5H_DIAG_SKIP_LN=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > $O/noln_$i.log 2>&1 || exit 1
done
for f in $O/fuse_*.log $O/sep_*.log $O/noln_*.log; do echo "$f $(tail -1 $f | python -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')"; done
export F5H_TRACE_WARM=1 F5H_TRACE_CALLS=2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/trace -o run -- \
  python tools/trace_c2.py run > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
python tools/trace_c2.py report $O/trace/run_kernel_trace.csv > $O/r03_c2_kernels.txt; head -24 $O/r03_c2_kernels.txt
