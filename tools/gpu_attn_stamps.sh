#!/bin/bash
# attn_pw_kernel: parity (op tests with F5H_ATTN=1), phase stamps (diagnostic build), kernel-trace timing of both variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
F5H_ATTN=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/t_attn.log 2>&1 && echo "attn tests ok" \
&& F5H_ATTN=1 F5H_LIB=f5-tts_amd/build/stamps/libf5h.so timeout -k 10 120 python tools/attn_stamps_pw.py > gpurun_out/stamps.txt 2>&1 && echo stamps ok \
&& F5H_ATTN=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/at1 -o run -- python tools/attn_time.py > gpurun_out/at1p.log 2>&1 && echo "prof1 ok" \
&& F5H_ATTN=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/at0 -o run -- python tools/attn_time.py > gpurun_out/at0p.log 2>&1 && echo "prof0 ok"
rc=$?; tail -2 gpurun_out/t_attn.log; exit $rc
