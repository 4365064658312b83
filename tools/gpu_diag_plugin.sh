#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-diag_plugin}; mkdir -p $O; export TMPDIR=/tmp
echo "== new lib"; timeout -k 10 200 python tools/diag_plugin_c2.py 2>&1 | grep -v amdgpu.ids | tee $O/new.log || exit 1
echo "== r05 lib"; F5H_LIB=$PWD/f5-tts_amd/f5_tts_amd/lib_r05/libf5h.so timeout -k 10 200 python tools/diag_plugin_c2.py 2>&1 | grep -v amdgpu.ids | tee $O/r05.log || exit 1
