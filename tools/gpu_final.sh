#!/bin/bash
# Round-end check of the tree as committed: GPU suite, smoke, default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/fin; export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/fin/gputest.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/fin/gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/fin/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/fin/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/fin/bench.log 2>&1 || exit 1
tail -1 gpurun_out/fin/bench.log
