#!/bin/bash
# Build libf5h.so of another git revision into f5-tts_amd/f5_tts_amd/lib_base/ (for one-box A/Bs through
# F5H_LIB, tools/gpu_ab.sh). Usage: tools/build_base.sh <rev> [dir under f5-tts_amd/f5_tts_amd, default lib_base]
set -e
cd "$(dirname "$0")/.."
REV=${1:?rev}
T=/tmp/f5h_base_$REV
rm -rf $T && mkdir -p $T
git archive $REV f5-tts_amd/csrc include | tar -x -C $T
make -C $T/f5-tts_amd/csrc -j8 OBJ_DIR=$T/obj OUT_DIR=$PWD/f5-tts_amd/f5_tts_amd/${2:-lib_base} > $T/build.log 2>&1
echo "built $REV -> f5-tts_amd/f5_tts_amd/${2:-lib_base}/libf5h.so"
