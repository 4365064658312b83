#!/bin/bash
# One-box interleaved A/B of two builds (cdna_hip_programming.md §5.4 rule 24): the base library
# (f5-tts_amd/f5_tts_amd/lib_base/libf5h.so, tools/build_base.sh) against the in-tree one, ROUNDS rounds of
# quick bench lines per config, attention probed live (PROBE, default attention). Output: gpurun_out/$OUT.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-ab}; mkdir -p $O; export TMPDIR=/tmp
BASE=$PWD/f5-tts_amd/f5_tts_amd/lib_base/libf5h.so
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
for i in $(seq 1 ${ROUNDS:-2}); do
  for c in ${CONFIGS:-c2}; do
    case $c in c2|c1) ST="--steps 10 --warmup 3";; *) ST="--steps 2 --warmup 1";; esac
    for arm in base new; do
      if [ $arm = base ]; then L=$BASE; else L=$PWD/f5-tts_amd/f5_tts_amd/lib/libf5h.so; fi
      F5H_LIB=$L timeout -k 10 600 python bench.py --config $c $ST --no-cpu-baseline --no-vocos --probe ${PROBE:-attention} \
        > $O/${c}_${arm}_$i.log 2>&1 || { echo "$c $arm $i failed"; exit 1; }
      echo "$c $arm $i $(tail -1 $O/${c}_${arm}_$i.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["ms_per_step"],2), r["kernel"], r.get("avg_launch_us"), r["frac"])')"
    done
  done
done
