#!/bin/bash
# One-box interleaved A/B of builds (cdna_hip_programming.md §5.4 rule 24): ARMS="name=dir ..." (default
# "base=lib_base new=lib", dirs under f5-tts_amd/f5_tts_amd/, tools/build_base.sh builds a revision into one),
# an arm may add environment settings: "name=dir:VAR=val,VAR2=val2";
# ROUNDS rounds of quick bench lines per config in CONFIGS, the class PROBE (default attention) probed live.
# Output: gpurun_out/$OUT.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-ab}; mkdir -p $O; export TMPDIR=/tmp
LD=$PWD/f5-tts_amd/f5_tts_amd
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
for i in $(seq 1 ${ROUNDS:-2}); do
  for c in ${CONFIGS:-c2}; do
    case $c in c2|c1) ST="--steps 10 --warmup 3";; *) ST="--steps 2 --warmup 1";; esac
    for arm in ${ARMS:-base=lib_base new=lib}; do
      n=${arm%%=*}; spec=${arm#*=}; dir=${spec%%:*}; L=$LD/$dir/libf5h.so
      EV=""; [ "$spec" != "$dir" ] && EV=$(echo ${spec#*:} | tr ',' ' ')
      env $EV F5H_LIB=$L timeout -k 10 600 python bench.py --config $c $ST --no-cpu-baseline --no-vocos --probe ${PROBE:-attention} \
        > $O/${c}_${n}_$i.log 2>&1 || { echo "$c $n $i failed"; exit 1; }
      echo "$c $n $i $(tail -1 $O/${c}_${n}_$i.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["ms_per_step"],2), r["kernel"], r.get("avg_launch_us"), r["frac"])')"
    done
  done
done
