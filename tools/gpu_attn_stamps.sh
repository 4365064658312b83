set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
F5H_LIB=f5-tts_amd/build/stamps/libf5h.so timeout -k 10 120 python tools/attn_stamps_pw.py > gpurun_out/stamps.txt 2>&1 && echo stamps ok \
&& F5H_ATTN=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/at1 -o run -- python tools/attn_time.py > gpurun_out/at1p.log 2>&1 && echo "prof1 ok"
