# usage: bash tools/overlap_runs.sh "F WF HWQ" ...   (k_trace launch concurrency in the N=8 root rehearsal)
cd /tmp && export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
for cfg in "$@"; do set -- $cfg
 GPU_MAX_HW_QUEUES=$3 MIRT_WG_FACTOR=$2 MIRT_GROUP_REHEARSE=8 timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/ov_$1_$2_$3 -o run --output-format csv -- python3 $R/tools/group_probe.py --tile 8 --frames 300 --inflight $1 || exit 1
 f=$(find $R/gpurun_out/ov_$1_$2_$3 -name '*kernel_trace.csv' | head -1); echo "F=$1 WF=$2 HWQ=$3"; python3 $R/tools/trace_overlap.py $f || exit 1
done
