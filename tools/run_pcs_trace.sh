set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_pcs -o run -- python3 tools/sumcheck_timeline.py 24 pcs > gpurun_out/${TAG}_pcs.log 2>&1
f=$(find gpurun_out/${TAG}_pcs -name "*kernel_trace.csv" | head -1)
python3 tools/timeline_summary.py $f 1 > gpurun_out/${TAG}_pcs_summary.txt
python3 tools/kernel_seq.py $f 1 > gpurun_out/${TAG}_pcs_seq.txt
grep "pcs prove" gpurun_out/${TAG}_pcs.log; cat gpurun_out/${TAG}_pcs_summary.txt; tail -1 gpurun_out/${TAG}_pcs_seq.txt
