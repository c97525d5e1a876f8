# FRI prove 2^25 under a kernel trace: per-kernel sequence of the last prove (dev tool)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_fri -o run -- python3 tools/fri_timeline.py 24 > gpurun_out/${TAG}_fri.log 2>&1
f=$(find gpurun_out/${TAG}_fri -name "*kernel_trace.csv" | head -1)
python3 tools/timeline_summary.py $f 1 > gpurun_out/${TAG}_fri_summary.txt
python3 tools/kernel_seq.py $f 1 > gpurun_out/${TAG}_fri_seq.txt
grep "fri prove" gpurun_out/${TAG}_fri.log; cat gpurun_out/${TAG}_fri_summary.txt
