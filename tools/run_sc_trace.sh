set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_kt -o run -- python3 tools/sumcheck_timeline.py 24 > gpurun_out/${TAG}_sc.log 2>&1
f=$(find gpurun_out/${TAG}_kt -name "*kernel_trace.csv" | head -1)
python3 tools/kernel_seq.py $f 1 > gpurun_out/${TAG}_seq_factored.txt
python3 tools/kernel_seq.py $f 2 > gpurun_out/${TAG}_seq_twotable.txt
cat gpurun_out/${TAG}_sc.log; tail -1 gpurun_out/${TAG}_seq_factored.txt
