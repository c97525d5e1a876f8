set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06i}
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt -o run -- python3 tools/sc_kt.py > gpurun_out/${T}_kt.log 2>&1 || { tail -20 gpurun_out/${T}_kt.log; exit 1; }
grep "_ms" gpurun_out/${T}_kt.log
f=$(find gpurun_out/${T}_kt -name "*kernel_stats.csv" | head -1); head -25 "$f" | cut -d, -f1-8
