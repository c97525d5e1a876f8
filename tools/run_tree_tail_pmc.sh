# SQ counters of the latency-bound Merkle tree tails (subtree_kernel,
# top_kernel) and the FRI fold-leaves kernel during a 2^25 FRI prove: VALU
# instructions per wave and wave cycles per VALU instruction (dev tool).
# usage: bash tools/run_tree_tail_pmc.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d gpurun_out/${TAG}_tail -o run -- python3 tools/fri_timeline.py 24 > gpurun_out/${TAG}_tail.log 2>&1
f=$(find gpurun_out/${TAG}_tail -name "*counter_collection.csv" | head -1)
python3 tools/pmc_kernels.py $(dirname $f) subtree_kernel top_kernel fri_fold_leaves_kernel > gpurun_out/${TAG}_tail_summary.txt 2>&1 || true
cat gpurun_out/${TAG}_tail_summary.txt
echo done
