set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06y}
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_failures.py tests/test_gpu_fullsize.py -k "sumcheck or pcs or config4 or gen_pows" > gpurun_out/${T}_t1.log 2>&1 || { grep -n "Error\|passed\|failed" gpurun_out/${T}_t1.log | tail -20; exit 1; }
tail -1 gpurun_out/${T}_t1.log
timeout -k 10 200 python tools/sumcheck_ab.py ${ABLIBS:-tools/variants/libNOXC.so multilinear_amd/libmlhip.so} > gpurun_out/${T}_ab.txt 2>&1; grep -v amdgpu gpurun_out/${T}_ab.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt -o run -- python3 tools/sc_kt.py > gpurun_out/${T}_kt.log 2>&1 || { tail -20 gpurun_out/${T}_kt.log; exit 1; }
grep "_ms" gpurun_out/${T}_kt.log
f=$(find gpurun_out/${T}_kt -name "*kernel_stats.csv" | head -1); grep -i "eq_tail\|eq_head\|fold_group\|corner_sums" "$f" | cut -d, -f1-4
