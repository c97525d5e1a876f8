set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06q}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "sumcheck or pcs" tests/test_gpu_failures.py tests/test_gpu_fullsize.py::test_config4_sumcheck_24_vars_vs_c_oracle tests/test_gpu_pcs_fullsize.py tests/test_gpu_pcs_fused.py > gpurun_out/${T}_t1.log 2>&1 || { grep -n "Error\|passed\|failed" gpurun_out/${T}_t1.log | tail -20; exit 1; }
tail -1 gpurun_out/${T}_t1.log
timeout -k 10 120 python tools/sumcheck_ab.py ${ABLIBS} > gpurun_out/${T}_ab.txt 2>&1; grep sumcheck gpurun_out/${T}_ab.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt -o run -- python3 tools/sc_kt.py > gpurun_out/${T}_kt.log 2>&1 || { tail -20 gpurun_out/${T}_kt.log; exit 1; }
grep "_ms" gpurun_out/${T}_kt.log
f=$(find gpurun_out/${T}_kt -name "*kernel_stats.csv" | head -1); grep -i "eq_tail\|eq_setup" "$f" | cut -d, -f1-4
