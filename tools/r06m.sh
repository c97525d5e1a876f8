set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06e}
timeout -k 10 120 python tools/coop_pipeline.py tools/variants/libPROF.so > gpurun_out/${T}_coop.txt 2>&1; cat gpurun_out/${T}_coop.txt | head -24; tail -14 gpurun_out/${T}_coop.txt
timeout -k 10 120 python tools/sumcheck_ab.py ${ABLIBS:-tools/variants/libBASE.so multilinear_amd/libmlhip.so tools/variants/libBASE.so multilinear_amd/libmlhip.so} > gpurun_out/${T}_ab.txt 2>&1; cat gpurun_out/${T}_ab.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "sumcheck or pcs" tests/test_gpu_failures.py > gpurun_out/${T}_t1.log 2>&1 || { grep -n "Error\|passed\|failed" gpurun_out/${T}_t1.log | tail -20; exit 1; }
tail -1 gpurun_out/${T}_t1.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py::test_config4_sumcheck_24_vars_vs_c_oracle tests/test_gpu_pcs_fullsize.py > gpurun_out/${T}_t2.log 2>&1 || { grep -n "Error\|passed\|failed" gpurun_out/${T}_t2.log | tail -20; exit 1; }
tail -1 gpurun_out/${T}_t2.log
