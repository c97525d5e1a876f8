set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python tools/coop_pipeline.py tools/variants/libPROF.so > gpurun_out/r06c_coop.txt 2>&1; tail -14 gpurun_out/r06c_coop.txt
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "inner_fold_step or huge_k or step_api or fold_step_gp" > gpurun_out/r06c_t1.log 2>&1 || { grep -n "MlhError\|Error\|passed\|failed" gpurun_out/r06c_t1.log | tail -20; exit 1; }
tail -2 gpurun_out/r06c_t1.log
