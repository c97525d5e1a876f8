set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python tools/coop_pipeline.py tools/variants/libPROF.so > gpurun_out/r06d_coop.txt 2>&1; tail -40 gpurun_out/r06d_coop.txt
timeout -k 10 120 python tools/sumcheck_ab.py tools/variants/libBASE.so multilinear_amd/libmlhip.so tools/variants/libBASE.so multilinear_amd/libmlhip.so > gpurun_out/r06d_ab.txt 2>&1; cat gpurun_out/r06d_ab.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "inner_fold_step or huge_k or step_api or fold_step_gp or sumcheck or pcs" > gpurun_out/r06d_t1.log 2>&1 || { grep -n "Error\|passed\|failed" gpurun_out/r06d_t1.log | tail -20; exit 1; }
tail -2 gpurun_out/r06d_t1.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k config4 tests/test_gpu_pcs_fullsize.py tests/test_gpu_failures.py > gpurun_out/r06d_t2.log 2>&1 || { grep -n "Error\|passed\|failed" gpurun_out/r06d_t2.log | tail -20; exit 1; }
tail -2 gpurun_out/r06d_t2.log
