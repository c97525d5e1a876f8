set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( while true; do date >> gpurun_out/r06a_hb.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "inner_fold_step or huge_k or step_api or fold_step_gp or batched" > gpurun_out/r06a_t1.log 2>&1 || { tail -40 gpurun_out/r06a_t1.log; exit 1; }
tail -2 gpurun_out/r06a_t1.log
MLH_TEST_PROGRESS=gpurun_out/r06a_prog.txt timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_sharded_threads_gpu.py -k config5 --durations=5 > gpurun_out/r06a_t2.log 2>&1 || { tail -40 gpurun_out/r06a_t2.log; exit 1; }
tail -8 gpurun_out/r06a_t2.log
timeout -k 10 700 python -u -m pytest -x -v --timeout 330 --timeout-method thread tests/test_bench_rehearsal_gpu.py --durations=5 > gpurun_out/r06a_t3.log 2>&1 || { tail -60 gpurun_out/r06a_t3.log; exit 1; }
tail -8 gpurun_out/r06a_t3.log
