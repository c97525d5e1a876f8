set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06y7}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_failures.py -k "config4 or sumcheck" > gpurun_out/${T}_t1.log 2>&1 || { grep -n "Error\|passed\|failed" gpurun_out/${T}_t1.log | tail -20; exit 1; }
tail -1 gpurun_out/${T}_t1.log
timeout -k 10 200 python tools/sumcheck_ab.py tools/variants/libNOOVL.so multilinear_amd/libmlhip.so > gpurun_out/${T}_ab.txt 2>&1; grep -v amdgpu gpurun_out/${T}_ab.txt
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_kt -o run -- python3 tools/sumcheck_ab.py multilinear_amd/libmlhip.so > gpurun_out/${T}_kt.log 2>&1 || { tail -20 gpurun_out/${T}_kt.log; exit 1; }
