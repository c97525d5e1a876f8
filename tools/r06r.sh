set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06r}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "fri or fold or pcs or batched" tests/test_gpu_fullsize.py tests/test_gpu_pcs_fullsize.py tests/test_gpu_pcs_fused.py > gpurun_out/${T}_t1.log 2>&1 || { grep -n "Error\|passed\|failed" gpurun_out/${T}_t1.log | tail -20; exit 1; }
tail -1 gpurun_out/${T}_t1.log
timeout -k 10 300 python tools/prove_ab.py ${ABLIBS} > gpurun_out/${T}_ab.txt 2>&1; cat gpurun_out/${T}_ab.txt | grep -v amdgpu
