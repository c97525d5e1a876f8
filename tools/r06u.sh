set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06u}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "fri or fold or pcs or batched" tests/test_gpu_pcs_fused.py > gpurun_out/${T}_t1.log 2>&1 || { grep -n "Error\|passed\|failed" gpurun_out/${T}_t1.log | tail -20; exit 1; }
tail -1 gpurun_out/${T}_t1.log
for v in PREV NEW; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_$v -o run -- python3 tools/prove_ab.py tools/variants/lib$v.so > gpurun_out/${T}_$v.log 2>&1 || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_CUR -o run -- python3 tools/prove_ab.py multilinear_amd/libmlhip.so > gpurun_out/${T}_CUR.log 2>&1 || exit 1
grep -h "fri_prove" gpurun_out/${T}_*.log
