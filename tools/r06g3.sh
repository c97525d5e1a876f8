set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06g3}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "progression or ntt_vs_c or intt_vs_c or forced_plans" > gpurun_out/${T}_t1.log 2>&1 || { grep -n "Error\|passed\|failed" gpurun_out/${T}_t1.log | tail -20; exit 1; }
tail -1 gpurun_out/${T}_t1.log
timeout -k 10 400 python tools/ntt_libab.py tools/variants/libNOGEO.so tools/variants/libLATE.so multilinear_amd/libmlhip.so tools/variants/libEARLY1.so > gpurun_out/${T}_ab.txt 2>&1; grep -v amdgpu gpurun_out/${T}_ab.txt | tail -30
