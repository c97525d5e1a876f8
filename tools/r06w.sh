set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06w}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "sumcheck or pcs" tests/test_gpu_failures.py tests/test_gpu_fullsize.py::test_config4_sumcheck_24_vars_vs_c_oracle > gpurun_out/${T}_t1.log 2>&1 || { grep -n "Error\|passed\|failed" gpurun_out/${T}_t1.log | tail -20; exit 1; }
tail -1 gpurun_out/${T}_t1.log
timeout -k 10 120 python tools/coop_pipeline.py tools/variants/libPROF.so > gpurun_out/${T}_coop.txt 2>&1 || { tail gpurun_out/${T}_coop.txt; exit 1; }
grep -v amdgpu gpurun_out/${T}_coop.txt | head -18; tail -12 gpurun_out/${T}_coop.txt
timeout -k 10 200 python tools/sumcheck_ab.py ${ABLIBS:-tools/variants/libPREV.so tools/variants/libOFF.so tools/variants/libK4.so multilinear_amd/libmlhip.so} > gpurun_out/${T}_ab.txt 2>&1; grep -v amdgpu gpurun_out/${T}_ab.txt
