cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "sumcheck or pcs or eq" > gpurun_out/fu_test.log 2>&1 || { tail -30 gpurun_out/fu_test.log; exit 1; }
tail -2 gpurun_out/fu_test.log
timeout -k 10 300 python tools/sumcheck_ab.py multilinear_amd/libmlhip.so tools/variants/libHEAD.so > gpurun_out/fu_ab.log 2>&1; cat gpurun_out/fu_ab.log
timeout -k 10 300 python tools/sumcheck_ab.py multilinear_amd/libmlhip.so tools/variants/libHEAD.so > gpurun_out/fu_ab2.log 2>&1; cat gpurun_out/fu_ab2.log
