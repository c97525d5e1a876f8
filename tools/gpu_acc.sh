cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 60 ./tools/sha2l_check > gpurun_out/acc.log 2>&1 && \
timeout -k 10 300 python tools/sumcheck_ab.py multilinear_amd/libmlhip.so tools/variants/libHEAD.so >> gpurun_out/acc.log 2>&1 && \
timeout -k 10 300 python tools/prove_ab.py multilinear_amd/libmlhip.so tools/variants/libHEAD.so >> gpurun_out/acc.log 2>&1 && \
timeout -k 10 120 python tools/coop_pipeline.py tools/variants/libPROF.so >> gpurun_out/acc.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sumcheck or merkle or fri or pcs" >> gpurun_out/acc.log 2>&1
rc=$?; tail -60 gpurun_out/acc.log; exit $rc
