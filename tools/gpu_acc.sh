cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 python tools/coop_pipeline.py tools/variants/libPROF.so > gpurun_out/cp.log 2>&1; cat gpurun_out/cp.log
timeout -k 10 60 ./tools/coop_bench > gpurun_out/cb.log 2>&1; tail -32 gpurun_out/cb.log
