cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 python tools/coop_pipeline.py tools/variants/libFNOSER.so > gpurun_out/cp.log 2>&1; head -12 gpurun_out/cp.log
