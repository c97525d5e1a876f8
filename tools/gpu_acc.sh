cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 python tools/coop_pipeline.py tools/variants/libPROF.so > gpurun_out/cp.log 2>&1; cat gpurun_out/cp.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sc_kt -o run -- python3 tools/sumcheck_ab.py multilinear_amd/libmlhip.so > gpurun_out/sc_kt.log 2>&1; tail -3 gpurun_out/sc_kt.log
