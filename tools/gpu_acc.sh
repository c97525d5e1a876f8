cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python tools/ntt_libab.py multilinear_amd/libmlhip.so tools/variants/libTA2.so > gpurun_out/ta_ab.log 2>&1; cat gpurun_out/ta_ab.log
