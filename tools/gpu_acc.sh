cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python tools/sumcheck_ab.py tools/variants/libREH0.so tools/variants/libREH1.so tools/variants/libREH2.so tools/variants/libHEAD.so > gpurun_out/fu_ab.log 2>&1; cat gpurun_out/fu_ab.log
timeout -k 10 300 python tools/sumcheck_ab.py tools/variants/libREH0.so tools/variants/libREH1.so tools/variants/libREH2.so > gpurun_out/fu_ab2.log 2>&1; cat gpurun_out/fu_ab2.log
