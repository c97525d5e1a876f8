set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt2 -o run -- python3 bench.py --steps 20 --no-cpu --strong-log 0 > gpurun_out/kt2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/valu2 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --fri-log 0 --strong-log 0 > gpurun_out/valu2.log 2>&1
ls gpurun_out/kt2 gpurun_out/valu2
