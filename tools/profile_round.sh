# Round profile set (run on the GPU box from the repo root):
#  kernel stats of the bench, separate FETCH_SIZE / WRITE_SIZE passes, and a
#  VALU-counter pass with kernel trace.  Summaries: tools/pmc_summary.py and
#  tools/valu_summary.py (run locally on the merged gpurun_out/).
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt -o run -- python3 bench.py --steps 20 --no-cpu > gpurun_out/kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras > gpurun_out/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras > gpurun_out/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/valu -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --fri-log 0 > gpurun_out/valu.log 2>&1
find gpurun_out -name "*.csv" | head -20
