# Round-6 counter passes of the NTT headline after the progression pass 0 (each
# rocprofv3 pass its own run under its own time limit; counters never combined
# with trace domains).  Summaries on the host:
#   python tools/pmc_summary.py <tag> gpurun_out/<tag>_kt gpurun_out/<tag>_fetch gpurun_out/<tag>_write 24
#   python tools/valu_summary.py <tag> gpurun_out/<tag>_valu
# usage: bash tools/run_r06_pmc.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r06p}
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras > gpurun_out/${TAG}_kt.log 2>&1 && echo "kt done" &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras > gpurun_out/${TAG}_fetch.log 2>&1 && echo "fetch done" &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras > gpurun_out/${TAG}_write.log 2>&1 && echo "write done" &&
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/${TAG}_valu -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --fri-log 0 --strong-log 0 > gpurun_out/${TAG}_valu.log 2>&1 && echo "valu done"
