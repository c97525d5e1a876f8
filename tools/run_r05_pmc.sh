# Round-5 counter passes of the committed tree (each rocprofv3 pass its own run
# under its own time limit; counters never combined with trace domains): the
# FETCH_SIZE / WRITE_SIZE passes of the NTT headline (pmc_ntt.json), the VALU
# pass of bench.py (valu_profile) and the config-4 sumcheck's FETCH/WRITE.
# The kernel-trace --stats run is tools/r05_check.sh's.  Summaries on the host:
#   python tools/pmc_summary.py <tag> gpurun_out/<tag>_kt gpurun_out/<tag>_fetch gpurun_out/<tag>_write 24
#   python tools/valu_summary.py <tag> gpurun_out/<tag>_valu
#   python tools/sumcheck_pmc.py <tag> gpurun_out/<tag>_scf gpurun_out/<tag>_scw 22
# usage: bash tools/run_r05_pmc.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r05}
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras > gpurun_out/${TAG}_fetch.log 2>&1 && echo "fetch done" &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras > gpurun_out/${TAG}_write.log 2>&1 && echo "write done" &&
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/${TAG}_valu -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --fri-log 0 --strong-log 0 > gpurun_out/${TAG}_valu.log 2>&1 && echo "valu done" &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_scf -o run -- python3 tools/sumcheck_ab.py multilinear_amd/libmlhip.so > gpurun_out/${TAG}_scf.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_scw -o run -- python3 tools/sumcheck_ab.py multilinear_amd/libmlhip.so > gpurun_out/${TAG}_scw.log 2>&1 && echo "sumcheck pmc done"
