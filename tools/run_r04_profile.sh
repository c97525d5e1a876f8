# Round-4 profile set of the committed tree (each rocprofv3 pass its own run
# under its own time limit; counters never combined with trace domains):
#  * kernel-trace --stats of bench.py (the live timer's numbers must agree),
#  * FETCH_SIZE and WRITE_SIZE passes of the NTT headline (pmc_ntt.json),
#  * the VALU pass of bench.py (valu_profile),
#  * FETCH_SIZE / WRITE_SIZE of the config-4 sumcheck (sumcheck_hbm_frac).
# Summaries on the build host:
#   python tools/pmc_summary.py <tag> gpurun_out/<tag>_kt gpurun_out/<tag>_fetch gpurun_out/<tag>_write 24
#   python tools/valu_summary.py <tag> gpurun_out/<tag>_valu
#   python tools/sumcheck_pmc.py <tag> gpurun_out/<tag>_scf gpurun_out/<tag>_scw 22
# usage: bash tools/run_r04_profile.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r04}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt -o run -- python3 bench.py --steps 20 --no-cpu > gpurun_out/${TAG}_kt.log 2>&1 && echo "kt done" &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras > gpurun_out/${TAG}_fetch.log 2>&1 && echo "fetch done" &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras > gpurun_out/${TAG}_write.log 2>&1 && echo "write done" &&
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/${TAG}_valu -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --fri-log 0 --strong-log 0 > gpurun_out/${TAG}_valu.log 2>&1 && echo "valu done" &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_scf -o run -- python3 tools/sumcheck_ab.py multilinear_amd/libmlhip.so > gpurun_out/${TAG}_scf.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_scw -o run -- python3 tools/sumcheck_ab.py multilinear_amd/libmlhip.so > gpurun_out/${TAG}_scw.log 2>&1 && echo "sumcheck pmc done"
