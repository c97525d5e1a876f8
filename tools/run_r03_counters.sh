# Round-3 counter passes (each rocprofv3 pass its own run, under its own
# time limit): sumcheck HBM traffic (FETCH_SIZE, WRITE_SIZE over
# tools/sumcheck_ab.py), the bench's VALU pass and the NTT stall passes.
# Raw CSVs land in gpurun_out/<tag>_*; summarise on the build host with
#   python tools/sumcheck_pmc.py <tag> gpurun_out/<tag>_scf gpurun_out/<tag>_scw 22
#   python tools/valu_summary.py <tag> gpurun_out/<tag>_valu
#   python tools/pmc_kernels.py gpurun_out/<tag>_stall ntt_pass  (and _stall2)
# usage: bash tools/run_r03_counters.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r03}
SC="python3 tools/sumcheck_ab.py multilinear_amd/libmlhip.so"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_scf -o run -- $SC > gpurun_out/${TAG}_scf.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_scw -o run -- $SC > gpurun_out/${TAG}_scw.log 2>&1 &&
echo "sumcheck PMC done" &&
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/${TAG}_valu -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --fri-log 0 --strong-log 0 > gpurun_out/${TAG}_valu.log 2>&1 &&
echo "VALU pass done" &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/${TAG}_stall -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras > gpurun_out/${TAG}_stall.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d gpurun_out/${TAG}_stall2 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras > gpurun_out/${TAG}_stall2.log 2>&1 &&
echo "stall passes done"
