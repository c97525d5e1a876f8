# Per-pass counter attribution of the 2^24 NTT passes:
# three rocprofv3 --pmc passes over the same short bench run, each in its own
# process with its own time limit; summarised by tools/ntt_attrib.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1
B="python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras --spinup-s 0.1"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LEVEL_WAVES SQ_BUSY_CYCLES TA_BUSY_avr GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/${TAG}_a -o run -- $B > gpurun_out/${TAG}_a.log 2>&1 || exit 11
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d gpurun_out/${TAG}_b -o run -- $B > gpurun_out/${TAG}_b.log 2>&1 || exit 12
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_max TD_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC --kernel-trace --output-format csv -d gpurun_out/${TAG}_c -o run -- $B > gpurun_out/${TAG}_c.log 2>&1 || exit 13
echo attrib_done
