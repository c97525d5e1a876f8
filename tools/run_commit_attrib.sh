# Counter attribution of the FRI commit's SHA-256 kernels (leaf_pairs_level2,
# level2) with the same three passes as tools/run_ntt_attrib.sh.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1
B="python3 tools/commit_drv.py 6"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INSTS_SMEM TA_BUSY_avr GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/${TAG}_a -o run -- $B > gpurun_out/${TAG}_a.log 2>&1 || exit 11
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d gpurun_out/${TAG}_b -o run -- $B > gpurun_out/${TAG}_b.log 2>&1 || exit 12
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_max TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC --kernel-trace --output-format csv -d gpurun_out/${TAG}_c -o run -- $B > gpurun_out/${TAG}_c.log 2>&1 || exit 13
echo attrib_done
