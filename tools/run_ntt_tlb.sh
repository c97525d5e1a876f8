# Address-translation counters of the NTT passes (is pass 0's 1-MiB row
# stride missing the UTCL1?).  usage: bash tools/run_ntt_tlb.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1
timeout -s KILL 60 rocprofv3 -L > gpurun_out/${TAG}_avail.txt 2>&1 || true
grep -o "TCP_UTCL[A-Z0-9_]*\|TCP_TCP_LATENCY[A-Z_]*\|TA_BUSY[a-z_]*\|TCP_PENDING[A-Z_]*" gpurun_out/${TAG}_avail.txt | sort -u > gpurun_out/${TAG}_names.txt || true
cat gpurun_out/${TAG}_names.txt
timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_PERMISSION_MISS_sum TCP_UTCL1_REQUEST_sum --output-format csv -d gpurun_out/${TAG}_tlb -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras > gpurun_out/${TAG}_tlb.log 2>&1
echo done
