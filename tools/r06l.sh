set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/shard_fri_diag.py "$1" 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06l_diag.txt
