set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06z1}
for v in T1 T2 IF32 CUR; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_$v -o run -- python3 tools/sumcheck_ab.py $( [ $v = CUR ] && echo multilinear_amd/libmlhip.so || echo tools/variants/lib$v.so ) > gpurun_out/${T}_$v.log 2>&1 || { tail -20 gpurun_out/${T}_$v.log; exit 1; }
grep sumcheck_eq gpurun_out/${T}_$v.log
done
