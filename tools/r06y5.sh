set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06y5}
timeout -k 10 200 python tools/sumcheck_ab.py tools/variants/libPREV.so tools/variants/libNOSPLIT.so tools/variants/libHB8.so multilinear_amd/libmlhip.so tools/variants/libHB32.so > gpurun_out/${T}_ab.txt 2>&1; grep -v amdgpu gpurun_out/${T}_ab.txt
for v in HB8 CUR HB32; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_$v -o run -- python3 tools/sumcheck_ab.py $( [ $v = CUR ] && echo multilinear_amd/libmlhip.so || echo tools/variants/lib$v.so ) > gpurun_out/${T}_$v.log 2>&1 || { tail -20 gpurun_out/${T}_$v.log; exit 1; }
done
