set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02o_gputest.log 2>&1 || { tail -30 gpurun_out/r02o_gputest.log; exit 1; }
tail -2 gpurun_out/r02o_gputest.log
timeout -k 10 300 python bench.py > gpurun_out/r02o_bench.json 2> gpurun_out/r02o_bench.err || { tail -20 gpurun_out/r02o_bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02o_kt -o run -- python3 bench.py --steps 20 --no-cpu > gpurun_out/r02o_kt.log 2>&1
echo done
