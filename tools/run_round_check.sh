set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${1:-r02u}_gputest.log 2>&1 || { tail -30 gpurun_out/${1:-r02u}_gputest.log; exit 1; }
tail -2 gpurun_out/${1:-r02u}_gputest.log
timeout -k 10 300 python bench.py > gpurun_out/${1:-r02u}_bench.json 2> gpurun_out/${1:-r02u}_bench.err || { tail -20 gpurun_out/${1:-r02u}_bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${1:-r02u}_kt -o run -- python3 bench.py --steps 20 --no-cpu > gpurun_out/${1:-r02u}_kt.log 2>&1
echo done
