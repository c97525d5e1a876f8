set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02d_gputest.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r02d_bench.json 2> gpurun_out/r02d_bench.err
