# usage: bash tools/gpu_quick.sh TAG "pytest -k expr" [bench]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1; K=$2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -3 gpurun_out/${TAG}_gputest.log
if [ "$3" = "bench" ]; then
  timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print({k:d[k] for k in ['value','ms_per_step','fri_commit_ms','sumcheck_ms','pcs_prove_ms','eq_table_ms']})"
fi
