# usage: bash tools/run_bench_prof.sh TAG  -- bench line + rocprofv3 kernel stats of the bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt -o run -- python3 bench.py --steps 20 --no-cpu > gpurun_out/${TAG}_kt.log 2>&1
echo done
