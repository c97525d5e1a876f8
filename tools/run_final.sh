# Round-end check of one committed tree, as the driver runs it: the full GPU
# suite, smoke(), bench.py (N = 1), a rocprofv3 kernel-trace of the bench, and
# the N = 2 gloo rehearsal of the multi-GPU bench script.  Every log starts
# with the tree's HEAD sha (passed by the caller: the box gets no .git).
# usage: bash tools/run_final.sh <tag> <sha>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1
SHA=$2
echo "HEAD $SHA" > gpurun_out/${TAG}_gputest.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread >> gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -2 gpurun_out/${TAG}_gputest.log
echo "HEAD $SHA" > gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" >> gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
T0=$SECONDS
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
echo "bench wall $((SECONDS - T0)) s" | tee gpurun_out/${TAG}_bench_wall.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt -o run -- python3 bench.py --steps 20 --no-cpu > gpurun_out/${TAG}_kt.log 2>&1 || { echo "rocprof pass failed"; exit 1; }
echo "HEAD $SHA" > gpurun_out/${TAG}_n2.log
MLH_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu > gpurun_out/${TAG}_n2.json 2>> gpurun_out/${TAG}_n2.log || { tail -30 gpurun_out/${TAG}_n2.log; exit 1; }
echo done
