# N = 2 rehearsal of the driver's multi-GPU bench on a one-GPU box: both ranks
# share cuda:0 and exchange through gloo (the script's logic, not a result).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export MLH_BENCH_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu > gpurun_out/n2_bench.json 2> gpurun_out/n2_bench.err || { tail -30 gpurun_out/n2_bench.err; exit 1; }
cat gpurun_out/n2_bench.json
