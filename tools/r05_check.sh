# Round-5 check on one box (ONE per round): the whole GPU
# suite, the N = 2 gloo rehearsal of the multi-GPU bench line, the N = 1 bench
# (with its CPU baselines) and its rocprofv3 kernel stats, smoke().
# usage: bash tools/r05_check.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -40 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -2 gpurun_out/${TAG}_gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
MLH_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/${TAG}_n2.json 2> gpurun_out/${TAG}_n2.err || { tail -30 gpurun_out/${TAG}_n2.err; exit 1; }
python -c "import json; d=[json.loads(l) for l in open('gpurun_out/${TAG}_n2.json') if l.startswith('{')][-1]; print({k: d.get(k) for k in ['value','comm','rccl_ranks','preflight','sharded_phases','sharded_ntt_verified']})"
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print({k:d.get(k) for k in ['value','ms_per_step','fri_commit_ms','fri_prove_ms','sumcheck_ms','pcs_prove_ms','pcs_verified','config5_rs_fri_prove_ms']}); print(d['roofline']['launch_avg_ms'], d['roofline']['frac'], d.get('cpu_baseline_fri_commit'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt -o run -- python3 bench.py --no-cpu > gpurun_out/${TAG}_kt.log 2>&1 || { tail -20 gpurun_out/${TAG}_kt.log; exit 1; }
echo check_done
