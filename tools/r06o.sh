set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06o}
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print({k:d.get(k) for k in ['value','ms_per_step','fri_commit_ms','fri_prove_ms','sumcheck_ms','pcs_prove_ms','pcs_verified','config5_rs_fri_prove_ms','eq_table_ms']}); r=d['roofline']; print(r['launch_avg_ms'], r['frac'], r.get('launch_timing_overhead_us')); print(d['kernels'])"
