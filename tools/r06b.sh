set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python tools/hip_diag.py > gpurun_out/r06b_diag.txt 2>&1; cat gpurun_out/r06b_diag.txt | sort -u
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -3
timeout -k 10 120 python tools/coop_pipeline.py tools/variants/libPROF.so > gpurun_out/r06b_coop.txt 2>&1; cat gpurun_out/r06b_coop.txt
