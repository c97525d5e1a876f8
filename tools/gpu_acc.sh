cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python tools/sumcheck_ab.py multilinear_amd/libmlhip.so tools/variants/libNONT.so multilinear_amd/libmlhip.so tools/variants/libNONT.so > gpurun_out/acc.log 2>&1 && \
for L in multilinear_amd/libmlhip.so tools/variants/libNONT.so; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pk -o run -- python3 tools/sumcheck_ab.py $L > gpurun_out/pk.log 2>&1 || exit 1
echo "== $L $(grep sumcheck_eq gpurun_out/pk.log | awk '{print $3}' | tr '\n' ' ')" >> gpurun_out/acc.log
python3 - gpurun_out/pk >> gpurun_out/acc.log <<'PY'
import csv, sys, glob
p = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(p)):
    n = r['Name']
    if any(k in n for k in ('eq_tail', 'fold_group_eq_kernel<6', 'corner_sums_lo', 'eq_setup')):
        print(f"  {n[:40]:40s} {int(r['Calls']):5d} avg {float(r['AverageNs'])/1e3:7.1f} us min {float(r['MinNs'])/1e3:7.1f}")
PY
rm -rf gpurun_out/pk
done
rc=$?; cat gpurun_out/acc.log; exit $rc
