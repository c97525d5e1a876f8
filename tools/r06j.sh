set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06j}; K=${2:-"production_shape and 2"}
export MLH_TEST_PROGRESS=gpurun_out/${T}_prog.txt
( while true; do date >> gpurun_out/${T}_hb.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 560 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_sharded_threads_gpu.py -k "$K" > gpurun_out/${T}_t.log 2>&1 || { tail -60 gpurun_out/${T}_t.log; tail -5 gpurun_out/${T}_prog.txt; exit 1; }
tail -3 gpurun_out/${T}_t.log; tail -4 gpurun_out/${T}_prog.txt
