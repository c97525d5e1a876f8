# Builds tools/bin/tree_tail_bench: merkle.hip with the per-level stamps
# (-DMLH_TREE_TS) + the library's other objects (make the library first).
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/bin /tmp/ttb
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function"
/opt/rocm/bin/hipcc $F -DMLH_TREE_TS -c multilinear_amd/csrc/merkle.hip -o /tmp/ttb/merkle.o
/opt/rocm/bin/hipcc $F -c tools/tree_tail_bench.hip -o /tmp/ttb/bench.o
OBJS=$(ls build/mlhip/*.o | grep -v '/merkle.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -o tools/bin/tree_tail_bench /tmp/ttb/bench.o /tmp/ttb/merkle.o $OBJS -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
