# HBM traffic per launch of the kernels matching a regex, from two counter-only rocprofv3 passes
# (FETCH_SIZE, then WRITE_SIZE: they do not fit one TCC pass) over a short config-4 bench.
# usage: bash tools/pmc_kernels.sh <kernel-regex> <tag>
set -e
ROOT=$GRAFT_REPO_ROOT
RE=$1; TAG=$2
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "$RE" --output-format csv \
    -d $ROOT/gpurun_out/pmck_${TAG}_$C -o run -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline \
    > $ROOT/gpurun_out/pmck_${TAG}_$C.log 2>&1
done
cd $ROOT && python tools/pmc_kernel_table.py gpurun_out/pmck_${TAG}_FETCH_SIZE gpurun_out/pmck_${TAG}_WRITE_SIZE
