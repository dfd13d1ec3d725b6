# SQ stall counters (one counter-only pass, kernel-filtered) over a python command, then a
# per-kernel table.  usage: bash tools/pmc_sq.sh <kernel-regex> <tag> <python args...>
set -e
ROOT=$GRAFT_REPO_ROOT
RE=$1; TAG=$2; shift 2
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --kernel-include-regex "$RE" --output-format csv \
  -d $ROOT/gpurun_out/sq_$TAG -o run -- python3 $ROOT/$1 "${@:2}" > $ROOT/gpurun_out/sq_$TAG.log 2>&1
cd $ROOT && python tools/sq_table.py gpurun_out/sq_$TAG
