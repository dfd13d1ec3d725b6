# kernel trace of the emulated per-rank step (bench.py --emulate-world W [...]): breakdown + one block's kernels
set -e
ROOT=$GRAFT_REPO_ROOT
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $ROOT/gpurun_out/prof_$TAG -o run -- python3 $ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > $ROOT/gpurun_out/pe_$TAG.log 2>&1
cd $ROOT && tail -1 gpurun_out/pe_$TAG.log | cut -c1-200
python tools/step_breakdown.py gpurun_out/prof_$TAG/run_results.db 4 70 > gpurun_out/pe_${TAG}_breakdown.txt
python tools/kernel_seq.py gpurun_out/prof_$TAG/run_results.db 5 > gpurun_out/pe_${TAG}_fwdblock.txt
python tools/kernel_seq.py gpurun_out/prof_$TAG/run_results.db -1 > gpurun_out/pe_${TAG}_bwd.txt
head -3 gpurun_out/pe_${TAG}_breakdown.txt
