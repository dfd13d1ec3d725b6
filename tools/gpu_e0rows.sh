# Block-0 prologue in row order (GASFM_E0_ROWS): its tests, the model fixtures, a same-box bench A/B,
# then a kernel-trace profile of the default bench.
set -e
mkdir -p gpurun_out
bash tools/gpu_env_ab.sh GASFM_E0_ROWS tests/test_gpu_edge_block.py tests/test_gpu_model.py tests/test_gpu_train_step.py
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e0 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_e0.log 2>&1
ls -R gpurun_out/prof_e0 | head -20
