# round 4: config-3 training step (4-scene union batch, device data path) after the host-side
# savings, with the capture floor beside it, and the host profile of the fixed union step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/train_step_bench.py --steps 20 --warmup 3 --capture-floor > gpurun_out/r4_cfg3.jsonl 2> gpurun_out/r4_cfg3.err || { tail -30 gpurun_out/r4_cfg3.err; exit 1; }
cat gpurun_out/r4_cfg3.jsonl
timeout -k 10 300 python -u tools/host_profile_union.py --steps 10 --same-thread --top 40 > gpurun_out/r4_host_prof_after.txt 2> gpurun_out/r4_host_prof_after.err || { tail -30 gpurun_out/r4_host_prof_after.err; exit 1; }
head -1 gpurun_out/r4_host_prof_after.txt
