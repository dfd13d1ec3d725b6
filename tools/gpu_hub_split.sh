# Round 6: the split point-hub backward -- its tests, the kernel bench (rocprof per kernel), config 4 / em8
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_point_block.py > gpurun_out/hub_split_tests.log 2>&1 || { tail -30 gpurun_out/hub_split_tests.log; exit 1; }
tail -1 gpurun_out/hub_split_tests.log
rm -rf gpurun_out/hubprof
(cd /tmp && TMPDIR=/tmp timeout -k 10 180 rocprofv3 --kernel-trace -d $R/gpurun_out/hubprof -o run -- python3 $R/tools/point_bench.py 25000 200000 > $R/gpurun_out/hubprof.log 2>&1) || { tail -20 gpurun_out/hubprof.log; exit 1; }
grep "kernel us" gpurun_out/hubprof.log
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/hub_split_c4.json 2> gpurun_out/hub_split_c4.err || { tail -20 gpurun_out/hub_split_c4.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/hub_split_c4.json').read().strip().splitlines()[-1]);print('c4 split', d['ms_per_step'])"
GASFM_PT_HUB_SPLIT=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/hub_onepass_c4.json 2> gpurun_out/hub_onepass_c4.err || { tail -20 gpurun_out/hub_onepass_c4.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/hub_onepass_c4.json').read().strip().splitlines()[-1]);print('c4 one-pass', d['ms_per_step'])"
timeout -k 10 300 python bench.py --emulate-world 8 --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/hub_split_em8.json 2> gpurun_out/hub_split_em8.err || { tail -20 gpurun_out/hub_split_em8.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/hub_split_em8.json').read().strip().splitlines()[-1]);print('em8 split', d['ms_per_step'])"
GASFM_PT_HUB_SPLIT=0 timeout -k 10 300 python bench.py --emulate-world 8 --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/hub_onepass_em8.json 2> gpurun_out/hub_onepass_em8.err || { tail -20 gpurun_out/hub_onepass_em8.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/hub_onepass_em8.json').read().strip().splitlines()[-1]);print('em8 one-pass', d['ms_per_step'])"
