# round-5 quick check: the distributed suite, the edge / model parity tests, then config 4 and the
# rank-0-of-8 proxy (prints as it goes: the silence watchdog sees progress)
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_distributed.py -m gpu > gpurun_out/r5c_dist.log 2>&1 || { grep -B5 -A40 "^E \|FAILED" gpurun_out/r5c_dist.log | grep -v "hostname\|amdgpu.ids\|Gloo" | head -100; exit 1; }
tail -1 gpurun_out/r5c_dist.log
timeout -k 10 900 $T tests -m gpu --deselect tests/test_distributed.py "$@" > gpurun_out/r5c_tests.log 2>&1 || { grep -B5 -A40 "^E \|FAILED" gpurun_out/r5c_tests.log | head -100; exit 1; }
tail -1 gpurun_out/r5c_tests.log
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r5c_c4.json 2> gpurun_out/r5c_c4.err || { tail -20 gpurun_out/r5c_c4.err; exit 1; }
tail -1 gpurun_out/r5c_c4.json | cut -c1-250
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --emulate-world 8 > gpurun_out/r5c_em8.json 2> gpurun_out/r5c_em8.err || { tail -20 gpurun_out/r5c_em8.err; exit 1; }
tail -1 gpurun_out/r5c_em8.json | cut -c1-250
