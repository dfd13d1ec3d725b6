set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5a_tests.log 2>&1 || { grep -B5 -A40 "^E \|FAILED\|Error" gpurun_out/r5a_tests.log | head -120; tail -3 gpurun_out/r5a_tests.log; exit 1; }
tail -1 gpurun_out/r5a_tests.log
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r5a_c4.json 2> gpurun_out/r5a_c4.err || { tail -20 gpurun_out/r5a_c4.err; exit 1; }
tail -1 gpurun_out/r5a_c4.json | cut -c1-300
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --emulate-world 8 > gpurun_out/r5a_em8.json 2> gpurun_out/r5a_em8.err || { tail -20 gpurun_out/r5a_em8.err; exit 1; }
tail -1 gpurun_out/r5a_em8.json | cut -c1-300
