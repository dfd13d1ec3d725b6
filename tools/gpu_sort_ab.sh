# Round 6: length-sorted items for the grouped point-direction forward -- tests, kernel bench, A/B
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_attn_dispatch.py tests/test_gpu_attention.py > gpurun_out/sort_tests.log 2>&1 || { tail -30 gpurun_out/sort_tests.log; exit 1; }
tail -1 gpurun_out/sort_tests.log
for w in 256 0; do
  GASFM_ATTN_SORT_WINDOW=$w timeout -k 10 120 python tools/attn_bench.py > gpurun_out/sort_attn_$w.txt 2>&1 || { tail -20 gpurun_out/sort_attn_$w.txt; exit 1; }
  echo "window $w"; grep proj2scenepoint gpurun_out/sort_attn_$w.txt
done
for w in 256 0 256 0; do
  GASFM_ATTN_SORT_WINDOW=$w timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/sort_c4_$w.json 2> gpurun_out/sort_c4_$w.err || { tail -20 gpurun_out/sort_c4_$w.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/sort_c4_$w.json').read().strip().splitlines()[-1]);print('c4 window $w', round(d['ms_per_step'],3), 'attn_fwd us', round(d['roofline_attention']['mean_us'],1), round(d['roofline_attention']['frac'],3))"
done
for w in 256 0; do
  GASFM_ATTN_SORT_WINDOW=$w timeout -k 10 300 python bench.py --emulate-world 8 --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/sort_em8_$w.json 2> gpurun_out/sort_em8_$w.err || { tail -20 gpurun_out/sort_em8_$w.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/sort_em8_$w.json').read().strip().splitlines()[-1]);print('em8 window $w', round(d['ms_per_step'],3), 'attn_fwd us', round(d['roofline_attention']['mean_us'],1), round(d['roofline_attention']['frac'],3))"
done
