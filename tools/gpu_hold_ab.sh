# Round 6: kernel timing with the stream held by a spin kernel (bench roofline mean_us) -- config 4 and the proxy,
# against the rocprof in-step durations of the same launches
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/hold_c4.json 2> gpurun_out/hold_c4.err || { tail -20 gpurun_out/hold_c4.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/hold_c4.json').read().strip().splitlines()[-1]);r=d['roofline'];a=d['roofline_attention'];print('c4', round(d['ms_per_step'],3), 'pbwd', round(r['mean_us'],1), round(r['frac'],3), 'attn', round(a['mean_us'],1), round(a['frac'],3), 'b2b', round(a['mean_us_back_to_back'],1))"
timeout -k 10 300 python bench.py --emulate-world 8 --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/hold_em8.json 2> gpurun_out/hold_em8.err || { tail -20 gpurun_out/hold_em8.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/hold_em8.json').read().strip().splitlines()[-1]);r=d['roofline'];a=d['roofline_attention'];print('em8', round(d['ms_per_step'],3), 'pbwd', round(r['mean_us'],1), round(r['frac'],3), 'attn', round(a['mean_us'],1), round(a['frac'],3), 'b2b', round(a['mean_us_back_to_back'],1))"
