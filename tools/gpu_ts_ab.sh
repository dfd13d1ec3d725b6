# same-box A/B of the training-step bench: ab_old/ (an older tree's Python, same library) vs this tree
set -e
mkdir -p gpurun_out
for r in 1 2; do
  for t in ab_old .; do
    (cd $t && timeout -k 10 300 python tools/train_step_bench.py --steps 6 --outliers 0.1 > $GRAFT_REPO_ROOT/gpurun_out/tsab_$r.log 2>&1)
    echo "$t: $(grep ms_per_step gpurun_out/tsab_$r.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['ms_per_step'],1), round(d['ms_data_prep'],1), round(d['ms_fwd_bwd_loss_errors'],1))")"
  done
done
