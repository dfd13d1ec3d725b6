# Kernel trace of the rank-0-of-8 proxy (or the bench with BENCH_ARGS) with each library given (gasfm_amd/<lib>): one step's
# breakdown per library, and the global attention / view chain / global chain kernels' means.
set -o pipefail
ROOT=$PWD
mkdir -p gpurun_out
for lib in "$@"; do
  (cd /tmp && TMPDIR=/tmp GASFM_LIB=$ROOT/gasfm_amd/$lib timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/pg_$lib -o run -- python3 $ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS---emulate-world 8}) > gpurun_out/pg_$lib.log 2>&1 || { tail -5 gpurun_out/pg_$lib.log; exit 1; }
  python tools/step_breakdown.py /tmp/pg_$lib/run_results.db 4 70 > gpurun_out/pg_${lib%.so}_breakdown.txt || exit 1
  echo "== $lib"; head -1 gpurun_out/pg_${lib%.so}_breakdown.txt
  grep -E "${PAT:-gatt|vc_|gnode}" gpurun_out/pg_${lib%.so}_breakdown.txt | grep -v "kernels  other" || true
done
