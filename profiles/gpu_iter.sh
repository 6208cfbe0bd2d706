# One build -> measure iteration: the named GPU tests, then bench lines of the given semantics.
#   bash profiles/gpu_iter.sh <outdir> "<pytest args>" "<sem1> <sem2> ..."
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/iter}
mkdir -p $OUT
if [ -n "$2" ]; then
  timeout -k 10 600 python3 -u -m pytest $2 -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
for sem in ${3:-vdbfusion}; do
  timeout -k 10 200 python3 bench.py --no-cpu --steps ${STEPS:-16} --semantics $sem $BENCH_ARGS > $OUT/bench_$sem.json 2> $OUT/bench_$sem.err || { tail -5 $OUT/bench_$sem.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$sem.json')); print('$sem', d['value'], d['kernel_ms_per_launch'])"
done
