# Single-walk front end: GPU parity suite, then the bench in both walk modes.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/walk}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for w in two single; do
  timeout -k 10 300 python3 bench.py --no-cpu --walk $w > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -20 $OUT/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$w.json')); print('$w', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'], d['roofline']['path_frac'])"
done
