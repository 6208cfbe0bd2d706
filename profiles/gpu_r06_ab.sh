#!/bin/bash
# Round 6: optional GPU test files, then an interleaved A/B of library builds.
# Usage: gpu_r06_ab.sh <tag> <rounds> name=lib ...   (lib "" = the real build)
# TESTS="tests/x.py tests/y.py" runs those GPU tests first (stops on failure).
# One bench line per (round, name) into gpurun_out/r06/<tag>/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06/$1; R=$2; shift 2
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS > $O/pytest.log 2>&1 \
    || { tail -30 $O/pytest.log; exit 1; }
  tail -3 $O/pytest.log
fi
for i in $(seq 1 $R); do
  for nl in "$@"; do
    n=${nl%%=*}; lib=${nl#*=}
    TSDF_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu --steps 32 $BENCH_ARGS > $O/${n}_$i.json 2> $O/${n}_$i.err || { tail -3 $O/${n}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${n}_$i.json')); print('${n}_$i', d['value'], d['ms_per_step'], d.get('serial_kernel_ms_per_launch'), (d.get('parity') or {}).get('bitwise'))"
  done
done
