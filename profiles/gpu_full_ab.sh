# Full GPU parity suite, then every variant build's bench line beside the default build.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/fab}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
STEPS=${STEPS:-32} bash profiles/variants.sh $OUT
