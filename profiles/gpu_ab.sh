# A/B round: parity tests of the default build, then every variant's bench line.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_growth.py tests/test_voxblox.py tests/test_literal.py -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
STEPS=${STEPS:-16} bash profiles/variants.sh $OUT
