# FETCH_SIZE / WRITE_SIZE calibration (profiles/tools/fetch_calib.hip), one counter per pass.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/calib}
mkdir -p $OUT
timeout -k 10 60 ./profiles/tools/fetch_calib > $OUT/bytes.json || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c -d $OUT/$c -o pmc --output-format csv -- ./profiles/tools/fetch_calib > $OUT/$c.log 2>&1 || { tail -5 $OUT/$c.log; exit 1; }
done
find $OUT -name '*counter_collection.csv'
