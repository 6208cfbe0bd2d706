# GPU parity suite, then the PCIe-inclusive host-pointer rate (profiles/host_path.py) with 1 and 4
# staging threads.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/host}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for t in 1 4; do
  TSDF_PACK_THREADS=$t timeout -k 10 300 python3 profiles/host_path.py > $OUT/host_path_t$t.json 2> $OUT/h$t.err || { tail -5 $OUT/h$t.err; exit 1; }
  echo "threads $t: $(cat $OUT/host_path_t$t.json)"
done
