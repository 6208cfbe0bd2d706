# Bench A/B of runtime settings and A/B builds, interleaved: every case runs ROUNDS times in turn
# (ABAB...), so drift on the box hits all cases alike.  A case is "name:VAR=v,VAR2=w" (environment
# for bench.py; TSDF_HIP_LIB=<path> selects an A/B build from `make variants`).
#   bash profiles/gpu_ab_env.sh <out> "base:" "wide:TSDF_COUNT_WIDE=1000000" ...
set -o pipefail
export TMPDIR=/tmp
O=$1; shift
mkdir -p "$O"
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in "$@"; do
    n=${c%%:*}; e=${c#*:}
    env $(echo "$e" | tr ',' ' ') timeout -k 10 200 python3 bench.py --steps ${STEPS:-32} --no-cpu \
        $BENCH_ARGS > "$O/${n}_$r.json" 2> "$O/${n}_$r.err" || { echo "$n failed"; tail -3 "$O/${n}_$r.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${n}_$r.json')); print('$n', $r, d['value'], d['ms_per_step'], d['kernel_ms_per_launch'])"
  done
done
