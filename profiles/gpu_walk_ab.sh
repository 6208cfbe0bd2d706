# Single-walk A/B: every variant build's bench line, then PMC traffic of the default build.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/walkab}
mkdir -p $OUT
STEPS=${STEPS:-16} bash profiles/variants.sh $OUT || exit 1
bash profiles/collect_pmc.sh $OUT/pmc > $OUT/pmc.log 2>&1 || exit 1
python3 -c "import json; d=json.load(open('$OUT/pmc/traffic.json'))['bytes_per_launch']; print({k: round(v/1e6) for k, v in d.items()}, round(sum(d.values())/1e6))"
