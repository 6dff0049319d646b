# Same-box A/B of bench.py lines: alternate two environment settings N times.
#   bash tools/ab_bench.sh TAG N "ENV_A" "ENV_B" [bench args...]
# e.g. bash tools/ab_bench.sh r06m 2 "MARLMAZE_WG_DMA=0" "" --no-cpu-baseline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; N=$2; A=$3; B=$4; shift 4
R=gpurun_out/$TAG; mkdir -p $R
for i in $(seq 1 $N); do
  for v in A B; do
    e=$A; [ $v = B ] && e=$B
    env $e timeout -k 10 300 python -u bench.py "$@" > $R/ab_${v}_$i.log 2>&1 || { tail -20 $R/ab_${v}_$i.log; exit 1; }
    tail -1 $R/ab_${v}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', '$e', round(d['value']/1e6,4), 'Msteps/s update', round(d['update_ms_per_iter'],2), 'rollout', round(d['rollout_ms_per_iter'],2))"
  done
done
