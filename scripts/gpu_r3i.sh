set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r3i; mkdir -p $O
for S in 1 16 24; do
  ONI_POST_SAMPLES=$S timeout -k 10 200 python -u tools/recall_probe.py --source flow --n 12500000 --wide > $O/flow_wide_S$S.json 2> $O/flow_wide_S$S.err || exit 1
done
for S in 16 24; do
  ONI_POST_SAMPLES=$S timeout -k 10 200 python -u tools/recall_probe.py --source proxy --n 2000000 --anomaly-kind rare > $O/proxy_S$S.json 2> $O/proxy_S$S.err || exit 1
  ONI_POST_SAMPLES=$S timeout -k 10 200 python -u tools/recall_probe.py --source flow --n 12500000 > $O/flow_S$S.json 2> $O/flow_S$S.err || exit 1
done
