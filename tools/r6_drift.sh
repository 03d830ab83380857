# Ego-drift ablation on the oracle (tools/drift_ablation.py): frames rendered on the GPU, one
# oracle process per configuration on the host cores.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 ${DRIFT_TIMEOUT:-900} python -u tools/drift_ablation.py --frames ${DRIFT_FRAMES:-3200} --out gpurun_out/drift > gpurun_out/drift.log 2>&1 || { tail -30 gpurun_out/drift.log; exit 1; }
tail -8 gpurun_out/drift.log
