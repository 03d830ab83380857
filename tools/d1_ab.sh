# D1 kernel A/B per edge count: the LDS kernel (MMT_PO_VARIANT=0), the register kernel (1), the
# light-trial kernel with lambda candidates (2, default).
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in ${NS:-400 1000 1500 2000}; do
  for v in ${VARIANTS:-0 1 2}; do
    MMT_PO_VARIANT=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/d1_${n}_$v -o run -- python tools/d1_bench.py $n 50 > gpurun_out/d1_${n}_$v.log 2>&1
    f=$(find gpurun_out/d1_${n}_$v -name '*kernel_stats.csv' -print -quit)
    echo "n=$n variant=$v $(grep -h k_pose_opt "$f" | cut -d, -f1-5)"
    rm -rf gpurun_out/d1_${n}_$v
  done
done
