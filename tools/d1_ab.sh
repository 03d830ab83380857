# D1 kernel A/B: the LDS kernel (MMT_PO_VARIANT=0) against the register kernel, per edge count.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in ${NS:-400 1000 1500 2000}; do
  for v in 0 1; do
    MMT_PO_VARIANT=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/d1_${n}_$v -o run -- python tools/d1_bench.py $n 50 > gpurun_out/d1_${n}_$v.log 2>&1
    f=$(find gpurun_out/d1_${n}_$v -name '*kernel_stats.csv' -print -quit)
    echo "n=$n variant=$v $(grep -h k_pose_opt "$f" | cut -d, -f1-5)"
    rm -rf gpurun_out/d1_${n}_$v
  done
done
