set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for e in 0 1; do
  if [ $e = 1 ]; then export MMT_OCT_ONE_PER_CU=1; fi
  rm -rf gpurun_out/oab
  MMT_ORB_SCHED=2 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/oab -o run -- python tools/orb_microbench.py 64 10 > gpurun_out/oab.log 2>&1
  echo "== one_per_cu=$e"; python tools/rocprof_summary.py gpurun_out/oab gpurun_out/oab_$e.csv | grep octree
  python tools/timeline.py gpurun_out/oab 0.7 | grep octree | tail -2
done
