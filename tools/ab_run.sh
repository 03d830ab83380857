# A/B timing of ORB kernels: default libmmt.so vs each libmmt_<sfx>.so given as arguments.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base "$@"; do
  if [ "$v" = base ]; then unset MMT_LIB_PATH; else export MMT_LIB_PATH=$PWD/multimot_track_amd/libmmt_$v.so; fi
  rm -rf gpurun_out/ab_$v
  timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/ab_$v -o run -- python tools/orb_microbench.py ${B:-64} 20 > gpurun_out/ab_$v.log 2>&1
  echo "== $v kitti: $(grep batch= gpurun_out/ab_$v.log)"
  python tools/dispatch_times.py gpurun_out/ab_$v/run_results.db | grep -v "k_resize"
  ORB_MB_SCENE=synthetic timeout -k 10 120 python tools/orb_microbench.py ${B:-64} 20 2>&1 | tail -1 | sed "s/^/== $v synthetic: /"
  timeout -k 10 120 python tools/orb_window_bench.py ${B:-64} 20 2>&1 | grep batch= | sed "s/^/== $v window: /"
done
