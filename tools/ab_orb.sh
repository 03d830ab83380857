# A/B kernel times of the ORB microbench: default libmmt.so vs libmmt_<sfx>.so builds
# (tools/ab_build.sh).  Usage (GPU box): bash tools/ab_orb.sh sfx...
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base "$@"; do
  if [ "$v" = base ]; then unset MMT_LIB_PATH; else export MMT_LIB_PATH=$PWD/multimot_track_amd/libmmt_$v.so; fi
  rm -rf gpurun_out/ab_$v
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_$v -o run -- python tools/orb_microbench.py 32 20 > gpurun_out/ab_$v.log 2>&1
  echo "== $v: $(grep batch= gpurun_out/ab_$v.log)"
  python tools/rocprof_summary.py gpurun_out/ab_$v gpurun_out/ab_${v}_stats.csv | grep mmt:: || true
done
