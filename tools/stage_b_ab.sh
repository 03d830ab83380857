set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for v in new base; do
  if [ $v = base ]; then export MMT_LIB_PATH=/root/repo/multimot_track_amd/libmmt_sbbase.so; fi
  rm -rf gpurun_out/sb_$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sb_$v -o run -- python bench.py --steps 3 --warmup 1 --chunk 32 --no-cpu > gpurun_out/sb_$v.json 2> gpurun_out/sb_$v.log
  python tools/rocprof_summary.py gpurun_out/sb_$v gpurun_out/sb_${v}_stats.csv | grep "k_obj_stage_b\|k_flow_lm" || true
  rm -rf gpurun_out/sb_$v
done
