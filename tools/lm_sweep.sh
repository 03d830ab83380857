set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in ${CFGS:-default 64x4 128x4 256x2 256x4 256x1}; do
  if [ "$cfg" = default ]; then unset MMT_LM_CONFIG; else export MMT_LM_CONFIG=$cfg; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lm_$cfg -- python3 tools/lm_microbench.py > gpurun_out/lm_$cfg.log 2>&1
  python3 tools/rocprof_summary.py /tmp/lm_$cfg gpurun_out/lm_$cfg.csv > /dev/null
done
