set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in ${CFGS:-default 64 128 256}; do
  if [ "$cfg" = default ]; then unset MMT_LM_THREADS; else export MMT_LM_THREADS=$cfg; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lm_$cfg -- python3 tools/lm_microbench.py > gpurun_out/lm_$cfg.log 2>&1
  python3 tools/rocprof_summary.py /tmp/lm_$cfg gpurun_out/lm_$cfg.csv > /dev/null
done
