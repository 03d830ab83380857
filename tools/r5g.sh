# Round 5: BA p3 one-wave LDL^T + p5 fold, KeyFrameCulling parity, k_fast multi-cell waves.
# LocalMapping / ORB / tracking tests, ba_bench, ORB window A/B over cells per wave, the batch-128
# ORB kernel summary, HBM traffic and SQ counters, k_fast phase clocks.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_localmap.py tests/test_gpu_track.py -m gpu -x -v --timeout 240 --timeout-method thread -k "orb or local_ba or localmap or map_graph or c3_long or culling" > gpurun_out/r5g_tests.log 2>&1 || { tail -40 gpurun_out/r5g_tests.log; exit 1; }
tail -3 gpurun_out/r5g_tests.log
MMT_BA_PROFILE=1 timeout -k 10 200 python tools/ba_bench.py --reps 64 > gpurun_out/r5g_ba.txt 2>&1 || { tail -20 gpurun_out/r5g_ba.txt; exit 1; }
tail -4 gpurun_out/r5g_ba.txt
for c in 1 4 1 4 8 2; do
  MMT_FAST_CPW=$c timeout -k 10 120 python tools/orb_window_bench.py 128 20 > gpurun_out/r5g_cpw$c.log 2>&1 || { tail -20 gpurun_out/r5g_cpw$c.log; exit 1; }
  echo "cpw=$c $(cat gpurun_out/r5g_cpw$c.log)"
done
# ORB window at batch 128 only: kernel trace summary (standalone kernel times: one stream)
rm -rf gpurun_out/orbk
MMT_ORB_SCHED=2 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/orbk -o run -- python tools/orb_window_bench.py 128 5 > gpurun_out/r5g_orbk.log 2>&1 || { tail -20 gpurun_out/r5g_orbk.log; exit 1; }
grep window_ms gpurun_out/r5g_orbk.log
find gpurun_out/orbk -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} gpurun_out/r5g_orb_kstats.csv
timeout -k 10 400 bash tools/orb_traffic.sh 128 > gpurun_out/r5g_orbt.log 2>&1 || { tail -20 gpurun_out/r5g_orbt.log; exit 1; }
cat gpurun_out/r5g_orbt.log
# k_fast phase clocks (libmmt_prof.so built with PROF_DEFS=-DMMT_FAST_PROFILE)
MMT_LIB_PATH=multimot_track_amd/libmmt_prof.so MMT_ORB_SCHED=2 timeout -k 10 120 python tools/orb_window_bench.py 128 1 > gpurun_out/r5g_fastprof.log 2>&1 || { tail -20 gpurun_out/r5g_fastprof.log; exit 1; }
grep -c fastprof gpurun_out/r5g_fastprof.log
# SQ counters per ORB kernel at batch 128
B=128 timeout -k 10 300 bash tools/orb_pmc_sq.sh r5sq > gpurun_out/r5g_sq.log 2>&1 || { tail -20 gpurun_out/r5g_sq.log; exit 1; }
cat gpurun_out/r5sq_summary.txt
