# k_fast tile stride A/B (MMT_FAST_FS 40 = libmmt.so, 48 / 52 / 96 = tools/ab_build.sh fsNN):
# interleaved orb_microbench rounds at batch 128, then per library a kernel-trace stats pass and an
# SQ pass with the LDS bank-conflict counter.  Usage: bash tools/r6_fs_ab.sh <tag>
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-fsab}
L=multimot_track_amd
libs="$PWD/$L/libmmt.so $PWD/$L/libmmt_fs48.so $PWD/$L/libmmt_fs52.so $PWD/$L/libmmt_fs96.so"
out=gpurun_out/${tag}.txt
: > $out
for r in 1 2 3; do
  for lib in $libs; do
    echo -n "$(basename $lib) " >> $out
    MMT_LIB_PATH=$lib timeout -k 10 120 python tools/orb_microbench.py 128 20 >> $out 2>&1
  done
done
for lib in $libs; do
  b=$(basename $lib .so)
  MMT_LIB_PATH=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_kt_$b -o run -- python tools/orb_microbench.py 128 10 > gpurun_out/${tag}_kt_$b.log 2>&1
  MMT_LIB_PATH=$lib timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/${tag}_sq_$b -o run -- python tools/orb_microbench.py 128 3 > gpurun_out/${tag}_sq_$b.log 2>&1
  python tools/pmc_summary.py gpurun_out/${tag}_sq_$b >> gpurun_out/${tag}_sq_summary.txt 2>&1 || true
done
cat $out
