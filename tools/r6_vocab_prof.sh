# Kernel trace of the vocabulary bench against the same run without the vocabulary (short runs);
# the rocpd databases are summarised on the box and removed (gpurun copies back <= 64 MiB).  Then
# the map profile (MMT_MAP_PROFILE=1) and the BA host phases (MMT_BA_PROFILE=1) of the vocabulary run.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-vp}
common="--steps 4 --warmup 5 --no-cpu --single-frames 0 --c2-steps 0"
for v in voc novoc; do
  extra=""
  [ $v = novoc ] && extra="--vocabulary="
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/${tag}_kt_$v -o run -- python bench.py $common $extra > gpurun_out/${tag}_kt_$v.json 2> gpurun_out/${tag}_kt_$v.err
  python tools/rocpd_summary.py /tmp/${tag}_kt_$v | grep -v "at::native\|Cijk_\|reduce_kernel" > gpurun_out/${tag}_kt_$v.txt 2>&1
  rm -rf /tmp/${tag}_kt_$v
done
MMT_MAP_PROFILE=1 MMT_BA_PROFILE=1 timeout -k 10 300 python bench.py $common > gpurun_out/${tag}_mp.json 2> gpurun_out/${tag}_mp.err
head -40 gpurun_out/${tag}_kt_voc.txt
head -40 gpurun_out/${tag}_kt_novoc.txt
grep -h "profile\]" gpurun_out/${tag}_mp.err | tail -8
