# Object path placement, interleaved in one process after the pose-opt launch order change:
# inline split (default), inline in the first chain (MMT_OBJ_SPLIT=0), worker thread (MMT_OBJ_THREAD=1)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u tools/ab_interleave.py --rounds 4 'MMT_OBJ_THREAD=0' 'MMT_OBJ_SPLIT=0' 'MMT_OBJ_THREAD=1' > gpurun_out/r5zg.txt 2>&1
tail -4 gpurun_out/r5zg.txt
