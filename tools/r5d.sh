# several sequences per GPU: the object streams' priority classes (MMT_D3_PRIO, MMT_RANSAC_CU_MASK)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "0 0" "1 0" "2 0" "0 1"; do
set -- $cfg
MMT_D3_PRIO=$1 MMT_RANSAC_CU_MASK=$2 timeout -k 10 400 python bench.py --seqs-per-gpu 4 --steps 4 --warmup 2 --no-cpu --single-frames 0 --c2-steps 0 --rank-parity-frames 0 > gpurun_out/r5d_$1_$2.json 2> gpurun_out/r5d_$1_$2.err || { tail -20 gpurun_out/r5d_$1_$2.err; exit 1; }
python -c "import json,sys; d=json.load(open('gpurun_out/r5d_$1_$2.json')); print('D3_PRIO', $1, 'CU_MASK', $2, d['value'], d['valid'], d['roofline']['launch_ms'])"
done
