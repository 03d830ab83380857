# several sequences per GPU against the hardware queue count (GPU_MAX_HW_QUEUES)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "8 0" "8 16" "8 32" "4 16"; do
set -- $cfg
timeout -k 10 500 python bench.py --seqs-per-gpu $1 --hw-queues $2 --steps 4 --warmup 2 --no-cpu --single-frames 0 --c2-steps 0 --rank-parity-frames 0 > gpurun_out/r5c_k$1_q$2.json 2> gpurun_out/r5c_k$1_q$2.err || { tail -20 gpurun_out/r5c_k$1_q$2.err; exit 1; }
python -c "import json,sys; d=json.load(open('gpurun_out/r5c_k$1_q$2.json')); print('K', $1, 'queues', d['config']['gpu_max_hw_queues'], d['value'], d['valid'], d['roofline']['launch_ms'])"
done
