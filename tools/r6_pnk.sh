# ProcessNewKeyFrame with the keyframe's BoW descent overlapped: the vocabulary / LocalMapping GPU
# tests, then the 8-step bench under MMT_MAP_PROFILE=1 (the PNK block times on stderr).
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-pnk}
timeout -k 10 600 python -u -m pytest tests/test_gpu_vocab.py tests/test_gpu_localmap.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
MMT_MAP_PROFILE=1 timeout -k 10 300 python bench.py --steps 8 --warmup 5 --no-cpu --single-frames 0 --c2-steps 0 > gpurun_out/${tag}_mp.json 2> gpurun_out/${tag}_mp.err
python -c "import json; d=json.load(open('gpurun_out/${tag}_mp.json')); print('bench', d['value'], d['valid'])"
grep -h "profile\]" gpurun_out/${tag}_mp.err
