# Round-5 close-out profile: the map branch's host stage times and kernel stats (map_profile.sh),
# then keyframe / other call times of the one-frame-per-call path
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/map_profile.sh r5z
timeout -k 10 300 python tools/one_frame_bench.py --frames 256 --start 8 > gpurun_out/r5z_one_frame.txt 2>&1
tail -8 gpurun_out/r5z_one_frame.txt
