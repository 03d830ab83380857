# Round-6 ORB evidence for the final build at batch 128: HBM traffic (FETCH_SIZE / WRITE_SIZE in
# separate --pmc passes), SQ counters per ORB kernel, and standalone kernel times (one stream).
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/orb_traffic.sh 128
B=128 bash tools/orb_pmc_sq.sh r6sq
B=128 bash tools/orb_sched.sh 2
rm -rf gpurun_out/r6sq_p1 gpurun_out/r6sq_p2 gpurun_out/sched_2
echo done
