set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for b in 32 48 64 96 128; do
  timeout -k 10 120 python tools/orb_window_bench.py $b 10 2>&1 | grep batch=
done
