# The -m gpu suite with the given test file(s) first (fail fast on new tests), then the rest.
# Usage: bash tools/r6_suite.sh <tag> [first test files...]
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
shift || true
IGN=()
for f in "$@"; do IGN+=("--ignore=$f"); done
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_first_$TAG.log 2>&1 || { tail -60 gpurun_out/gpu_first_$TAG.log; exit 1; }
  tail -3 gpurun_out/gpu_first_$TAG.log
fi
timeout -k 10 700 python -u -m pytest tests "${IGN[@]}" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -60 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -3 gpurun_out/gpu_tests_$TAG.log
