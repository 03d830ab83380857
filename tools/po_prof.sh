# D1 phase clocks inside the tracker (MMT_PO_PROFILE build, tools/build_prof_lib.sh)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MMT_LIB_PATH=multimot_track_amd/libmmt_prof.so timeout -k 10 300 python bench.py --steps 2 --warmup 1 --chunk 64 --no-cpu --single-frames 0 --c2-steps 0 > gpurun_out/po_prof.json 2> gpurun_out/po_prof.err
grep -c "po profile" gpurun_out/po_prof.err
