# A/B with the vocabulary, map profile of the 8-step bench (MMT_MAP_PROFILE=1), interleaved twice:
# the LocalMapping stream at normal / the greatest priority (MMT_LM_PRIO), and the local BA's
# heavy-point threshold 8 (libmmt.so) / 4 / 2 (tools/ab_build.sh h4|h2 --src mmt_ba.hip).
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-ab}
L=$PWD/multimot_track_amd
common="--steps 8 --warmup 5 --no-cpu --single-frames 0 --c2-steps 0"
for r in 1 2; do
  for v in base:libmmt.so:normal high:libmmt.so:high h4:libmmt_h4.so:normal h2:libmmt_h2.so:normal; do
    n=${v%%:*}; rest=${v#*:}; lib=${rest%%:*}; p=${rest#*:}
    MMT_LIB_PATH=$L/$lib MMT_LM_PRIO=$p MMT_MAP_PROFILE=1 timeout -k 10 300 python bench.py $common > gpurun_out/${tag}_${n}_$r.json 2> gpurun_out/${tag}_${n}_$r.err
    echo "$n $r $(python -c "import json; print(json.load(open('gpurun_out/${tag}_${n}_$r.json'))['value'])") $(grep -h 'host wall us per keyframe' gpurun_out/${tag}_${n}_$r.err | grep -o 'LocalBundleAdjustment [0-9.]*') $(grep -h 'per keyframe, us' gpurun_out/${tag}_${n}_$r.err | tr ',' '\n' | grep -E 'PNK ComputeBoW' | tr -d '\n')"
  done
done
