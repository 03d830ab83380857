# A/B experiment: relink libmmt with one source rebuilt under extra defines.
# usage: tools/ab_build.sh <suffix> [--src mmt_lm.hip] <hipcc defines...>
#        -> multimot_track_amd/libmmt_<suffix>.so   (default source: mmt_orb.hip)
set -e
cd "$(dirname "$0")/.."
sfx=$1; shift
src=mmt_orb.hip
if [ "$1" = "--src" ]; then src=$2; shift 2; fi
B=multimot_track_amd/build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt "$@" -c multimot_track_amd/csrc/$src -o $B/${src%.hip}_$sfx.o
objs=$(ls $B/*.hip.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o multimot_track_amd/libmmt_$sfx.so $objs $B/${src%.hip}_$sfx.o
