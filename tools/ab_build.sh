# A/B experiment: relink libmmt with mmt_orb.hip rebuilt under extra defines.
# usage: tools/ab_build.sh <suffix> <hipcc defines...>   -> multimot_track_amd/libmmt_<suffix>.so
set -e
cd "$(dirname "$0")/.."
sfx=$1; shift
B=multimot_track_amd/build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt "$@" -c multimot_track_amd/csrc/mmt_orb.hip -o $B/mmt_orb_$sfx.o
objs=$(ls $B/*.hip.o | grep -v mmt_orb.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o multimot_track_amd/libmmt_$sfx.so $objs $B/mmt_orb_$sfx.o
