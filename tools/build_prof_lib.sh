# libmmt_prof.so: libmmt built with extra defines (default -DMMT_PO_PROFILE), for
# MMT_LIB_PATH=multimot_track_amd/libmmt_prof.so runs of tools/.
set -e
cd "$(dirname "$0")/../multimot_track_amd"
D=${PROF_DEFS:--DMMT_PO_PROFILE}
mkdir -p /tmp/mmt_prof_build
for f in csrc/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
    -fhip-fp32-correctly-rounded-divide-sqrt -Xarch_host -mpopcnt $D -c $f -o /tmp/mmt_prof_build/$(basename $f).o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o libmmt_prof.so /tmp/mmt_prof_build/*.o
