# Builds mh_micro binaries for kernel variants: VARIANTS="name:-DFLAGS ..." (default: current code)
set -e
cd "$(dirname "$0")"
C=../../pet_posterior_distribution_amd/csrc
for v in ${VARIANTS:-base:}; do
  name=${v%%:*}; flags=$(echo "${v#*:}" | tr "," " ")
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../include -DMH_VARIANT="\"$name\"" -mllvm -disable-machine-licm $flags \
    mh_micro.cpp $C/mh_kernels.hip -x hip $C/mh_api.cpp -o mh_micro_$name &
done
wait
