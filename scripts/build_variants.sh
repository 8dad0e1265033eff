#!/bin/bash
# Build A/B variants of libdervet_hip.so into scripts/_variants/ (dev helper; see scripts/probe_iter.py).
set -e
cd "$(dirname "$0")/.."
mkdir -p scripts/_variants
C=der-vet_amd/csrc
for v in "$@"; do
  name=${v%%:*}; defs=${v#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -Wno-unused-value \
    $defs -o scripts/_variants/lib_$name.so $C/dvh_api.cpp $C/dvh_kernels.hip $C/dvh_band.hip $C/dvh_chain.hip $C/dvh_build.hip $C/dvh_sweep.hip $C/dvh_series.hip $C/dvh_route.hip $C/dvh_large.hip $C/dvh_outage.hip $C/dvh_validate.cpp &
done
wait
