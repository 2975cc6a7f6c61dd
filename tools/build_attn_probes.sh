#!/bin/bash
# Lab builds of the span library with attn_prefill.hip compiled under extra defines (timing-only
# variants such as AP_PROBE=n, wrong output) -> tools/probe_libs/libinferd_span_<name>.so; select
# one with INFERD_LIB.   usage: tools/build_attn_probes.sh name='-DAP_PROBE=1 ...' ...
set -e
cd "$(dirname "$0")/../inferd_amd/csrc"
make -j8 >/dev/null
mkdir -p ../../tools/probe_libs
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -Wall -Wno-unused-result -fno-honor-nans \
    -fno-slp-vectorize $flags -c attn_prefill.hip -o build/attn_prefill_lab_$name.o 2>/dev/null
  objs=$(ls build/*.o | grep -v attn_prefill)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../../tools/probe_libs/libinferd_span_$name.so $objs build/attn_prefill_lab_$name.o
done
