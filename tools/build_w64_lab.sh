#!/bin/bash
# Lab builds of the span library whose prefill attention is the one-wave-per-SIMD body of
# tools/labsrc/attn_w64.hip, compiled under extra defines ->
# tools/probe_libs/libinferd_span_<name>.so (tools/attn_ab.py / tools/span_ab.py load them).
#   usage: tools/build_w64_lab.sh name='-DFOO=1 ...' ...
set -e
cd "$(dirname "$0")/../inferd_amd/csrc"
make -j8 >/dev/null
mkdir -p ../../tools/probe_libs
F="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -Wall -Wno-unused-result -fno-honor-nans -fno-slp-vectorize"
/opt/rocm/bin/hipcc $F -DATTN_W64 -c attention.hip -o build/attention_lab_w64.o
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  /opt/rocm/bin/hipcc $F $flags -c ../../tools/labsrc/attn_w64.hip -o build/attn_w64_lab_$name.o
  objs="build/elementwise.o build/gemm.o build/span.o build/kvtable.o build/probe.o"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../../tools/probe_libs/libinferd_span_$name.so $objs \
    build/attention_lab_w64.o build/attn_w64_lab_$name.o
done
