#!/bin/bash
# Lab builds of the span library with ONE source compiled under extra defines (timing-only or
# layout variants) -> tools/probe_libs/libinferd_span_<name>.so; select one with INFERD_LIB.
#   usage: tools/build_probes.sh <source.hip> name='-DFOO=1 ...' ...
set -e
src=$1; shift
cd "$(dirname "$0")/../inferd_amd/csrc"
make -j8 >/dev/null
mkdir -p ../../tools/probe_libs
base=${src%.hip}
extra=""
case $base in attention|attn_prefill) extra="-fno-honor-nans -fno-slp-vectorize";; esac
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -Wall -Wno-unused-result $extra \
    $flags -c $src -o build/${base}_lab_$name.o
  objs=$(ls build/*.o | grep -v "_lab_" | grep -v "/$base.o")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../../tools/probe_libs/libinferd_span_$name.so $objs build/${base}_lab_$name.o
done
