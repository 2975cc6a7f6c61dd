#!/bin/bash
# A/B decode bench on one box: alternate the in-tree library with tools/ab/libbase.so
# (a build of the previous source), N rounds each; prints value and ms/step per run.
# usage: tools/ab_bench.sh [rounds] [extra bench args...]
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
n=${1:-2}; shift
for i in $(seq 1 "$n"); do
  for v in new base; do
    if [ $v = base ]; then export INFERD_LIB=$PWD/tools/ab/libbase.so; else unset INFERD_LIB; fi
    timeout -k 10 200 python bench.py --steps 32 --warmup 4 --no-cpu-baseline --no-profile --no-prefill-line "$@" > gpurun_out/ab_$v$i.log 2>&1 || exit $?
    python3 -c "import json,sys
for l in open('gpurun_out/ab_$v$i.log'):
    if l.startswith('{'): d=json.loads(l); print('$v$i', d['value'], d['ms_per_step'])"
  done
done
