#!/bin/bash
export KB_DIAGNOSTICS=1   # (the engine reads its KB_* switches only with this opt-in)
# Same-box A/B of the current build against other builds in lib/ (libkbengine_<v>.so):
# c3 bench lines alternated so box drift shows.  Usage: gpurun -- 'bash tools/gpu_ab.sh <tag> v1 v2 ...'
set -u
T=${1:-x}; shift
O=gpurun_out/$T
mkdir -p $O
b() { timeout -k 10 300 "$@" --no-cpu-baseline; }
ok=0
for rep in 1 2; do
  b python bench.py --steps 1000 > $O/c3_cur$rep.json 2> $O/err_cur$rep || exit 1
  for v in "$@"; do
    KB_ENGINE_LIB=kafkabalancer_amd/lib/libkbengine_$v.so KB_ABI_ANY=1 b python bench.py --steps 1000 > $O/c3_$v$rep.json 2> $O/err_$v$rep || exit 1
  done
done
