#!/bin/bash
export KB_DIAGNOSTICS=1   # (the engine reads its KB_* switches only with this opt-in)
# Same-box A/B of the current build against lib/libkbengine_prev.so on one workload:
# usage: gpurun -- 'bash tools/gpu_ab_wl.sh <tag> <workload> <steps>'
set -u
T=$1; W=$2; S=$3
O=gpurun_out/$T
mkdir -p $O
P="env KB_ENGINE_LIB=kafkabalancer_amd/lib/libkbengine_prev.so KB_ABI_ANY=1"
b() { timeout -k 10 300 "$@" --no-cpu-baseline; }
b python bench.py --workload $W --steps $S > $O/${W}_cur1.json 2> $O/e1 &&
b $P python bench.py --workload $W --steps $S > $O/${W}_prev1.json 2> $O/e2 &&
b python bench.py --workload $W --steps $S > $O/${W}_cur2.json 2> $O/e3 &&
b $P python bench.py --workload $W --steps $S > $O/${W}_prev2.json 2> $O/e4
