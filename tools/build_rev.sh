#!/bin/bash
export KB_DIAGNOSTICS=1   # (the engine reads its KB_* switches only with this opt-in)
# Diagnostic: build libkbengine.so of a git revision as kafkabalancer_amd/lib/libkbengine_<name>.so
# (A/B timing against the working tree in one GPU call: tools/exp_step.sh new=- old=libkbengine_<name>.so)
REV=${1:-HEAD}; NAME=${2:-prev}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT" || exit 1
T=$(mktemp -d)
mkdir -p $T/kafkabalancer_amd/csrc $T/include
for f in kernels.hip engine.cpp engine_dev.h kernels_api.h wave_ops.h; do
  git show $REV:kafkabalancer_amd/csrc/$f > $T/kafkabalancer_amd/csrc/$f || exit 1
done
git show $REV:include/kbengine.h > $T/include/kbengine.h || exit 1
(cd $T/kafkabalancer_amd/csrc && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -w -shared \
    -o $ROOT/kafkabalancer_amd/lib/libkbengine_$NAME.so kernels.hip engine.cpp) || exit 1
rm -rf $T
echo built kafkabalancer_amd/lib/libkbengine_$NAME.so
