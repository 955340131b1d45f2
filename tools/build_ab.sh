#!/bin/bash
# Build the library from csrc/ as of git revision REV into camels-diffusion-model_amd/lib/ab/<name>.so, for A/B timing
# on one GPU box (CDM_LIB=<that path> python bench.py ...).   bash tools/build_ab.sh REV NAME
set -e
REV=$1; NAME=$2
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p $T/csrc $T/include
git -C $R archive $REV camels-diffusion-model_amd/csrc include | tar -x -C $T
mkdir -p $R/camels-diffusion-model_amd/lib/ab
objs=""
for f in $T/camels-diffusion-model_amd/csrc/*.hip; do
  o=$T/$(basename $f).o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $EXTRA -I $T/camels-diffusion-model_amd/csrc -I $T/include -Wno-unused-result -c $f -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o $R/camels-diffusion-model_amd/lib/ab/$NAME.so
rm -rf $T
echo built $R/camels-diffusion-model_amd/lib/ab/$NAME.so
