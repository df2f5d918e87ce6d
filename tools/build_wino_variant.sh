#!/bin/bash
# A/B builds of librrin_hip.so that differ only in one source's compile flags:
#   tools/build_wino_variant.sh NAME "FLAGS" [SRC (default conv_wino)]  ->  ab/librrin_hip_NAME.so
set -e
cd "$(dirname "$0")/.."
make -s -j8 >/dev/null 2>&1 || make -j8
mkdir -p build/ab ab
NOPK="-Xclang -target-feature -Xclang -packed-fp32-ops"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Iinclude $NOPK $2 \
  -c rrin_amd/csrc/${3:-conv_wino}.hip -o build/ab/${3:-conv_wino}_$1.o 2>&1 | grep -v "recognized feature" || true
objs=$(ls build/obj/*.o | grep -v "/${3:-conv_wino}.o")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ab/librrin_hip_$1.so $objs build/ab/${3:-conv_wino}_$1.o
echo "ab/librrin_hip_$1.so"
