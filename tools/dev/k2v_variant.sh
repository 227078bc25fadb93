#!/bin/bash
# K2V measurement variant: align_refv.hip rebuilt with extra -D flags into build/<dir>/libsvo_hip.so (the other objects
# from build/), after the same VGPR-fence and wait-state checks as the product build.
# usage: [SRC=other.hip] tools/dev/k2v_variant.sh <dir> -DFOO=1 ...   then SVO_LIB_DIR=semi-direct-visual-odometry_amd/build/<dir>
set -e
cd "$(dirname "$0")/../../semi-direct-visual-odometry_amd"
d=build/$1; shift
mkdir -p "$d"
F="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Wall -Wno-unused-function -Wno-unused-result"
src=${SRC:-csrc/align_refv.hip}
/opt/rocm/bin/hipcc $F "$@" -I csrc --cuda-device-only -S -o "$d/align_refv.s" "$src"
python3 ../tools/check_vreg_fence.py "$d/align_refv.s" > /dev/null
python3 ../tools/check_wait_states.py "$d/align_refv.s" > /dev/null
/opt/rocm/bin/hipcc $F "$@" -I csrc -c -o "$d/align_refv.o" "$src"
objs=$(ls build/*.o | grep -v align_refv.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$d/libsvo_hip.so" $objs "$d/align_refv.o"
echo "built $d"
