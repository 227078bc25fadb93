# a K2V variant library (argument 1: name, the rest: extra hipcc flags, e.g. -DSVO_QG=8) under
# semi-direct-visual-odometry_amd/build/var_<name>: align_refv rebuilt (fence and wait-state checked), the other objects
# taken from the product build; used by the same-box A/B scripts of this directory
set -e
cd /root/repo/semi-direct-visual-odometry_amd
D=build/var_$1; shift
mkdir -p $D
F="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Wall -Wno-unused-function -Wno-unused-result $*"
/opt/rocm/bin/hipcc $F --cuda-device-only -S -o $D/align_refv.s csrc/align_refv.hip
python3 ../tools/check_vreg_fence.py $D/align_refv.s > $D/fence.txt
python3 ../tools/check_wait_states.py $D/align_refv.s >> $D/fence.txt
/opt/rocm/bin/hipcc $F -c -o $D/align_refv.o csrc/align_refv.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libsvo_hip.so build/capi.o build/align.o build/align_ref.o $D/align_refv.o build/pyramid.o build/feature_align.o build/depth_filter.o build/feature_select.o build/pose_ba.o
cp build/libsvo_synth.so $D/ 
echo built $D
