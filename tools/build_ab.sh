#!/bin/bash
# Build A/B variants of librtamd.so with extra device defines: raytracert_amd/ab/lib_<name>.so.
# (kernel flags as the Makefile: KFLAGS -fno-slp-vectorize)
# Usage: tools/build_ab.sh name1 "-DFOO=1 -DBAR=2" name2 "-DFOO=2" ...   (run on the CPU host)
set -e
cd "$(dirname "$0")/../raytracert_amd"
mkdir -p ab build
rm -f ab/lib_*.so
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -I../include -Icsrc -Ibuild"
while [ $# -ge 2 ]; do
  N=$1; D=$2; shift 2
  /opt/rocm/bin/hipcc $HIPFLAGS $D -c csrc/rt_kernels.hip -o ab/k_$N.o &
  # BVH builder knobs (RT_BVH_*) need their own bvh.o
  case "$D" in *RT_BVH_*) /opt/rocm/bin/hipcc $HIPFLAGS -pthread $D -c csrc/bvh.cpp -o ab/b_$N.o & ;; esac
done
wait
for o in ab/k_*.o; do
  N=${o#ab/k_}; N=${N%.o}
  B=build/bvh.o; [ -f ab/b_$N.o ] && B=ab/b_$N.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o ab/lib_$N.so $o build/rt_capi.o build/rt_comm.o build/scene_loader.o build/obj_parallel.o $B -ldl
  rm -f $o ab/b_$N.o
done
ls ab
