#!/bin/bash
# Build A/B variants of liblgs_hip.so with extra -D flags into ablib/ab_<name>.so
# (loaded by bench.py / tests through LGS_LIB).  Usage: tools/ab_build.sh name "-DFLAG=1 ..."
set -e
cd "$(dirname "$0")/../my-lidar-graph-slam_amd/csrc"
name=$1; shift
OUT=/tmp/abbuild/ab_$name
mkdir -p ../../ablib /tmp/abbuild
mkdir -p $OUT
FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -fno-fast-math -fno-gpu-rdc -Wno-unused-result -Wno-unused-value -I../../include -I. $*"
for f in *.hip; do
  /opt/rocm/bin/hipcc $FLAGS -c -o $OUT/${f%.hip}.o $f &
done
g++ -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -c -o $OUT/host_simd.o host_simd.cpp &
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT.so $OUT/*.o && mv $OUT.so ../../ablib/ab_$name.so
rm -rf $OUT
echo built ablib/ab_$name.so
