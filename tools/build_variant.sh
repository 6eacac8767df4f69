#!/bin/bash
# Build libcrnn_hip_<name>.so from the current objects with linear.hip recompiled under extra flags
# (GEMM-template A/B without a full rebuild):  tools/build_variant.sh <name> -DKEY=V ...
set -e
name=$1; shift
cd "$(dirname "$0")/../rcnn-ocr_amd/csrc"
obj=../../build/obj_$name
mkdir -p $obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -Wno-unused-result "$@" -c linear.hip -o $obj/linear.o
objs=$(ls ../../build/obj/*.o | grep -v /linear.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../crnn_hip/libcrnn_hip_$name.so $objs $obj/linear.o
