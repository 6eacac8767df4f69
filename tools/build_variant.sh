#!/bin/bash
# Build libcrnn_hip_<name>.so from the current objects with some sources recompiled under extra flags
# (A/B without touching the default library):  SRCS="conv.hip" tools/build_variant.sh <name> -DKEY=V ...
# (SRCS defaults to linear.hip)
set -e
name=$1; shift
srcs=${SRCS:-linear.hip}
cd "$(dirname "$0")/../rcnn-ocr_amd/csrc"
obj=../../build/obj_$name
mkdir -p $obj
skip=""
for s in $srcs; do
  o=$obj/${s%.hip}.o
  # the Makefile's device flags (NOPK: no packed fp32 ops) so that a variant differs only in the flags under test
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -Wno-unused-result \
    -Xclang -target-feature -Xclang -packed-fp32-ops "$@" -c $s -o $o
  skip="$skip|/${s%.hip}.o"
done
objs=$(ls ../../build/obj/*.o | grep -Ev "(${skip#|})$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../crnn_hip/libcrnn_hip_$name.so $objs $obj/*.o
