#!/bin/bash
# Build the current csrc tree as an A/B variant library abvar/libflcodec_<tag>.so (loaded
# with FLC_LIB_VARIANT=<tag>); the product libflcodec.so is untouched.   usage: [XFLAGS=-D...] tools/ab_build.sh <tag>
set -e
tag=$1
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=/tmp/ab_$tag
rm -rf $tmp && mkdir -p $tmp/flpytorch_amd $tmp/include
cp -r $root/flpytorch_amd/csrc $tmp/flpytorch_amd/ && rm -rf $tmp/flpytorch_amd/csrc/build $tmp/flpytorch_amd/csrc/build_tuning
cp $root/include/flcodec.h $tmp/include/
mkdir -p $root/abvar
make -s -j8 -C $tmp/flpytorch_amd/csrc BUILD=$tmp/build OUT=$root/abvar/libflcodec_$tag.so XFLAGS="$XFLAGS"
echo "built abvar/libflcodec_$tag.so"
