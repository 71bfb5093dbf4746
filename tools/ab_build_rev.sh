#!/bin/bash
# Build the library of git revision <rev> as an A/B variant abvar/libflcodec_<tag>.so
# (loaded with FLC_LIB_VARIANT=<tag>; its C ABI must match the tree's).   usage: tools/ab_build_rev.sh <rev> <tag>
set -e
rev=$1; tag=$2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=/tmp/abrev_$tag
rm -rf $tmp && mkdir -p $tmp
git -C $root archive $rev flpytorch_amd/csrc include | tar -x -C $tmp
mkdir -p $root/abvar
make -s -j8 -C $tmp/flpytorch_amd/csrc BUILD=$tmp/build OUT=$root/abvar/libflcodec_$tag.so
echo "built abvar/libflcodec_$tag.so from $(git -C $root rev-parse --short $rev)"
