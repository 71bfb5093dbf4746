#!/bin/bash
# Build libflcodec from a git revision into flpytorch_amd/libflcodec_<tag>.so (for A/B timing
# against the working tree's build on the same GPU box).   usage: tools/ab_build.sh <rev> <tag> [--tuning]
# --tuning: a -DFLC_TUNING build, the only kind that reads the FLC_* layout / probe switches
set -e
rev=$1; tag=$2; tune=${3:+TUNING=1}
root=$(cd "$(dirname "$0")/.." && pwd)
wt=/tmp/flc_ab_$tag
rm -rf "$wt"; git -C "$root" worktree prune
git -C "$root" worktree add --detach "$wt" "$rev" > /dev/null
make -C "$wt/flpytorch_amd/csrc" -j8 $tune > /dev/null
cp "$wt/flpytorch_amd/libflcodec${tune:+_tuning}.so" "$root/flpytorch_amd/libflcodec_$tag.so"
git -C "$root" worktree remove --force "$wt"
echo "built $rev -> flpytorch_amd/libflcodec_$tag.so"
