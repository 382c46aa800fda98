#!/bin/bash
# A/B baseline: libmj423gpu.so of an earlier commit, built from `git archive` (build container):
#   tools/build_commit.sh COMMIT NAME  -> tools/variants/NAME/libmj423gpu.so (git-ignored, travels to the box)
set -e
commit=$1; name=$2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$commit" mjpeg423-video-decoder-software_amd include | tar -x -C "$tmp"
make -C "$tmp/mjpeg423-video-decoder-software_amd" -j8 libmj423gpu.so > /dev/null
mkdir -p "$root/tools/variants/$name"
cp "$tmp/mjpeg423-video-decoder-software_amd/libmj423gpu.so" "$root/tools/variants/$name/"
rm -rf "$tmp"
echo "$root/tools/variants/$name/libmj423gpu.so"
