#!/bin/bash
# Build an A/B variant of libicgpu.so from the current sources plus a patch
# (a probe or an alternative kept out of the product sources):
#   tools/build_patched.sh NAME tools/patches/X.patch [more patches...]  ->  ab/libicgpu_NAME.so
# Load it with IC_LIBRARY=ab/libicgpu_NAME.so (bench.py, tools/ab_lib_args.sh).
set -e
name=${1:?name}; shift
here=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
mkdir -p "$tmp/x"
cp -r "$here/include" "$tmp/"
cp -r "$here/iterative_cleaner_amd/csrc" "$tmp/x/csrc"
rm -f "$tmp"/x/csrc/*.o "$tmp"/x/csrc/*.s
for p in "$@"; do
    (cd "$tmp/x/csrc" && patch -p1 --quiet < "$here/$p")
done
mkdir -p "$here/ab"
make -s -C "$tmp/x/csrc" -j8 OUT="$here/ab/libicgpu_$name.so"
rm -rf "$tmp"
echo "$here/ab/libicgpu_$name.so"
