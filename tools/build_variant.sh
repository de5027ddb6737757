#!/bin/bash
# Build an A/B variant of libicgpu.so with extra compile definitions:
#   tools/build_variant.sh NAME -DFOO=1 ...   ->  ab/libicgpu_NAME.so (travels with gpurun)
# Load it with IC_LIBRARY=ab/libicgpu_NAME.so (bench.py, tests).
set -e
name=$1; shift
here=$(cd "$(dirname "$0")/.." && pwd)
obj=$(mktemp -d)
cd "$here/iterative_cleaner_amd/csrc"
for f in ic_kernels ic_session ic_comm; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
        -I../../include "$@" -c $f.hip -o "$obj/$f.o"
done
mkdir -p "$here/ab"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$here/ab/libicgpu_$name.so" "$obj"/*.o
rm -rf "$obj"
echo "$here/ab/libicgpu_$name.so"
