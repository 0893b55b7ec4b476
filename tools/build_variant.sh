#!/bin/bash
# Build an experiment copy of libsrk.so with extra compiler defines, for A/B runs through SRK_LIB:
#   tools/build_variant.sh NAME -DFOO=1 ...   ->  tools/_exp/libsrk_NAME.so
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/tools/_exp/$name
mkdir -p "$out"
objs=()
for src in "$root"/speechrecognitionproject_amd/csrc/*.hip "$root"/speechrecognitionproject_amd/csrc/*.cpp; do
  o=$out/$(basename "$src").o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -mllvm -disable-promote-alloca-to-lds \
    -I "$root/include" "$@" -c "$src" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 "${objs[@]}" -o "$root/tools/_exp/libsrk_$name.so"
echo "$root/tools/_exp/libsrk_$name.so"
