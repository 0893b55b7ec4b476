#!/bin/bash
# Build an experiment copy of libsrk.so with extra compiler defines, for A/B runs through SRK_LIB:
#   [SRCS="gemm"] tools/build_variant.sh NAME -DFOO=1 ...   ->  tools/_exp/libsrk_NAME.so
# SRCS: basenames (no suffix) of the sources to recompile with the defines; the other objects come
# from the main build (speechrecognitionproject_amd/_build, run the build first).  Default: all.
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/tools/_exp/$name
mkdir -p "$out"
objs=()
for src in "$root"/speechrecognitionproject_amd/csrc/*.hip "$root"/speechrecognitionproject_amd/csrc/*.cpp; do
  base=$(basename "$src"); stem=${base%.*}
  o=$out/$base.o
  if [ -n "$SRCS" ] && [[ " $SRCS " != *" $stem "* ]]; then
    cp "$root/speechrecognitionproject_amd/_build/$base.o" "$o" 2>/dev/null || cp "$root/speechrecognitionproject_amd/_build/$stem.o" "$o"
  else
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -mllvm -disable-promote-alloca-to-lds \
      -I "$root/include" "$@" -c "$src" -o "$o" &
  fi
  objs+=("$o")
done
objs+=("$root/speechrecognitionproject_amd/_build/stamp.cpp.o")   # srk_source_stamp (the main build's)
for job in $(jobs -p); do wait "$job" || { echo "variant $name: a compile failed" >&2; exit 1; }; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 "${objs[@]}" -o "$root/tools/_exp/libsrk_$name.so"
echo "$root/tools/_exp/libsrk_$name.so"
