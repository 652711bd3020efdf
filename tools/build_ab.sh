#!/usr/bin/env bash
# Build an A/B variant of the product library into a3-reliable-transport_amd/lib/ab/<name>.so
#   tools/build_ab.sh <name> [extra hipcc flags...]      (current source)
#   AB_REV=<git rev> tools/build_ab.sh <name> [flags]    (the kernel sources at a revision)
set -eu
cd "$(dirname "$0")/.."
name="$1"; shift
PKG=a3-reliable-transport_amd
SRC=$PKG/csrc
if [ -n "${AB_REV:-}" ]; then
  SRC=$(mktemp -d)
  for f in crc32_kernels.hip wtp_host.cpp crc32_math.hpp; do git show "$AB_REV:$PKG/csrc/$f" > "$SRC/$f"; done
fi
mkdir -p $PKG/lib/ab $PKG/build/ab
F="-O3 -std=c++20 -fPIC --offload-arch=gfx950 -I$PWD/include -DWTP_AB_BUILD=1 $*"
/opt/rocm/bin/hipcc $F -c -o $PKG/build/ab/$name.k.o $SRC/crc32_kernels.hip
/opt/rocm/bin/hipcc $F -x hip -c -o $PKG/build/ab/$name.h.o $SRC/wtp_host.cpp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $PKG/lib/ab/$name.so $PKG/build/ab/$name.k.o $PKG/build/ab/$name.h.o
echo "built $PKG/lib/ab/$name.so"
