#!/bin/bash
# Build the working tree's library with extra compiler flags into multimodal-pl_amd/u3d/<name>.so (diagnostic
# builds, e.g. -DU3D_WRING_M16=0): tools/build_variant.sh NAME "FLAGS"
set -e
NAME=$1; FLAGS=$2
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/u3d_var.XXXX)
mkdir -p "$T/multimodal-pl_amd/u3d"
cp -r "$R/multimodal-pl_amd/csrc" "$T/multimodal-pl_amd/" && rm -rf "$T/multimodal-pl_amd/csrc/build"
cp -r "$R/include" "$T/"
make -s -C "$T/multimodal-pl_amd/csrc" -j8 CXXFLAGS_EXTRA="$FLAGS" >/dev/null
cp "$T/multimodal-pl_amd/u3d/libu3d.so" "$R/multimodal-pl_amd/u3d/$NAME.so"
rm -rf "$T"
echo "built working tree + [$FLAGS] -> multimodal-pl_amd/u3d/$NAME.so"
