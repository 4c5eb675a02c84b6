#!/bin/bash
# Build the library of another revision (default HEAD, i.e. without the working-tree changes) as
# multimodal-pl_amd/u3d/libu3d_ab.so for an A/B run on one box: tools/build_ab.sh [rev]
set -e
REV=${1:-HEAD}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/u3d_ab.XXXX)
git -C "$R" archive "$REV" multimodal-pl_amd/csrc include | tar -x -C "$T"
mkdir -p "$T/multimodal-pl_amd/u3d"
make -s -C "$T/multimodal-pl_amd/csrc" -j8 >/dev/null
cp "$T/multimodal-pl_amd/u3d/libu3d.so" "$R/multimodal-pl_amd/u3d/libu3d_ab.so"
rm -rf "$T"
echo "built $REV -> multimodal-pl_amd/u3d/libu3d_ab.so"
