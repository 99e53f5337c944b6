#!/bin/bash
# Build libivc.so from a git revision (or "work" = the working tree) into ab/<name>.so for
# same-process A/B timing on the GPU box (tools/ab/ab_intra.py).  ab/ is git-ignored (*.so).
set -e
REV=$1; NAME=$2; shift 2
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
SRC=$(mktemp -d)
mkdir -p "$SRC/ivclab_amd"
if [ "$REV" = work ]; then
  cp -r "$ROOT/ivclab_amd/csrc" "$SRC/ivclab_amd/" && cp -r "$ROOT/include" "$SRC/"
else
  mkdir -p "$SRC/ivclab_amd/csrc" "$SRC/include"
  for f in $(git -C "$ROOT" ls-tree --name-only "$REV" ivclab_amd/csrc/ include/); do
    git -C "$ROOT" show "$REV:$f" > "$SRC/$f"
  done
fi
mkdir -p "$ROOT/ab"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math \
  "$@" -o "$ROOT/ab/$NAME.so" "$SRC"/ivclab_amd/csrc/*.hip
rm -rf "$SRC"
echo "built ab/$NAME.so"
