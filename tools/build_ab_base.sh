#!/bin/bash
# Build a committed revision's kernel library into tools/_ab/libretr_base.so (A/B timing only:
# RETR_AB_LIB=tools/_ab/libretr_base.so makes retr_amd._lib load it instead of the working tree's).
# Uses the working tree's Makefile, so both libraries get the same per-file flags (the attention
# and decode objects' -amdgpu-mfma-vgpr-form: a plain hipcc loop without it gave a base library
# whose attention kernels were ~10 % slower -- it confounded round 6's first base/tree A/Bs).
#   usage: bash tools/build_ab_base.sh [rev]        (default HEAD)
set -e
REPO=$(cd "$(dirname "$0")/.." && pwd)
REV=${1:-HEAD}
TMP=$(mktemp -d)
git -C "$REPO" archive "$REV" retr_amd/csrc include | tar -x -C "$TMP"
mkdir -p "$REPO/tools/_ab"
(cd "$TMP" && make -s -f "$REPO/Makefile" -j8 LIB="$REPO/tools/_ab/libretr_base.so" \
   "$REPO/tools/_ab/libretr_base.so" 2>&1 | grep -E "error" || true)
rm -rf "$TMP"
test -f "$REPO/tools/_ab/libretr_base.so"
echo "built $REPO/tools/_ab/libretr_base.so from $(git -C "$REPO" rev-parse --short "$REV")"
