#!/bin/bash
# Build libptmi.so from a git revision as an A/B variant (not product):
#   bash tools/build_ref_variant.sh REV NAME [DEFS]
# -> path-tracer-python_amd/ptmi/_lib/variants/libptmi_NAME.so, compiled from
#    REV's csrc/ and include/ with REV's Makefile flags (plus DEFS).
set -eu
REV=$1; NAME=$2; DEFS=${3:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d /tmp/ptmi_ref.XXXXXX)
git -C "$ROOT" archive "$REV" path-tracer-python_amd/csrc include | tar -x -C "$TMP"
OUT="$ROOT/path-tracer-python_amd/ptmi/_lib/variants"
mkdir -p "$OUT"
make -s -C "$TMP/path-tracer-python_amd/csrc" variant NAME="$NAME" DEFS="$DEFS" VOUT="$TMP/out" > /dev/null
cp "$TMP/out/libptmi_$NAME.so" "$OUT/libptmi_$NAME.so"
rm -rf "$TMP"
echo "$OUT/libptmi_$NAME.so"
