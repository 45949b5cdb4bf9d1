#!/bin/bash
# Build an A/B variant of liblpa_hip.so: the current csrc with sed expressions applied
# (each argument after the name is one `sed -i` program for lpa_iter.hip), into
# build/ab/<name>/liblpa_hip.so (loaded with LPA_LIB_PATH by tools/bench_env_ab.sh).
#   tools/ab_variant.sh <name> 's/a/b/' ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/community-detection-outlier-detection-through-massive-graph-mining-over-apache-spark._amd
name=$1; shift
W=/tmp/abv_$name
rm -rf "$W" && mkdir -p "$W/pkg/csrc" "$W/include" "$ROOT/build/ab/$name"
cp "$PKG"/csrc/*.hip "$PKG"/csrc/*.h "$PKG"/csrc/*.cpp "$PKG"/csrc/Makefile "$W/pkg/csrc/"
cp "$ROOT"/include/*.h "$W/include/"
for e in "$@"; do sed -i "$e" "$W/pkg/csrc/lpa_iter.hip"; done
make -s -C "$W/pkg/csrc" -j8 OUT="$ROOT/build/ab/$name/liblpa_hip.so" BUILD="$W/build" "$ROOT/build/ab/$name/liblpa_hip.so"
echo "built build/ab/$name/liblpa_hip.so"
