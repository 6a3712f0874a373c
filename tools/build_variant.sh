#!/bin/bash
# Build the product library from a source tree with extra compile flags into abl/<name>/; copy it to
# abv/libpitt_seg_<name>.so for tools/gpu_ab.sh: bash tools/build_variant.sh <name> "<-D flags>" [source csrc dir]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; FLAGS=$2; SRC=${3:-$ROOT/pitt_object_table_segmentation_amd/csrc}
mkdir -p "$ROOT/abl/$NAME"
make -C "$SRC" -j8 BUILD="build_v_$NAME" OUT="$ROOT/abl/$NAME" EXTRA="$FLAGS" all
