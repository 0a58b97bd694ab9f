#!/bin/bash
# Build libmeshsearch.so variants that differ in SOURCE files (CPU container, cross-compile): for each
# "name:dir" the tree mesh_amd/csrc is copied to build/src_<name>/mesh_amd/csrc, the files in `dir` replace
# their namesakes, and the copy is built into build/variants/<name>.so (EXTRA flags after a second colon).
#   VARIANTS="base:/tmp/v_base;line:/tmp/v_line:-DFOO=1" bash scripts/build_src_variants.sh
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
[ -n "${KEEP:-}" ] || rm -rf "$R/build/variants" "$R"/build/src_*
mkdir -p "$R/build/variants"
IFS=';' read -ra VS <<< "${VARIANTS:?set VARIANTS}"
for v in "${VS[@]}"; do
  IFS=':' read -r name dir flags <<< "$v"
  S="$R/build/src_$name"
  rm -rf "$S"
  mkdir -p "$S/mesh_amd" "$S/include"
  cp -r "$R/mesh_amd/csrc" "$S/mesh_amd/csrc"
  cp "$R/include/meshsearch.h" "$S/include/"
  [ -n "$dir" ] && cp "$dir"/* "$S/mesh_amd/csrc/"
  make -s -j8 -C "$S/mesh_amd/csrc" BUILD="$S/obj" OUT="$R/build/variants/$name.so" EXTRA="${flags:-}"
  echo "built $name (sources: ${dir:-tree}, flags: ${flags:-none})"
done
