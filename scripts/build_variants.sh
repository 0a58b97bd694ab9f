#!/bin/bash
# Build tuning variants of libmeshsearch.so into build/variants/<name>.so (CPU container, cross-compile);
# scripts/gpu_check.sh's `variants` stage benches each one (10M C3 queries) via MESH_AMD_LIB.
#   VARIANTS="name:FLAGS;name2:FLAGS2" bash scripts/build_variants.sh
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
[ -n "${KEEP:-}" ] || rm -rf "$R/build/variants"
mkdir -p "$R/build/variants"
IFS=';' read -ra VS <<< "${VARIANTS:?set VARIANTS}"
for v in "${VS[@]}"; do
  name=${v%%:*}
  flags=${v#*:}
  make -s -j8 -C "$R/mesh_amd/csrc" BUILD="$R/build/v_$name" OUT="$R/build/variants/$name.so" EXTRA="$flags"
  echo "built $name ($flags)"
done
