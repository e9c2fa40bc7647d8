#!/bin/bash
# Build the product library of another source state for a same-box A/B:
#   tools/build_variant.sh <git-rev> <name>  ->  tiledb_amd/libtiledb_amd_<name>.so
# (load it with TDBG_LIB=libtiledb_amd_<name>.so; never shipped)
set -e
REV=$1; NAME=$2
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/tdbg_var_XXXX)
git -C "$R" archive "$REV" tiledb_amd/csrc tiledb_amd/build.py tiledb_amd/__init__.py include | tar -x -C "$T"
(cd "$T" && python3 -c "import sys; sys.path.insert(0, 'tiledb_amd'); import build; build.build(force=True)")
cp "$T/tiledb_amd/libtiledb_amd.so" "$R/tiledb_amd/libtiledb_amd_$NAME.so"
rm -rf "$T"
echo "built tiledb_amd/libtiledb_amd_$NAME.so from $REV"
