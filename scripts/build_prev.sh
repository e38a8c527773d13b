#!/bin/bash
# Build the library of an earlier commit as tools/libagn_prev.so for in-process
# A/B runs (scripts/ab_prev.py): -Bsymbolic keeps its internal calls inside
# itself when it is loaded next to the current library.
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$ROOT" archive "$REV" antidote_amd/csrc include | tar -x -C "$T"
cd "$T/antidote_amd/csrc"
make -s -j8 $(ls *.hip | sed 's/\.hip$/.o/; s/^/build\//')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-Bsymbolic -o "$ROOT/tools/libagn_prev.so" \
    build/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$T"
echo "built tools/libagn_prev.so from $REV"
