#!/bin/bash
# Build the engine library of git revision $1 (default HEAD) into
# tools/ab/libbase.so, for interleaved A/B runs against the working tree
# (tools/ab.sh).  CPU only (hipcc cross-compiles for gfx950).
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
D=$(mktemp -d)
mkdir -p $D/esslivedata_amd/csrc $D/include tools/ab
for f in $(git ls-tree --name-only $REV esslivedata_amd/csrc/) include/lde.h; do git show $REV:$f > $D/$f; done
objs=""
for f in $D/esslivedata_amd/csrc/*.hip $D/esslivedata_amd/csrc/*.cpp; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$D/include -c $f -o $f.o &
  objs="$objs $f.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined -Wl,-Bsymbolic $objs -o tools/ab/libbase.so
rm -rf $D
echo tools/ab/libbase.so from $REV
