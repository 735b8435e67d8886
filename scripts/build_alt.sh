#!/bin/bash
# Build an A/B variant of the kernel library: the in-tree objects with ONE source replaced.
#   bash scripts/build_alt.sh <variant.hip> <replaced-object-name> [outdir]
# e.g. bash scripts/build_alt.sh /tmp/vE.hip hw_scan foremast_amd/ops/_lib/ab
set -eu
cd "$(dirname "$0")/.."
src=$1; name=$2; out=${3:-foremast_amd/ops/_lib/ab}
python -m foremast_amd.ops.build > /dev/null
mkdir -p "$out"
F="-O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=fast -munsafe-fp-atomics -Wno-unused-result -Werror=return-type"
cp "$src" "$out/$name.hip"   # compiled from $out: its includes resolve to csrc/, not to the source's directory
/opt/rocm/bin/hipcc $F -I foremast_amd/ops/csrc -c "$out/$name.hip" -o "$out/$name.o"
objs=$(ls foremast_amd/ops/_lib/obj/*.o | grep -v "/$name.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/libforemast_hip.so" $objs "$out/$name.o"
echo "$out/libforemast_hip.so"
