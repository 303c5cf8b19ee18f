#!/bin/bash
# Build an A/B variant of libpdeinv.so: one kernel source replaced (a file path, or a git revision of the
# in-tree file as REV:path), extra hipcc flags allowed; the other objects are the current in-tree build.
# Usage: [REPLACE=<object basename>] bash tools/build_var.sh <name> <source.hip | REV:csrc-relative-path> [hipcc flags...]
set -e
cd "$(dirname "$0")/.."
B=pde-inverse-problem_amd/_build
C=pde-inverse-problem_amd/csrc
name=$1; src=$2; shift 2
mkdir -p $B/var
case $src in
  *:*) rev=${src%%:*}; f=${src#*:}; git show "$rev:$C/$f" > $C/.var_$name.hip; src=$C/.var_$name.hip; obj=$(basename $f .hip) ;;
  *) obj=${REPLACE:-$(basename $src .hip)} ;;
esac
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -munsafe-fp-atomics \
  -ffp-contract=fast-honor-pragmas -I$C "$@" -c $src -o $B/var/$name.o
objs=$(ls $B/*.o | grep -v "/$obj.o$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs $B/var/$name.o -o $B/var/$name.so -ldl
rm -f $C/.var_$name.hip $B/var/$name.o
echo built $B/var/$name.so
