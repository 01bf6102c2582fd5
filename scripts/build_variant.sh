#!/bin/bash
# Experiment library from a git revision's sources (A/B against the working tree on one box):
#   scripts/build_variant.sh <name> <rev> [extra hipcc flags]  ->  sclmd_amd/_lib/libhipgle_<name>.so
# e.g. scripts/build_variant.sh base HEAD~1 ; the working tree's own: make experiments EXPNAME=cur
set -eo pipefail
name=${1:?name}; rev=${2:?rev}; shift 2
src=build/src_$name
rm -rf $src && mkdir -p $src/sclmd_amd/csrc $src/include build/$name
for f in $(git ls-tree --name-only $rev sclmd_amd/csrc/) $(git ls-tree --name-only $rev include/); do
  git show $rev:$f > $src/$f
done
objs=""
for f in $src/sclmd_amd/csrc/*.hip; do
  o=build/$name/$(basename ${f%.hip}).o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -Wno-unused-value \
    -DGLE_EXPERIMENTS "$@" -c -o $o $f &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o sclmd_amd/_lib/libhipgle_$name.so $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built sclmd_amd/_lib/libhipgle_$name.so from $rev"
