#!/bin/bash
# Build a variant of libnkhip.so whose fused Arnoldi kernel is compiled with extra flags:
#   scripts/arn_variant_build.sh <name> [hipcc flags...]  ->  nkhip/libnkhip_<name>.so
# (e.g. -DARN_NV_ONLY=24 for a one-basis-length build in seconds); A/B on the GPU box with
# scripts/arn_variants.sh.  Needs the objects of a normal `make` in build/.
set -e
name=$1; shift
cd "$(dirname "$0")/../iterative-solvers-summer-2020_amd"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I/opt/rocm/include "$@" \
    -c csrc/arnoldi.hip -o build/arnoldi_$name.o
objs=$(ls build/*.o | grep -v 'arnoldi' ; echo build/arnoldi_$name.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o nkhip/libnkhip_$name.so $objs \
    -L/opt/rocm/lib -lrccl -lamdhip64 -Wl,-rpath,/opt/rocm/lib
echo "built nkhip/libnkhip_$name.so"
