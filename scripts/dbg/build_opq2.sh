#!/bin/bash
# Diagnostic builds for the ARN_OPQ=2 question (round 6): the bounds-checked library and the
# product library with the stencil coefficients and x0 pinned through "+s" asm constraints.
#   nkhip/libnkhip_check_opq2.so  (-DNKHIP_ARN_CHECK -DARN_OPQ=2)
#   nkhip/libnkhip_opq2.so        (-DARN_OPQ=2)
set -eu
cd "$(dirname "$0")/../../iterative-solvers-summer-2020_amd"
make -s all
FLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-variable -Wno-unused-but-set-variable -Wno-unused-value -Wno-unused-result --offload-arch=gfx950 -I/opt/rocm/include"
OTHERS="build/stencil.o build/krylov.o build/arnctl.o build/droplet.o build/peer.o build/nk_solver.o build/lgmres.o build/sh_problem.o build/droplet_problem.o build/mems_problem.o build/shlin.o build/comm.o build/capi.o"
/opt/rocm/bin/hipcc $FLAGS -DNKHIP_ARN_CHECK -DARN_OPQ=2 -c csrc/arnoldi.hip -o build/arnoldi_check_opq2.o &
/opt/rocm/bin/hipcc $FLAGS -DARN_OPQ=2 -c csrc/arnoldi.hip -o build/arnoldi_opq2.o &
wait
for v in check_opq2 opq2; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o nkhip/libnkhip_$v.so $OTHERS \
      build/arnoldi_$v.o -L/opt/rocm/lib -lrccl -lamdhip64 -Wl,-rpath,/opt/rocm/lib
done
ls -la nkhip/libnkhip_check_opq2.so nkhip/libnkhip_opq2.so
