#!/bin/bash
# Build meep_nl_amd/libmnl.so for gfx950 (MI355X).  hipcc for the kernels,
# g++ for the host side (see mnl_host.cpp header for why): mnl_host.cpp (orchestration, C-ABI),
# mnl_dft.cpp (DFT monitors), mnl_io.cpp (checkpoints, slices, energy), mnl_comm.cpp (RCCL / IPC).
set -e
HERE="$(cd "$(dirname "$0")" && pwd)"
OUT=${MNL_OUT:-"$HERE/../libmnl.so"}
ROCM=${ROCM_PATH:-/opt/rocm}
TMP=${MNL_OBJ:-"$HERE/_obj"}
mkdir -p "$TMP"
ARCH=${MNL_ARCH:-gfx950}
hipcc --offload-arch=$ARCH $MNL_KFLAGS -O3 -ffp-contract=off -fPIC -std=c++17 -Wall \
  -c "$HERE/mnl_kernels.hip" -o "$TMP/mnl_kernels.o"
CXXF="$MNL_KFLAGS -O2 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -Wall -Wno-unused-result -D__HIP_PLATFORM_AMD__ -I$ROCM/include"
g++ $CXXF -c "$HERE/mnl_host.cpp" -o "$TMP/mnl_host.o"
g++ $CXXF -c "$HERE/mnl_dft.cpp" -o "$TMP/mnl_dft.o"
g++ $CXXF -c "$HERE/mnl_io.cpp" -o "$TMP/mnl_io.o"
g++ $CXXF -c "$HERE/mnl_comm.cpp" -o "$TMP/mnl_comm.o"
# Link with g++ so the host's complex arithmetic (__muldc3 / __divdc3 of
# std::complex) comes from libgcc as in the reference (and the oracle), not
# from clang's compiler-rt, whose complex division rounds differently.
g++ -shared -fPIC -o "$OUT" "$TMP/mnl_kernels.o" "$TMP/mnl_host.o" "$TMP/mnl_dft.o" "$TMP/mnl_io.o" "$TMP/mnl_comm.o" \
  -L$ROCM/lib -lamdhip64 -lrccl -lrt -Wl,-rpath,$ROCM/lib
echo "built $OUT"
