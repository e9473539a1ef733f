#!/bin/bash
# Build an experimental kernel variant into meep_nl_amd/variants/<name>/libmnl.so
#   tools/build_variant.sh <name> "<hipcc -D flags>"
# Select it at run time with MNL_LIB_VARIANT=<name> (meep_nl_amd/_lib.py).
set -e
cd "$(dirname "$0")/.."
mkdir -p meep_nl_amd/variants/$1/_obj
MNL_OUT=$PWD/meep_nl_amd/variants/$1/libmnl.so MNL_OBJ=$PWD/meep_nl_amd/variants/$1/_obj \
  MNL_KFLAGS="$2" bash meep_nl_amd/csrc/build.sh
