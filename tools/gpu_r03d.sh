#!/bin/bash
# Round-3: per-body timing of the tile kernel (tools/tile_bodies.py) in the default build
# and in a build whose tile kernel holds the lean body only (register-allocation effect);
# 512^3 waveguide, 512^3 vacuum, 256^3 C2.
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python tools/tile_bodies.py > gpurun_out/r03d_tb_wg.log 2>&1 || exit $?
timeout -k 10 300 python tools/tile_bodies.py --vacuum > gpurun_out/r03d_tb_vac.log 2>&1 || exit $?
timeout -k 10 300 python tools/tile_bodies.py --vacuum --size 256 > gpurun_out/r03d_tb_c2.log 2>&1 || exit $?
MNL_LIB_VARIANT=lean1 timeout -k 10 300 python tools/tile_bodies.py > gpurun_out/r03d_tb_wg_lean1.log 2>&1 || exit $?
MNL_LIB_VARIANT=lean1 timeout -k 10 300 python tools/tile_bodies.py --vacuum > gpurun_out/r03d_tb_vac_lean1.log 2>&1 || exit $?
grep -H "^mask" gpurun_out/r03d_tb_*.log
