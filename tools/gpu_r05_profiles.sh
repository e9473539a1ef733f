#!/bin/bash
# Round-5 profiles of the current kernel source (one gpurun call): rocprofv3 kernel stats and the
# FETCH_SIZE / WRITE_SIZE passes (separate runs; never combined with traces) of the 512^3
# headline pair and of the 256^3 sub-configs, then tools/pmc_summary.py on the CPU side.
#   gpurun --timeout 1200 -- 'bash tools/gpu_r05_profiles.sh'
cd "$(dirname "$0")/.." || exit 1
H="--no-cpu --no-extra --no-tune --steps 20 --warmup 4 --no-smi"
set -e
bash tools/gpu.sh "prof:r05p_512::$H" "pmc:r05p_512_fetch:FETCH_SIZE:$H" "pmc:r05p_512_write:WRITE_SIZE:$H"
for wl in c2 kerr kerr_nr; do
  A="--workload $wl --size 256 $H"
  bash tools/gpu.sh "prof:r05p_${wl}::$A" "pmc:r05p_${wl}_fetch:FETCH_SIZE:$A" "pmc:r05p_${wl}_write:WRITE_SIZE:$A"
done
