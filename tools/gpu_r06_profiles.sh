#!/bin/bash
# Round-6 profiles of the current kernel source (one gpurun call): rocprofv3 kernel-trace stats
# and the FETCH_SIZE / WRITE_SIZE passes (separate runs; never combined with traces) of the 512^3
# headline pair, the flux bench and the 256^3 sub-configs; summaries on the CPU side with
# tools/pmc_pairs.py (pairs) and tools/pmc_summary.py (one-step configs).
#   gpurun --timeout 1200 -- 'bash tools/gpu_r06_profiles.sh [tags...]'
cd "$(dirname "$0")/.." || exit 1
H="--no-cpu --no-extra --no-tune --steps 20 --warmup 4 --no-smi"
set -e
ALL=" $* "
want() { [ "$ALL" = "  " ] || [[ "$ALL" == *" $1 "* ]]; }
run3() {  # tag, env, args
  bash tools/gpu.sh "prof:$1:$2:$3" "pmce:$1_fetch:${2:-X=0}:FETCH_SIZE:$3" "pmce:$1_write:${2:-X=0}:WRITE_SIZE:$3"
}
if want 512; then run3 r06p_512 "" "$H"; fi
if want flux4; then run3 r06p_flux4 "" "$H --flux 4 --nfreq 50"; fi
if want c2; then run3 r06p_c2 "" "--workload c2 --size 256 $H"; fi
if want kerr; then run3 r06p_kerr_1s "MNL_TB_POL=0" "--workload kerr --size 256 $H"; fi
if want kerrtb; then run3 r06p_kerr_tb "" "--workload kerr --size 256 $H"; fi
if want kerrnr; then run3 r06p_kerr_nr "" "--workload kerr_nr --size 256 $H"; fi
echo "profiles done"
