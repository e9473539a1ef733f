#!/bin/bash
# z-chunk sweep of the fused kernels on the 256^3 configs (C2 vacuum, C4 Kerr)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for wl in vacuum kerr; do
for z in 8 12 16 24; do
  MNL_FUSED_ZCHUNK=$z timeout -k 10 120 python bench.py --size 256 --workload $wl --steps 40 --warmup 5 --no-cpu --no-extra > gpurun_out/z_${wl}_$z.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/z_${wl}_$z.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$wl z=$z', d['ms_per_step'], r['avg_launch_ms'], r['general_kernel']['avg_launch_ms'])"
done
done
