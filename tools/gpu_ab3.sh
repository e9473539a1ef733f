cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
V1=MNL_TILE_STEP=0
V2=MNL_TILE_STEP=1,MNL_ZCUT_STEP=1,MNL_ZCHUNK_STEP=0
V3=MNL_TILE_STEP=1,MNL_ZCUT_STEP=0,MNL_ZCHUNK_STEP=0
timeout -k 10 400 python tools/ab_inproc.py $V1 $V2 $V3 -- --vacuum > gpurun_out/ab3_vac.log 2>&1 || exit $?
cat gpurun_out/ab3_vac.log
timeout -k 10 400 python tools/ab_inproc.py $V1 $V2 $V3 > gpurun_out/ab3_wg.log 2>&1 || exit $?
cat gpurun_out/ab3_wg.log
timeout -k 10 400 python tools/ab_inproc.py $V1 $V2 $V3 -- --workload c2 --size 256 > gpurun_out/ab3_c2.log 2>&1 || exit $?
cat gpurun_out/ab3_c2.log
timeout -k 10 400 python tools/ab_inproc.py $V1 $V2 $V3 -- --workload kerr --size 256 > gpurun_out/ab3_kerr.log 2>&1 || exit $?
cat gpurun_out/ab3_kerr.log
timeout -k 10 300 python tools/tile_bodies.py --vacuum > gpurun_out/tb_vac.log 2>&1 || exit $?
grep -E "^mask|body . *: [1-9]|^tile: " gpurun_out/tb_vac.log | awk '!seen[$0]++'
