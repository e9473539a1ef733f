cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/pmcb; mkdir -p $OUT
for m in 1 2; do
  for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_FLAT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR" "FETCH_SIZE" "WRITE_SIZE"; do
    n=$(echo $pass | cut -d' ' -f1)
    MNL_TILE_BODY_MASK=$m timeout -s KILL 120 rocprofv3 --pmc $pass -d $OUT/m${m}_$n -o run --output-format csv -- python3 tools/tile_one.py --vacuum > $OUT/m${m}_$n.log 2>&1 || { echo "fail $m $n"; tail -5 $OUT/m${m}_$n.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, collections
for m in (1, 2):
    agg = collections.defaultdict(float); cnt = collections.defaultdict(int)
    for fn in glob.glob(f'gpurun_out/pmcb/m{m}_*/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(fn)):
            if 'fused_tile_kernel' not in r['Kernel_Name']: continue
            agg[r['Counter_Name']] += float(r['Counter_Value']); cnt[r['Counter_Name']] += 1
    print('mask', m, {k: round(v / max(1, cnt[k] / max(1, 1)) ) for k, v in sorted(agg.items())})
    print('   dispatch-rows', dict(cnt))
PY
