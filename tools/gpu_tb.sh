cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/tile_bodies.py --vacuum > gpurun_out/tb_vac.log 2>&1 || exit $?
grep -E "^mask|body . *: [1-9]|^tile: " gpurun_out/tb_vac.log | awk '!seen[$0]++'
timeout -k 10 300 python tools/tile_bodies.py --size 256 > gpurun_out/tb_256.log 2>&1 || exit $?
grep -E "^mask|body . *: [1-9]|^tile: " gpurun_out/tb_256.log | awk '!seen[$0]++'
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/tb_bench.json 2> gpurun_out/tb_bench.err || exit $?
python -c "
import json; d=json.load(open('gpurun_out/tb_bench.json'))
print(d['ms_per_step'], d['config']['model_fraction_of_peak'], d['roofline']['avg_launch_ms'])
for k,v in d['configs'].items(): print(k, v.get('ms_per_step'), v.get('model_fraction_of_peak'), v['roofline']['avg_launch_ms'], v['roofline'].get('general_kernel',{}).get('avg_launch_ms'))
"
timeout -k 10 600 python -u -m pytest tests/test_gpu_nr_defer.py -x -q --timeout 500 --timeout-method thread -rf > gpurun_out/nr_defer.log 2>&1; tail -3 gpurun_out/nr_defer.log
