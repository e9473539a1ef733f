cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for B in 1 4 16; do
  MNL_DFT_BLOCK=$B timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pv$B -o run --output-format csv -- python3 bench.py --steps 32 --warmup 3 --flux 4 --nfreq 50 --no-cpu > gpurun_out/pv$B.log 2>&1 || exit 1
done
