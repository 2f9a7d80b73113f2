cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for g in 1024 768 512; do
  MW_KBLOCKS=$g timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/grid_$g.json 2>/dev/null || exit 1
  echo "G=$g"; python -c "import json;d=json.load(open('gpurun_out/grid_$g.json'));print(d['ms_per_step']);[print(' ',k,v['mean_ms']) for k,v in d['kernels'].items()]"
done
