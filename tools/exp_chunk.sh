cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/exp1
for v in c4 c8 c16 ""; do
  if [ -n "$v" ]; then export DDR_LIB=$PWD/ddr_amd/lib/libddr_mc_$v.so; else unset DDR_LIB; fi
  timeout -k 10 180 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/exp1/b_$v.log 2>&1 || exit $?
  echo "$v" $(grep '^{' gpurun_out/exp1/b_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels'])")
done
